// CPU-baseline timers of the oracle restatement for bench.py (test infrastructure):
// the configurations whose CPU path is not a plain extract + ComputeStereoMatches.
//   config 4: the TUM-VI KannalaBrandt8 stereo Frame (Frame.cc:1034-1125): ExtractORB of the left and
//             right image with vLappingArea {0, 511} (:1059-1062; two std::threads in the reference's
//             split), then ComputeStereoFishEyeMatches' descriptor stage (:1126-1151: knnMatch(k = 2) of
//             the lapping rows + the 0.7 ratio test); the KannalaBrandt8 TriangulateMatches after it is
//             the camera model's and not timed on either side.
#include <chrono>
#include <cstdint>
#include <thread>
#include <vector>

#include "../include/orbfe.h"

extern "C" {
void* oro_create(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh);
void oro_destroy(void* h);
int oro_extract(void* h, const uint8_t* img, int w, int hgt, int stride, int lap0, int lap1, orbfe_keypoint* kps,
                int cap, uint8_t* desc, int* n_out);
int oro_stereo_knn_ratio(const uint8_t* L, int32_t nl, const uint8_t* R, int32_t nr, float ratio, int32_t* out_train,
                         int32_t* out_dist);
}

namespace {

struct Fisheye {
    void* el;
    void* er;
    int cap;
    std::vector<orbfe_keypoint> kl, kr;
    std::vector<uint8_t> dl, dr;
    std::vector<int32_t> t, d;
    Fisheye(int nf, float sf, int nlevels, int ini, int mn) : cap(nf + 3 * nlevels + 64) {
        el = oro_create(nf, sf, nlevels, ini, mn);
        er = oro_create(nf, sf, nlevels, ini, mn);
        kl.resize(cap);
        kr.resize(cap);
        dl.resize((size_t)cap * 32);
        dr.resize((size_t)cap * 32);
        t.resize(cap);
        d.resize(cap);
    }
    ~Fisheye() {
        oro_destroy(el);
        oro_destroy(er);
    }
    // one frame; returns the ratio-test survivors (descMatches)
    int frame(const uint8_t* L, const uint8_t* R, int w, int h, int lap0, int lap1, bool lr_split) {
        int nl = 0, nr = 0, ml = 0, mr = 0;
        if (lr_split) {
            std::thread a([&] { ml = oro_extract(el, L, w, h, w, lap0, lap1, kl.data(), cap, dl.data(), &nl); });
            std::thread b([&] { mr = oro_extract(er, R, w, h, w, lap0, lap1, kr.data(), cap, dr.data(), &nr); });
            a.join();
            b.join();
        } else {
            ml = oro_extract(el, L, w, h, w, lap0, lap1, kl.data(), cap, dl.data(), &nl);
            mr = oro_extract(er, R, w, h, w, lap0, lap1, kr.data(), cap, dr.data(), &nr);
        }
        if (ml < 0 || mr < 0 || nl > cap || nr > cap) return 0;
        // the lapping-area rows [monoIndex, n) of each side (Frame.cc:1129-1133)
        return oro_stereo_knn_ratio(dl.data() + (size_t)ml * 32, nl - ml, dr.data() + (size_t)mr * 32, nr - mr, 0.7f,
                                    t.data(), d.data());
    }
};

}  // namespace

extern "C" {

// nframes frames one after another (lr_split: the two extractions on two per-frame threads);
// *ms_per_frame = mean wall time per frame. Returns the total ratio-test survivors.
long oro_bench_fisheye_latency(const uint8_t* L, const uint8_t* R, int nframes, int w, int h, int nfeatures, float sf,
                               int nlevels, int ini, int mn, int lap0, int lap1, int lr_split, double* ms_per_frame) {
    Fisheye f(nfeatures, sf, nlevels, ini, mn);
    long tot = 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < nframes; i++)
        tot += f.frame(L + (size_t)i * w * h, R + (size_t)i * w * h, w, h, lap0, lap1, lr_split != 0);
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (ms_per_frame) *ms_per_frame = nframes > 0 ? ms / nframes : 0.0;
    return tot;
}

// Throughput: nthreads workers, one frame at a time each (frames i, i + nthreads, ...);
// *ms_total = wall time. Returns the total ratio-test survivors.
long oro_bench_fisheye(const uint8_t* L, const uint8_t* R, int nframes, int w, int h, int nfeatures, float sf,
                       int nlevels, int ini, int mn, int lap0, int lap1, int nthreads, double* ms_total) {
    std::vector<long> tot(nthreads > 0 ? nthreads : 1, 0);
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> ws;
    for (int t = 0; t < (int)tot.size(); t++)
        ws.emplace_back([&, t] {
            Fisheye f(nfeatures, sf, nlevels, ini, mn);
            for (int i = t; i < nframes; i += (int)tot.size())
                tot[t] += f.frame(L + (size_t)i * w * h, R + (size_t)i * w * h, w, h, lap0, lap1, false);
        });
    for (auto& w_ : ws) w_.join();
    if (ms_total) *ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    long s = 0;
    for (long v : tot) s += v;
    return s;
}

}  // extern "C"
