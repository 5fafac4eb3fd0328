// The Tracking frame of tests/native/tracking_loop.h on the CPU restatement (oracle/liborb_oracle.so):
// the CPU baseline of bench.py's tracking_frame leg and the reference of the GPU-vs-CPU sequence parity
// test (tests/test_capi_consumer.py). Frame(stereo) extracts the left and right images on two
// std::threads started per frame, as Frame.cc:122-125 does, then runs ComputeStereoMatches (:141).
// usage: tracking_cpu <frames> <seq.bin> [out.bin]   (seq.bin: the sequence job of capi_frontend)
#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <string>
#include <stdexcept>
#include <thread>
#include <vector>

#include "orbfe.h"
#include "tracking_kb8.h"
#include "tracking_loop.h"

// oracle/orb_oracle.cpp, orb_oracle_match.cpp (KeyPoint records are the 28-byte cv::KeyPoint layout)
extern "C" {
void* oro_create(int nfeatures, float scaleFactor, int nlevels, int iniTh, int minTh);
void oro_destroy(void* h);
void oro_level_info(void* h, float* scale, float* inv_scale, float* sigma2, float* inv_sigma2, int* per_level,
                    int* umax16);
int oro_extract(void* h, const uint8_t* img, int w, int hgt, int stride, int lap0, int lap1, orbfe_keypoint* kps,
                int cap, uint8_t* desc, int* n_out);
int oro_stereo_match(void* hL, void* hR, const orbfe_keypoint* kL, const uint8_t* dL, int N, const orbfe_keypoint* kR,
                     const uint8_t* dR, int Nr, float bf, float fx, float* uRight, float* depth);
int oro_sbp_lastframe(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs_in, const orbfe_proj_point* pts,
                      int32_t n_pts, float th, int32_t bForward, int32_t bBackward, int32_t checkOri);
int oro_search_local_points(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts, int32_t n,
                            int32_t* mvp, const int32_t* mvp_obs, float th, int32_t bFarPoints, float thFarPoints,
                            float nnratio, int32_t* n_to_match);
int oro_stereo_knn_ratio(const uint8_t* L, int32_t nl, const uint8_t* R, int32_t nr, float ratio, int32_t* out_train,
                         int32_t* out_dist);
int oro_sbp_lastframe_stereo(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs_in,
                             const orbfe_proj_point* pts, const float* right_uv, int32_t n_pts, float th,
                             int32_t bForward, int32_t bBackward, int32_t checkOri);
int oro_sbp_lastframe_pose(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs_in, const orbfe_last_point* lp,
                           int32_t n_pts, const orbfe_pose* Tcw, const orbfe_pose* Trl, const orbfe_camera_model* cam,
                           float th, int32_t bForward, int32_t bBackward, int32_t checkOri);
int oro_search_local_points_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* mvp_obs, float th,
                                int32_t bFarPoints, float thFarPoints, float nnratio, int32_t* n_to_match);
}

namespace {

struct CpuApi {
    void* el;
    void* er;
    int w, h, cap;
    float bf, fx;
    int frame(const uint8_t* L, const uint8_t* R, trk::FrameData& f) {
        f.keys.resize(cap);
        f.keys_r.resize(cap);
        f.desc.resize((size_t)cap * 32);
        f.desc_r.resize((size_t)cap * 32);
        int nl = 0, nr = 0;
        std::thread tl([&] { f.mono_l = oro_extract(el, L, w, h, w, 0, 0, f.keys.data(), cap, f.desc.data(), &nl); });
        std::thread tr([&] { f.mono_r = oro_extract(er, R, w, h, w, 0, 0, f.keys_r.data(), cap, f.desc_r.data(), &nr); });
        tl.join();
        tr.join();
        if (nl > cap || nr > cap) throw std::runtime_error("keypoint capacity");
        f.keys.resize(nl);
        f.desc.resize((size_t)nl * 32);
        f.keys_r.resize(nr);
        f.desc_r.resize((size_t)nr * 32);
        f.ur.assign(nl, -1.f);
        f.depth.assign(nl, -1.f);
        f.nstereo = oro_stereo_match(el, er, f.keys.data(), f.desc.data(), nl, f.keys_r.data(), f.desc_r.data(), nr, bf,
                                     fx, f.ur.data(), f.depth.data());
        return f.nstereo;
    }
    int sbp_last(const orbfe_frame* F, int32_t* mvp, const int32_t* obs, const orbfe_proj_point* pts, int n, float th,
                 int fwd, int bwd, int ori) {
        return oro_sbp_lastframe(F, mvp, obs, pts, n, th, fwd, bwd, ori);
    }
    int local_points(const orbfe_frame* F, const orbfe_camera* c, const orbfe_map_point_3d* pts, int n, int32_t* mvp,
                     const int32_t* obs, float th, int bFar, float thFar, float ratio, int32_t* ntm) {
        return oro_search_local_points(F, c, pts, n, mvp, obs, th, bFar, thFar, ratio, ntm);
    }
    // the two-camera Tracking frame (tests/native/tracking_kb8.h) on the restatement
    int frame_kb8(const uint8_t* L, const uint8_t* R, trk::FrameKB8& f) {
        std::vector<orbfe_keypoint> kl(cap), kr(cap);
        std::vector<uint8_t> dl((size_t)cap * 32), dr((size_t)cap * 32);
        int nl = 0, nr = 0;
        std::thread tl([&] { f.mono_l = oro_extract(el, L, w, h, w, 0, 511, kl.data(), cap, dl.data(), &nl); });
        std::thread tr([&] { f.mono_r = oro_extract(er, R, w, h, w, 0, 511, kr.data(), cap, dr.data(), &nr); });
        tl.join();
        tr.join();
        if (nl > cap || nr > cap) throw std::runtime_error("keypoint capacity");
        f.nl = nl;
        f.nr = nr;
        f.mono_l = std::max(f.mono_l, 0);
        f.mono_r = std::max(f.mono_r, 0);
        const int ql = nl - f.mono_l, qr = nr - f.mono_r;
        std::vector<int32_t> train(std::max(ql, 0), -1), dist(std::max(ql, 0), -1);
        if (ql > 0 && qr > 0)
            oro_stereo_knn_ratio(dl.data() + (size_t)f.mono_l * 32, ql, dr.data() + (size_t)f.mono_r * 32, qr, 0.7f,
                                 train.data(), dist.data());
        f.keys.assign(kl.begin(), kl.begin() + nl);
        f.keys.insert(f.keys.end(), kr.begin(), kr.begin() + nr);
        f.desc.assign(dl.begin(), dl.begin() + (size_t)nl * 32);
        f.desc.insert(f.desc.end(), dr.begin(), dr.begin() + (size_t)nr * 32);
        f.nstereo = trk::fisheye_links(f, train);
        return f.nstereo;
    }
    int sbp_last_pose(const orbfe_frame* F, int32_t* mvp, const int32_t* obs, const orbfe_last_point* pts, int n,
                      const orbfe_pose* Tcw, const orbfe_pose* Trl, const orbfe_camera_model* cam, float th) {
        return oro_sbp_lastframe_pose(F, mvp, obs, pts, n, Tcw, Trl, cam, th, 0, 0, 1);
    }
    int local_points_rig(const orbfe_frame* F, const orbfe_camera* c, const orbfe_stereo_rig* rig,
                         const orbfe_map_point_3d* pts, int n, int32_t* mvp, const int32_t* obs, float th,
                         int32_t* ntm) {
        return oro_search_local_points_rig(F, c, rig, pts, n, mvp, obs, th, 0, 50.f, 0.8f, ntm);
    }
};

}  // namespace

int main(int argc, char** argv) {
    // --kb8: the KannalaBrandt8 two-camera Tracking frame (tests/native/tracking_kb8.h)
    const bool kb8 = argc >= 2 && std::string(argv[1]) == "--kb8";
    if (kb8) {
        argv++;
        argc--;
    }
    if (argc != 3 && argc != 4) {
        fprintf(stderr, "usage: tracking_cpu [--kb8] <frames> <seq.bin> [out.bin]\n");
        return 2;
    }
    try {
        FILE* f = fopen(argv[2], "rb");
        if (!f) throw std::runtime_error("cannot open job");
        int32_t hdr[6];
        float c[6];
        if (fread(hdr, 4, 6, f) != 6 || fread(c, 4, 6, f) != 6 || hdr[0] != 0x5342524f)
            throw std::runtime_error("not a sequence job");
        const int w = hdr[1], h = hdr[2], nf = hdr[3], npairs = hdr[4], window = hdr[5];
        std::vector<uint8_t> px((size_t)npairs * 2 * w * h);
        if (npairs <= 0 || fread(px.data(), 1, px.size(), f) != px.size()) throw std::runtime_error("short job images");
        fclose(f);
        void* el = oro_create(nf, 1.2f, 8, 20, 7);
        void* er = oro_create(nf, 1.2f, 8, 20, 7);
        std::vector<float> scale(8);
        oro_level_info(el, scale.data(), nullptr, nullptr, nullptr, nullptr, nullptr);
        const int cap = nf + 3 * 8 + 64;
        CpuApi api{el, er, w, h, cap, c[4], c[0]};
        const trk::Cam cam{c[0], c[1], c[2], c[3], c[4], c[5]};
        auto L = [&](int k) { return px.data() + (size_t)(k % npairs) * 2 * w * h; };
        auto R = [&](int k) { return px.data() + (size_t)(k % npairs) * 2 * w * h + (size_t)w * h; };
        const int rc = kb8 ? trk::run_sequence_kb8(api, cam, w, h, scale, window, atoi(argv[1]), npairs, L, R,
                                                   argc == 4 ? argv[3] : nullptr,
                                                   "cpu: oracle restatement, KannalaBrandt8 two-camera frame (2 "
                                                   "extraction threads, kNN + ratio, then the matchers)")
                           : trk::run_sequence(api, cam, w, h, scale, window, atoi(argv[1]), npairs, L, R,
                                               argc == 4 ? argv[3] : nullptr,
                                               "cpu: oracle restatement (2 extraction threads per frame, then the "
                                               "matchers on the calling thread)");
        oro_destroy(el);
        oro_destroy(er);
        return rc;
    } catch (const std::exception& e) {
        fprintf(stderr, "tracking_cpu: %s\n", e.what());
        return 1;
    }
}
