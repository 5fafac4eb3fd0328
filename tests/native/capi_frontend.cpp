// A compiled C++ consumer of the C-ABI (include/orbfe.h only, linked against liborbfe.so): the call
// sequence the drop-in shims make (shim/ORBextractor_orbfe.cc, shim/ORBmatcher_orbfe.cc), on plain
// C++ stand-ins for the ORB-SLAM3 objects because OpenCV / Eigen are absent here:
//   ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) + getters   ORBextractor.cc:409-469
//   ORBextractor::operator()(image, mask, keys, desc, vLappingArea)                  ORBextractor.cc:1086-1168
//   Frame::Frame(stereo): two operator() calls, then ComputeStereoMatches             Frame.cc:101-197, 811-981
//   ORBmatcher(0.8).SearchByProjection(F, vpMapPoints, th) through a MapPoint* <-> handle table
//                                                                                     ORBmatcher.cc:43-213
// usage: capi_frontend <job.bin> <out.bin>
//        capi_frontend --latency <frames> <seq.bin>   (one JSON line: per-frame drop-in latency, both forms)
//        capi_frontend --tracking <frames> <seq.bin> [out.bin]   (one JSON line: a Tracking frame, split)
//   job: int32 w, h, nfeatures, n_mps, th_x100; float bf, fx; u8 left[w*h], u8 right[w*h]
//   out: per side {int32 monoIndex, n; keypoints n x 28 B; descriptors n x 32 B}; int32 levels;
//        float scale[levels]; stereo {int32 nmatch; float uR[nL]; float depth[nL]};
//        map points {n_mps x orbfe_map_point}; int32 nmatches; int32 mvp[nL] (map point ids, -1)
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "orbfe.h"
#include "orbfe_glue.h"   // shim/: the drop-in shim's own call sequence (Frame(stereo), SearchLocalPoints)
#include "tracking_kb8.h"
#include "tracking_loop.h"

namespace {

struct KeyPoint {   // cv::KeyPoint
    float x, y, size, angle, response;
    int32_t octave, class_id;
};
static_assert(sizeof(KeyPoint) == sizeof(orbfe_keypoint), "cv::KeyPoint layout (28 B)");

// std::vector descriptor sink for orbfe_glue::frame_stereo (the shim's is a cv::Mat)
struct VecRows {
    std::vector<uint8_t>& v;
    uint8_t* rows(int cap) {
        v.resize((size_t)cap * 32);
        return v.data();
    }
    void keep(int n) { v.resize((size_t)n * 32); }
};

void check(int rc, const char* what) {
    if (rc < 0 && rc != ORBFE_E_EMPTY) throw std::runtime_error(std::string(what) + " failed: " + std::to_string(rc));
}

// ORB_SLAM3::ORBextractor as the shim implements it
class ORBextractor {
public:
    ORBextractor(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST) : nlevels_(nlevels) {
        check(orbfe_extractor_create(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, &h_), "create");
        mvScaleFactor.resize(nlevels);
        mvInvScaleFactor.resize(nlevels);
        mvLevelSigma2.resize(nlevels);
        mvInvLevelSigma2.resize(nlevels);
        check(orbfe_extractor_scale_info(h_, mvScaleFactor.data(), mvInvScaleFactor.data(), mvLevelSigma2.data(),
                                         mvInvLevelSigma2.data(), nullptr),
              "scale_info");
    }
    ~ORBextractor() { orbfe_extractor_destroy(h_); }
    int operator()(const uint8_t* img, int w, int h, int step, std::vector<KeyPoint>& keys, std::vector<uint8_t>& desc,
                   const int lap[2]) {
        const int cap = orbfe_extractor_capacity(h_, w, h);
        check(cap, "capacity");
        keys.resize(cap);
        desc.resize((size_t)cap * 32);
        int n = 0;
        const int mono = orbfe_extract(h_, img, w, h, step, lap[0], lap[1], reinterpret_cast<orbfe_keypoint*>(keys.data()),
                                       desc.data(), cap, &n);
        if (mono == ORBFE_E_EMPTY) { keys.clear(); desc.clear(); return -1; }
        check(mono, "extract");
        keys.resize(n);
        desc.resize((size_t)n * 32);
        return mono;
    }
    int GetLevels() const { return nlevels_; }
    orbfe_extractor* handle() const { return h_; }
    std::vector<float> mvScaleFactor, mvInvScaleFactor, mvLevelSigma2, mvInvLevelSigma2;

private:
    orbfe_extractor* h_ = nullptr;
    int nlevels_;
};

struct MapPoint {   // the tracking fields SearchByProjection reads (MapPoint.h:172-180)
    float mTrackProjX, mTrackProjY, mTrackProjXR, mTrackViewCos, mTrackDepth;
    int mnTrackScaleLevel;
    bool mbTrackInView, bad;
    int observations;
    int32_t mnId;
    uint8_t desc[32];
};

struct Frame {   // Frame(stereo): Frame.cc:101-197
    std::vector<KeyPoint> mvKeys, mvKeysRight;
    std::vector<uint8_t> mDescriptors, mDescriptorsRight;
    std::vector<float> mvuRight, mvDepth;
    std::vector<MapPoint*> mvpMapPoints;
    int monoLeft = 0, monoRight = 0, nStereo = 0;
    float mnMinX = 0, mnMaxX = 0, mnMinY = 0, mnMaxY = 0, mbf, mfx;
    ORBextractor *left, *right;
    Frame(const uint8_t* L, const uint8_t* R, int w, int h, ORBextractor* el, ORBextractor* er, float bf, float fx)
        : mbf(bf), mfx(fx), left(el), right(er) {
        const int lap[2] = {0, 0};
        monoLeft = (*left)(L, w, h, w, mvKeys, mDescriptors, lap);    // ExtractORB(0, ...)
        monoRight = (*right)(R, w, h, w, mvKeysRight, mDescriptorsRight, lap);   // ExtractORB(1, ...)
        const int N = (int)mvKeys.size();
        mvuRight.assign(N, -1.f);
        mvDepth.assign(N, -1.f);
        // ComputeStereoMatches through the library (the shim's Frame reroute, kOrbfeStereoRerouted)
        nStereo = orbfe_stereo_match(left->handle(), right->handle(), bf, fx, mvuRight.data(), mvDepth.data());
        check(nStereo, "stereo_match");
        mvpMapPoints.assign(N, nullptr);
        mnMaxX = (float)w;   // ComputeImageBounds without distortion
        mnMaxY = (float)h;
    }
};

// MapPoint* <-> int32 handle table of shim/ORBmatcher_orbfe.cc
struct Handles {
    std::vector<MapPoint*> table;
    std::unordered_map<MapPoint*, int32_t> id;
    int32_t of(MapPoint* p) {
        if (!p) return -1;
        auto it = id.find(p);
        if (it != id.end()) return it->second;
        const int32_t h = (int32_t)table.size();
        table.push_back(p);
        id.emplace(p, h);
        return h;
    }
    MapPoint* at(int32_t h) const { return h < 0 ? nullptr : table[h]; }
};

// ORBmatcher(nnratio).SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints) as the shim does it
int SearchByProjection(Frame& F, const std::vector<MapPoint*>& vpMapPoints, float th, float nnratio,
                       std::vector<orbfe_map_point>& q_out) {
    Handles H;
    const int N = (int)F.mvKeys.size();
    std::vector<int32_t> mvp(N), obs(N);
    for (int i = 0; i < N; i++) {
        mvp[i] = H.of(F.mvpMapPoints[i]);
        obs[i] = F.mvpMapPoints[i] ? F.mvpMapPoints[i]->observations : 0;
    }
    std::vector<orbfe_map_point> q(vpMapPoints.size());
    for (size_t i = 0; i < vpMapPoints.size(); i++) {
        const MapPoint* p = vpMapPoints[i];
        orbfe_map_point& r = q[i];
        memset(&r, 0, sizeof(r));
        r.proj_x = p->mTrackProjX; r.proj_y = p->mTrackProjY; r.proj_xr = p->mTrackProjXR;
        r.view_cos = p->mTrackViewCos; r.depth = p->mTrackDepth; r.scale_level = p->mnTrackScaleLevel;
        r.flags = (p->mbTrackInView ? ORBFE_MP_IN_VIEW : 0) | (p->bad ? ORBFE_MP_BAD : 0);
        r.observations = p->observations;
        r.id = H.of(const_cast<MapPoint*>(p));
        r.scale_level_r = -1;
        if (p->mbTrackInView && !p->bad) memcpy(r.desc, p->desc, 32);
    }
    orbfe_frame fr;
    memset(&fr, 0, sizeof(fr));
    fr.n = N;
    fr.keys = reinterpret_cast<const orbfe_keypoint*>(F.mvKeys.data());
    fr.desc = F.mDescriptors.data();
    fr.uright = F.mvuRight.data();
    fr.min_x = F.mnMinX; fr.max_x = F.mnMaxX; fr.min_y = F.mnMinY; fr.max_y = F.mnMaxY;
    fr.nlevels = F.left->GetLevels();
    fr.scale_factors = F.left->mvScaleFactor.data();
    fr.mbf = F.mbf;
    const int n = orbfe_search_by_projection_local(&fr, mvp.data(), obs.data(), q.data(), (int)q.size(), th, 0, 0.f,
                                                   nnratio);
    check(n, "search_by_projection_local");
    for (int i = 0; i < N; i++) F.mvpMapPoints[i] = H.at(mvp[i]);
    // the records with the caller's map point ids (not the call's handles) for the checker
    for (size_t i = 0; i < q.size(); i++) q[i].id = vpMapPoints[i]->mnId;
    q_out = q;
    return n;
}

struct Lcg {   // deterministic map points without <random>'s implementation-defined distributions
    uint64_t s;
    uint32_t next() { s = s * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(s >> 33); }
    float unit() { return (next() & 0xFFFFFF) / 16777216.0f; }
};

double median(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

// Sequence job (bench.py dropin leg): int32 magic 'ORBS', w, h, nfeatures, npairs, window; float fx,
// fy, cx, cy, bf, tx; then npairs x (u8 left[w*h], u8 right[w*h]) of synth_stereo_sequence.
struct SeqJob {
    int w = 0, h = 0, nf = 0, npairs = 0, window = 6;
    trk::Cam cam{};
    std::vector<uint8_t> px;
    const uint8_t* left(int k) const { return px.data() + (size_t)(k % npairs) * 2 * w * h; }
    const uint8_t* right(int k) const { return left(k) + (size_t)w * h; }
};

SeqJob read_seq(const char* job) {
    FILE* f = fopen(job, "rb");
    if (!f) throw std::runtime_error("cannot open job");
    int32_t hdr[6];
    float c[6];
    if (fread(hdr, 4, 6, f) != 6 || fread(c, 4, 6, f) != 6) throw std::runtime_error("short job header");
    if (hdr[0] != 0x5342524f) throw std::runtime_error("not a sequence job");
    SeqJob j;
    j.w = hdr[1];
    j.h = hdr[2];
    j.nf = hdr[3];
    j.npairs = hdr[4];
    j.window = hdr[5];
    j.cam = trk::Cam{c[0], c[1], c[2], c[3], c[4], c[5]};
    j.px.resize((size_t)j.npairs * 2 * j.w * j.h);
    if (j.npairs <= 0 || fread(j.px.data(), 1, j.px.size(), f) != j.px.size()) throw std::runtime_error("short job images");
    fclose(f);
    return j;
}

// The drop-in path at batch 1, a stereo Frame at a time over the job's sequence (frame k = pair k mod
// npairs), in the two forms the shim can take:
//   frame call: orbfe_frame_stereo, Frame::Frame(stereo) in one library call (Frame.cc:101-141);
//   threads:    exactly as Tracking builds a stereo Frame (Frame.cc:122-141): the left and right
//               ORBextractor::operator() on two std::threads started per frame (ExtractORB), joined,
//               then ComputeStereoMatches (orbfe_stereo_match).
// Host images in, host keypoints / descriptors / uR / depth out. Per form: wall time per frame without
// event timing (medians), then a second pass with the library's call timing (HIP events on the
// stream: upload / kernels / result copies) for the split; host = timed wall - the device-side path.
int latency(int frames, const char* job) {
    const SeqJob J = read_seq(job);
    const int w = J.w, h = J.h, nf = J.nf;
    ORBextractor el(nf, 1.2f, 8, 20, 7), er(nf, 1.2f, 8, 20, 7);
    const int cap = orbfe_extractor_capacity(el.handle(), w, h);
    check(cap, "capacity");
    const int warm = 5;
    std::string out = "{";
    for (int form = 0; form < 2; form++) {   // 0 = frame call, 1 = threads
        std::vector<double> wall_plain, wall, ext, st, up, ker, cp, sker, scp, host;
        int nkp = 0, nst = 0;
        for (int it = 0; it < 2 * (warm + frames); it++) {
            const bool timed = it >= warm + frames;
            if (it == 0 || it == warm + frames) {
                check(orbfe_set_stage_timing(el.handle(), timed), "timing");
                check(orbfe_set_stage_timing(er.handle(), timed), "timing");
            }
            const int k = timed ? it - (warm + frames) : it;
            const uint8_t* L = J.left(k);
            const uint8_t* R = J.right(k);
            std::vector<KeyPoint> kl, kr;
            std::vector<uint8_t> dl, dr;
            std::vector<float> ur, dp;
            double tl = 0, tr = 0;
            int ns = 0;
            const auto t0 = std::chrono::steady_clock::now();
            auto t1 = t0;
            if (form == 0) {   // the shim's Frame(stereo) (shim/Frame_orbfe.cc -> orbfe_glue::frame_stereo)
                int ml = 0, mr = 0;
                VecRows sl{dl}, sr{dr};
                ns = orbfe_glue::frame_stereo(el.handle(), er.handle(), L, R, w, h, w, J.cam.bf, J.cam.fx, kl, sl, &ml, kr,
                                              sr, &mr, ur, dp);
                check(ns, "frame_stereo");
                t1 = std::chrono::steady_clock::now();
            } else {
                const int lap[2] = {0, 0};
                std::thread thL([&] {
                    const auto a = std::chrono::steady_clock::now();
                    el(L, w, h, w, kl, dl, lap);
                    tl = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
                });
                std::thread thR([&] {
                    const auto a = std::chrono::steady_clock::now();
                    er(R, w, h, w, kr, dr, lap);
                    tr = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
                });
                thL.join();
                thR.join();
                t1 = std::chrono::steady_clock::now();
                ur.assign(kl.size(), -1.f);
                dp.assign(kl.size(), -1.f);
                ns = orbfe_stereo_match(el.handle(), er.handle(), J.cam.bf, J.cam.fx, ur.data(), dp.data());
                check(ns, "stereo_match");
            }
            const auto t2 = std::chrono::steady_clock::now();
            if (k < warm) continue;
            if (!timed) {
                wall_plain.push_back(std::chrono::duration<double, std::milli>(t2 - t0).count());
                continue;
            }
            float a[5], b[5];
            check(orbfe_get_call_timing(el.handle(), a), "call_timing");
            check(orbfe_get_call_timing(er.handle(), b), "call_timing");
            const double fw = std::chrono::duration<double, std::milli>(t2 - t0).count();
            wall.push_back(fw);
            if (form == 0) {   // {upload, extraction kernels, result copies, stereo kernels}
                ext.push_back(std::chrono::duration<double, std::milli>(t1 - t0).count());
                st.push_back(0.0);
                up.push_back(a[0]);
                ker.push_back(a[1]);
                cp.push_back(a[2]);
                sker.push_back(a[3]);
                scp.push_back(0.0);
                host.push_back(fw - (a[0] + a[1] + a[2] + a[3]));
            } else {
                const bool lslow = tl >= tr;   // the extraction's critical side is the slower thread's
                const float* c = lslow ? a : b;
                ext.push_back(std::max(tl, tr));
                st.push_back(std::chrono::duration<double, std::milli>(t2 - t1).count());
                up.push_back(c[0]);
                ker.push_back(c[1]);
                cp.push_back(c[2]);
                sker.push_back(a[3]);
                scp.push_back(a[4]);
                host.push_back(fw - (c[0] + c[1] + c[2] + a[3] + a[4]));
            }
            nkp = (int)(kl.size() + kr.size());
            nst = ns;
        }
        char buf[1024];
        snprintf(buf, sizeof(buf),
                 "%s\"%s\": {\"frame_ms\": %.4f, \"frame_ms_min\": %.4f, \"frame_ms_timed\": %.4f, "
                 "\"extract_lr_ms\": %.4f, \"stereo_ms\": %.4f, \"keypoints_lr\": %d, \"stereo_matches\": %d, "
                 "\"split_ms\": {\"upload\": %.4f, \"extract_kernels\": %.4f, \"result_copies\": %.4f, "
                 "\"stereo_kernels\": %.4f, \"stereo_copies\": %.4f, \"host\": %.4f}}",
                 form ? ", " : "", form ? "threads" : "frame_call", median(wall_plain),
                 *std::min_element(wall_plain.begin(), wall_plain.end()), median(wall), median(ext), median(st), nkp,
                 nst, median(up), median(ker), median(cp), median(sker), median(scp), median(host));
        out += buf;
    }
    char tail[256];
    snprintf(tail, sizeof(tail), ", \"frames\": %d, \"distinct_pairs\": %d, \"width\": %d, \"height\": %d, \"nfeatures\": %d}",
             frames, J.npairs, w, h, nf);
    printf("%s%s\n", out.c_str(), tail);
    return 0;
}

// The library as trk::Tracker's Api (tests/native/tracking_loop.h)
struct GpuApi {
    ORBextractor& el;
    ORBextractor& er;
    int w, h, cap;
    float bf, fx;
    // Frame(stereo) as the shim builds it (shim/Frame_orbfe.cc: orbfe_glue::frame_stereo)
    int frame(const uint8_t* L, const uint8_t* R, trk::FrameData& f) {
        VecRows sl{f.desc}, sr{f.desc_r};
        const int ns = orbfe_glue::frame_stereo(el.handle(), er.handle(), L, R, w, h, w, bf, fx, f.keys, sl, &f.mono_l,
                                                f.keys_r, sr, &f.mono_r, f.ur, f.depth);
        check(ns, "frame_stereo");
        f.nstereo = ns;
        frame_id = host_view ? 0 : orbfe_extractor_frame_id(el.handle());   // the shim keeps it in the Frame
        return ns;
    }
    uint64_t frame_id = 0;   // the current frame's id: its searches read it in HBM (orbfe_frame_device_view)
    bool host_view = false;  // --tracking-hostview: the searches read the caller's copy (A/B)
    // diagnostic run (--tracking-diag): device time (HIP events around the call's kernels) and the
    // fixed-point passes of every matcher call
    bool diag = false;
    std::vector<double> d_sbp, d_loc, p_sbp, p_loc, w_sbp, w_loc;
    std::vector<orbfe_map_point> track;   // SearchLocalPoints' isInFrustum records
    void note(std::vector<double>& dv, std::vector<double>& pv) {
        if (!diag) return;
        dv.push_back(orbfe_matcher_last_ms());
        long long st[3];
        orbfe_matcher_last_stats(st);
        pv.push_back((double)st[2]);
    }
    int sbp_last(const orbfe_frame* F, int32_t* mvp, const int32_t* obs, const orbfe_proj_point* pts, int n, float th,
                 int fwd, int bwd, int ori) {
        const auto t0 = std::chrono::steady_clock::now();
        const int r = orbfe_glue::on_current_frame(el.handle(), frame_id, *F, [&](const orbfe_frame* V) {
            return orbfe_search_by_projection_lastframe(V, mvp, obs, pts, n, th, fwd, bwd, ori);
        });
        if (diag) w_sbp.push_back(trk::ms_since(t0));
        check(r, "search_by_projection_lastframe");
        note(d_sbp, p_sbp);
        return r;
    }
    int local_points(const orbfe_frame* F, const orbfe_camera* c, const orbfe_map_point_3d* pts, int n, int32_t* mvp,
                     const int32_t* obs, float th, int bFar, float thFar, float ratio, int32_t* ntm) {
        const auto t0 = std::chrono::steady_clock::now();
        // SearchLocalPoints as the shim calls it (shim/Tracking_orbfe.cc: orbfe_glue::local_points, the
        // isInFrustum records returned for the MapPoint side effects); nnratio is the reference's 0.8
        (void)ratio;
        const int r = orbfe_glue::on_current_frame(el.handle(), frame_id, *F, [&](const orbfe_frame* V) {
            return orbfe_glue::local_points(V, c, nullptr, pts, n, mvp, obs, th, bFar != 0, thFar, track, ntm);
        });
        if (diag) w_loc.push_back(trk::ms_since(t0));
        check(r, "search_local_points");
        note(d_loc, p_loc);
        return r;
    }
};

// The library as trk::TrackerKB8's Api (tests/native/tracking_kb8.h): Frame(stereo, KB8) the way the
// reference builds it (two ExtractORB threads with vLappingArea {0, 511}, then the kNN + ratio stage of
// ComputeStereoFishEyeMatches over the lapping rows), the two-camera SearchByProjection(LastFrame) and
// SearchLocalPoints through the shim glue with the rig
struct GpuApiKB8 {
    ORBextractor& el;
    ORBextractor& er;
    int w, h;
    std::vector<orbfe_map_point> track;
    int frame_kb8(const uint8_t* L, const uint8_t* R, trk::FrameKB8& f) {
        // both extractions (vLappingArea {0, 511}) and the kNN ratio test in one library call
        std::vector<KeyPoint> kl, kr;
        std::vector<uint8_t> dl, dr;
        std::vector<int32_t> l2r, dist;
        VecRows sl{dl}, sr{dr};
        check(orbfe_glue::frame_fisheye(el.handle(), er.handle(), L, R, w, h, w, 0, 511, 0.7f, kl, sl, &f.mono_l, kr,
                                        sr, &f.mono_r, l2r, dist),
              "frame_fisheye");
        f.nl = (int)kl.size();
        f.nr = (int)kr.size();
        f.mono_l = std::max(f.mono_l, 0);
        f.mono_r = std::max(f.mono_r, 0);
        std::vector<int32_t> train(std::max(f.nl - f.mono_l, 0), -1);
        for (int q = 0; q < (int)train.size(); q++)
            if (l2r[q + f.mono_l] >= 0) train[q] = l2r[q + f.mono_l] - f.mono_r;
        f.keys.resize(f.nl + f.nr);
        memcpy(f.keys.data(), kl.data(), kl.size() * sizeof(KeyPoint));
        memcpy(f.keys.data() + f.nl, kr.data(), kr.size() * sizeof(KeyPoint));
        f.desc.resize((size_t)(f.nl + f.nr) * 32);
        memcpy(f.desc.data(), dl.data(), (size_t)f.nl * 32);
        memcpy(f.desc.data() + (size_t)f.nl * 32, dr.data(), (size_t)f.nr * 32);
        f.nstereo = trk::fisheye_links(f, train);
        return f.nstereo;
    }
    int sbp_last_pose(const orbfe_frame* F, int32_t* mvp, const int32_t* obs, const orbfe_last_point* pts, int n,
                      const orbfe_pose* Tcw, const orbfe_pose* Trl, const orbfe_camera_model* cam, float th) {
        const int r = orbfe_search_by_projection_lastframe_pose(F, mvp, obs, pts, n, Tcw, Trl, cam, th, 0, 0, 1);
        check(r, "search_by_projection_lastframe_pose");
        return r;
    }
    int local_points_rig(const orbfe_frame* F, const orbfe_camera* c, const orbfe_stereo_rig* rig,
                         const orbfe_map_point_3d* pts, int n, int32_t* mvp, const int32_t* obs, float th,
                         int32_t* ntm) {
        const int r = orbfe_glue::local_points(F, c, rig, pts, n, mvp, obs, th, false, 50.f, track, ntm);
        check(r, "search_local_points_track (rig)");
        return r;
    }
};

}  // namespace

int tracking_kb8(int frames, const char* job, const char* out_path) {
    const SeqJob J = read_seq(job);
    ORBextractor el(J.nf, 1.2f, 8, 20, 7), er(J.nf, 1.2f, 8, 20, 7);
    GpuApiKB8 api{el, er, J.w, J.h, {}};
    return trk::run_sequence_kb8(api, J.cam, J.w, J.h, el.mvScaleFactor, J.window, frames, J.npairs,
                                 [&](int k) { return J.left(k); }, [&](int k) { return J.right(k); }, out_path,
                                 "gpu: liborbfe.so C-ABI, KannalaBrandt8 two-camera frame (orbfe_frame_fisheye, "
                                 "orbfe_search_by_projection_lastframe_pose, "
                                 "orbfe_search_local_points_track with the rig)");
}

int tracking(int frames, const char* job, const char* out_path, bool diag, bool host_view = false) {
    const SeqJob J = read_seq(job);
    ORBextractor el(J.nf, 1.2f, 8, 20, 7), er(J.nf, 1.2f, 8, 20, 7);
    const int cap = orbfe_extractor_capacity(el.handle(), J.w, J.h);
    check(cap, "capacity");
    GpuApi api{el, er, J.w, J.h, cap, J.cam.bf, J.cam.fx};
    api.diag = diag;
    api.host_view = host_view;
    if (diag) {
        orbfe_matcher_set_timing(1);
        orbfe_matcher_set_stats(1);
    }
    const int rc = trk::run_sequence(api, J.cam, J.w, J.h, el.mvScaleFactor, J.window, frames, J.npairs,
                                     [&](int k) { return J.left(k); }, [&](int k) { return J.right(k); }, out_path,
                                     "gpu: liborbfe.so C-ABI through the shim glue (shim/orbfe_glue.h: orbfe_frame_stereo, "
                                     "orbfe_search_local_points_track) + orbfe_search_by_projection_lastframe");
    if (diag)
        printf("{\"diag\": {\"sbp_last_wall_ms\": %.4f, \"sbp_last_device_ms\": %.4f, \"sbp_last_passes\": %.1f, "
               "\"local_wall_ms\": %.4f, \"local_device_ms\": %.4f, \"local_passes\": %.1f}}\n",
               median(api.w_sbp), median(api.d_sbp), median(api.p_sbp), median(api.w_loc), median(api.d_loc),
               median(api.p_loc));
    return rc;
}


int main(int argc, char** argv) {
    if ((argc == 4 || argc == 5) && (std::string(argv[1]) == "--tracking" || std::string(argv[1]) == "--tracking-diag" ||
                                     std::string(argv[1]) == "--tracking-hostview")) {
        try {
            return tracking(atoi(argv[2]), argv[3], argc == 5 ? argv[4] : nullptr, std::string(argv[1]) == "--tracking-diag",
                            std::string(argv[1]) == "--tracking-hostview");
        } catch (const std::exception& e) {
            fprintf(stderr, "capi_frontend: %s\n", e.what());
            return 1;
        }
    }
    if ((argc == 4 || argc == 5) && std::string(argv[1]) == "--tracking-kb8") {
        try {
            return tracking_kb8(atoi(argv[2]), argv[3], argc == 5 ? argv[4] : nullptr);
        } catch (const std::exception& e) {
            fprintf(stderr, "capi_frontend: %s\n", e.what());
            return 1;
        }
    }
    if (argc == 4 && std::string(argv[1]) == "--latency") {
        try {
            return latency(atoi(argv[2]), argv[3]);
        } catch (const std::exception& e) {
            fprintf(stderr, "capi_frontend: %s\n", e.what());
            return 1;
        }
    }
    if (argc != 3) { fprintf(stderr, "usage: capi_frontend job.bin out.bin | --latency frames job.bin\n"); return 2; }
    try {
        FILE* f = fopen(argv[1], "rb");
        if (!f) throw std::runtime_error("cannot open job");
        int32_t hdr[5];
        float cam[2];
        if (fread(hdr, 4, 5, f) != 5 || fread(cam, 4, 2, f) != 2) throw std::runtime_error("short job header");
        const int w = hdr[0], h = hdr[1], nf = hdr[2], n_mps = hdr[3];
        const float th = hdr[4] / 100.f;
        std::vector<uint8_t> L((size_t)w * h), R((size_t)w * h);
        if (fread(L.data(), 1, L.size(), f) != L.size() || fread(R.data(), 1, R.size(), f) != R.size())
            throw std::runtime_error("short job images");
        fclose(f);
        ORBextractor el(nf, 1.2f, 8, 20, 7), er(nf, 1.2f, 8, 20, 7);   // mpORBextractorLeft / Right
        Frame F(L.data(), R.data(), w, h, &el, &er, cam[0], cam[1]);
        // local map: noisy copies of the frame's own keypoints (as Tracking would project them)
        Lcg rng{12345};
        std::vector<MapPoint> pts(n_mps);
        std::vector<MapPoint*> vp(n_mps);
        const int N = (int)F.mvKeys.size();
        for (int i = 0; i < n_mps; i++) {
            MapPoint& p = pts[i];
            const int k = (int)(rng.next() % (uint32_t)N);
            const KeyPoint& kp = F.mvKeys[k];
            p.mTrackProjX = kp.x + (rng.unit() - 0.5f) * 2.f;
            p.mTrackProjY = kp.y + (rng.unit() - 0.5f) * 2.f;
            p.mTrackProjXR = F.mvuRight[k] >= 0 ? F.mvuRight[k] + (rng.unit() - 0.5f) : p.mTrackProjX - 20.f * rng.unit();
            p.mTrackViewCos = 0.99f + 0.01f * rng.unit();
            p.mTrackDepth = 1.f + 10.f * rng.unit();
            p.mnTrackScaleLevel = kp.octave;
            p.mbTrackInView = (rng.next() % 10) != 0;
            p.bad = (rng.next() % 50) == 0;
            p.observations = (int)(rng.next() % 5);
            p.mnId = 1000 + i;
            memcpy(p.desc, F.mDescriptors.data() + (size_t)k * 32, 32);
            for (int b = 0; b < 12; b++) {
                const uint32_t bit = rng.next() % 256;
                p.desc[bit >> 3] ^= (uint8_t)(1u << (bit & 7));
            }
            vp[i] = &p;
        }
        std::vector<orbfe_map_point> q;
        const int nmatches = SearchByProjection(F, vp, th, 0.8f, q);
        FILE* o = fopen(argv[2], "wb");
        if (!o) throw std::runtime_error("cannot open out");
        auto w32 = [&](int32_t v) { fwrite(&v, 4, 1, o); };
        for (int side = 0; side < 2; side++) {
            const std::vector<KeyPoint>& k = side ? F.mvKeysRight : F.mvKeys;
            const std::vector<uint8_t>& d = side ? F.mDescriptorsRight : F.mDescriptors;
            w32(side ? F.monoRight : F.monoLeft);
            w32((int32_t)k.size());
            fwrite(k.data(), sizeof(KeyPoint), k.size(), o);
            fwrite(d.data(), 1, d.size(), o);
        }
        w32(el.GetLevels());
        fwrite(el.mvScaleFactor.data(), 4, el.mvScaleFactor.size(), o);
        w32(F.nStereo);
        fwrite(F.mvuRight.data(), 4, F.mvuRight.size(), o);
        fwrite(F.mvDepth.data(), 4, F.mvDepth.size(), o);
        fwrite(q.data(), sizeof(orbfe_map_point), q.size(), o);
        w32(nmatches);
        for (MapPoint* p : F.mvpMapPoints) w32(p ? p->mnId : -1);
        fclose(o);
    } catch (const std::exception& e) {
        fprintf(stderr, "capi_frontend: %s\n", e.what());
        return 1;
    }
    return 0;
}
