// OpenCV-free core of the drop-in shim: the library calls behind Frame::Frame(stereo) and
// Tracking::SearchLocalPoints, written once over plain types. The shim's replacements
// (shim/Frame_orbfe.cc, shim/Tracking_orbfe.cc) instantiate them with cv::KeyPoint / cv::Mat, and the
// compiled C-ABI consumer that bench.py times (tests/native/capi_frontend.cpp: dropin_latency_ms,
// tracking_frame_ms) instantiates them with its stand-in types, so the measured drop-in path runs
// this code. Header-only, C++14 (the reference's standard, CMakeLists.txt:16-29).
#pragma once
#include <cstdint>
#include <cstring>
#include <vector>

#include "orbfe.h"

namespace orbfe_glue {

// Frame::Frame(imLeft, imRight, ...) (Frame.cc:101-141): the two ExtractORB threads (:122-125,
// vLappingArea {0, 0}) and ComputeStereoMatches (:141) as ONE orbfe_frame_stereo call (both images
// up in one pinned block, one two-image launch chain with the stereo kernels, one result copy).
//   Key  : a 28-byte record with cv::KeyPoint's layout (cv::KeyPoint itself in the shim);
//   Desc : a descriptor sink with uint8_t* rows(int cap) (a continuous cap x 32 buffer) and
//          void keep(int n) (keep the first n rows).
// On success: kl / kr / ur / depth hold mvKeys, mvKeysRight, mvuRight, mvDepth (uR / depth -1 = no
// match, Frame.cc:813-814), mono_* the operator() return values, and the pre-cut stereo match count
// is returned. An empty image gives no keypoints and monoIndex -1, as operator() (ORBextractor.cc:
// 1090-1091). A negative return is a library status; the caller then runs the reference's body.
template <class Key, class Desc>
int frame_stereo(orbfe_extractor* hl, orbfe_extractor* hr, const uint8_t* img_l, const uint8_t* img_r, int width,
                 int height, int stride, float mbf, float fx, std::vector<Key>& kl, Desc& dl, int* mono_l,
                 std::vector<Key>& kr, Desc& dr, int* mono_r, std::vector<float>& ur, std::vector<float>& depth) {
    static_assert(sizeof(Key) == sizeof(orbfe_keypoint), "cv::KeyPoint layout (28 B) expected");
    if (width <= 0 || height <= 0 || !img_l || !img_r) {
        kl.clear(); kr.clear(); ur.clear(); depth.clear();
        dl.keep(0); dr.keep(0);
        *mono_l = *mono_r = -1;
        return 0;
    }
    const int cap = orbfe_extractor_capacity(hl, width, height);
    if (cap < 0) return cap;
    kl.resize(cap);
    kr.resize(cap);
    ur.resize(cap);
    depth.resize(cap);
    int nl = 0, nr = 0;
    const int ns = orbfe_frame_stereo(hl, hr, img_l, img_r, width, height, stride, mbf, fx,
                                      reinterpret_cast<orbfe_keypoint*>(kl.data()), dl.rows(cap), cap, &nl, mono_l,
                                      reinterpret_cast<orbfe_keypoint*>(kr.data()), dr.rows(cap), cap, &nr, mono_r,
                                      ur.data(), depth.data());
    if (ns < 0) return ns;
    kl.resize(nl);
    kr.resize(nr);
    dl.keep(nl);
    dr.keep(nr);
    ur.resize(nl);
    depth.resize(nl);
    return ns;
}

// Frame::Frame(imLeft, imRight, ..., KannalaBrandt8) (Frame.cc:1034-1105) up to the descriptor stage
// of ComputeStereoFishEyeMatches (:1126-1151): the two ExtractORB threads with each camera's
// vLappingArea (:1059-1062; one pair for both images here, as the batched engine) and knnMatch(k = 2)
// + ratio over the lapping rows as ONE orbfe_frame_fisheye call. On success l2r[i] is the right
// keypoint (absolute index) left keypoint i's ratio test keeps, -1 otherwise, dist[i] its Hamming
// distance; the return value is the number kept. The triangulation and depth checks that follow in
// the reference (:1153-1176) need the camera models and stay with the caller.
template <class Key, class Desc>
int frame_fisheye(orbfe_extractor* hl, orbfe_extractor* hr, const uint8_t* img_l, const uint8_t* img_r, int width,
                  int height, int stride, int lap0, int lap1, float ratio, std::vector<Key>& kl, Desc& dl, int* mono_l,
                  std::vector<Key>& kr, Desc& dr, int* mono_r, std::vector<int32_t>& l2r,
                  std::vector<int32_t>& dist) {
    static_assert(sizeof(Key) == sizeof(orbfe_keypoint), "cv::KeyPoint layout (28 B) expected");
    if (width <= 0 || height <= 0 || !img_l || !img_r) {
        kl.clear(); kr.clear(); l2r.clear(); dist.clear();
        dl.keep(0); dr.keep(0);
        *mono_l = *mono_r = -1;
        return 0;
    }
    const int cap = orbfe_extractor_capacity(hl, width, height);
    if (cap < 0) return cap;
    kl.resize(cap);
    kr.resize(cap);
    l2r.resize(cap);
    dist.resize(cap);
    int nl = 0, nr = 0;
    const int ng = orbfe_frame_fisheye(hl, hr, img_l, img_r, width, height, stride, lap0, lap1, ratio,
                                       reinterpret_cast<orbfe_keypoint*>(kl.data()), dl.rows(cap), cap, &nl, mono_l,
                                       reinterpret_cast<orbfe_keypoint*>(kr.data()), dr.rows(cap), cap, &nr, mono_r,
                                       l2r.data(), dist.data());
    if (ng < 0) return ng;
    kl.resize(nl);
    kr.resize(nr);
    dl.keep(nl);
    dr.keep(nr);
    l2r.resize(nl);
    dist.resize(nl);
    return ng;
}

// The pose part of Frame::isInFrustum's inputs (Frame.cc:512-586): Rcw row-major, tcw, Ow = the
// camera centre; fx..cy the pinhole parameters (unused with a rig), mfLogScaleFactor, and the
// viewing-cosine limit SearchLocalPoints passes (0.5, Tracking.cc:3415).
inline orbfe_camera camera(const float* Rcw_rowmajor, const float* tcw, const float* Ow, float fx, float fy, float cx,
                           float cy, float log_scale_factor, float view_cos_limit) {
    orbfe_camera c;
    memset(&c, 0, sizeof(c));
    memcpy(c.Rcw, Rcw_rowmajor, sizeof(c.Rcw));
    memcpy(c.tcw, tcw, sizeof(c.tcw));
    memcpy(c.Ow, Ow, sizeof(c.Ow));
    c.fx = fx; c.fy = fy; c.cx = cx; c.cy = cy;
    c.log_scale_factor = log_scale_factor;
    c.view_cos_limit = view_cos_limit;
    return c;
}

// Tracking::SearchLocalPoints' second loop and matcher call (Tracking.cc:3404-3452) over the points
// that loop visits, in mvpLocalMapPoints order: isInFrustum + SearchByProjection(F, points, th,
// bFarPoints, thFarPoints) with nnratio 0.8 in one device pass. mvp / obs are the frame's slots
// (handles, -1 = NULL) and their Observations(); mvp is updated in place. track[i] receives point i's
// isInFrustum record, from which the caller applies the loop's side effects. rig NULL = a pinhole
// single-camera frame. Returns nmatches (or a negative status) and *n_to_match = nToMatch.
inline int local_points(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                        const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* obs, float th,
                        bool bFarPoints, float thFarPoints, std::vector<orbfe_map_point>& track, int32_t* n_to_match) {
    track.resize((size_t)n);
    return orbfe_search_local_points_track(F, cam, rig, pts, n, mvp, obs, th, bFarPoints ? 1 : 0, thFarPoints, 0.8f,
                                           n_to_match, track.data());
}

// Tracking's searches on the CURRENT frame read it in HBM when the extractor still holds it: call(F)
// runs with the device view of the frame the last orbfe_frame_stereo on `left` produced
// (orbfe_frame_device_view; `frame_id` = orbfe_extractor_frame_id(left) right after that call, 0 =
// none), the bounds and mbf taken from `host`; a view the library cannot take for this call (a
// stale id, a search shape outside the one-workgroup path) falls back to call(&host), the host view.
template <class Call>
int on_current_frame(orbfe_extractor* left, uint64_t frame_id, const orbfe_frame& host, Call&& call) {
    if (left && frame_id) {
        orbfe_frame dv = host;
        if (orbfe_frame_device_view(left, frame_id, &dv) == ORBFE_OK) {
            const int r = call(&dv);
            if (r != ORBFE_E_ARG) return r;
        }
    }
    return call(&host);
}

}  // namespace orbfe_glue
