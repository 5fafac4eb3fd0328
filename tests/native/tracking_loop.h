// The per-frame front-end work of Tracking::Track for a stereo camera in its steady state, over a
// seeded synthetic stereo sequence (orb_slam3_ros_amd/synth.py: synth_stereo_sequence), written once
// against an "Api" of the three calls Tracking makes into the ORB front-end:
//   Frame::Frame(stereo): ExtractORB x 2 + ComputeStereoMatches          Frame.cc:101-141
//   TrackWithMotionModel: SearchByProjection(CurrentFrame, LastFrame, th = 7 for stereo, retried at
//                         2 th below 20 matches)                         Tracking.cc:2893-2935
//   TrackLocalMap -> SearchLocalPoints: isInFrustum over the local map points not already matched,
//                         then SearchByProjection(F, vpLocalMapPoints, th = 1 for stereo)
//                                                                         Tracking.cc:3382-3452
// tests/native/capi_frontend.cpp instantiates it with the library's C-ABI (the GPU path),
// tests/native/tracking_cpu.cpp with the CPU restatement in oracle/ (the CPU baseline and the parity
// reference of the whole sequence). The bookkeeping between the calls (the caller's projection of the
// last frame's points with the motion-model pose, the map-point snapshots, the new points a stereo
// keyframe would create) is plain host code shared by both, so both runs see the same inputs whenever
// the calls return the same outputs.
//
// Geometry (synth_stereo_sequence): a fronto-parallel plane at depth bf / disp, a rectified pinhole
// rig translating along +x by shift * Z / fx per frame (image content moves `shift` px per frame), so
// the constant-velocity motion model is exact and Tcw = [I | -Ow_k].
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "orbfe.h"

namespace trk {

struct Cam {
    float fx, fy, cx, cy, bf;
    float tx;   // camera x translation per frame (metres)
};

struct MapPoint {
    float pos[3], normal[3], min_dist, max_dist;
    uint8_t desc[32];
    int32_t obs;
    int last_seen;   // last frame whose mvpMapPoints held it (or that created it)
};

struct FrameData {
    std::vector<orbfe_keypoint> keys, keys_r;
    std::vector<uint8_t> desc, desc_r;
    std::vector<float> ur, depth;
    std::vector<int32_t> mvp;
    int mono_l = 0, mono_r = 0, nstereo = 0;
};

struct Stats {
    double frame_ms = 0, sbp_ms = 0, local_ms = 0, total_ms = 0;
    int n_left = 0, n_right = 0, n_stereo = 0;
    int n_last_pts = 0, sbp_matches = 0, sbp_th = 0;
    int n_local_pts = 0, n_to_match = 0, local_matches = 0;
};

inline double ms_since(std::chrono::steady_clock::time_point t) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

template <class Api>
class Tracker {
public:
    Tracker(Api& api, const Cam& cam, int w, int h, const std::vector<float>& scale, int window)
        : api_(api), cam_(cam), w_(w), h_(h), scale_(scale), window_(window) {
        log_sf_ = (float)std::log(scale.size() > 1 ? scale[1] : 1.2f);   // Frame::mfLogScaleFactor
    }

    // One frame; mvp_out (may be null) receives the frame's mvpMapPoints after SearchLocalPoints.
    Stats step(const uint8_t* L, const uint8_t* R, std::vector<int32_t>* mvp_out) {
        Stats st;
        FrameData cur;
        const auto t0 = std::chrono::steady_clock::now();
        st.n_stereo = api_.frame(L, R, cur);
        st.frame_ms = ms_since(t0);
        st.n_left = (int)cur.keys.size();
        st.n_right = (int)cur.keys_r.size();
        const int N = st.n_left;
        const float Ox = k_ * cam_.tx;   // camera centre (Ox, 0, 0); Rcw = I, tcw = -Ow
        orbfe_frame fr;
        memset(&fr, 0, sizeof(fr));
        fr.n = N;
        fr.keys = cur.keys.data();
        fr.desc = cur.desc.data();
        fr.uright = cur.ur.data();
        fr.min_x = 0.f;
        fr.max_x = (float)w_;
        fr.min_y = 0.f;
        fr.max_y = (float)h_;
        fr.nlevels = (int)scale_.size();
        fr.scale_factors = scale_.data();
        fr.mbf = cam_.bf;
        cur.mvp.assign(N, -1);
        std::vector<int32_t> obs(N, 0);
        // TrackWithMotionModel (the last frame's points projected with the motion-model pose)
        const auto t1 = std::chrono::steady_clock::now();
        if (have_last_) {
            std::vector<orbfe_proj_point> pts;
            pts.reserve(last_.keys.size());
            for (size_t i = 0; i < last_.keys.size(); i++) {
                const int32_t id = last_.mvp[i];
                if (id < 0) continue;
                const MapPoint& p = points_[id];
                orbfe_proj_point q;
                memset(&q, 0, sizeof(q));
                const float xc = p.pos[0] - Ox, yc = p.pos[1], zc = p.pos[2];
                q.invzc = 1.0f / zc;
                q.u = cam_.fx * xc / zc + cam_.cx;   // Pinhole::project
                q.v = cam_.fy * yc / zc + cam_.cy;
                q.valid = q.invzc >= 0 && q.u >= fr.min_x && q.u <= fr.max_x && q.v >= fr.min_y && q.v <= fr.max_y;
                q.octave = last_.keys[i].octave;
                q.angle = last_.keys[i].angle;
                q.observations = p.obs;
                q.id = id;
                memcpy(q.desc, p.desc, 32);
                pts.push_back(q);
            }
            st.n_last_pts = (int)pts.size();
            st.sbp_th = 7;
            st.sbp_matches = api_.sbp_last(&fr, cur.mvp.data(), obs.data(), pts.data(), (int)pts.size(), 7.f, 0, 0, 1);
            if (st.sbp_matches < 20) {   // wider window (Tracking.cc:2928-2935)
                std::fill(cur.mvp.begin(), cur.mvp.end(), -1);
                st.sbp_th = 14;
                st.sbp_matches = api_.sbp_last(&fr, cur.mvp.data(), obs.data(), pts.data(), (int)pts.size(), 14.f, 0, 0, 1);
            }
        }
        st.sbp_ms = ms_since(t1);
        // UpdateLocalPoints (untimed, Tracking.cc:3496-3527, a separate step of TrackLocalMap): the
        // local map = the points held by any of the last `window` frames (the reference takes the
        // points of the covisible keyframes)
        std::vector<int32_t> local_ids;
        for (size_t j = 0; j < points_.size(); j++)
            if (points_[j].last_seen >= k_ - window_) local_ids.push_back((int32_t)j);
        // SearchLocalPoints (Tracking.cc:3382-3452): the frame's matched points skipped, the local
        // points snapshotted (isInFrustum's inputs), the projection + search
        std::vector<uint8_t> held(points_.size(), 0);
        const auto t2 = std::chrono::steady_clock::now();
        {
            for (int i = 0; i < N; i++)
                if (cur.mvp[i] >= 0) {
                    held[cur.mvp[i]] = 1;   // mnLastFrameSeen = current frame: not projected
                    obs[i] = points_[cur.mvp[i]].obs;
                }
            std::vector<orbfe_map_point_3d> lm;
            lm.reserve(local_ids.size());
            for (const int32_t j : local_ids) {
                const MapPoint& p = points_[j];
                orbfe_map_point_3d r;
                memset(&r, 0, sizeof(r));
                memcpy(r.pos, p.pos, 12);
                memcpy(r.normal, p.normal, 12);
                r.min_dist = p.min_dist;
                r.max_dist = p.max_dist;
                r.flags = held[j] ? ORBFE_MP_SKIP : 0;
                r.observations = p.obs;
                r.id = (int32_t)j;
                memcpy(r.desc, p.desc, 32);
                lm.push_back(r);
            }
            st.n_local_pts = (int)lm.size();
            orbfe_camera c;
            memset(&c, 0, sizeof(c));
            c.Rcw[0] = c.Rcw[4] = c.Rcw[8] = 1.f;
            c.tcw[0] = -Ox;
            c.Ow[0] = Ox;
            c.fx = cam_.fx;
            c.fy = cam_.fy;
            c.cx = cam_.cx;
            c.cy = cam_.cy;
            c.log_scale_factor = log_sf_;
            c.view_cos_limit = 0.5f;
            int32_t ntm = 0;
            st.local_matches = lm.empty() ? 0
                                          : api_.local_points(&fr, &c, lm.data(), (int)lm.size(), cur.mvp.data(),
                                                              obs.data(), 1.f, 0, 50.f, 0.8f, &ntm);
            st.n_to_match = ntm;
        }
        st.local_ms = ms_since(t2);
        st.total_ms = ms_since(t0);
        if (mvp_out) *mvp_out = cur.mvp;
        // keyframe bookkeeping (untimed): the frame's points are seen now, and a new point for every
        // stereo keypoint without one
        for (int i = 0; i < N; i++)
            if (cur.mvp[i] >= 0) points_[cur.mvp[i]].last_seen = k_;
        for (int i = 0; i < N; i++) {
            if (cur.mvp[i] >= 0 || !(cur.depth[i] > 0)) continue;
            const orbfe_keypoint& kp = cur.keys[i];
            const float z = cur.depth[i];
            MapPoint p;
            p.pos[0] = Ox + (kp.x - cam_.cx) * z / cam_.fx;
            p.pos[1] = (kp.y - cam_.cy) * z / cam_.fy;
            p.pos[2] = z;
            const float d0 = p.pos[0] - Ox, d1 = p.pos[1], d2 = p.pos[2];
            const float dist = std::sqrt(d0 * d0 + d1 * d1 + d2 * d2);
            p.normal[0] = d0 / dist;
            p.normal[1] = d1 / dist;
            p.normal[2] = d2 / dist;
            p.max_dist = dist * scale_[kp.octave];   // MapPoint::UpdateNormalAndDepth (MapPoint.cc:482-487)
            p.min_dist = p.max_dist / scale_.back();
            memcpy(p.desc, cur.desc.data() + (size_t)i * 32, 32);
            p.obs = 2;
            p.last_seen = k_;
            cur.mvp[i] = (int32_t)points_.size();
            points_.push_back(p);
        }
        last_ = std::move(cur);
        have_last_ = true;
        k_++;
        return st;
    }

private:
    Api& api_;
    Cam cam_;
    int w_, h_;
    std::vector<float> scale_;
    int window_;
    float log_sf_;
    std::vector<MapPoint> points_;
    FrameData last_;
    bool have_last_ = false;
    int k_ = 0;
};

inline double median_of(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? 0.0 : v[v.size() / 2];
}

// Runs the tracker over frames 0 .. frames-1 of a sequence (frames <= npairs: the motion model needs
// consecutive frames), the first kWarm frames untimed; prints one JSON line of medians (per-frame wall
// times of the three calls and the frame) and, when out_path is set, writes per frame {n_left,
// n_right, n_stereo, sbp_th, sbp_matches, n_to_match, local_matches, mvp[n_left]} (int32) for the
// GPU-vs-CPU parity test.
template <class Api, class FL, class FR>
int run_sequence(Api& api, const Cam& cam, int w, int h, const std::vector<float>& scale, int window, int frames,
                 int npairs, FL left, FR right, const char* out_path, const char* label) {
    constexpr int kWarm = 5;
    if (frames > npairs || frames <= kWarm) throw std::runtime_error("tracking: need kWarm < frames <= npairs");
    Tracker<Api> T(api, cam, w, h, scale, window);
    FILE* o = out_path ? fopen(out_path, "wb") : nullptr;
    if (out_path && !o) throw std::runtime_error("cannot open out");
    std::vector<double> fm, sm, lm, tm;
    double nl = 0, nst = 0, nlast = 0, nsbp = 0, nloc = 0, ntm = 0, nlm = 0;
    int cnt = 0;
    std::vector<int32_t> mvp;
    for (int k = 0; k < frames; k++) {
        const Stats s = T.step(left(k), right(k), &mvp);
        if (o) {
            const int32_t rec[7] = {s.n_left, s.n_right, s.n_stereo, s.sbp_th, s.sbp_matches, s.n_to_match, s.local_matches};
            fwrite(rec, 4, 7, o);
            fwrite(mvp.data(), 4, mvp.size(), o);
        }
        if (k < kWarm) continue;
        fm.push_back(s.frame_ms);
        sm.push_back(s.sbp_ms);
        lm.push_back(s.local_ms);
        tm.push_back(s.total_ms);
        nl += s.n_left;
        nst += s.n_stereo;
        nlast += s.n_last_pts;
        nsbp += s.sbp_matches;
        nloc += s.local_matches;
        ntm += s.n_to_match;
        nlm += s.n_local_pts;
        cnt++;
    }
    if (o) fclose(o);
    printf("{\"path\": \"%s\", \"frames_timed\": %d, \"tracking_frame_ms\": %.4f, \"split_ms\": {\"frame_stereo\": %.4f, "
           "\"search_by_projection_last_frame\": %.4f, \"search_local_points\": %.4f}, \"mean\": {\"keypoints_left\": %.1f, "
           "\"stereo_matches\": %.1f, \"last_frame_points\": %.1f, \"last_frame_matches\": %.1f, \"local_map_points\": %.1f, "
           "\"local_to_match\": %.1f, \"local_matches\": %.1f}}\n",
           label, cnt, median_of(tm), median_of(fm), median_of(sm), median_of(lm), nl / cnt, nst / cnt, nlast / cnt,
           nsbp / cnt, nlm / cnt, ntm / cnt, nloc / cnt);
    return 0;
}

}  // namespace trk
