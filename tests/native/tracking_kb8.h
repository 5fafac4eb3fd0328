// The per-frame front-end work of Tracking::Track for a KannalaBrandt8 two-camera rig (BASELINE config 4,
// TUM-VI stereo(-inertial), Nleft != -1), over a seeded synthetic 512x512 stereo sequence, written once
// against an "Api" of the calls Tracking makes into the ORB front-end, like tracking_loop.h:
//   Frame::Frame(stereo, KB8) (Frame.cc:1034-1105): ExtractORB x 2 with vLappingArea {0, 511}
//       (:1059-1062), ComputeStereoFishEyeMatches' descriptor stage (:1126-1151: knnMatch k = 2 over
//       the lapping rows, ratio 0.7) -> mvLeftToRightMatch / mvRightToLeftMatch
//   TrackWithMotionModel: SearchByProjection(CurrentFrame, LastFrame, th 7, retried at 14 below 20
//       matches) with the right-camera projections (ORBmatcher.cc:1676-1887, :1794-1858)
//   TrackLocalMap -> SearchLocalPoints: isInFrustum(Checks) for both cameras over the local map
//       points not matched yet, then SearchByProjection(F, local map, th) with the right-camera branch
//       (Tracking.cc:3382-3452, Frame.cc:1168-1242, ORBmatcher.cc:43-213); th 2 = a stereo-inertial
//       map after the second inertial BA (Tracking.cc:3434-3437)
// tests/native/capi_frontend.cpp instantiates it with the library (--tracking-kb8), tracking_cpu.cpp
// with the CPU restatement; the bookkeeping between the calls is shared host code, so both runs see
// the same inputs whenever the calls return the same outputs.
//
// Geometry: the rectified sequence of tracking_loop.h (a plane at disparity SEQ_DISP, the rig moving
// SEQ_SHIFT px per frame) seen through a KannalaBrandt8 model whose coefficients are tan's Taylor
// series (k0..k3 = 1/3, 2/15, 17/315, 62/2835: theta_d(theta) ~ tan(theta) within 0.04 % over the
// image), so the synthetic pinhole-rendered images and the fisheye projections agree; the right camera
// is the left one translated by the baseline (Trl = [I | (-b, 0, 0)]). TriangulateMatches (the KB8
// depth check after the ratio test, a CPU post-filter of the camera model) is replaced by the
// sequence's known depth: every ratio-test pair is a stereo match.
#pragma once
#include <cmath>

#include "tracking_loop.h"

namespace trk {

struct Kb8 {
    float fx, fy, cx, cy, k0, k1, k2, k3;
};

// KannalaBrandt8::project (KannalaBrandt8.cpp:67-82), as the shim calls it on the host
inline void kb8_project(const Kb8& c, float x, float y, float z, float* u, float* v) {
    const float x2_plus_y2 = x * x + y * y;
    const float theta = atan2f(sqrtf(x2_plus_y2), z);
    const float psi = atan2f(y, x);
    const float theta2 = theta * theta, theta3 = theta * theta2, theta5 = theta3 * theta2, theta7 = theta5 * theta2,
                theta9 = theta7 * theta2;
    const float r = theta + c.k0 * theta3 + c.k1 * theta5 + c.k2 * theta7 + c.k3 * theta9;
    *u = c.fx * r * cosf(psi) + c.cx;
    *v = c.fy * r * sinf(psi) + c.cy;
}

inline orbfe_camera_model kb8_model(const Kb8& c) {
    orbfe_camera_model m;
    memset(&m, 0, sizeof(m));
    m.type = ORBFE_CAM_KANNALA_BRANDT8;
    const float p[8] = {c.fx, c.fy, c.cx, c.cy, c.k0, c.k1, c.k2, c.k3};
    memcpy(m.params, p, sizeof(p));
    return m;
}

// Frame(stereo, KB8): keys = mvKeys ++ mvKeysRight, desc likewise, the stereo links
struct FrameKB8 {
    std::vector<orbfe_keypoint> keys;
    std::vector<uint8_t> desc;
    std::vector<int32_t> l2r, r2l, mvp;
    int nl = 0, nr = 0, mono_l = 0, mono_r = 0, nstereo = 0;
};

// ComputeStereoFishEyeMatches' bookkeeping (Frame.cc:1144-1160) from the kNN stage's per-query
// train index (right lapping row, -1 = failed ratio test): queries in order, the later one keeps a
// right keypoint two queries chose (mvRightToLeftMatch is overwritten)
inline int fisheye_links(FrameKB8& f, const std::vector<int32_t>& train) {
    f.l2r.assign(f.nl, -1);
    f.r2l.assign(f.nr, -1);
    int n = 0;
    for (int q = 0; q < (int)train.size(); q++) {
        if (train[q] < 0) continue;
        const int il = q + f.mono_l, ir = train[q] + f.mono_r;
        f.l2r[il] = ir;
        f.r2l[ir] = il;
        n++;
    }
    return n;
}

template <class Api>
class TrackerKB8 {
public:
    TrackerKB8(Api& api, const Cam& cam, int w, int h, const std::vector<float>& scale, int window)
        : api_(api), cam_(cam), w_(w), h_(h), scale_(scale), window_(window) {
        log_sf_ = (float)std::log(scale.size() > 1 ? scale[1] : 1.2f);
        kb_ = Kb8{cam.fx, cam.fy, cam.cx, cam.cy, 1.f / 3.f, 2.f / 15.f, 17.f / 315.f, 62.f / 2835.f};
        b_ = cam.bf / cam.fx;
        memset(&rig_, 0, sizeof(rig_));
        rig_.left = kb8_model(kb_);
        rig_.right = kb8_model(kb_);
        rig_.Rrl[0] = rig_.Rrl[4] = rig_.Rrl[8] = 1.f;
        rig_.trl[0] = -b_;
        rig_.tlr[0] = b_;
        rig_.Rwc[0] = rig_.Rwc[4] = rig_.Rwc[8] = 1.f;
    }

    Stats step(const uint8_t* L, const uint8_t* R, std::vector<int32_t>* mvp_out) {
        Stats st;
        FrameKB8 cur;
        const auto t0 = std::chrono::steady_clock::now();
        st.n_stereo = api_.frame_kb8(L, R, cur);
        st.frame_ms = ms_since(t0);
        st.n_left = cur.nl;
        st.n_right = cur.nr;
        const int N = cur.nl + cur.nr;
        const float Ox = k_ * cam_.tx;   // camera centre (Ox, 0, 0); Rcw = I, tcw = -Ow
        orbfe_frame fr;
        memset(&fr, 0, sizeof(fr));
        fr.n = N;
        fr.keys = cur.keys.data();
        fr.desc = cur.desc.data();
        fr.min_x = 0.f;
        fr.max_x = (float)w_;
        fr.min_y = 0.f;
        fr.max_y = (float)h_;
        fr.nlevels = (int)scale_.size();
        fr.scale_factors = scale_.data();
        fr.mbf = cam_.bf;
        fr.two_cams = 1;
        fr.nleft = cur.nl;
        fr.l2r = cur.l2r.data();
        fr.r2l = cur.r2l.data();
        cur.mvp.assign(N, -1);
        std::vector<int32_t> obs(N, 0);
        // TrackWithMotionModel: the last frame's points (both cameras' slots), projected by the search
        // itself (orbfe_search_by_projection_lastframe_pose: x3Dc = Tcw * x3Dw, mpCamera->project for the
        // left window and for Trl * x3Dc, ORBmatcher.cc:1702-1718, 1794-1796); Rcw = I here, so Tcw is
        // the quaternion (0, 0, 0, 1) with tcw = -Ow, and Trl the rig's baseline
        const auto t1 = std::chrono::steady_clock::now();
        if (have_last_) {
            std::vector<orbfe_last_point> pts;
            for (int i = 0; i < (int)last_.mvp.size(); i++) {
                const int32_t id = last_.mvp[i];
                if (id < 0) continue;
                const MapPoint& p = points_[id];
                orbfe_last_point q;
                memset(&q, 0, sizeof(q));
                memcpy(q.pos, p.pos, 12);
                const orbfe_keypoint& kp = last_.keys[i];   // mvKeys[i] or mvKeysRight[i - Nleft]
                q.octave = kp.octave;
                q.angle = kp.angle;
                q.observations = p.obs;
                q.id = id;
                q.valid = 1;
                memcpy(q.desc, p.desc, 32);
                pts.push_back(q);
            }
            orbfe_pose Tcw, Trl;
            memset(&Tcw, 0, sizeof(Tcw));
            memset(&Trl, 0, sizeof(Trl));
            Tcw.q[3] = Trl.q[3] = 1.f;
            Tcw.t[0] = -Ox;
            Trl.t[0] = -b_;
            const orbfe_camera_model cam = kb8_model(kb_);
            st.n_last_pts = (int)pts.size();
            st.sbp_th = 7;
            st.sbp_matches = api_.sbp_last_pose(&fr, cur.mvp.data(), obs.data(), pts.data(), (int)pts.size(), &Tcw,
                                                &Trl, &cam, 7.f);
            if (st.sbp_matches < 20) {
                std::fill(cur.mvp.begin(), cur.mvp.end(), -1);
                st.sbp_th = 14;
                st.sbp_matches = api_.sbp_last_pose(&fr, cur.mvp.data(), obs.data(), pts.data(), (int)pts.size(),
                                                    &Tcw, &Trl, &cam, 14.f);
            }
        }
        st.sbp_ms = ms_since(t1);
        std::vector<int32_t> local_ids;   // UpdateLocalPoints (untimed)
        for (size_t j = 0; j < points_.size(); j++)
            if (points_[j].last_seen >= k_ - window_) local_ids.push_back((int32_t)j);
        std::vector<uint8_t> held(points_.size(), 0);
        const auto t2 = std::chrono::steady_clock::now();
        {
            for (int i = 0; i < N; i++)
                if (cur.mvp[i] >= 0) {
                    held[cur.mvp[i]] = 1;
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
                r.id = j;
                memcpy(r.desc, p.desc, 32);
                lm.push_back(r);
            }
            st.n_local_pts = (int)lm.size();
            orbfe_camera c;
            memset(&c, 0, sizeof(c));
            c.Rcw[0] = c.Rcw[4] = c.Rcw[8] = 1.f;
            c.tcw[0] = -Ox;
            c.Ow[0] = Ox;
            c.log_scale_factor = log_sf_;
            c.view_cos_limit = 0.5f;
            int32_t ntm = 0;
            st.local_matches = lm.empty() ? 0
                                          : api_.local_points_rig(&fr, &c, &rig_, lm.data(), (int)lm.size(),
                                                                  cur.mvp.data(), obs.data(), 2.f, &ntm);
            st.n_to_match = ntm;
        }
        st.local_ms = ms_since(t2);
        st.total_ms = ms_since(t0);
        if (mvp_out) *mvp_out = cur.mvp;
        // keyframe bookkeeping (untimed): seen points; a new point at the sequence's depth for every
        // left keypoint with a stereo partner and no point (held by both of the pair's slots)
        for (int i = 0; i < N; i++)
            if (cur.mvp[i] >= 0) points_[cur.mvp[i]].last_seen = k_;
        const float z = cam_.bf / (float)16;   // SEQ_DISP
        for (int i = 0; i < cur.nl; i++) {
            const int ir = cur.l2r[i];
            if (cur.mvp[i] >= 0 || ir < 0 || cur.mvp[cur.nl + ir] >= 0) continue;
            const orbfe_keypoint& kp = cur.keys[i];
            MapPoint p;
            p.pos[0] = Ox + (kp.x - cam_.cx) * z / cam_.fx;   // the plane's point (pinhole ~ this KB8 model)
            p.pos[1] = (kp.y - cam_.cy) * z / cam_.fy;
            p.pos[2] = z;
            const float d0 = p.pos[0] - Ox, d1 = p.pos[1], d2 = p.pos[2];
            const float dist = std::sqrt(d0 * d0 + d1 * d1 + d2 * d2);
            p.normal[0] = d0 / dist;
            p.normal[1] = d1 / dist;
            p.normal[2] = d2 / dist;
            p.max_dist = dist * scale_[kp.octave];
            p.min_dist = p.max_dist / scale_.back();
            memcpy(p.desc, cur.desc.data() + (size_t)i * 32, 32);
            p.obs = 2;
            p.last_seen = k_;
            cur.mvp[i] = cur.mvp[cur.nl + ir] = (int32_t)points_.size();
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
    float log_sf_, b_;
    Kb8 kb_;
    orbfe_stereo_rig rig_;
    std::vector<MapPoint> points_;
    FrameKB8 last_;
    bool have_last_ = false;
    int k_ = 0;
};

// run_sequence of tracking_loop.h for the two-camera tracker (same JSON line and record format; the
// per-frame mvp covers both cameras' slots)
template <class Api, class FL, class FR>
int run_sequence_kb8(Api& api, const Cam& cam, int w, int h, const std::vector<float>& scale, int window, int frames,
                     int npairs, FL left, FR right, const char* out_path, const char* label) {
    constexpr int kWarm = 5;
    if (frames > npairs || frames <= kWarm) throw std::runtime_error("tracking: need kWarm < frames <= npairs");
    TrackerKB8<Api> T(api, cam, w, h, scale, window);
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
    printf("{\"path\": \"%s\", \"frames_timed\": %d, \"tracking_frame_ms\": %.4f, \"split_ms\": {\"frame_stereo_kb8\": %.4f, "
           "\"search_by_projection_last_frame\": %.4f, \"search_local_points\": %.4f}, \"mean\": {\"keypoints_left\": %.1f, "
           "\"stereo_matches\": %.1f, \"last_frame_points\": %.1f, \"last_frame_matches\": %.1f, \"local_map_points\": %.1f, "
           "\"local_to_match\": %.1f, \"local_matches\": %.1f}}\n",
           label, cnt, median_of(tm), median_of(fm), median_of(sm), median_of(lm), nl / cnt, nst / cnt, nlast / cnt,
           nsbp / cnt, nlm / cnt, ntm / cnt, nloc / cnt);
    return 0;
}

}  // namespace trk
