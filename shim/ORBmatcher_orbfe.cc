// Replacement bodies for the Tracking-thread ORBmatcher methods (orb_slam3/src/ORBmatcher.cc) on
// top of liborbfe.so (Frame::ComputeStereoMatches and the stereo Frame's one-call extraction are in
// shim/Frame_orbfe.cc, Tracking::SearchLocalPoints in shim/Tracking_orbfe.cc). The original bodies
// of the replaced methods stay in ORBmatcher.cc / Frame.cc renamed *_cpu: every replacement checks
// the library's return code and, on an error (no device, a capacity or argument limit), logs the
// reason once and runs the *_cpu body instead, so a failure never reaches Tracking as a negative
// nmatches or a silently monocular frame. Both camera layouts are handled on the device: Nleft ==
// -1 frames and the KannalaBrandt8 two-camera frames (Nleft != -1: keys mvKeys ++ mvKeysRight,
// mvLeftToRightMatch / mvRightToLeftMatch).
// Built inside the ORB-SLAM3 tree; this repository compiles it with -fsyntax-only against stand-in
// headers (tests/shim_stubs/, tests/test_shim_compile.py). See INTEGRATION.md.
#include "ORBmatcher.h"

#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>

#include <orbfe.h>

#include "orbfe_glue.h"
#include "orbfe_slam_types.h"

#include "Frame.h"
#include "KeyFrame.h"
#include "ORBextractor.h"
#include "MapPoint.h"

using namespace std;

namespace ORB_SLAM3 {

namespace {

// MapPoint* <-> int32 handle table for one call (the C-ABI carries handles, -1 = NULL).
struct Handles {
    vector<MapPoint*> table;
    unordered_map<MapPoint*, int32_t> id;
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

// One log line per (call site, error code): `what` names the call site; the caller then runs the
// CPU body. A repeated failure of one method never silences the first failure of another.
bool failed(int rc, const char* what) {
    if (rc >= 0) return false;
    static std::mutex mu;
    static std::set<std::pair<std::string, int>> seen;
    bool first;
    {
        std::lock_guard<std::mutex> lk(mu);
        first = seen.emplace(what, rc).second;
    }
    if (first)
        fprintf(stderr, "[orbfe] %s returned %d (%s); running the CPU implementation\n", what, rc,
                rc == ORBFE_E_ARG ? "argument / capacity limit" : rc == ORBFE_E_DEVICE ? "HIP device error"
                : rc == ORBFE_E_CAPACITY ? "capacity" : "error");
    return true;
}

// Frame fields the matchers read (Frame.h). Single camera: mvKeysUn and mDescriptors borrowed.
// Two cameras (Nleft != -1): keys = mvKeys ++ mvKeysRight (AssignFeaturesToGrid's keypoints,
// Frame.cc:401-403) in `keys`, the stereo links borrowed.
orbfe_frame frame_view(const Frame& F, vector<cv::KeyPoint>& keys) {
    orbfe_frame f;
    memset(&f, 0, sizeof(f));
    f.n = F.N;
    if (F.Nleft == -1) {
        f.keys = reinterpret_cast<const orbfe_keypoint*>(F.mvKeysUn.data());
    } else {
        keys.assign(F.mvKeys.begin(), F.mvKeys.end());
        keys.insert(keys.end(), F.mvKeysRight.begin(), F.mvKeysRight.end());
        f.keys = reinterpret_cast<const orbfe_keypoint*>(keys.data());
        f.two_cams = 1;
        f.nleft = F.Nleft;
        f.l2r = F.mvLeftToRightMatch.data();
        f.r2l = F.mvRightToLeftMatch.data();
    }
    f.desc = F.mDescriptors.data;   // N x 32, continuous
    f.uright = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
    f.min_x = Frame::mnMinX; f.max_x = Frame::mnMaxX; f.min_y = Frame::mnMinY; f.max_y = Frame::mnMaxY;
    f.nlevels = F.mnScaleLevels;
    f.scale_factors = F.mvScaleFactors.data();
    f.mbf = F.mbf;
    return f;
}

void slots_of(const Frame& F, Handles& H, vector<int32_t>& mvp, vector<int32_t>* obs) {
    mvp.resize(F.N);
    if (obs) obs->resize(F.N);
    for (int i = 0; i < F.N; i++) {
        MapPoint* p = F.mvpMapPoints[i];
        mvp[i] = H.of(p);
        if (obs) (*obs)[i] = p ? p->Observations() : 0;
    }
}

void copy_desc(const cv::Mat& d, uint8_t out[32]) { memcpy(out, d.ptr<uint8_t>(0), 32); }

// keypoint i of a frame / keyframe in the reference's side-aware lookup
// the left extractor's handle (the device view of the frame it produced last)
orbfe_extractor* handle_of(const Frame& F) {
    return F.mpORBextractorLeft ? static_cast<orbfe_extractor*>(F.mpORBextractorLeft->OrbfeHandle()) : nullptr;
}

const cv::KeyPoint& key_of(const Frame& F, int i) {
    return F.Nleft == -1 ? F.mvKeysUn[i] : i < F.Nleft ? F.mvKeys[i] : F.mvKeysRight[i - F.Nleft];
}

}  // namespace

// ORBmatcher.cc:43-213
int ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, const float th,
                                   const bool bFarPoints, const float thFarPoints) {
    Handles H;
    vector<int32_t> mvp, obs;
    slots_of(F, H, mvp, &obs);
    vector<orbfe_map_point> q(vpMapPoints.size());
    for (size_t i = 0; i < vpMapPoints.size(); i++) {
        MapPoint* p = vpMapPoints[i];
        orbfe_map_point& r = q[i];
        memset(&r, 0, sizeof(r));
        r.proj_x = p->mTrackProjX; r.proj_y = p->mTrackProjY; r.proj_xr = p->mTrackProjXR;
        r.view_cos = p->mTrackViewCos; r.depth = p->mTrackDepth; r.scale_level = p->mnTrackScaleLevel;
        r.flags = (p->mbTrackInView ? ORBFE_MP_IN_VIEW : 0) | (p->isBad() ? ORBFE_MP_BAD : 0);
        if (F.Nleft != -1) {
            r.flags |= p->mbTrackInViewR ? ORBFE_MP_IN_VIEW_R : 0;
            r.proj_yr = p->mTrackProjYR;
            r.view_cos_r = p->mTrackViewCosR;
            r.scale_level_r = p->mnTrackScaleLevelR;
        }
        r.observations = p->Observations();
        r.id = H.of(p);
        if ((r.flags & (ORBFE_MP_IN_VIEW | ORBFE_MP_IN_VIEW_R)) && !(r.flags & ORBFE_MP_BAD))
            copy_desc(p->GetDescriptor(), r.desc);
    }
    vector<cv::KeyPoint> keys;
    const orbfe_frame fr = frame_view(F, keys);
    // the current frame in HBM when its extractor still holds it (single camera)
    const int n = orbfe_glue::on_current_frame(handle_of(F), F.Nleft == -1 ? F.mnOrbfeFrameId : 0, fr,
                                               [&](const orbfe_frame* V) {
        return orbfe_search_by_projection_local(V, mvp.data(), obs.data(), q.data(), (int)q.size(), th, bFarPoints,
                                                thFarPoints, mfNNratio);
    });
    if (failed(n, "orbfe_search_by_projection_local"))
        return SearchByProjection_cpu(F, vpMapPoints, th, bFarPoints, thFarPoints);
    for (int i = 0; i < F.N; i++) F.mvpMapPoints[i] = H.at(mvp[i]);
    return n;
}

// ORBmatcher.cc:1676-1887: the projection (Tcw * x3Dw, mpCamera->project for the left window and for
// GetRelativePoseTrl() * x3Dc, :1702-1718, 1794-1796) runs on the device with the search
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
    const Sophus::SE3f Tcw = CurrentFrame.GetPose();
    const Eigen::Vector3f twc = Tcw.inverse().translation();
    const Eigen::Vector3f tlc = LastFrame.GetPose() * twc;
    const bool bForward = tlc(2) > CurrentFrame.mb && !bMono;
    const bool bBackward = -tlc(2) > CurrentFrame.mb && !bMono;
    const bool two = CurrentFrame.Nleft != -1;
    Handles H;
    vector<int32_t> mvp, obs;
    slots_of(CurrentFrame, H, mvp, &obs);
    vector<orbfe_last_point> q(LastFrame.N);
    for (int i = 0; i < LastFrame.N; i++) {
        orbfe_last_point& r = q[i];
        memset(&r, 0, sizeof(r));
        MapPoint* p = LastFrame.mvpMapPoints[i];
        if (!p || LastFrame.mvbOutlier[i]) continue;   // valid = 0
        const Eigen::Vector3f x3Dw = p->GetWorldPos();
        r.pos[0] = x3Dw(0); r.pos[1] = x3Dw(1); r.pos[2] = x3Dw(2);
        // nLastOctave and kpLF (:1721-1722, :1765-1767)
        r.octave = (LastFrame.Nleft == -1 || i < LastFrame.Nleft) ? LastFrame.mvKeys[i].octave
                                                                   : LastFrame.mvKeysRight[i - LastFrame.Nleft].octave;
        r.angle = key_of(LastFrame, i).angle;
        r.valid = 1;
        r.observations = p->Observations();
        r.id = H.of(p);
        copy_desc(p->GetDescriptor(), r.desc);
    }
    const orbfe_pose pcw = orbfe_shim::pose_of(Tcw);
    const orbfe_pose prl = two ? orbfe_shim::pose_of(CurrentFrame.GetRelativePoseTrl()) : pcw;
    const orbfe_camera_model cam = orbfe_shim::model_of(CurrentFrame.mpCamera);
    vector<cv::KeyPoint> keys;
    const orbfe_frame fr = frame_view(CurrentFrame, keys);
    const int n = orbfe_glue::on_current_frame(handle_of(CurrentFrame), two ? 0 : CurrentFrame.mnOrbfeFrameId, fr,
                                               [&](const orbfe_frame* V) {
        return orbfe_search_by_projection_lastframe_pose(V, mvp.data(), obs.data(), q.data(), (int)q.size(), &pcw,
                                                         two ? &prl : nullptr, &cam, th, bForward, bBackward,
                                                         mbCheckOrientation);
    });
    if (failed(n, "orbfe_search_by_projection_lastframe_pose"))
        return SearchByProjection_cpu(CurrentFrame, LastFrame, th, bMono);
    for (int i = 0; i < CurrentFrame.N; i++) CurrentFrame.mvpMapPoints[i] = H.at(mvp[i]);
    return n;
}

// ORBmatcher.cc:1889-2010 (no right-camera branch: the left grid of a two-camera frame)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, KeyFrame* pKF, const set<MapPoint*>& sAlreadyFound,
                                   const float th, const int ORBdist) {
    const Sophus::SE3f Tcw = CurrentFrame.GetPose();
    const Eigen::Vector3f Ow = Tcw.inverse().translation();
    const vector<MapPoint*> vpMPs = pKF->GetMapPointMatches();
    Handles H;
    vector<int32_t> mvp;
    slots_of(CurrentFrame, H, mvp, nullptr);
    vector<orbfe_proj_point> q(vpMPs.size());
    for (size_t i = 0; i < vpMPs.size(); i++) {
        orbfe_proj_point& r = q[i];
        memset(&r, 0, sizeof(r));
        MapPoint* p = vpMPs[i];
        if (!p || p->isBad() || sAlreadyFound.count(p)) continue;
        const Eigen::Vector3f x3Dw = p->GetWorldPos();
        const Eigen::Vector3f x3Dc = Tcw * x3Dw;
        const Eigen::Vector2f uv = CurrentFrame.mpCamera->project(x3Dc);
        if (uv(0) < CurrentFrame.mnMinX || uv(0) > CurrentFrame.mnMaxX) continue;
        if (uv(1) < CurrentFrame.mnMinY || uv(1) > CurrentFrame.mnMaxY) continue;
        const float dist3D = (x3Dw - Ow).norm();
        if (dist3D < p->GetMinDistanceInvariance() || dist3D > p->GetMaxDistanceInvariance()) continue;
        r.u = uv(0); r.v = uv(1);
        r.octave = p->PredictScale(dist3D, &CurrentFrame);
        r.angle = pKF->mvKeysUn[i].angle;
        r.valid = 1;
        r.id = H.of(p);
        copy_desc(p->GetDescriptor(), r.desc);
    }
    vector<cv::KeyPoint> keys;
    const orbfe_frame fr = frame_view(CurrentFrame, keys);
    const int n = orbfe_search_by_projection_kf(&fr, mvp.data(), q.data(), (int)q.size(), th,
                                                ORBdist, mbCheckOrientation);
    if (failed(n, "orbfe_search_by_projection_kf"))
        return SearchByProjection_cpu(CurrentFrame, pKF, sAlreadyFound, th, ORBdist);
    for (int i = 0; i < CurrentFrame.N; i++) CurrentFrame.mvpMapPoints[i] = H.at(mvp[i]);
    return n;
}

// ORBmatcher.cc:648-763 (monocular initialisation: single-camera frames)
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
                                        vector<int>& vnMatches12, int windowSize) {
    static_assert(sizeof(cv::Point2f) == 8, "Point2f layout");
    vector<cv::KeyPoint> k1, k2;
    const orbfe_frame f1 = frame_view(F1, k1), f2 = frame_view(F2, k2);
    vector<cv::Point2f> prev(vbPrevMatched);
    vector<int> m12(F1.mvKeysUn.size(), -1);
    const int n = orbfe_search_for_initialization(&f1, &f2, reinterpret_cast<float*>(prev.data()), m12.data(),
                                                  windowSize, mfNNratio, mbCheckOrientation);
    if (failed(n, "orbfe_search_for_initialization"))
        return SearchForInitialization_cpu(F1, F2, vbPrevMatched, vnMatches12, windowSize);
    vbPrevMatched.swap(prev);
    vnMatches12.swap(m12);
    return n;
}

// ORBmatcher.cc:223-425
int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches) {
    const vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    Handles H;
    vector<int32_t> kf_mp(vpMapPointsKF.size());
    for (size_t i = 0; i < vpMapPointsKF.size(); i++) {
        MapPoint* p = vpMapPointsKF[i];
        kf_mp[i] = (p && !p->isBad()) ? H.of(p) : -1;
    }
    // kp of the KF index (:327-329): mvKeysUn, or by side for a two-camera KF
    vector<cv::KeyPoint> kf_keys;
    if (pKF->mpCamera2) {
        kf_keys.resize(vpMapPointsKF.size());
        for (size_t i = 0; i < kf_keys.size(); i++)
            kf_keys[i] = (int)i >= pKF->NLeft ? pKF->mvKeysRight[i - pKF->NLeft] : pKF->mvKeys[i];
    }
    auto flatten = [](const DBoW2::FeatureVector& fv, vector<uint32_t>& ids, vector<int32_t>& off,
                      vector<uint32_t>& idx) {
        off.push_back(0);
        for (const auto& kv : fv) {
            ids.push_back(kv.first);
            idx.insert(idx.end(), kv.second.begin(), kv.second.end());
            off.push_back((int32_t)idx.size());
        }
    };
    vector<uint32_t> kid, kidx, fid, fidx;
    vector<int32_t> koff, foff;
    flatten(pKF->mFeatVec, kid, koff, kidx);
    flatten(F.mFeatVec, fid, foff, fidx);
    const orbfe_feature_vector kfv{(int32_t)kid.size(), kid.data(), koff.data(), kidx.data()};
    const orbfe_feature_vector ffv{(int32_t)fid.size(), fid.data(), foff.data(), fidx.data()};
    vector<int32_t> out(F.N, -1);
    vector<cv::KeyPoint> keys;
    const orbfe_frame fr = frame_view(F, keys);
    const int n = orbfe_search_by_bow(
        reinterpret_cast<const orbfe_keypoint*>(pKF->mpCamera2 ? kf_keys.data() : pKF->mvKeysUn.data()),
        pKF->mDescriptors.data, kf_mp.data(), (int)kf_mp.size(), &kfv, &fr, &ffv, out.data(), mfNNratio,
        mbCheckOrientation);
    if (failed(n, "orbfe_search_by_bow")) return SearchByBoW_cpu(pKF, F, vpMapPointMatches);
    vpMapPointMatches.assign(F.N, nullptr);
    for (int i = 0; i < F.N; i++) vpMapPointMatches[i] = H.at(out[i]);
    return n;
}

}  // namespace ORB_SLAM3
