// Tracking::SearchLocalPoints (orb_slam3/src/Tracking.cc:3382-3452) on top of liborbfe.so: the
// isInFrustum loop over the local map and SearchByProjection(F, vpLocalMapPoints, th) become ONE
// device call (orbfe_search_local_points_track through shim/orbfe_glue.h), after which this file
// applies the loop's side effects on the MapPoints in the reference's order. Built inside the
// ORB-SLAM3 tree; this repository compiles it with -fsyntax-only against stand-in headers
// (tests/test_shim_compile.py). INTEGRATION.md §2: the original body stays in Tracking.cc renamed
// SearchLocalPoints_cpu (declared in Tracking.h) and is not called by this file; the fallback below
// runs the frustum loop and the matcher call only, because the first loop's side effects have
// already happened by then.
#include "Tracking.h"

#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>

#include <orbfe.h>

#include "Atlas.h"
#include "Frame.h"
#include "LocalMapping.h"
#include "MapPoint.h"
#include "ORBextractor.h"
#include "ORBmatcher.h"
#include "orbfe_glue.h"
#include "orbfe_slam_types.h"

using namespace std;

namespace ORB_SLAM3 {

namespace {

void log_fallback(int rc, const char* what) {   // one line per (call site, code), as the matcher shims
    static std::mutex mu;
    static std::set<std::pair<std::string, int>> seen;
    bool first;
    {
        std::lock_guard<std::mutex> lk(mu);
        first = seen.emplace(what, rc).second;
    }
    if (first) fprintf(stderr, "[orbfe] %s returned %d; running the CPU implementation\n", what, rc);
}

// MapPoint* <-> int32 handle table for one call (see ORBmatcher_orbfe.cc)
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

void rowmajor(const Eigen::Matrix3f& R, float* out) {
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) out[3 * r + c] = R(r, c);
}

}  // namespace

void Tracking::SearchLocalPoints() {
    Frame& F = mCurrentFrame;
    // Do not search map points already matched (:3384-3402, unchanged)
    for (vector<MapPoint*>::iterator vit = F.mvpMapPoints.begin(), vend = F.mvpMapPoints.end(); vit != vend; vit++) {
        MapPoint* pMP = *vit;
        if (!pMP) continue;
        if (pMP->isBad()) {
            *vit = static_cast<MapPoint*>(NULL);
        } else {
            pMP->IncreaseVisible();
            pMP->mnLastFrameSeen = F.mnId;
            pMP->mbTrackInView = false;
            pMP->mbTrackInViewR = false;
        }
    }
    // the points the frustum loop visits (:3407-3413), in mvpLocalMapPoints order; the others
    // cannot match (seen this frame: mbTrackInView false; bad: skipped by the matcher)
    Handles H;
    vector<MapPoint*> pts;
    vector<orbfe_map_point_3d> recs;
    pts.reserve(mvpLocalMapPoints.size());
    recs.reserve(mvpLocalMapPoints.size());
    for (MapPoint* pMP : mvpLocalMapPoints) {
        if (pMP->mnLastFrameSeen == F.mnId || pMP->isBad()) continue;
        orbfe_map_point_3d r;
        memset(&r, 0, sizeof(r));
        const Eigen::Vector3f X = pMP->GetWorldPos(), n = pMP->GetNormal();
        for (int k = 0; k < 3; k++) { r.pos[k] = X(k); r.normal[k] = n(k); }
        r.min_dist = pMP->GetMinDistance();   // accessors INTEGRATION.md §2 adds to MapPoint.h
        r.max_dist = pMP->GetMaxDistance();
        r.observations = pMP->Observations();
        r.id = H.of(pMP);
        r.track_depth = pMP->mTrackDepth;
        memcpy(r.desc, pMP->GetDescriptor().data, 32);
        pts.push_back(pMP);
        recs.push_back(r);
    }
    // the search radius factor (:3429-3448, unchanged)
    int th = 1;
    if (mSensor == System::RGBD || mSensor == System::IMU_RGBD) th = 3;
    if (mpAtlas->isImuInitialized()) {
        if (mpAtlas->GetCurrentMap()->GetIniertialBA2()) th = 2;
        else th = 6;
    } else if (!mpAtlas->isImuInitialized() &&
               (mSensor == System::IMU_MONOCULAR || mSensor == System::IMU_STEREO || mSensor == System::IMU_RGBD)) {
        th = 10;
    }
    if (F.mnId < mnLastRelocFrameId + 2) th = 5;
    if (mState == LOST || mState == RECENTLY_LOST) th = 15;

    // the frame as the matchers see it (ORBmatcher_orbfe.cc frame_view) and its slots
    vector<cv::KeyPoint> keys;
    orbfe_frame fr;
    memset(&fr, 0, sizeof(fr));
    fr.n = F.N;
    if (F.Nleft == -1) {
        fr.keys = reinterpret_cast<const orbfe_keypoint*>(F.mvKeysUn.data());
    } else {
        keys.assign(F.mvKeys.begin(), F.mvKeys.end());
        keys.insert(keys.end(), F.mvKeysRight.begin(), F.mvKeysRight.end());
        fr.keys = reinterpret_cast<const orbfe_keypoint*>(keys.data());
        fr.two_cams = 1;
        fr.nleft = F.Nleft;
        fr.l2r = F.mvLeftToRightMatch.data();
        fr.r2l = F.mvRightToLeftMatch.data();
    }
    fr.desc = F.mDescriptors.data;
    fr.uright = F.mvuRight.empty() ? nullptr : F.mvuRight.data();
    fr.min_x = Frame::mnMinX; fr.max_x = Frame::mnMaxX; fr.min_y = Frame::mnMinY; fr.max_y = Frame::mnMaxY;
    fr.nlevels = F.mnScaleLevels;
    fr.scale_factors = F.mvScaleFactors.data();
    fr.mbf = F.mbf;
    vector<int32_t> mvp(F.N), obs(F.N);
    for (int i = 0; i < F.N; i++) {
        MapPoint* p = F.mvpMapPoints[i];
        mvp[i] = H.of(p);
        obs[i] = p ? p->Observations() : 0;
    }
    // isInFrustum's inputs: the pose, the camera models and, for a two-camera frame, the rig
    // (Frame.cc:512-586, 1168-1242)
    const Sophus::SE3f Tcw = F.GetPose();
    float Rcw[9], tcw[3], Ow[3];
    rowmajor(Tcw.rotationMatrix(), Rcw);
    const Eigen::Vector3f t = Tcw.translation(), O = F.GetCameraCenter();
    for (int k = 0; k < 3; k++) { tcw[k] = t(k); Ow[k] = O(k); }
    const orbfe_camera cam = orbfe_glue::camera(Rcw, tcw, Ow, 0.f, 0.f, 0.f, 0.f, F.mfLogScaleFactor, 0.5f);
    orbfe_stereo_rig rig;
    memset(&rig, 0, sizeof(rig));
    rig.left = orbfe_shim::model_of(F.mpCamera);
    if (F.Nleft != -1) {
        rig.right = orbfe_shim::model_of(F.mpCamera2);
        const Sophus::SE3f Trl = F.GetRelativePoseTrl(), Tlr = F.GetRelativePoseTlr();
        rowmajor(Trl.rotationMatrix(), rig.Rrl);
        const Eigen::Vector3f trl = Trl.translation(), tlr = Tlr.translation();
        for (int k = 0; k < 3; k++) { rig.trl[k] = trl(k); rig.tlr[k] = tlr(k); }
        rowmajor(F.GetRotationInverse(), rig.Rwc);
    }
    vector<orbfe_map_point> track;
    int32_t nToMatch = 0;
    // the current frame in HBM while its extractor still holds it (single camera, Frame_orbfe.cc)
    orbfe_extractor* hl = F.mpORBextractorLeft ? static_cast<orbfe_extractor*>(F.mpORBextractorLeft->OrbfeHandle()) : nullptr;
    const int n = orbfe_glue::on_current_frame(hl, F.Nleft == -1 ? F.mnOrbfeFrameId : 0, fr, [&](const orbfe_frame* V) {
        return orbfe_glue::local_points(V, &cam, &rig, recs.data(), (int32_t)recs.size(), mvp.data(), obs.data(),
                                        (float)th, mpLocalMapper->mbFarPoints, mpLocalMapper->mThFarPoints, track,
                                        &nToMatch);
    });
    if (n < 0) {
        // the frustum loop and the matcher call of the reference (:3404-3452); the first loop's
        // side effects above have already happened
        log_fallback(n, "orbfe_search_local_points_track");
        int nToMatchCpu = 0;
        for (MapPoint* pMP : pts) {
            if (F.isInFrustum(pMP, 0.5)) {
                pMP->IncreaseVisible();
                nToMatchCpu++;
            }
            if (pMP->mbTrackInView) F.mmProjectPoints[pMP->mnId] = cv::Point2f(pMP->mTrackProjX, pMP->mTrackProjY);
        }
        if (nToMatchCpu > 0) {
            ORBmatcher matcher(0.8);
            matcher.SearchByProjection(F, mvpLocalMapPoints, th, mpLocalMapper->mbFarPoints,
                                       mpLocalMapper->mThFarPoints);
        }
        return;
    }
    // the frustum loop's side effects, in point order (:3415-3424; Frame.cc:512-586 for the fields:
    // a single-camera point's projection is written once it falls in the image, the two-camera
    // views' fields only when they pass; mTrackDepthR, which nothing reads, is not carried)
    for (size_t i = 0; i < pts.size(); i++) {
        MapPoint* pMP = pts[i];
        const orbfe_map_point& r = track[i];
        const bool inL = (r.flags & ORBFE_MP_IN_VIEW) != 0, inR = (r.flags & ORBFE_MP_IN_VIEW_R) != 0;
        pMP->mbTrackInView = inL;
        pMP->mTrackDepth = r.depth;
        if (F.Nleft == -1) {
            pMP->mTrackProjX = r.proj_x;
            pMP->mTrackProjY = r.proj_y;
            if (inL) {
                pMP->mTrackProjXR = r.proj_xr;
                pMP->mnTrackScaleLevel = r.scale_level;
                pMP->mTrackViewCos = r.view_cos;
            }
        } else {
            pMP->mbTrackInViewR = inR;
            pMP->mnTrackScaleLevel = r.scale_level;
            pMP->mnTrackScaleLevelR = r.scale_level_r;
            if (inL) {
                pMP->mTrackProjX = r.proj_x;
                pMP->mTrackProjY = r.proj_y;
                pMP->mTrackViewCos = r.view_cos;
            }
            if (inR) {
                pMP->mTrackProjXR = r.proj_xr;
                pMP->mTrackProjYR = r.proj_yr;
                pMP->mTrackViewCosR = r.view_cos_r;
            }
        }
        if (inL || inR) pMP->IncreaseVisible();
        if (inL) F.mmProjectPoints[pMP->mnId] = cv::Point2f(r.proj_x, r.proj_y);
    }
    // SearchByProjection's result (:3451): the slots the search assigned
    if (nToMatch > 0)
        for (int i = 0; i < F.N; i++) F.mvpMapPoints[i] = H.at(mvp[i]);
}

}  // namespace ORB_SLAM3
