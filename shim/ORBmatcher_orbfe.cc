// Replacement bodies for the Tracking-thread ORBmatcher methods (orb_slam3/src/ORBmatcher.cc)
// and Frame::ComputeStereoMatches (Frame.cc:811-981) on top of liborbfe.so. The original
// bodies of these methods are removed from ORBmatcher.cc / Frame.cc; every other method
// (SearchForTriangulation, Fuse, SearchBySim3, ...) keeps its CPU code. The KannalaBrandt8
// branches (F.Nleft != -1) keep the original code, renamed *_cpu.
// Built inside the ORB-SLAM3 tree; NOT compiled in this repository's container (no OpenCV /
// Eigen / Sophus here). See INTEGRATION.md.
#include "ORBmatcher.h"

#include <cstring>
#include <unordered_map>

#include <orbfe.h>

#include "Frame.h"
#include "KeyFrame.h"
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

// Frame fields the matchers read (Frame.h); mvKeysUn and mDescriptors stay borrowed.
orbfe_frame frame_view(const Frame& F) {
    orbfe_frame f;
    f.n = F.N;
    f.keys = reinterpret_cast<const orbfe_keypoint*>(F.mvKeysUn.data());
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

}  // namespace

// ORBmatcher.cc:43-213
int ORBmatcher::SearchByProjection(Frame& F, const vector<MapPoint*>& vpMapPoints, const float th,
                                   const bool bFarPoints, const float thFarPoints) {
    if (F.Nleft != -1) return SearchByProjection_cpu(F, vpMapPoints, th, bFarPoints, thFarPoints);
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
        r.observations = p->Observations();
        r.id = H.of(p);
        if (r.flags == ORBFE_MP_IN_VIEW) copy_desc(p->GetDescriptor(), r.desc);
    }
    const orbfe_frame fr = frame_view(F);
    const int n = orbfe_search_by_projection_local(&fr, mvp.data(), obs.data(), q.data(), (int)q.size(),
                                                   th, bFarPoints, thFarPoints, mfNNratio);
    for (int i = 0; i < F.N; i++) F.mvpMapPoints[i] = H.at(mvp[i]);
    return n;
}

// ORBmatcher.cc:1676-1887 (projection with Tcw stays on the host, as in the reference)
int ORBmatcher::SearchByProjection(Frame& CurrentFrame, const Frame& LastFrame, const float th, const bool bMono) {
    if (CurrentFrame.Nleft != -1 || LastFrame.Nleft != -1)
        return SearchByProjection_cpu(CurrentFrame, LastFrame, th, bMono);
    const Sophus::SE3f Tcw = CurrentFrame.GetPose();
    const Eigen::Vector3f twc = Tcw.inverse().translation();
    const Eigen::Vector3f tlc = LastFrame.GetPose() * twc;
    const bool bForward = tlc(2) > CurrentFrame.mb && !bMono;
    const bool bBackward = -tlc(2) > CurrentFrame.mb && !bMono;
    Handles H;
    vector<int32_t> mvp, obs;
    slots_of(CurrentFrame, H, mvp, &obs);
    vector<orbfe_proj_point> q(LastFrame.N);
    for (int i = 0; i < LastFrame.N; i++) {
        orbfe_proj_point& r = q[i];
        memset(&r, 0, sizeof(r));
        MapPoint* p = LastFrame.mvpMapPoints[i];
        if (!p || LastFrame.mvbOutlier[i]) continue;   // valid = 0
        const Eigen::Vector3f x3Dc = Tcw * p->GetWorldPos();
        r.invzc = 1.0 / x3Dc(2);
        const Eigen::Vector2f uv = CurrentFrame.mpCamera->project(x3Dc);
        r.u = uv(0); r.v = uv(1);
        r.octave = LastFrame.mvKeys[i].octave;
        r.angle = LastFrame.mvKeysUn[i].angle;
        r.valid = 1;
        r.observations = p->Observations();
        r.id = H.of(p);
        copy_desc(p->GetDescriptor(), r.desc);
    }
    const orbfe_frame fr = frame_view(CurrentFrame);
    const int n = orbfe_search_by_projection_lastframe(&fr, mvp.data(), obs.data(), q.data(),
                                                       (int)q.size(), th, bForward, bBackward, mbCheckOrientation);
    for (int i = 0; i < CurrentFrame.N; i++) CurrentFrame.mvpMapPoints[i] = H.at(mvp[i]);
    return n;
}

// ORBmatcher.cc:1889-2010
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
    const orbfe_frame fr = frame_view(CurrentFrame);
    const int n = orbfe_search_by_projection_kf(&fr, mvp.data(), q.data(), (int)q.size(), th,
                                                ORBdist, mbCheckOrientation);
    for (int i = 0; i < CurrentFrame.N; i++) CurrentFrame.mvpMapPoints[i] = H.at(mvp[i]);
    return n;
}

// ORBmatcher.cc:648-763
int ORBmatcher::SearchForInitialization(Frame& F1, Frame& F2, vector<cv::Point2f>& vbPrevMatched,
                                        vector<int>& vnMatches12, int windowSize) {
    vnMatches12.assign(F1.mvKeysUn.size(), -1);
    static_assert(sizeof(cv::Point2f) == 8, "Point2f layout");
    const orbfe_frame f1 = frame_view(F1), f2 = frame_view(F2);
    return orbfe_search_for_initialization(&f1, &f2,
                                           reinterpret_cast<float*>(vbPrevMatched.data()), vnMatches12.data(),
                                           windowSize, mfNNratio, mbCheckOrientation);
}

// ORBmatcher.cc:223-425 (pinhole path)
int ORBmatcher::SearchByBoW(KeyFrame* pKF, Frame& F, vector<MapPoint*>& vpMapPointMatches) {
    if (F.Nleft != -1) return SearchByBoW_cpu(pKF, F, vpMapPointMatches);
    const vector<MapPoint*> vpMapPointsKF = pKF->GetMapPointMatches();
    Handles H;
    vector<int32_t> kf_mp(vpMapPointsKF.size());
    for (size_t i = 0; i < vpMapPointsKF.size(); i++) {
        MapPoint* p = vpMapPointsKF[i];
        kf_mp[i] = (p && !p->isBad()) ? H.of(p) : -1;
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
    const orbfe_frame fr = frame_view(F);
    const int n = orbfe_search_by_bow(reinterpret_cast<const orbfe_keypoint*>(pKF->mvKeysUn.data()),
                                      pKF->mDescriptors.data, kf_mp.data(), (int)kf_mp.size(), &kfv,
                                      &fr, &ffv, out.data(), mfNNratio, mbCheckOrientation);
    vpMapPointMatches.assign(F.N, nullptr);
    for (int i = 0; i < F.N; i++) vpMapPointMatches[i] = H.at(out[i]);
    return n;
}

// Frame.cc:811-981 (replaces the body of Frame::ComputeStereoMatches; lives in Frame.cc)
//   void Frame::ComputeStereoMatches() {
//       mvuRight = vector<float>(N, -1.0f);
//       mvDepth = vector<float>(N, -1.0f);
//       orbfe_stereo_match(static_cast<orbfe_extractor*>(mpORBextractorLeft->mpOrbfe),
//                          static_cast<orbfe_extractor*>(mpORBextractorRight->mpOrbfe),
//                          mbf, fx, mvuRight.data(), mvDepth.data());
//   }

}  // namespace ORB_SLAM3
