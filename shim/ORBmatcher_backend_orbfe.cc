// Replacement bodies for the LocalMapping / LoopClosing ORBmatcher methods
// (orb_slam3/src/ORBmatcher.cc:427-646, 765-1674) and MapPoint::ComputeDistinctiveDescriptors
// (MapPoint.cc:329-403) on top of liborbfe.so. Keyframes with a second camera
// (KannalaBrandt8 stereo, NLeft != -1) go to the library's two-camera entry points
// (orbfe_search_by_bow_kf2, orbfe_fuse_rig, orbfe_search_by_projection_sim3_rig, orbfe_search_by_sim3,
// orbfe_search_for_triangulation with bCoarse, orbfe_search_for_triangulation_epi with the camera
// models' epipolarConstrain called back on this thread). The original bodies, renamed *_cpu, run only
// for SearchForTriangulation(bCoarse = false) between a one-camera and a two-camera keyframe (the
// reference reads R12 / t12 uninitialised there, ORBmatcher.cc:925-940, 1036-1074) and, after one
// logged line per call site and error code, whenever the library returns an error.
// Built inside the ORB-SLAM3 tree; this repository compiles it with -fsyntax-only against stand-in
// headers (tests/shim_stubs/, tests/test_shim_compile.py). See INTEGRATION.md §4.
#include "ORBmatcher.h"

#include <cstdio>
#include <cstring>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>

#include <orbfe.h>

#include "orbfe_slam_types.h"

#include "KeyFrame.h"
#include "MapPoint.h"

using namespace std;

namespace ORB_SLAM3 {

namespace {

struct Handles {   // MapPoint* <-> int32 (see ORBmatcher_orbfe.cc)
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

// One log line per (call site, error code), as ORBmatcher_orbfe.cc.
bool failed(int rc, const char* what) {
    if (rc >= 0) return false;
    static std::mutex mu;
    static std::set<std::pair<std::string, int>> seen;
    bool first;
    {
        std::lock_guard<std::mutex> lk(mu);
        first = seen.emplace(what, rc).second;
    }
    if (first) fprintf(stderr, "[orbfe] %s returned %d; running the CPU implementation\n", what, rc);
    return true;
}

// Keyframe fields the matchers read. Single camera: mvKeysUn borrowed. Two cameras (NLeft != -1):
// keys = mvKeys ++ mvKeysRight in `keys` (the reference's per-side keypoint selection), the stereo
// links borrowed.
orbfe_frame kf_view(KeyFrame* K, vector<cv::KeyPoint>& keys) {
    orbfe_frame f;
    memset(&f, 0, sizeof(f));
    f.n = K->N;
    if (K->NLeft == -1) {
        f.keys = reinterpret_cast<const orbfe_keypoint*>(K->mvKeysUn.data());
    } else {
        keys.assign(K->mvKeys.begin(), K->mvKeys.end());
        keys.insert(keys.end(), K->mvKeysRight.begin(), K->mvKeysRight.end());
        f.keys = reinterpret_cast<const orbfe_keypoint*>(keys.data());
        f.two_cams = 1;
        f.nleft = K->NLeft;
        f.l2r = K->mvLeftToRightMatch.data();
        f.r2l = K->mvRightToLeftMatch.data();
    }
    f.desc = K->mDescriptors.data;
    f.uright = K->mvuRight.empty() ? nullptr : K->mvuRight.data();
    f.min_x = K->mnMinX; f.max_x = K->mnMaxX; f.min_y = K->mnMinY; f.max_y = K->mnMaxY;
    f.nlevels = K->mnScaleLevels;
    f.scale_factors = K->mvScaleFactors.data();
    f.mbf = K->mbf;
    return f;
}

using orbfe_shim::model_of;
using orbfe_shim::pose_of;

orbfe_kf_camera kf_camera(KeyFrame* K, const Sophus::SE3f& Tcw, const Eigen::Vector3f& Ow) {
    orbfe_kf_camera c;
    c.Tcw = pose_of(Tcw);
    c.Ow[0] = Ow(0); c.Ow[1] = Ow(1); c.Ow[2] = Ow(2);
    c.fx = K->fx; c.fy = K->fy; c.cx = K->cx; c.cy = K->cy;
    c.log_scale_factor = K->mfLogScaleFactor;
    return c;
}

// GetMinDistance / GetMaxDistance: two accessors added to MapPoint.h.
orbfe_map_point_3d point_3d(MapPoint* p, int32_t id, int32_t flags) {
    orbfe_map_point_3d m;
    memset(&m, 0, sizeof(m));
    m.id = id;
    if (!p) return m;
    const Eigen::Vector3f X = p->GetWorldPos(), n = p->GetNormal();
    for (int k = 0; k < 3; k++) { m.pos[k] = X(k); m.normal[k] = n(k); }
    m.min_dist = p->GetMinDistance();
    m.max_dist = p->GetMaxDistance();
    m.flags = flags | (p->isBad() ? ORBFE_MP_BAD : 0);
    m.observations = p->Observations();
    m.track_depth = p->mTrackDepth;
    memcpy(m.desc, p->GetDescriptor().data, 32);
    return m;
}

struct FlatFV {   // DBoW2::FeatureVector flattened (ORBmatcher_orbfe.cc has the same helper)
    vector<uint32_t> ids, idx;
    vector<int32_t> off;
    orbfe_feature_vector v;
    explicit FlatFV(const DBoW2::FeatureVector& fv) {
        off.push_back(0);
        for (const auto& kv : fv) {
            ids.push_back(kv.first);
            idx.insert(idx.end(), kv.second.begin(), kv.second.end());
            off.push_back((int32_t)idx.size());
        }
        v.n_nodes = (int32_t)ids.size();
        v.node_ids = ids.data();
        v.offsets = off.data();
        v.indices = idx.data();
    }
};

// SearchForTriangulation's epipolar test through the camera models: the camera pair and relative pose
// the reference selects by the keypoints' sides (ORBmatcher.cc:925-940, 1036-1074); single-camera
// keyframes use T12 (slot ll) and mvKeysUn.
struct EpiCtx {
    KeyFrame* k1;
    KeyFrame* k2;
    Eigen::Matrix3f R[4];   // ll, lr, rl, rr
    Eigen::Vector3f t[4];
};
int32_t epipolar_cb(void* c, int32_t idx1, int32_t idx2) {
    const EpiCtx* e = static_cast<const EpiCtx*>(c);
    const bool s1 = e->k1->NLeft == -1, s2 = e->k2->NLeft == -1;
    const bool r1 = !s1 && idx1 >= e->k1->NLeft, r2 = !s2 && idx2 >= e->k2->NLeft;
    const cv::KeyPoint& kp1 = s1 ? e->k1->mvKeysUn[idx1] : r1 ? e->k1->mvKeysRight[idx1 - e->k1->NLeft] : e->k1->mvKeys[idx1];
    const cv::KeyPoint& kp2 = s2 ? e->k2->mvKeysUn[idx2] : r2 ? e->k2->mvKeysRight[idx2 - e->k2->NLeft] : e->k2->mvKeys[idx2];
    GeometricCamera* c1 = r1 ? e->k1->mpCamera2 : e->k1->mpCamera;
    GeometricCamera* c2 = r2 ? e->k2->mpCamera2 : e->k2->mpCamera;
    const int sel = (r1 ? 2 : 0) + (r2 ? 1 : 0);
    return c1->epipolarConstrain(c2, kp1, kp2, e->R[sel], e->t[sel], e->k1->mvLevelSigma2[kp1.octave],
                                 e->k2->mvLevelSigma2[kp2.octave]) ? 1 : 0;
}

}  // namespace

int ORBmatcher::SearchByBoW(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12) {
    Handles H;
    const vector<MapPoint*> v1 = pKF1->GetMapPointMatches(), v2 = pKF2->GetMapPointMatches();
    vector<int32_t> m1(v1.size()), m2(v2.size()), out(v1.size());
    for (size_t i = 0; i < v1.size(); i++) m1[i] = (v1[i] && !v1[i]->isBad()) ? H.of(v1[i]) : -1;
    for (size_t i = 0; i < v2.size(); i++) m2[i] = (v2[i] && !v2[i]->isBad()) ? H.of(v2[i]) : -1;
    FlatFV f1(pKF1->mFeatVec), f2(pKF2->mFeatVec);
    vector<cv::KeyPoint> keys1, keys2;   // two cameras: the right indices are skipped (:800-819)
    const orbfe_frame k1 = kf_view(pKF1, keys1), k2 = kf_view(pKF2, keys2);
    const int n = orbfe_search_by_bow_kf2(k1.keys, pKF1->mDescriptors.data, m1.data(), pKF1->N, pKF1->NLeft, &f1.v,
                                          k2.keys, pKF2->mDescriptors.data, m2.data(), pKF2->N, pKF2->NLeft, &f2.v,
                                          out.data(), mfNNratio, mbCheckOrientation);
    if (failed(n, "orbfe_search_by_bow_kf2")) return SearchByBoW_cpu(pKF1, pKF2, vpMatches12);
    vpMatches12.assign(v1.size(), static_cast<MapPoint*>(nullptr));
    for (size_t i = 0; i < v1.size(); i++) vpMatches12[i] = H.at(out[i]);
    return n;
}

int ORBmatcher::SearchForTriangulation(KeyFrame* pKF1, KeyFrame* pKF2, vector<pair<size_t, size_t>>& vMatchedPairs,
                                       const bool bOnlyStereo, const bool bCoarse) {
    const bool two1 = pKF1->mpCamera2 != nullptr, two2 = pKF2->mpCamera2 != nullptr;
    // one keyframe with a second camera, the other without: the reference's fine test reads R12 / t12
    // uninitialised (they are set only when both have one, :1036-1074); its own body keeps that
    if (two1 != two2 && !bCoarse)
        return SearchForTriangulation_cpu(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse);
    // the per-call constants, computed exactly as the reference does (ORBmatcher.cc:913-940,
    // Pinhole.cpp:109-112)
    const Sophus::SE3f T1w = pKF1->GetPose(), T2w = pKF2->GetPose(), Tw2 = pKF2->GetPoseInverse();
    const Eigen::Vector3f C2 = T2w * pKF1->GetCameraCenter();
    const Eigen::Vector2f ep = pKF2->mpCamera->project(C2);
    const bool pin = pKF1->mpCamera->GetType() == GeometricCamera::CAM_PINHOLE &&
                     pKF2->mpCamera->GetType() == GeometricCamera::CAM_PINHOLE;
    if (!bCoarse && (two1 || !pin)) {
        // a camera model's own test (KannalaBrandt8::epipolarConstrain -> TriangulateMatches, an
        // Eigen JacobiSVD) runs here, called back by the library on the candidates the device lists
        // until the first that passes
        EpiCtx e;
        e.k1 = pKF1;
        e.k2 = pKF2;
        if (two1) {
            const Sophus::SE3f Tr1w = pKF1->GetRightPose(), Twr2 = pKF2->GetRightPoseInverse();
            const Sophus::SE3f T[4] = {T1w * Tw2, T1w * Twr2, Tr1w * Tw2, Tr1w * Twr2};   // ll, lr, rl, rr
            for (int k = 0; k < 4; k++) {
                e.R[k] = T[k].rotationMatrix();
                e.t[k] = T[k].translation();
            }
        } else {
            const Sophus::SE3f T12 = T1w * Tw2;
            e.R[0] = T12.rotationMatrix();
            e.t[0] = T12.translation();
        }
        vector<int32_t> m1(pKF1->N), m2(pKF2->N), out(pKF1->N);
        for (int i = 0; i < pKF1->N; i++) m1[i] = pKF1->GetMapPoint(i) ? 1 : -1;
        for (int i = 0; i < pKF2->N; i++) m2[i] = pKF2->GetMapPoint(i) ? 1 : -1;
        FlatFV f1(pKF1->mFeatVec), f2(pKF2->mFeatVec);
        vector<cv::KeyPoint> keys1, keys2;
        const orbfe_frame k1 = kf_view(pKF1, keys1), k2 = kf_view(pKF2, keys2);
        const float epv[2] = {ep(0), ep(1)};
        const int n = orbfe_search_for_triangulation_epi(&k1, m1.data(), &f1.v, &k2, m2.data(), &f2.v, epv, bOnlyStereo,
                                                         mbCheckOrientation, epipolar_cb, &e, out.data());
        if (failed(n, "orbfe_search_for_triangulation_epi"))
            return SearchForTriangulation_cpu(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse);
        vMatchedPairs.clear();
        vMatchedPairs.reserve(n);
        for (int i = 0; i < pKF1->N; i++)
            if (out[i] >= 0) vMatchedPairs.push_back(make_pair((size_t)i, (size_t)out[i]));
        return n;
    }
    const Sophus::SE3f T12 = T1w * Tw2;
    const Eigen::Matrix3f R12 = T12.rotationMatrix();
    const Eigen::Vector3f t12 = T12.translation();
    const Eigen::Matrix3f K1 = pKF1->mpCamera->toK_(), K2 = pKF2->mpCamera->toK_();
    const Eigen::Matrix3f F = K1.transpose().inverse() * Sophus::SO3f::hat(t12) * R12 * K2.inverse();
    float F12[9], epv[2] = {ep(0), ep(1)};
    for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) F12[3 * r + c] = F(r, c);
    vector<int32_t> m1(pKF1->N), m2(pKF2->N), out(pKF1->N);
    for (int i = 0; i < pKF1->N; i++) m1[i] = pKF1->GetMapPoint(i) ? 1 : -1;
    for (int i = 0; i < pKF2->N; i++) m2[i] = pKF2->GetMapPoint(i) ? 1 : -1;
    FlatFV f1(pKF1->mFeatVec), f2(pKF2->mFeatVec);
    vector<cv::KeyPoint> keys1, keys2;
    const orbfe_frame k1 = kf_view(pKF1, keys1), k2 = kf_view(pKF2, keys2);
    const int n = orbfe_search_for_triangulation(&k1, m1.data(), &f1.v, &k2, m2.data(), &f2.v, F12, epv,
                                                 pKF2->mvLevelSigma2.data(), bOnlyStereo, bCoarse,
                                                 mbCheckOrientation, out.data());
    if (failed(n, "orbfe_search_for_triangulation"))
        return SearchForTriangulation_cpu(pKF1, pKF2, vMatchedPairs, bOnlyStereo, bCoarse);
    vMatchedPairs.clear();
    vMatchedPairs.reserve(n);
    for (int i = 0; i < pKF1->N; i++)
        if (out[i] >= 0) vMatchedPairs.push_back(make_pair((size_t)i, (size_t)out[i]));
    return n;
}

int ORBmatcher::Fuse(KeyFrame* pKF, const vector<MapPoint*>& vpMapPoints, const float th, const bool bRight) {
    // pCamera / Tcw / Ow as the reference selects them (:1154-1163)
    const orbfe_camera_model model = model_of(bRight ? pKF->mpCamera2 : pKF->mpCamera);
    const orbfe_kf_camera cam = bRight ? kf_camera(pKF, pKF->GetRightPose(), pKF->GetRightCameraCenter())
                                       : kf_camera(pKF, pKF->GetPose(), pKF->GetCameraCenter());
    vector<orbfe_map_point_3d> q(vpMapPoints.size());
    for (size_t i = 0; i < vpMapPoints.size(); i++) {
        MapPoint* p = vpMapPoints[i];
        q[i] = point_3d(p, p ? 0 : -1, (p && p->IsInKeyFrame(pKF)) ? ORBFE_MP_SKIP : 0);
    }
    vector<int32_t> best(q.size()), dist(q.size());   // best: NLeft + right index with bRight (:1283)
    vector<cv::KeyPoint> keys;
    const orbfe_frame kf = kf_view(pKF, keys);
    if (failed(orbfe_fuse_rig(&kf, &cam, &model, pKF->mvInvLevelSigma2.data(), q.data(), (int)q.size(), th, 0,
                              bRight, best.data(), dist.data()), "orbfe_fuse_rig"))
        return Fuse_cpu(pKF, vpMapPoints, th, bRight);
    // the reference's commit, in point order; the isBad / IsInKeyFrame gate is re-read because an
    // earlier commit (Replace / AddObservation) may have changed it
    int nFused = 0;
    for (size_t i = 0; i < vpMapPoints.size(); i++) {
        MapPoint* pMP = vpMapPoints[i];
        if (best[i] < 0 || !pMP || pMP->isBad() || pMP->IsInKeyFrame(pKF)) continue;
        MapPoint* pMPinKF = pKF->GetMapPoint(best[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) {
                if (pMPinKF->Observations() > pMP->Observations()) pMP->Replace(pMPinKF);
                else pMPinKF->Replace(pMP);
            }
        } else {
            pMP->AddObservation(pKF, best[i]);
            pKF->AddMapPoint(pMP, best[i]);
        }
        nFused++;
    }
    return nFused;
}

int ORBmatcher::Fuse(KeyFrame* pKF, Sophus::Sim3f& Scw, const vector<MapPoint*>& vpPoints, float th,
                     vector<MapPoint*>& vpReplacePoint) {
    const Sophus::SE3f Tcw = Sophus::SE3f(Scw.rotationMatrix(), Scw.translation() / Scw.scale());
    const orbfe_kf_camera cam = kf_camera(pKF, Tcw, Tcw.inverse().translation());
    const set<MapPoint*> spAlreadyFound = pKF->GetMapPoints();
    vector<orbfe_map_point_3d> q(vpPoints.size());
    for (size_t i = 0; i < vpPoints.size(); i++)
        q[i] = point_3d(vpPoints[i], 0, spAlreadyFound.count(vpPoints[i]) ? ORBFE_MP_SKIP : 0);
    vector<int32_t> best(q.size()), dist(q.size());
    vector<cv::KeyPoint> keys;
    const orbfe_frame kf = kf_view(pKF, keys);   // a two-camera keyframe: its left grid (:1397)
    const orbfe_camera_model model = model_of(pKF->mpCamera);
    if (failed(orbfe_fuse_rig(&kf, &cam, &model, nullptr, q.data(), (int)q.size(), th, 1, 0, best.data(),
                              dist.data()), "orbfe_fuse_rig(Scw)"))
        return Fuse_cpu(pKF, Scw, vpPoints, th, vpReplacePoint);
    int nFused = 0;
    for (size_t i = 0; i < vpPoints.size(); i++) {
        if (best[i] < 0) continue;
        MapPoint* pMP = vpPoints[i];
        MapPoint* pMPinKF = pKF->GetMapPoint(best[i]);
        if (pMPinKF) {
            if (!pMPinKF->isBad()) vpReplacePoint[i] = pMPinKF;
        } else {
            pMP->AddObservation(pKF, best[i]);
            pKF->AddMapPoint(pMP, best[i]);
        }
        nFused++;
    }
    return nFused;
}

int ORBmatcher::SearchByProjection(KeyFrame* pKF, Sophus::Sim3f& Scw, const vector<MapPoint*>& vpPoints,
                                   vector<MapPoint*>& vpMatched, int th, float ratioHamming) {
    // pKF->mpCamera->project (:465) with the keyframe's model; a two-camera keyframe's left grid
    const orbfe_camera_model model = model_of(pKF->mpCamera);
    const Sophus::SE3f Tcw = Sophus::SE3f(Scw.rotationMatrix(), Scw.translation() / Scw.scale());
    const orbfe_kf_camera cam = kf_camera(pKF, Tcw, Tcw.inverse().translation());
    Handles H;
    vector<orbfe_map_point_3d> q(vpPoints.size());
    for (size_t i = 0; i < vpPoints.size(); i++) q[i] = point_3d(vpPoints[i], H.of(vpPoints[i]), 0);
    vector<int32_t> m(vpMatched.size());
    for (size_t k = 0; k < vpMatched.size(); k++) m[k] = H.of(vpMatched[k]);
    vector<cv::KeyPoint> keys;
    const orbfe_frame kf = kf_view(pKF, keys);
    const int n = orbfe_search_by_projection_sim3_rig(&kf, &cam, &model, q.data(), (int)q.size(), nullptr, th,
                                                      ratioHamming, m.data(), nullptr);
    if (failed(n, "orbfe_search_by_projection_sim3_rig"))
        return SearchByProjection_cpu(pKF, Scw, vpPoints, vpMatched, th, ratioHamming);
    for (size_t k = 0; k < vpMatched.size(); k++) vpMatched[k] = H.at(m[k]);
    return n;
}

int ORBmatcher::SearchBySim3(KeyFrame* pKF1, KeyFrame* pKF2, vector<MapPoint*>& vpMatches12, const Sophus::Sim3f& S12,
                             const float th) {
    // every camera with the pinhole expression on pKF1's intrinsics (:1514-1519,1594-1599); two-camera
    // keyframes on their left grids
    Handles H;
    const vector<MapPoint*> v1 = pKF1->GetMapPointMatches(), v2 = pKF2->GetMapPointMatches();
    vector<orbfe_map_point_3d> p1(v1.size()), p2(v2.size());
    for (size_t i = 0; i < v1.size(); i++) p1[i] = point_3d(v1[i], H.of(v1[i]), 0);
    for (size_t i = 0; i < v2.size(); i++) p2[i] = point_3d(v2[i], H.of(v2[i]), 0);
    vector<int32_t> m12(v1.size()), idx2(v1.size(), -1);
    for (size_t i = 0; i < v1.size(); i++) {
        m12[i] = H.of(vpMatches12[i]);
        if (vpMatches12[i]) idx2[i] = get<0>(vpMatches12[i]->GetIndexInKeyFrame(pKF2));
    }
    orbfe_kf_camera c1 = kf_camera(pKF1, pKF1->GetPose(), pKF1->GetCameraCenter());
    orbfe_kf_camera c2 = kf_camera(pKF2, pKF2->GetPose(), pKF2->GetCameraCenter());
    const orbfe_pose s12 = pose_of(S12), s21 = pose_of(S12.inverse());
    vector<cv::KeyPoint> keys1, keys2;
    const orbfe_frame k1 = kf_view(pKF1, keys1), k2 = kf_view(pKF2, keys2);
    const int n = orbfe_search_by_sim3(&k1, &k2, p1.data(), p2.data(), &c1, &c2, &s12, &s21, th, m12.data(),
                                       idx2.data());
    if (failed(n, "orbfe_search_by_sim3")) return SearchBySim3_cpu(pKF1, pKF2, vpMatches12, S12, th);
    for (size_t i = 0; i < v1.size(); i++) vpMatches12[i] = H.at(m12[i]);
    return n;
}

// MapPoint::ComputeDistinctiveDescriptors for the points LocalMapping updates in one step
// (MapPointCulling / SearchInNeighbors call it per point; batching them is the caller's choice).
void ComputeDistinctiveDescriptorsBatch(const vector<MapPoint*>& points) {
    vector<uint8_t> desc;
    vector<int32_t> off(1, 0);
    for (size_t p = 0; p < points.size(); p++) {
        if (points[p]->isBad()) {   // mbBad: the reference returns without touching the descriptor
            off.push_back((int32_t)(desc.size() / 32));
            continue;
        }
        for (const auto& obs : points[p]->GetObservations()) {
            KeyFrame* pKF = obs.first;
            if (pKF->isBad()) continue;
            const int left = get<0>(obs.second), right = get<1>(obs.second);
            for (int idx : {left, right}) {
                if (idx < 0) continue;
                const uint8_t* row = pKF->mDescriptors.ptr<uint8_t>(idx);
                desc.insert(desc.end(), row, row + 32);
            }
        }
        off.push_back((int32_t)(desc.size() / 32));
    }
    vector<int32_t> best(points.size());
    if (failed(orbfe_distinctive_descriptors(desc.data(), off.data(), (int)points.size(), best.data()),
               "orbfe_distinctive_descriptors")) {
        for (MapPoint* p : points) p->ComputeDistinctiveDescriptors();
        return;
    }
    for (size_t p = 0; p < points.size(); p++)
        if (best[p] >= 0) points[p]->SetDescriptor(&desc[32 * ((size_t)off[p] + best[p])]);   // under mMutexFeatures
}

}  // namespace ORB_SLAM3
