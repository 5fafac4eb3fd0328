// ============================================================================================
// orb_oracle_match.cpp — CPU ORACLE of the Tracking-thread ORBmatcher methods (test
// infrastructure only; see orb_oracle.cpp's header for the rules and the parity status).
// Literal sequential restatements over the flattened snapshot structs of include/orbfe.h:
//   Frame::AssignFeaturesToGrid / PosInGrid  Frame.cc:385-416, 725-735   -> Grid
//   Frame::GetFeaturesInArea                 Frame.cc:657-723            -> Grid::area()
//   ORBmatcher::SearchByProjection (local)   ORBmatcher.cc:43-213        -> oro_sbp_local()
//   ORBmatcher::RadiusByViewingCos           ORBmatcher.cc:215-221
//   ORBmatcher::SearchByBoW(KF, F)           ORBmatcher.cc:223-425       -> oro_search_by_bow()
//   ORBmatcher::SearchForInitialization      ORBmatcher.cc:648-763       -> oro_search_for_init()
//   ORBmatcher::SearchByBoW(KF, KF)          ORBmatcher.cc:765-903       -> oro_search_by_bow_kf()
//   MapPoint::ComputeDistinctiveDescriptors  MapPoint.cc:329-403         -> oro_distinctive_descriptors()
//   ORBmatcher::SearchForTriangulation       ORBmatcher.cc:907-1146      -> oro_search_for_triangulation()
//   Pinhole::epipolarConstrain               Pinhole.cpp:107-129
//   ORBmatcher::Fuse(KF, vpMapPoints)        ORBmatcher.cc:1148-1337     -> oro_fuse(sim3 = 0)
//   ORBmatcher::Fuse(KF, Scw, ...)           ORBmatcher.cc:1339-1455     -> oro_fuse(sim3 = 1)
//   ORBmatcher::SearchByProjection (Sim3)    ORBmatcher.cc:427-646       -> oro_sbp_sim3()
//   ORBmatcher::SearchBySim3                 ORBmatcher.cc:1457-1674     -> oro_search_by_sim3()
//   Sophus SO3/RxSO3 point action            so3.hpp:358-367, rxso3.hpp:265-273
//   ORBmatcher::SearchByProjection (frame)   ORBmatcher.cc:1676-1887     -> oro_sbp_lastframe()
//   ORBmatcher::SearchByProjection (KF)      ORBmatcher.cc:1889-2010     -> oro_sbp_kf()
//   ORBmatcher::ComputeThreeMaxima           ORBmatcher.cc:2012-2053     -> three_maxima()
//   Frame::ComputeStereoFishEyeMatches kNN   Frame.cc:1126-1151          -> oro_stereo_knn_ratio()
//   Frame::isInFrustum (pinhole)             Frame.cc:512-570            -> oro_is_in_frustum()
//   Frame::isInFrustum (any camera model, both branches), isInFrustumChecks
//                                            Frame.cc:512-586, 1168-1242 -> oro_is_in_frustum_rig()
//   KannalaBrandt8::project (float)          KannalaBrandt8.cpp:67-82    -> kb8_project()
//   MapPoint::PredictScale                   MapPoint.cc:531-546
//   Tracking::SearchLocalPoints (projection + SearchByProjection)  Tracking.cc:3404-3453
//                                                                        -> oro_search_local_points()
// Two-camera frames (F.Nleft != -1, orbfe_frame.two_cams) follow the reference's Nleft branches of
// SearchByProjection (local map :95-209, last frame :1727-1858) and SearchByBoW(KF, F) (:270-386):
// keys[0, nleft) = mvKeys with the left grid mGrid, keys[nleft, n) = mvKeysRight with mGridRight
// (AssignFeaturesToGrid :399-413, GetFeaturesInArea(..., bRight) :657-723). Grid keeps GLOBAL row
// indices (right row = nleft + the reference's right index).
// ============================================================================================
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <vector>

#include "../include/orbfe.h"

namespace oracle {
int hamming(const uint8_t* a, const uint8_t* b);
}

namespace {

const int TH_HIGH = 100, TH_LOW = 50, HISTO_LENGTH = 30;

// Eigen 3.3's 3-term sums in fixed-size expressions (a product's coefficient, norm(), dot()): the
// non-vectorised redux halves the range, sum(a, b, c) = a + (b + c) (Eigen/src/Core/Redux.h
// redux_novec_unroller; ProductEvaluators.h lazy coeff = (lhs.row(i).transpose().cwiseProduct(
// rhs.col(j))).sum()). The reference's Eigen is focal's libeigen3-dev 3.3.7 (Dockerfile:19).
static inline float eig_sum3(float a, float b, float c) { return a + (b + c); }

struct CamModel {
    int type;
    float p[8];
};

// GeometricCamera::project(const Eigen::Vector3f&): Pinhole.cpp:43-49 (fx * x / z + cx) and
// KannalaBrandt8.cpp:67-82 (atan2f / sqrtf explicit; cos(psi) / sin(psi) of a float resolve to
// cosf / sinf, as for computeOrbDescriptor's rotation), float arithmetic in source order.
static void cam_project(const CamModel& m, const float* Pc, float& u, float& v) {
    if (m.type == ORBFE_CAM_KANNALA_BRANDT8) {
        const float x2_plus_y2 = Pc[0] * Pc[0] + Pc[1] * Pc[1];
        const float theta = atan2f(sqrtf(x2_plus_y2), Pc[2]);
        const float psi = atan2f(Pc[1], Pc[0]);
        const float theta2 = theta * theta;
        const float theta3 = theta * theta2;
        const float theta5 = theta3 * theta2;
        const float theta7 = theta5 * theta2;
        const float theta9 = theta7 * theta2;
        const float r = theta + m.p[4] * theta3 + m.p[5] * theta5 + m.p[6] * theta7 + m.p[7] * theta9;
        u = m.p[0] * r * cosf(psi) + m.p[2];
        v = m.p[1] * r * sinf(psi) + m.p[3];
        return;
    }
    u = m.p[0] * Pc[0] / Pc[2] + m.p[2];
    v = m.p[1] * Pc[1] / Pc[2] + m.p[3];
}


struct Grid {
    const orbfe_frame* F;
    float invw, invh;
    std::vector<size_t> cell[ORBFE_GRID_COLS][ORBFE_GRID_ROWS];
    // side: -1 all rows (Nleft == -1), 0 the left rows [0, nleft) (mGrid), 1 the right rows (mGridRight)
    explicit Grid(const orbfe_frame* f, int side = -1) : F(f) {
        invw = static_cast<float>(ORBFE_GRID_COLS) / (F->max_x - F->min_x);
        invh = static_cast<float>(ORBFE_GRID_ROWS) / (F->max_y - F->min_y);
        const int i0 = side == 1 ? F->nleft : 0, i1 = side == 0 ? F->nleft : F->n;
        for (int i = i0; i < i1; i++) {
            const orbfe_keypoint& kp = F->keys[i];
            int px = (int)std::round((kp.x - F->min_x) * invw);
            int py = (int)std::round((kp.y - F->min_y) * invh);
            if (px < 0 || px >= ORBFE_GRID_COLS || py < 0 || py >= ORBFE_GRID_ROWS) continue;
            cell[px][py].push_back(i);
        }
    }
    std::vector<size_t> area(float x, float y, float r, int minLevel, int maxLevel) const {
        std::vector<size_t> v;
        const float fx = r, fy = r;
        const int nMinCellX = std::max(0, (int)std::floor((x - F->min_x - fx) * invw));
        if (nMinCellX >= ORBFE_GRID_COLS) return v;
        const int nMaxCellX = std::min(ORBFE_GRID_COLS - 1, (int)std::ceil((x - F->min_x + fx) * invw));
        if (nMaxCellX < 0) return v;
        const int nMinCellY = std::max(0, (int)std::floor((y - F->min_y - fy) * invh));
        if (nMinCellY >= ORBFE_GRID_ROWS) return v;
        const int nMaxCellY = std::min(ORBFE_GRID_ROWS - 1, (int)std::ceil((y - F->min_y + fy) * invh));
        if (nMaxCellY < 0) return v;
        const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
        for (int ix = nMinCellX; ix <= nMaxCellX; ix++)
            for (int iy = nMinCellY; iy <= nMaxCellY; iy++) {
                const std::vector<size_t>& c = cell[ix][iy];
                for (size_t j = 0; j < c.size(); j++) {
                    const orbfe_keypoint& kp = F->keys[c[j]];
                    if (bCheckLevels) {
                        if (kp.octave < minLevel) continue;
                        if (maxLevel >= 0 && kp.octave > maxLevel) continue;
                    }
                    const float distx = kp.x - x, disty = kp.y - y;
                    if (std::fabs(distx) < fx && std::fabs(disty) < fy) v.push_back(c[j]);
                }
            }
        return v;
    }
};

void three_maxima(const std::vector<int>* histo, int L, int& ind1, int& ind2, int& ind3) {
    int max1 = 0, max2 = 0, max3 = 0;
    for (int i = 0; i < L; i++) {
        const int s = (int)histo[i].size();
        if (s > max1) {
            max3 = max2; max2 = max1; max1 = s;
            ind3 = ind2; ind2 = ind1; ind1 = i;
        } else if (s > max2) {
            max3 = max2; max2 = s;
            ind3 = ind2; ind2 = i;
        } else if (s > max3) {
            max3 = s; ind3 = i;
        }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
}

int rot_bin(float a1, float a2) {
    const float factor = 1.0f / HISTO_LENGTH;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)std::round(rot * factor);
    if (bin == HISTO_LENGTH) bin = 0;
    return bin;
}

float radius_by_viewing_cos(const float& viewCos) { return viewCos > 0.998 ? 2.5f : 4.0f; }

}  // namespace

extern "C" {

int oro_sbp_local(const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs_in, const orbfe_map_point* mps,
                  int32_t n_mps, float th, int32_t bFarPoints, float thFarPoints, float nnratio) {
    const bool two = F->two_cams != 0;   // F.Nleft != -1
    const int Nleft = F->nleft;
    Grid grid(F, two ? 0 : -1);
    Grid gridR(F, two ? 1 : -1);
    std::vector<int32_t> obs(mvp_obs_in, mvp_obs_in + F->n);
    auto put = [&](int slot, const orbfe_map_point& mp) { mvp[slot] = mp.id; obs[slot] = mp.observations; };
    int nmatches = 0;
    const bool bFactor = th != 1.0;
    for (int iMP = 0; iMP < n_mps; iMP++) {
        const orbfe_map_point& mp = mps[iMP];
        const bool inView = (mp.flags & ORBFE_MP_IN_VIEW) != 0, inViewR = two && (mp.flags & ORBFE_MP_IN_VIEW_R);
        if (!inView && !inViewR) continue;
        if (bFarPoints && mp.depth > thFarPoints) continue;
        if (mp.flags & ORBFE_MP_BAD) continue;
        if (inView) {
            const int nPredictedLevel = mp.scale_level;
            float r = radius_by_viewing_cos(mp.view_cos);
            if (bFactor) r *= th;
            const std::vector<size_t> vIndices =
                grid.area(mp.proj_x, mp.proj_y, r * F->scale_factors[nPredictedLevel], nPredictedLevel - 1, nPredictedLevel);
            if (!vIndices.empty()) {
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (size_t idx : vIndices) {
                    if (mvp[idx] >= 0 && obs[idx] > 0) continue;
                    if (!two && F->uright && F->uright[idx] > 0) {
                        const float er = std::fabs(mp.proj_xr - F->uright[idx]);
                        if (er > r * F->scale_factors[nPredictedLevel]) continue;
                    }
                    const int dist = oracle::hamming(mp.desc, F->desc + idx * 32);
                    // octave: mvKeysUn[idx] / mvKeys[idx] / mvKeysRight[idx - Nleft] == keys[idx]
                    if (dist < bestDist) {
                        bestDist2 = bestDist; bestDist = dist;
                        bestLevel2 = bestLevel; bestLevel = F->keys[idx].octave;
                        bestIdx = (int)idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = F->keys[idx].octave;
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= TH_HIGH) {
                    if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;   // skips the right search too
                    if (bestLevel != bestLevel2 || bestDist <= nnratio * bestDist2) {
                        put(bestIdx, mp);
                        if (two && F->l2r[bestIdx] != -1) {   // the stereo partner in the right camera
                            put(F->l2r[bestIdx] + Nleft, mp);
                            nmatches++;
                        }
                        nmatches++;
                    }
                }
            }
        }
        if (two && inViewR) {
            const int nPredictedLevel = mp.scale_level_r;
            if (nPredictedLevel != -1) {
                const float r = radius_by_viewing_cos(mp.view_cos_r);   // not scaled by th (:141)
                const std::vector<size_t> vIndices = gridR.area(mp.proj_xr, mp.proj_yr,
                                                                r * F->scale_factors[nPredictedLevel],
                                                                nPredictedLevel - 1, nPredictedLevel);
                if (vIndices.empty()) continue;
                int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
                for (size_t idx : vIndices) {   // global rows: idx + Nleft in the reference's numbering
                    if (mvp[idx] >= 0 && obs[idx] > 0) continue;
                    const int dist = oracle::hamming(mp.desc, F->desc + idx * 32);
                    if (dist < bestDist) {
                        bestDist2 = bestDist; bestDist = dist;
                        bestLevel2 = bestLevel; bestLevel = F->keys[idx].octave;
                        bestIdx = (int)idx;
                    } else if (dist < bestDist2) {
                        bestLevel2 = F->keys[idx].octave;
                        bestDist2 = dist;
                    }
                }
                if (bestDist <= TH_HIGH) {
                    if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) continue;
                    if (F->r2l[bestIdx - Nleft] != -1) {
                        put(F->r2l[bestIdx - Nleft], mp);
                        nmatches++;
                    }
                    put(bestIdx, mp);
                    nmatches++;
                }
            }
        }
    }
    return nmatches;
}

int oro_sbp_lastframe_stereo(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs_in,
                             const orbfe_proj_point* pts, const float* right_uv, int32_t n_pts, float th,
                             int32_t bForward, int32_t bBackward, int32_t checkOri) {
    const bool two = cur->two_cams != 0;   // CurrentFrame.Nleft != -1
    Grid grid(cur, two ? 0 : -1);
    Grid gridR(cur, two ? 1 : -1);
    std::vector<int32_t> obs(mvp_obs_in, mvp_obs_in + cur->n);
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    for (int i = 0; i < n_pts; i++) {
        const orbfe_proj_point& p = pts[i];
        if (!p.valid) continue;
        if (p.invzc < 0) continue;
        if (p.u < cur->min_x || p.u > cur->max_x) continue;
        if (p.v < cur->min_y || p.v > cur->max_y) continue;
        const int nLastOctave = p.octave;
        const float radius = th * cur->scale_factors[nLastOctave];
        std::vector<size_t> v2;
        if (bForward) v2 = grid.area(p.u, p.v, radius, nLastOctave, -1);
        else if (bBackward) v2 = grid.area(p.u, p.v, radius, 0, nLastOctave);
        else v2 = grid.area(p.u, p.v, radius, nLastOctave - 1, nLastOctave + 1);
        if (v2.empty()) continue;   // skips the right-camera search as well
        int bestDist = 256, bestIdx2 = -1;
        for (size_t i2 : v2) {
            if (mvp[i2] >= 0 && obs[i2] > 0) continue;
            if (!two && cur->uright && cur->uright[i2] > 0) {
                const float ur = p.u - cur->mbf * p.invzc;
                const float er = std::fabs(ur - cur->uright[i2]);
                if (er > radius) continue;
            }
            const int dist = oracle::hamming(p.desc, cur->desc + i2 * 32);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = (int)i2; }
        }
        if (bestDist <= TH_HIGH) {
            mvp[bestIdx2] = p.id;
            obs[bestIdx2] = p.observations;
            nmatches++;
            if (checkOri) rotHist[rot_bin(p.angle, cur->keys[bestIdx2].angle)].push_back(bestIdx2);
        }
        if (two) {   // :1794-1858, the projection into the right camera comes from the caller
            const float ur = right_uv[2 * i], vr = right_uv[2 * i + 1];
            std::vector<size_t> w2;
            if (bForward) w2 = gridR.area(ur, vr, radius, nLastOctave, -1);
            else if (bBackward) w2 = gridR.area(ur, vr, radius, 0, nLastOctave);
            else w2 = gridR.area(ur, vr, radius, nLastOctave - 1, nLastOctave + 1);
            int bestDistR = 256, bestIdxR = -1;
            for (size_t i2 : w2) {   // global rows (i2 + Nleft in the reference)
                if (mvp[i2] >= 0 && obs[i2] > 0) continue;
                const int dist = oracle::hamming(p.desc, cur->desc + i2 * 32);
                if (dist < bestDistR) { bestDistR = dist; bestIdxR = (int)i2; }
            }
            if (bestDistR <= TH_HIGH) {
                mvp[bestIdxR] = p.id;
                obs[bestIdxR] = p.observations;
                nmatches++;
                if (checkOri) rotHist[rot_bin(p.angle, cur->keys[bestIdxR].angle)].push_back(bestIdxR);
            }
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++)
            if (i != ind1 && i != ind2 && i != ind3)
                for (int k : rotHist[i]) { mvp[k] = -1; nmatches--; }
    }
    return nmatches;
}

int oro_sbp_lastframe(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs_in, const orbfe_proj_point* pts,
                      int32_t n_pts, float th, int32_t bForward, int32_t bBackward, int32_t checkOri) {
    if (cur->two_cams) return -1;   // needs the right-camera projections (oro_sbp_lastframe_stereo)
    return oro_sbp_lastframe_stereo(cur, mvp, mvp_obs_in, pts, nullptr, n_pts, th, bForward, bBackward, checkOri);
}

int oro_sbp_kf(const orbfe_frame* cur, int32_t* mvp, const orbfe_proj_point* pts, int32_t n_pts, float th,
               int32_t ORBdist, int32_t checkOri) {
    Grid grid(cur);
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    for (int i = 0; i < n_pts; i++) {
        const orbfe_proj_point& p = pts[i];
        if (!p.valid) continue;
        const int nPredictedLevel = p.octave;
        const float radius = th * cur->scale_factors[nPredictedLevel];
        const std::vector<size_t> v2 = grid.area(p.u, p.v, radius, nPredictedLevel - 1, nPredictedLevel + 1);
        if (v2.empty()) continue;
        int bestDist = 256, bestIdx2 = -1;
        for (size_t i2 : v2) {
            if (mvp[i2] >= 0) continue;
            const int dist = oracle::hamming(p.desc, cur->desc + i2 * 32);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = (int)i2; }
        }
        if (bestDist <= ORBdist) {
            mvp[bestIdx2] = p.id;
            nmatches++;
            if (checkOri) rotHist[rot_bin(p.angle, cur->keys[bestIdx2].angle)].push_back(bestIdx2);
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++)
            if (i != ind1 && i != ind2 && i != ind3)
                for (int k : rotHist[i]) { mvp[k] = -1; nmatches--; }
    }
    return nmatches;
}

int oro_search_for_init(const orbfe_frame* F1, const orbfe_frame* F2, float* prev, int32_t* m12, int32_t windowSize,
                        float nnratio, int32_t checkOri) {
    Grid grid2(F2);
    int nmatches = 0;
    for (int i = 0; i < F1->n; i++) m12[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    std::vector<int> vMatchedDistance(F2->n, INT_MAX), vnMatches21(F2->n, -1);
    for (int i1 = 0; i1 < F1->n; i1++) {
        const orbfe_keypoint& kp1 = F1->keys[i1];
        const int level1 = kp1.octave;
        if (level1 > 0) continue;
        const std::vector<size_t> v2 = grid2.area(prev[2 * i1], prev[2 * i1 + 1], (float)windowSize, level1, level1);
        if (v2.empty()) continue;
        int bestDist = INT_MAX, bestDist2 = INT_MAX, bestIdx2 = -1;
        for (size_t i2 : v2) {
            const int dist = oracle::hamming(F1->desc + (size_t)i1 * 32, F2->desc + i2 * 32);
            if (vMatchedDistance[i2] <= dist) continue;
            if (dist < bestDist) { bestDist2 = bestDist; bestDist = dist; bestIdx2 = (int)i2; }
            else if (dist < bestDist2) bestDist2 = dist;
        }
        if (bestDist <= TH_LOW) {
            if (bestDist < (float)bestDist2 * nnratio) {
                if (vnMatches21[bestIdx2] >= 0) { m12[vnMatches21[bestIdx2]] = -1; nmatches--; }
                m12[i1] = bestIdx2;
                vnMatches21[bestIdx2] = i1;
                vMatchedDistance[bestIdx2] = bestDist;
                nmatches++;
                if (checkOri) rotHist[rot_bin(F1->keys[i1].angle, F2->keys[bestIdx2].angle)].push_back(i1);
            }
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int idx1 : rotHist[i])
                if (m12[idx1] >= 0) { m12[idx1] = -1; nmatches--; }
        }
    }
    for (int i1 = 0; i1 < F1->n; i1++)
        if (m12[i1] >= 0) { prev[2 * i1] = F2->keys[m12[i1]].x; prev[2 * i1 + 1] = F2->keys[m12[i1]].y; }
    return nmatches;
}

int oro_search_by_bow(const orbfe_keypoint* kf_keys, const uint8_t* kf_desc, const int32_t* kf_mp, int32_t kf_n,
                      const orbfe_feature_vector* kfv, const orbfe_frame* F, const orbfe_feature_vector* ffv,
                      int32_t* out, float nnratio, int32_t checkOri) {
    (void)kf_n;
    for (int i = 0; i < F->n; i++) out[i] = -1;
    std::vector<int> rotHist[HISTO_LENGTH];
    int nmatches = 0;
    // std::map iteration with lower_bound jumps == ordered merge-join on equal node ids
    int a = 0, b = 0;
    while (a < kfv->n_nodes && b < ffv->n_nodes) {
        if (kfv->node_ids[a] == ffv->node_ids[b]) {
            for (int ia = kfv->offsets[a]; ia < kfv->offsets[a + 1]; ia++) {
                const unsigned realIdxKF = kfv->indices[ia];
                const int mp = kf_mp[realIdxKF];
                if (mp < 0) continue;
                const uint8_t* dKF = kf_desc + (size_t)realIdxKF * 32;
                int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
                int bestDist1R = 256, bestIdxFR = -1, bestDist2R = 256;
                for (int ib = ffv->offsets[b]; ib < ffv->offsets[b + 1]; ib++) {
                    const unsigned realIdxF = ffv->indices[ib];
                    if (out[realIdxF] >= 0) continue;
                    const int dist = oracle::hamming(dKF, F->desc + (size_t)realIdxF * 32);
                    if (!F->two_cams) {
                        if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = (int)realIdxF; }
                        else if (dist < bestDist2) bestDist2 = dist;
                    } else {   // :288-313
                        const bool left = (int)realIdxF < F->nleft;
                        if (left && dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = (int)realIdxF; }
                        else if (left && dist < bestDist2) bestDist2 = dist;
                        if (!left && dist < bestDist1R) { bestDist2R = bestDist1R; bestDist1R = dist; bestIdxFR = (int)realIdxF; }
                        else if (!left && dist < bestDist2R) bestDist2R = dist;
                    }
                }
                if (bestDist1 <= TH_LOW) {
                    if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                        out[bestIdxF] = mp;
                        if (checkOri) rotHist[rot_bin(kf_keys[realIdxKF].angle, F->keys[bestIdxF].angle)].push_back(bestIdxF);
                        nmatches++;
                    }
                    if (bestDist1R <= TH_LOW) {
                        // the reference's ratio test here ends in "|| true" (:359): always taken
                        out[bestIdxFR] = mp;
                        if (checkOri) rotHist[rot_bin(kf_keys[realIdxKF].angle, F->keys[bestIdxFR].angle)].push_back(bestIdxFR);
                        nmatches++;
                    }
                }
            }
            a++;
            b++;
        } else if (kfv->node_ids[a] < ffv->node_ids[b]) {
            while (a < kfv->n_nodes && kfv->node_ids[a] < ffv->node_ids[b]) a++;
        } else {
            while (b < ffv->n_nodes && ffv->node_ids[b] < kfv->node_ids[a]) b++;
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int k : rotHist[i]) { out[k] = -1; nmatches--; }
        }
    }
    return nmatches;
}

// vbMatched2 / vpMatches12 are indexed by keypoint; the std::map walk is the same merge-join as
// the KF-F variant. Note the strict bestDist1 < TH_LOW here (<= in the KF-F variant).
// nleft1 / nleft2: NLeft of a keyframe with a second camera (-1: none); its right indices are skipped
// (ORBmatcher.cc:800-802, 817-819: idx >= mvKeysUn.size() == NLeft).
int oro_search_by_bow_kf2(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                          int32_t nleft1, const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2,
                          const uint8_t* desc2, const int32_t* mp2, int32_t n2, int32_t nleft2,
                          const orbfe_feature_vector* fv2, int32_t* out12, float nnratio, int32_t checkOri) {
    const unsigned lim1 = (unsigned)(nleft1 >= 0 ? nleft1 : n1), lim2 = (unsigned)(nleft2 >= 0 ? nleft2 : n2);
    std::vector<int> rotHist[HISTO_LENGTH];
    std::vector<char> vbMatched2(n2 > 0 ? n2 : 1, 0);
    for (int i = 0; i < n1; i++) out12[i] = -1;
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int ia = fv1->offsets[a]; ia < fv1->offsets[a + 1]; ia++) {
                const unsigned idx1 = fv1->indices[ia];
                if (idx1 >= lim1) continue;
                if (mp1[idx1] < 0) continue;   // !pMP1 || pMP1->isBad()
                const uint8_t* d1 = desc1 + (size_t)idx1 * 32;
                int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
                for (int ib = fv2->offsets[b]; ib < fv2->offsets[b + 1]; ib++) {
                    const unsigned idx2 = fv2->indices[ib];
                    if (idx2 >= lim2) continue;
                    if (vbMatched2[idx2] || mp2[idx2] < 0) continue;
                    const int dist = oracle::hamming(d1, desc2 + (size_t)idx2 * 32);
                    if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdx2 = (int)idx2; }
                    else if (dist < bestDist2) bestDist2 = dist;
                }
                if (bestDist1 < TH_LOW) {
                    if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
                        out12[idx1] = mp2[bestIdx2];
                        vbMatched2[bestIdx2] = 1;
                        if (checkOri) rotHist[rot_bin(keys1[idx1].angle, keys2[bestIdx2].angle)].push_back((int)idx1);
                        nmatches++;
                    }
                }
            }
            a++;
            b++;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) {
            while (a < fv1->n_nodes && fv1->node_ids[a] < fv2->node_ids[b]) a++;
        } else {
            while (b < fv2->n_nodes && fv2->node_ids[b] < fv1->node_ids[a]) b++;
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int k : rotHist[i]) { out12[k] = -1; nmatches--; }
        }
    }
    return nmatches;
}

int oro_search_by_bow_kf(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                         const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2, const uint8_t* desc2,
                         const int32_t* mp2, int32_t n2, const orbfe_feature_vector* fv2, int32_t* out12,
                         float nnratio, int32_t checkOri) {
    return oro_search_by_bow_kf2(keys1, desc1, mp1, n1, -1, fv1, keys2, desc2, mp2, n2, -1, fv2, out12, nnratio,
                                 checkOri);
}

// Distances[N][N] (symmetric, zero diagonal), each row sorted, median = row[0.5 * (N - 1)] with the
// index truncated, first row with the strictly smallest median wins.
int oro_distinctive_descriptors(const uint8_t* desc, const int32_t* offsets, int32_t n_points, int32_t* best) {
    for (int p = 0; p < n_points; p++) {
        const int N = offsets[p + 1] - offsets[p];
        if (N == 0) { best[p] = -1; continue; }
        const uint8_t* d = desc + (size_t)offsets[p] * 32;
        std::vector<std::vector<float>> Distances(N, std::vector<float>(N));
        for (int i = 0; i < N; i++) {
            Distances[i][i] = 0;
            for (int j = i + 1; j < N; j++) {
                const int distij = oracle::hamming(d + (size_t)i * 32, d + (size_t)j * 32);
                Distances[i][j] = distij;
                Distances[j][i] = distij;
            }
        }
        int BestMedian = INT_MAX, BestIdx = 0;
        for (int i = 0; i < N; i++) {
            std::vector<int> vDists(Distances[i].begin(), Distances[i].end());
            std::sort(vDists.begin(), vDists.end());
            const int median = vDists[(size_t)(0.5 * (N - 1))];
            if (median < BestMedian) { BestMedian = median; BestIdx = i; }
        }
        best[p] = BestIdx;
    }
    return n_points;
}

// ---- back-end projections ----
// Sophus point action in Eigen's evaluation order (no contraction). RxSO3's scale is
// quaternion().squaredNorm(), which Eigen reduces as one SSE packet: (x*x + z*z) + (y*y + w*w).
static void pose_apply(const orbfe_pose& P, const float p[3], float o[3]) {
    const float vx = P.q[0], vy = P.q[1], vz = P.q[2], w = P.q[3];
    float uv[3] = {vy * p[2] - vz * p[1], vz * p[0] - vx * p[2], vx * p[1] - vy * p[0]};
    for (int k = 0; k < 3; k++) uv[k] += uv[k];
    const float c[3] = {vy * uv[2] - vz * uv[1], vz * uv[0] - vx * uv[2], vx * uv[1] - vy * uv[0]};
    if (P.kind == ORBFE_SIM3) {
        const float sc = (vx * vx + vz * vz) + (vy * vy + w * w);
        for (int k = 0; k < 3; k++) o[k] = (sc * p[k] + (w * uv[k] + c[k])) + P.t[k];
    } else {
        for (int k = 0; k < 3; k++) o[k] = ((p[k] + w * uv[k]) + c[k]) + P.t[k];
    }
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) with its projection (ORBmatcher.cc:1695-1718,
// 1794-1796): x3Dc = Tcw * x3Dw (Sophus SE3f action), invzc = 1.0 / x3Dc(2) (the double literal makes
// the division double), uv = mpCamera->project(x3Dc); a two-camera frame's right-camera window around
// mpCamera->project(Trl * x3Dc); then the host-projected search above.
int oro_sbp_lastframe_pose(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs_in, const orbfe_last_point* lp,
                           int32_t n_pts, const orbfe_pose* Tcw, const orbfe_pose* Trl, const orbfe_camera_model* cam,
                           float th, int32_t bForward, int32_t bBackward, int32_t checkOri) {
    const bool two = cur->two_cams != 0;
    CamModel M{cam->type, {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}};
    for (int k = 0; k < 8; k++) M.p[k] = cam->params[k];
    orbfe_pose T = *Tcw, R;
    T.kind = ORBFE_SE3;
    if (two) {
        R = *Trl;
        R.kind = ORBFE_SE3;
    }
    std::vector<orbfe_proj_point> pts((size_t)n_pts);
    std::vector<float> ruv((size_t)n_pts * 2, 0.f);
    for (int i = 0; i < n_pts; i++) {
        const orbfe_last_point& p = lp[i];
        orbfe_proj_point& q = pts[i];
        memset(&q, 0, sizeof(q));
        q.octave = p.octave;
        q.angle = p.angle;
        q.observations = p.observations;
        q.id = p.id;
        memcpy(q.desc, p.desc, 32);
        if (!p.valid) continue;   // pMP == NULL or an outlier
        q.valid = 1;
        float c[3];
        pose_apply(T, p.pos, c);
        q.invzc = (float)(1.0 / (double)c[2]);
        if (q.invzc < 0) continue;   // skipped by the search as the reference's `continue`
        cam_project(M, c, q.u, q.v);
        if (two) {
            float cr[3];
            pose_apply(R, c, cr);
            cam_project(M, cr, ruv[2 * i], ruv[2 * i + 1]);
        }
    }
    return oro_sbp_lastframe_stereo(cur, mvp, mvp_obs_in, pts.data(), two ? ruv.data() : nullptr, n_pts, th, bForward,
                                    bBackward, checkOri);
}

static bool kf_in_image(const orbfe_frame* F, float x, float y) {   // KeyFrame::IsInImage (KeyFrame.cc:753-756)
    return x >= F->min_x && x < F->max_x && y >= F->min_y && y < F->max_y;
}

static int predict_scale(float max_dist, float dist, float logsf, int nlevels) {   // MapPoint.cc:514-529
    const float ratio = max_dist / dist;
    int nScale = (int)std::ceil(logf(ratio) / logsf);
    if (nScale < 0) nScale = 0;
    else if (nScale >= nlevels) nScale = nlevels - 1;
    return nScale;
}

// Pinhole::epipolarConstrain with F12 precomputed (the value is the same on every call).
static bool epipolar(const orbfe_keypoint& kp1, const orbfe_keypoint& kp2, const float* F, float unc) {
    const float a = kp1.x * F[0] + kp1.y * F[3] + F[6];
    const float b = kp1.x * F[1] + kp1.y * F[4] + F[7];
    const float c = kp1.x * F[2] + kp1.y * F[5] + F[8];
    const float num = a * kp2.x + b * kp2.y + c;
    const float den = a * a + b * b;
    if (den == 0) return false;
    const float dsqr = num * num / den;
    return dsqr < 3.84 * unc;
}

typedef int32_t (*oro_epipolar_fn)(void* ctx, int32_t idx1, int32_t idx2);

// epi != NULL: pCamera1->epipolarConstrain(pCamera2, kp1, kp2, R12, t12, sigma1, sigma2) as the
// caller evaluates it for the keypoint pair (idx1, idx2) (two-camera keyframes with bCoarse false,
// ORBmatcher.cc:1036-1074); NULL: the pinhole test on F12.
static int search_for_triangulation(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                    const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                    const float* F12, const float* ep, const float* level_sigma2_2, int32_t bOnlyStereo,
                                    int32_t bCoarse, int32_t checkOri, int32_t* matches12, oro_epipolar_fn epi,
                                    void* ctx) {
    std::vector<int> rotHist[HISTO_LENGTH];
    for (int i = 0; i < KF1->n; i++) matches12[i] = -1;
    int nmatches = 0;
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int ia = fv1->offsets[a]; ia < fv1->offsets[a + 1]; ia++) {
                const unsigned idx1 = fv1->indices[ia];
                if (mp1[idx1] >= 0) continue;   // a MapPoint is already there
                // keys = mvKeysUn, or mvKeys ++ mvKeysRight with a second camera (ORBmatcher.cc:979-984)
                const bool bStereo1 = !KF1->two_cams && KF1->uright && KF1->uright[idx1] >= 0;
                if (bOnlyStereo && !bStereo1) continue;
                const orbfe_keypoint& kp1 = KF1->keys[idx1];
                const uint8_t* d1 = KF1->desc + (size_t)idx1 * 32;
                int bestDist = TH_LOW, bestIdx2 = -1;
                for (int ib = fv2->offsets[b]; ib < fv2->offsets[b + 1]; ib++) {
                    const unsigned idx2 = fv2->indices[ib];
                    if (mp2[idx2] >= 0) continue;   // vbMatched2 is never set by the reference
                    const bool bStereo2 = !KF2->two_cams && KF2->uright && KF2->uright[idx2] >= 0;
                    if (bOnlyStereo && !bStereo2) continue;
                    const int dist = oracle::hamming(d1, KF2->desc + (size_t)idx2 * 32);
                    if (dist > TH_LOW || dist > bestDist) continue;
                    const orbfe_keypoint& kp2 = KF2->keys[idx2];
                    if (!bStereo1 && !bStereo2 && !KF1->two_cams) {
                        const float distex = ep[0] - kp2.x;
                        const float distey = ep[1] - kp2.y;
                        if (distex * distex + distey * distey < 100 * KF2->scale_factors[kp2.octave]) continue;
                    }
                    if (bCoarse || (epi ? epi(ctx, (int32_t)idx1, (int32_t)idx2) != 0
                                        : epipolar(kp1, kp2, F12, level_sigma2_2[kp2.octave]))) {
                        bestIdx2 = (int)idx2;
                        bestDist = dist;
                    }
                }
                if (bestIdx2 >= 0) {
                    matches12[idx1] = bestIdx2;
                    nmatches++;
                    if (checkOri) rotHist[rot_bin(kp1.angle, KF2->keys[bestIdx2].angle)].push_back((int)idx1);
                }
            }
            a++;
            b++;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) {
            while (a < fv1->n_nodes && fv1->node_ids[a] < fv2->node_ids[b]) a++;
        } else {
            while (b < fv2->n_nodes && fv2->node_ids[b] < fv1->node_ids[a]) b++;
        }
    }
    if (checkOri) {
        int ind1 = -1, ind2 = -1, ind3 = -1;
        three_maxima(rotHist, HISTO_LENGTH, ind1, ind2, ind3);
        for (int i = 0; i < HISTO_LENGTH; i++) {
            if (i == ind1 || i == ind2 || i == ind3) continue;
            for (int k : rotHist[i]) { matches12[k] = -1; nmatches--; }
        }
    }
    return nmatches;
}

int oro_search_for_triangulation(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                 const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                 const float* F12, const float* ep, const float* level_sigma2_2, int32_t bOnlyStereo,
                                 int32_t bCoarse, int32_t checkOri, int32_t* matches12) {
    return search_for_triangulation(KF1, mp1, fv1, KF2, mp2, fv2, F12, ep, level_sigma2_2, bOnlyStereo, bCoarse,
                                    checkOri, matches12, nullptr, nullptr);
}

int oro_search_for_triangulation_epi(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                     const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                     const float* ep, int32_t bOnlyStereo, int32_t checkOri, oro_epipolar_fn epi,
                                     void* ctx, int32_t* matches12) {
    return search_for_triangulation(KF1, mp1, fv1, KF2, mp2, fv2, nullptr, ep, nullptr, bOnlyStereo, 0, checkOri,
                                    matches12, epi, ctx);
}

// The search half of both Fuse overloads; best_dist = -1 when no candidate survived the checks.
// model: pCamera (mpCamera, or mpCamera2 with bRight; NULL = pinhole from cam); bRight searches the
// right grid of a two-camera keyframe and reports global indices (idx += NLeft, ORBmatcher.cc:1283).
int oro_fuse_rig(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_camera_model* model,
                 const float* inv_level_sigma2, const orbfe_map_point_3d* pts, int32_t n, float th, int32_t sim3,
                 int32_t bRight, int32_t* best_idx, int32_t* best_dist) {
    const Grid grid(KF, KF->two_cams ? (bRight ? 1 : 0) : -1);
    CamModel M{ORBFE_CAM_PINHOLE, {cam->fx, cam->fy, cam->cx, cam->cy, 0.f, 0.f, 0.f, 0.f}};
    if (model) {
        M.type = model->type;
        memcpy(M.p, model->params, sizeof(M.p));
    }
    const float* uright = KF->two_cams ? nullptr : KF->uright;   // KannalaBrandt8 keyframes: mvuRight == -1
    int nFused = 0;
    for (int i = 0; i < n; i++) {
        best_idx[i] = -1;
        best_dist[i] = -1;
        const orbfe_map_point_3d& mp = pts[i];
        if (mp.id < 0) continue;   // !pMP
        if (mp.flags & (ORBFE_MP_BAD | ORBFE_MP_SKIP)) continue;
        float p3Dc[3];
        pose_apply(cam->Tcw, mp.pos, p3Dc);
        if (p3Dc[2] < 0.0f) continue;
        const float invz = 1 / p3Dc[2];
        float u, v;
        cam_project(M, p3Dc, u, v);   // pCamera->project (Pinhole: fx * x / z + cx)
        if (!kf_in_image(KF, u, v)) continue;
        const float ur = u - KF->mbf * invz;
        const float maxDistance = 1.2f * mp.max_dist, minDistance = 0.8f * mp.min_dist;
        const float PO[3] = {mp.pos[0] - cam->Ow[0], mp.pos[1] - cam->Ow[1], mp.pos[2] - cam->Ow[2]};
        const float dist3D = std::sqrt(eig_sum3(PO[0] * PO[0], PO[1] * PO[1], PO[2] * PO[2]));
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const float dotn = eig_sum3(PO[0] * mp.normal[0], PO[1] * mp.normal[1], PO[2] * mp.normal[2]);
        if (dotn < 0.5 * dist3D) continue;
        const int nPredictedLevel = predict_scale(mp.max_dist, dist3D, cam->log_scale_factor, KF->nlevels);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        const std::vector<size_t> vIndices = grid.area(u, v, radius, -1, -1);
        if (vIndices.empty()) continue;
        int bestDist = sim3 ? INT_MAX : 256, bestIdx = -1;
        for (size_t idx : vIndices) {
            const orbfe_keypoint& kp = KF->keys[idx];
            const int kpLevel = kp.octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            if (!sim3) {
                if (uright && uright[idx] >= 0) {
                    const float ex = u - kp.x, ey = v - kp.y, er = ur - uright[idx];
                    const float e2 = ex * ex + ey * ey + er * er;
                    if (e2 * inv_level_sigma2[kpLevel] > 7.8) continue;
                } else {
                    const float ex = u - kp.x, ey = v - kp.y;
                    const float e2 = ex * ex + ey * ey;
                    if (e2 * inv_level_sigma2[kpLevel] > 5.99) continue;
                }
            }
            const int dist = oracle::hamming(mp.desc, KF->desc + idx * 32);
            if (dist < bestDist) { bestDist = dist; bestIdx = (int)idx; }
        }
        if (bestIdx >= 0) best_dist[i] = bestDist;
        if (bestDist <= TH_LOW) {
            best_idx[i] = bestIdx;
            nFused++;
        }
    }
    return nFused;
}

int oro_fuse(const orbfe_frame* KF, const orbfe_kf_camera* cam, const float* inv_level_sigma2,
             const orbfe_map_point_3d* pts, int32_t n, float th, int32_t sim3, int32_t* best_idx, int32_t* best_dist) {
    return oro_fuse_rig(KF, cam, nullptr, inv_level_sigma2, pts, n, th, sim3, 0, best_idx, best_dist);
}

// model: pKF->mpCamera for the first overload (pKF->mpCamera->project, ORBmatcher.cc:465; NULL = the
// pinhole expression with cam's intrinsics); the vpPointsKFs overload always projects with
// fx * x * invz + cx (:571-576). A two-camera keyframe is searched on its left grid with mvKeys
// (KeyFrame::GetFeaturesInArea(.., bRight = false), KeyFrame.cc:707-751).
int oro_sbp_sim3_rig(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_camera_model* model,
                     const orbfe_map_point_3d* pts, int32_t n, const int32_t* point_kfs, int32_t th,
                     float ratioHamming, int32_t* matched, int32_t* matched_kf) {
    const Grid grid(KF, KF->two_cams ? 0 : -1);
    CamModel M{ORBFE_CAM_PINHOLE, {cam->fx, cam->fy, cam->cx, cam->cy, 0.f, 0.f, 0.f, 0.f}};
    if (model) {
        M.type = model->type;
        memcpy(M.p, model->params, sizeof(M.p));
    }
    std::vector<int32_t> found;
    for (int k = 0; k < KF->n; k++)
        if (matched[k] >= 0) found.push_back(matched[k]);
    std::sort(found.begin(), found.end());
    int nmatches = 0;
    for (int iMP = 0; iMP < n; iMP++) {
        const orbfe_map_point_3d& mp = pts[iMP];
        if (mp.id < 0) continue;   // NULL entry (the reference dereferences it; the API skips it)
        if ((mp.flags & ORBFE_MP_BAD) || std::binary_search(found.begin(), found.end(), mp.id)) continue;
        float p3Dc[3];
        pose_apply(cam->Tcw, mp.pos, p3Dc);
        if (p3Dc[2] < 0.0) continue;
        float u, v;
        if (!point_kfs) {
            cam_project(M, p3Dc, u, v);   // pKF->mpCamera->project (Pinhole: fx * x / z + cx)
        } else {
            const float invz = 1 / p3Dc[2];
            const float x = p3Dc[0] * invz, y = p3Dc[1] * invz;
            u = cam->fx * x + cam->cx;
            v = cam->fy * y + cam->cy;
        }
        if (!kf_in_image(KF, u, v)) continue;
        const float maxDistance = 1.2f * mp.max_dist, minDistance = 0.8f * mp.min_dist;
        const float PO[3] = {mp.pos[0] - cam->Ow[0], mp.pos[1] - cam->Ow[1], mp.pos[2] - cam->Ow[2]};
        const float dist = std::sqrt(eig_sum3(PO[0] * PO[0], PO[1] * PO[1], PO[2] * PO[2]));
        if (dist < minDistance || dist > maxDistance) continue;
        const float dotn = eig_sum3(PO[0] * mp.normal[0], PO[1] * mp.normal[1], PO[2] * mp.normal[2]);
        if (dotn < 0.5 * dist) continue;
        const int nPredictedLevel = predict_scale(mp.max_dist, dist, cam->log_scale_factor, KF->nlevels);
        const float radius = th * KF->scale_factors[nPredictedLevel];
        const std::vector<size_t> vIndices = grid.area(u, v, radius, -1, -1);
        if (vIndices.empty()) continue;
        int bestDist = 256, bestIdx = -1;
        for (size_t idx : vIndices) {
            if (matched[idx] >= 0) continue;
            const int kpLevel = KF->keys[idx].octave;
            if (kpLevel < nPredictedLevel - 1 || kpLevel > nPredictedLevel) continue;
            const int d = oracle::hamming(mp.desc, KF->desc + idx * 32);
            if (d < bestDist) { bestDist = d; bestIdx = (int)idx; }
        }
        if (bestDist <= TH_LOW * ratioHamming) {
            matched[bestIdx] = mp.id;
            if (point_kfs && matched_kf) matched_kf[bestIdx] = point_kfs[iMP];
            nmatches++;
        }
    }
    return nmatches;
}

int oro_sbp_sim3(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_map_point_3d* pts, int32_t n,
                 const int32_t* point_kfs, int32_t th, float ratioHamming, int32_t* matched, int32_t* matched_kf) {
    return oro_sbp_sim3_rig(KF, cam, nullptr, pts, n, point_kfs, th, ratioHamming, matched, matched_kf);
}

// One direction of SearchBySim3: points of A transformed by TAw then SBA, searched in B.
static void sim3_side(const orbfe_frame* B, const Grid& gridB, const orbfe_map_point_3d* ptsA, int nA,
                      const std::vector<char>& already, const orbfe_pose& TAw, const orbfe_pose& SBA,
                      const orbfe_kf_camera* cam1, float logsfB, float th, std::vector<int>& vnMatch) {
    vnMatch.assign(nA, -1);
    for (int i = 0; i < nA; i++) {
        const orbfe_map_point_3d& mp = ptsA[i];
        if (mp.id < 0 || already[i]) continue;
        if (mp.flags & ORBFE_MP_BAD) continue;
        float pA[3], pB[3];
        pose_apply(TAw, mp.pos, pA);
        pose_apply(SBA, pA, pB);
        if (pB[2] < 0.0) continue;
        const float invz = (float)(1.0 / (double)pB[2]);
        const float x = pB[0] * invz, y = pB[1] * invz;
        const float u = cam1->fx * x + cam1->cx, v = cam1->fy * y + cam1->cy;
        if (!kf_in_image(B, u, v)) continue;
        const float maxDistance = 1.2f * mp.max_dist, minDistance = 0.8f * mp.min_dist;
        const float dist3D = std::sqrt(eig_sum3(pB[0] * pB[0], pB[1] * pB[1], pB[2] * pB[2]));
        if (dist3D < minDistance || dist3D > maxDistance) continue;
        const int nPredictedLevel = predict_scale(mp.max_dist, dist3D, logsfB, B->nlevels);
        const float radius = th * B->scale_factors[nPredictedLevel];
        const std::vector<size_t> vIndices = gridB.area(u, v, radius, -1, -1);
        if (vIndices.empty()) continue;
        int bestDist = INT_MAX, bestIdx = -1;
        for (size_t idx : vIndices) {
            const int oct = B->keys[idx].octave;
            if (oct < nPredictedLevel - 1 || oct > nPredictedLevel) continue;
            const int d = oracle::hamming(mp.desc, B->desc + idx * 32);
            if (d < bestDist) { bestDist = d; bestIdx = (int)idx; }
        }
        if (bestDist <= TH_HIGH) vnMatch[i] = bestIdx;
    }
}

int oro_search_by_sim3(const orbfe_frame* KF1, const orbfe_frame* KF2, const orbfe_map_point_3d* pts1,
                       const orbfe_map_point_3d* pts2, const orbfe_kf_camera* cam1, const orbfe_kf_camera* cam2,
                       const orbfe_pose* S12, const orbfe_pose* S21, float th, int32_t* matches12,
                       const int32_t* matched_idx2) {
    const int N1 = KF1->n, N2 = KF2->n;
    std::vector<char> already1(N1, 0), already2(N2, 0);
    for (int i = 0; i < N1; i++)
        if (matches12[i] >= 0) {
            already1[i] = 1;
            const int idx2 = matched_idx2 ? matched_idx2[i] : -1;
            if (idx2 >= 0 && idx2 < N2) already2[idx2] = 1;
        }
    // pKF->GetFeaturesInArea(u, v, r): the left grid (mvKeys) of a two-camera keyframe; every
    // camera projects with pKF1's fx, fy, cx, cy (ORBmatcher.cc:1459-1462,1514-1519,1594-1599)
    const Grid g1(KF1, KF1->two_cams ? 0 : -1), g2(KF2, KF2->two_cams ? 0 : -1);
    std::vector<int> vnMatch1, vnMatch2;
    sim3_side(KF2, g2, pts1, N1, already1, cam1->Tcw, *S21, cam1, cam2->log_scale_factor, th, vnMatch1);
    sim3_side(KF1, g1, pts2, N2, already2, cam2->Tcw, *S12, cam1, cam1->log_scale_factor, th, vnMatch2);
    int nFound = 0;
    for (int i1 = 0; i1 < N1; i1++) {
        const int idx2 = vnMatch1[i1];
        if (idx2 >= 0 && vnMatch2[idx2] == i1) {
            matches12[i1] = pts2[idx2].id;
            nFound++;
        }
    }
    return nFound;
}

// BFMatcher(NORM_HAMMING).knnMatch(k=2): per query the two smallest distances, earlier train index
// first on ties; accept when (float)d0 < (double)d1 * ratio (Frame.cc:1151 multiplies by 0.7).
int oro_stereo_knn_ratio(const uint8_t* L, int32_t nl, const uint8_t* R, int32_t nr, float ratio, int32_t* out_train,
                         int32_t* out_dist) {
    int good = 0;
    for (int i = 0; i < nl; i++) {
        int d0 = INT_MAX, d1 = INT_MAX, t0 = -1;
        for (int j = 0; j < nr; j++) {
            const int d = oracle::hamming(L + (size_t)i * 32, R + (size_t)j * 32);
            if (d < d0) { d1 = d0; d0 = d; t0 = j; }
            else if (d < d1) d1 = d;
        }
        out_train[i] = -1;
        out_dist[i] = -1;
        if (nr >= 2 && (float)d0 < (float)d1 * (double)ratio) { out_train[i] = t0; out_dist[i] = d0; good++; }
    }
    return good;
}


// The checks of one view (isInFrustum's Nleft == -1 branch up to its writes, or isInFrustumChecks):
// returns the stage reached: 0 behind the camera, 1 outside the image, 2 outside the distance /
// viewing limits, 3 in view.
struct View {
    float u, v, depth, invz, view_cos;
    int level;
};
static int frustum_view(const orbfe_frame* F, const orbfe_camera* c, const float* R, const float* t, const float* Ow,
                        const CamModel& m, const orbfe_map_point_3d& p, View& o) {
    const float P0 = p.pos[0], P1 = p.pos[1], P2 = p.pos[2];
    float Pc[3];
    for (int i = 0; i < 3; i++) Pc[i] = eig_sum3(R[3 * i] * P0, R[3 * i + 1] * P1, R[3 * i + 2] * P2) + t[i];
    o.depth = std::sqrt(eig_sum3(Pc[0] * Pc[0], Pc[1] * Pc[1], Pc[2] * Pc[2]));
    o.invz = 1.0f / Pc[2];
    if (Pc[2] < 0.0f) return 0;
    cam_project(m, Pc, o.u, o.v);
    if (o.u < F->min_x || o.u > F->max_x) return 1;
    if (o.v < F->min_y || o.v > F->max_y) return 1;
    const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;   // Get{Max,Min}DistanceInvariance
    const float PO0 = P0 - Ow[0], PO1 = P1 - Ow[1], PO2 = P2 - Ow[2];
    const float dist = std::sqrt(eig_sum3(PO0 * PO0, PO1 * PO1, PO2 * PO2));
    if (dist < minDistance || dist > maxDistance) return 2;
    o.view_cos = eig_sum3(PO0 * p.normal[0], PO1 * p.normal[1], PO2 * p.normal[2]) / dist;
    if (o.view_cos < c->view_cos_limit) return 2;
    // MapPoint::PredictScale (MapPoint.cc:531-546): log(float) resolves to logf
    const float ratio = p.max_dist / dist;
    int nScale = (int)std::ceil(logf(ratio) / c->log_scale_factor);
    if (nScale < 0) nScale = 0;
    else if (nScale >= F->nlevels) nScale = F->nlevels - 1;
    o.level = nScale;
    return 3;
}

// Frame::isInFrustum (Frame.cc:512-586). Nleft == -1: mTrackProjX / Y = -1, then the projection
// once it is in the image, the rest when every check passes. Nleft != -1: both views through
// isInFrustumChecks (Frame.cc:1168-1242), levels reset to -1, each view's fields written only when
// it passes (failed-view fields: projections -1 here; the reference leaves the previous values).
static bool is_in_frustum(const orbfe_frame* F, const orbfe_camera* c, const orbfe_stereo_rig* rig,
                          const orbfe_map_point_3d& p, orbfe_map_point& t) {
    CamModel L{ORBFE_CAM_PINHOLE, {c->fx, c->fy, c->cx, c->cy, 0.f, 0.f, 0.f, 0.f}};
    if (rig) {
        L.type = rig->left.type;
        memcpy(L.p, rig->left.params, sizeof(L.p));
    }
    View o{};
    if (!F->two_cams) {
        t.flags &= ~ORBFE_MP_IN_VIEW;
        t.proj_x = -1;
        t.proj_y = -1;
        const int st = frustum_view(F, c, c->Rcw, c->tcw, c->Ow, L, p, o);
        if (st >= 2) {
            t.proj_x = o.u;
            t.proj_y = o.v;
        }
        if (st < 3) return false;
        t.flags |= ORBFE_MP_IN_VIEW;
        t.proj_xr = o.u - F->mbf * o.invz;
        t.depth = o.depth;
        t.scale_level = o.level;
        t.view_cos = o.view_cos;
        return true;
    }
    t.flags &= ~(ORBFE_MP_IN_VIEW | ORBFE_MP_IN_VIEW_R);
    t.scale_level = -1;
    t.scale_level_r = -1;
    t.proj_x = t.proj_y = t.proj_xr = t.proj_yr = -1;
    bool in = false;
    if (frustum_view(F, c, c->Rcw, c->tcw, c->Ow, L, p, o) == 3) {
        t.flags |= ORBFE_MP_IN_VIEW;
        t.proj_x = o.u;
        t.proj_y = o.v;
        t.scale_level = o.level;
        t.view_cos = o.view_cos;
        t.depth = o.depth;
        in = true;
    }
    // right view: mR = Rrl * mRcw, mt = Rrl * mtcw + trl, twc = mRwc * mTlr.translation() + mOw
    float R2[9], t2[3], Ow2[3];
    const float* A = rig->Rrl;
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
            R2[3 * i + j] = eig_sum3(A[3 * i] * c->Rcw[j], A[3 * i + 1] * c->Rcw[3 + j], A[3 * i + 2] * c->Rcw[6 + j]);
        t2[i] = eig_sum3(A[3 * i] * c->tcw[0], A[3 * i + 1] * c->tcw[1], A[3 * i + 2] * c->tcw[2]) + rig->trl[i];
        Ow2[i] = eig_sum3(rig->Rwc[3 * i] * rig->tlr[0], rig->Rwc[3 * i + 1] * rig->tlr[1], rig->Rwc[3 * i + 2] * rig->tlr[2]) +
                 c->Ow[i];
    }
    CamModel Rm{rig->right.type, {}};
    memcpy(Rm.p, rig->right.params, sizeof(Rm.p));
    if (frustum_view(F, c, R2, t2, Ow2, Rm, p, o) == 3) {
        t.flags |= ORBFE_MP_IN_VIEW_R;
        t.proj_xr = o.u;
        t.proj_yr = o.v;
        t.scale_level_r = o.level;
        t.view_cos_r = o.view_cos;
        in = true;
    }
    return in;
}

int oro_is_in_frustum_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                          const orbfe_map_point_3d* pts, int32_t n, orbfe_map_point* track) {
    int nToMatch = 0;
    for (int i = 0; i < n; i++) {
        const orbfe_map_point_3d& p = pts[i];
        orbfe_map_point& t = track[i];
        memset(&t, 0, sizeof(t));
        t.depth = p.track_depth;   // mTrackDepth persists unless a left view passes (Frame.cc:565,1237)
        t.flags = p.flags & ORBFE_MP_BAD;
        t.observations = p.observations;
        t.id = p.id;
        memcpy(t.desc, p.desc, 32);
        if (F->two_cams) { t.scale_level = -1; t.scale_level_r = -1; t.proj_x = t.proj_y = t.proj_xr = t.proj_yr = -1; }
        else { t.proj_x = t.proj_y = -1; t.scale_level_r = -1; }
        if (p.flags & ORBFE_MP_SKIP) continue;   // mnLastFrameSeen == current: mbTrackInView = false
        if (p.flags & ORBFE_MP_BAD) continue;
        if (is_in_frustum(F, cam, rig, p, t)) nToMatch++;
    }
    return nToMatch;
}

int oro_is_in_frustum(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts, int32_t n,
                      orbfe_map_point* track) {
    return oro_is_in_frustum_rig(F, cam, nullptr, pts, n, track);
}

int oro_search_local_points_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* mvp_obs, float th,
                                int32_t bFarPoints, float thFarPoints, float nnratio, int32_t* n_to_match) {
    std::vector<orbfe_map_point> track(n > 0 ? n : 1);
    const int nToMatch = oro_is_in_frustum_rig(F, cam, rig, pts, n, track.data());
    if (n_to_match) *n_to_match = nToMatch;
    if (nToMatch <= 0) return 0;
    return oro_sbp_local(F, mvp, mvp_obs, track.data(), n, th, bFarPoints, thFarPoints, nnratio);
}

int oro_search_local_points(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts, int32_t n,
                            int32_t* mvp, const int32_t* mvp_obs, float th, int32_t bFarPoints, float thFarPoints,
                            float nnratio, int32_t* n_to_match) {
    return oro_search_local_points_rig(F, cam, nullptr, pts, n, mvp, mvp_obs, th, bFarPoints, thFarPoints, nnratio,
                                       n_to_match);
}

}  // extern "C"
