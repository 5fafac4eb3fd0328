// Back-end ORBmatcher pieces on CDNA4; included into orbfe_engine.hip after the
// matcher (per-thread arena / stream helpers, rotation histogram helpers, level grids).
//  * SearchByBoW(KF1, KF2) (ORBmatcher.cc:765-903): like SearchByBoW(KF, F) one thread walks one
//    shared vocabulary node; vbMatched2 is node-local because a KF2 index lives in one node.
//  * MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403): one wave per map point, the
//    point's descriptors staged in LDS, every row's median found by a wave-wide counting search.
//  * SearchForTriangulation (ORBmatcher.cc:907-1146): vbMatched2 is never set by the reference, so
//    every KF1 keypoint of a shared node is an independent work item (one thread each).
//  * Fuse x2 (:1148-1455), SearchByProjection Sim3 x2 (:427-646), SearchBySim3 (:1457-1674): one
//    geometry kernel (Sophus pose action, projection, IsInImage, distance / viewing checks,
//    PredictScale) writes a 16-byte projection record per point; one search kernel scans the
//    keyframe's level-restricted grid. SearchByProjection's "keypoint already matched" dependency
//    is triangular and uses the matcher's fixed-point passes.
#pragma once

__global__ __launch_bounds__(MT_NT) void k_bow_kfkf(const int* pairs, int npairs, const int* off1, const uint32_t* idx1s,
                                                    const int* off2, const uint32_t* idx2s, const int32_t* mp1,
                                                    const int32_t* mp2, const uint32_t* d1, const uint32_t* d2,
                                                    float nnratio, int* matched2, int* out_idx, int lim1, int lim2) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npairs) return;
    const int a = pairs[2 * t], b = pairs[2 * t + 1];
    for (int ia = off1[a]; ia < off1[a + 1]; ia++) {
        const unsigned i1 = idx1s[ia];
        if ((int)i1 >= lim1) continue;   // a two-camera KF's right indices (ORBmatcher.cc:800-802)
        if (mp1[i1] < 0) continue;
        uint32_t q[8];
#pragma unroll
        for (int w = 0; w < 8; w++) q[w] = d1[8 * i1 + w];
        int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
        for (int ib = off2[b]; ib < off2[b + 1]; ib++) {
            const unsigned i2 = idx2s[ib];
            if ((int)i2 >= lim2) continue;   // (ORBmatcher.cc:817-819)
            if (matched2[i2] || mp2[i2] < 0) continue;
            int dist = 0;
#pragma unroll
            for (int w = 0; w < 8; w++) dist += __popc(q[w] ^ d2[8 * i2 + w]);
            if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdx2 = (int)i2; }
            else if (dist < bestDist2) bestDist2 = dist;
        }
        if (bestDist1 < MT_TH_LOW && static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) {
            out_idx[i1] = bestIdx2;
            matched2[bestIdx2] = 1;
        }
    }
}

__global__ __launch_bounds__(1024) void k_bow_kfkf_commit(const OrbKeyPoint* k1, const OrbKeyPoint* k2, int n1,
                                                          const int32_t* mp2, int checkOri, const int* out_idx,
                                                          int* out12, int* result) {
    __shared__ int s_hist[MT_HISTO];
    __shared__ unsigned s_keep;
    __shared__ int s_n;
    if (threadIdx.x < MT_HISTO) s_hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_n = 0;
    SYNC();
    for (int i = threadIdx.x; i < n1; i += blockDim.x) {
        const int j = out_idx[i];
        if (j >= 0 && checkOri) atomicAdd(&s_hist[mt_rot_bin(k1[i].angle, k2[j].angle)], 1);
    }
    SYNC();
    if (threadIdx.x == 0) s_keep = checkOri ? mt_three_maxima_keep(s_hist) : 0xFFFFFFFFu;
    SYNC();
    int cnt = 0;
    for (int i = threadIdx.x; i < n1; i += blockDim.x) {
        const int j = out_idx[i];
        int o = -1;
        if (j >= 0 && (!checkOri || ((s_keep >> mt_rot_bin(k1[i].angle, k2[j].angle)) & 1u))) o = mp2 ? mp2[j] : j;
        out12[i] = o;
        cnt += o >= 0 ? 1 : 0;
    }
    atomicAdd(&s_n, cnt);
    SYNC();
    if (threadIdx.x == 0) result[0] = s_n;
}

#define DD_MAXN 2048   // descriptors per point accepted by the API
#define DD_LDS_N 256   // descriptors per point staged in LDS (larger points read L2-resident global rows)
__global__ __launch_bounds__(256) void k_distinctive(const uint32_t* desc, const int* offsets, int np, int* best) {
    __shared__ uint4 s_d[4][2 * DD_LDS_N];   // one slice per wave, 2 x uint4 per descriptor
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + wave;
    if (p >= np) return;
    const int o0 = offsets[p], N = offsets[p + 1] - o0;
    if (N <= 0) {
        if (lane == 0) best[p] = -1;
        return;
    }
    uint4* sd = s_d[wave];
    const bool lds = N <= DD_LDS_N;
    if (lds) {
        for (int i = lane; i < 2 * N; i += 64) sd[i] = ((const uint4*)(desc + 8 * (size_t)o0))[i];
        WAVE_SYNC();
    }
    auto row = [&](int i, uint32_t (&r)[8]) {
        if (lds) {
            const uint4 a = sd[2 * i], b = sd[2 * i + 1];
            r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w; r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
        } else {
#pragma unroll
            for (int w = 0; w < 8; w++) r[w] = desc[8 * ((size_t)o0 + i) + w];
        }
    };
    const int kth = (N - 1) / 2;   // vDists[0.5 * (N - 1)], index truncated
    int bestMedian = INT_MAX, bestIdx = 0;
    for (int i = 0; i < N; i++) {
        uint32_t ri[8];
        row(i, ri);
        // the row's distances, 64 per chunk; the kth smallest = min v with #(d <= v) > kth
        int lo = 0, hi = 256;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            int c = 0;
            for (int j0 = 0; j0 < N; j0 += 64) {
                const int j = j0 + lane;
                int d = 1 << 20;
                if (j < N) {
                    uint32_t rj[8];
                    row(j, rj);
                    d = 0;
#pragma unroll
                    for (int w = 0; w < 8; w++) d += __popc(ri[w] ^ rj[w]);
                }
                c += __popcll(__ballot(d <= mid));
            }
            if (c > kth) hi = mid; else lo = mid + 1;
        }
        if (lo < bestMedian) { bestMedian = lo; bestIdx = i; }
    }
    if (lane == 0) best[p] = bestIdx;
}

// ---- back-end projections ----
// (be_pose_apply, the Sophus point action, lives in orbfe_matcher.hip: the last-frame search uses it too)

#define BE_PRJ_PINHOLE 0   // Pinhole::project: fx * x / z + cx
#define BE_PRJ_INVZ_F 1    // invz = 1 / z (float); u = fx * (x * invz) + cx
#define BE_PRJ_INVZ_D 2    // invz = (float)(1.0 / z)
#define BE_PRJ_MODEL 3     // GeometricCamera::project of cam_type (Pinhole == BE_PRJ_PINHOLE, KannalaBrandt8)
struct KfGeom {
    orbfe_pose T, S;
    int two;               // apply S after T (SearchBySim3)
    float Ow[3];
    float fx, fy, cx, cy, logsf, mbf;
    float kb[4];           // BE_PRJ_MODEL with a KannalaBrandt8 camera: k0..k3
    int cam_type;          // BE_PRJ_MODEL: ORBFE_CAM_*
    float minx, maxx, miny, maxy;
    int nlevels, proj, dist_cam, view;
    int skip_flags;        // ORBFE_MP_* flags that exclude a point (id < 0 = NULL always does)
};
struct KfProj {
    float u, v, ur;
    int level;             // -1: rejected before the search
};

__global__ __launch_bounds__(MT_NT) void k_kf_geom(KfGeom g, const orbfe_map_point_3d* pts, int n,
                                                   const uint8_t* skip, KfProj* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    KfProj r{0.f, 0.f, 0.f, -1};
    const orbfe_map_point_3d& mp = pts[i];
    do {
        if (mp.id < 0 || (mp.flags & g.skip_flags) || (skip && skip[i])) break;
        const float P[3] = {mp.pos[0], mp.pos[1], mp.pos[2]};
        float pc[3];
        be_pose_apply(g.T, P, pc);
        if (g.two) {
            const float a[3] = {pc[0], pc[1], pc[2]};
            be_pose_apply(g.S, a, pc);
        }
        if (pc[2] < 0.0f) break;
        const float invz = g.proj == BE_PRJ_INVZ_D ? (float)(1.0 / (double)pc[2]) : 1.0f / pc[2];
        float u, v;
        if (g.proj == BE_PRJ_PINHOLE) {
            u = g.fx * pc[0] / pc[2] + g.cx;
            v = g.fy * pc[1] / pc[2] + g.cy;
        } else if (g.proj == BE_PRJ_MODEL) {
            const CamModelDev m{g.cam_type, g.fx, g.fy, g.cx, g.cy, {g.kb[0], g.kb[1], g.kb[2], g.kb[3]}};
            const float2 uv = mt_cam_project(m, pc[0], pc[1], pc[2]);
            u = uv.x;
            v = uv.y;
        } else {
            const float x = pc[0] * invz, y = pc[1] * invz;
            u = g.fx * x + g.cx;
            v = g.fy * y + g.cy;
        }
        if (!(u >= g.minx && u < g.maxx && v >= g.miny && v < g.maxy)) break;   // KeyFrame::IsInImage
        const float maxDistance = 1.2f * mp.max_dist, minDistance = 0.8f * mp.min_dist;
        float dist;
        float PO[3] = {0.f, 0.f, 0.f};
        if (g.dist_cam) {
            dist = sqrtf(eig_sum3(pc[0] * pc[0], pc[1] * pc[1], pc[2] * pc[2]));
        } else {
            PO[0] = P[0] - g.Ow[0]; PO[1] = P[1] - g.Ow[1]; PO[2] = P[2] - g.Ow[2];
            dist = sqrtf(eig_sum3(PO[0] * PO[0], PO[1] * PO[1], PO[2] * PO[2]));
        }
        if (dist < minDistance || dist > maxDistance) break;
        if (g.view) {
            const float dotn = eig_sum3(PO[0] * mp.normal[0], PO[1] * mp.normal[1], PO[2] * mp.normal[2]);
            if ((double)dotn < 0.5 * (double)dist) break;
        }
        const float ratio = mp.max_dist / dist;
        int nScale = (int)ceilf(glibc_logf(ratio) / g.logsf);
        if (nScale < 0) nScale = 0;
        else if (nScale >= g.nlevels) nScale = g.nlevels - 1;
        r.u = u;
        r.v = v;
        r.ur = u - g.mbf * invz;
        r.level = nScale;
    } while (0);
    out[i] = r;
}

// Best keypoint in the radius among octaves [level-1, level] (strict-< first minimum), optional
// Fuse stereo / mono reprojection gate, optional "already matched" blocking (fixed-point passes).
__global__ __launch_bounds__(MT_NT) void k_kf_search(FrameDev fr, const KfProj* pj, const orbfe_map_point_3d* pts,
                                                     int nq, float th, int reproj, const float* inv_sigma2,
                                                     int init_best, float max_acc, const int* blocked0,
                                                     const int* first, int* assign, int* out_dist, int* changed,
                                                     int cell_off = 0) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const KfProj p = pj[q];
    int result = -1, bestIdx = -1, bestDist = init_best;
    if (p.level >= 0) {
        const float radius = th * fr.scale[p.level];
        const orbfe_map_point_3d& mp = pts[q];
        // cell_off = MT_NCELL: a two-camera keyframe's right grid (GetFeaturesInArea(.., bRight), KeyFrame.cc:707-751)
        mt_for_area(fr, fr.pcstart + p.level * fr.gstride_c + cell_off, fr.pcidx + p.level * fr.gstride_i, p.u, p.v, radius, -1,
                    -1, [&](int idx, const OrbKeyPoint& kp) {
            if (blocked0 && (blocked0[idx] || first[idx] < q)) return;
            if (reproj) {
                const float ex = p.u - kp.x, ey = p.v - kp.y;
                if (fr.uright && fr.uright[idx] >= 0) {
                    const float er = p.ur - fr.uright[idx];
                    const float e2 = ex * ex + ey * ey + er * er;
                    if ((double)(e2 * inv_sigma2[kp.octave]) > 7.8) return;
                } else {
                    const float e2 = ex * ex + ey * ey;
                    if ((double)(e2 * inv_sigma2[kp.octave]) > 5.99) return;
                }
            }
            const int dist = mt_hamming(mp.desc, fr.desc + 8 * idx);
            if (dist < bestDist) { bestDist = dist; bestIdx = idx; }
        });
        if (bestIdx >= 0 && (float)bestDist <= max_acc) result = bestIdx;
    }
    if (out_dist) out_dist[q] = bestIdx >= 0 ? bestDist : -1;
    if (result != assign[q]) {
        assign[q] = result;
        if (changed) mt_flag_changed(changed);
    }
}

__global__ void k_kf_commit(const int* assign, int nq, const orbfe_map_point_3d* pts, const int32_t* point_kfs,
                            int32_t* matched, int32_t* matched_kf, int* count) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int a = q < nq ? assign[q] : -1;
    if (a >= 0) {
        matched[a] = pts[q].id;
        if (point_kfs) matched_kf[a] = point_kfs[q];
    }
    const unsigned long long m = __ballot(a >= 0);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, __popcll(m));
}

__global__ void k_count_ge0(const int* v, int n, int* count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long m = __ballot(i < n && v[i] >= 0);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, __popcll(m));
}

__global__ void k_sim3_agree(const int* vn1, int n1, const int* vn2, const orbfe_map_point_3d* pts2, int32_t* m12,
                             int* count) {
    const int i1 = blockIdx.x * blockDim.x + threadIdx.x;
    bool ok = false;
    if (i1 < n1) {
        const int idx2 = vn1[i1];
        if (idx2 >= 0 && vn2[idx2] == i1) {
            m12[i1] = pts2[idx2].id;
            ok = true;
        }
    }
    const unsigned long long m = __ballot(ok);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, __popcll(m));
}

// ---- SearchForTriangulation ----
struct TriArgs {
    float F[9], ep[2];
    int bOnlyStereo, bCoarse;
    int two1, two2;        // KF1 / KF2 have a second camera (mpCamera2): bStereo false, no epipole test for KF1
};
__global__ __launch_bounds__(MT_NT) void k_tri(const int2* items, int nitems, const uint32_t* idx1s, const int* off2,
                                               const uint32_t* idx2s, const OrbKeyPoint* k1, const OrbKeyPoint* k2,
                                               const uint32_t* d1, const uint32_t* d2, const float* ur1,
                                               const float* ur2, const int32_t* mp1, const int32_t* mp2,
                                               const float* scale2, const float* sigma2_2, TriArgs a, int* out_idx) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nitems) return;
    const int2 it = items[t];
    const unsigned i1 = idx1s[it.x];
    if (mp1[i1] >= 0) return;
    const bool bStereo1 = !a.two1 && ur1 && ur1[i1] >= 0;   // (!pKF1->mpCamera2 && mvuRight >= 0)
    if (a.bOnlyStereo && !bStereo1) return;
    const OrbKeyPoint kp1 = k1[i1];
    uint32_t q[8];
#pragma unroll
    for (int w = 0; w < 8; w++) q[w] = d1[8 * i1 + w];
    // epipolar line of kp1 in KF2 (Pinhole::epipolarConstrain, Pinhole.cpp:114-117)
    const float la = kp1.x * a.F[0] + kp1.y * a.F[3] + a.F[6];
    const float lb = kp1.x * a.F[1] + kp1.y * a.F[4] + a.F[7];
    const float lc = kp1.x * a.F[2] + kp1.y * a.F[5] + a.F[8];
    int bestDist = MT_TH_LOW, bestIdx2 = -1;
    for (int ib = off2[it.y]; ib < off2[it.y + 1]; ib++) {
        const unsigned i2 = idx2s[ib];
        if (mp2[i2] >= 0) continue;
        const bool bStereo2 = !a.two2 && ur2 && ur2[i2] >= 0;
        if (a.bOnlyStereo && !bStereo2) continue;
        int dist = 0;
#pragma unroll
        for (int w = 0; w < 8; w++) dist += __popc(q[w] ^ d2[8 * i2 + w]);
        if (dist > MT_TH_LOW || dist > bestDist) continue;
        const OrbKeyPoint kp2 = k2[i2];
        if (!bStereo1 && !bStereo2 && !a.two1) {
            const float distex = a.ep[0] - kp2.x, distey = a.ep[1] - kp2.y;
            if (distex * distex + distey * distey < 100 * scale2[kp2.octave]) continue;
        }
        bool ok = a.bCoarse != 0;
        if (!ok) {
            const float num = la * kp2.x + lb * kp2.y + lc;
            const float den = la * la + lb * lb;
            if (den != 0) {
                const float dsqr = num * num / den;
                ok = (double)dsqr < 3.84 * (double)sigma2_2[kp2.octave];
            }
        }
        if (ok) { bestIdx2 = (int)i2; bestDist = dist; }
    }
    if (bestIdx2 >= 0) out_idx[i1] = bestIdx2;
}

// SearchForTriangulation with the caller's epipolar test (bCoarse false on keyframes with a second
// camera, whose KannalaBrandt8 test is a host-side JacobiSVD triangulation): one thread per KF1
// keypoint of a shared node lists the node's KF2 candidates that pass every other gate of the
// reference's loop (ORBmatcher.cc:1002-1033: no map point, bOnlyStereo, dist <= TH_LOW, the epipole
// distance), sorted by (dist ascending, node order descending). The loop keeps a candidate when its
// dist <= bestDist and the epipolar test passes, so its result is the LAST passing candidate of the
// smallest passing dist: the first passing entry of this order. seg_off[t] = the item's segment (its
// node's size), cnt[t] = candidates listed, cand = KF2 indices.
__global__ __launch_bounds__(MT_NT) void k_tri_cand(const int2* items, int nitems, const int* seg_off,
                                                    const uint32_t* idx1s, const int* off2, const uint32_t* idx2s,
                                                    const OrbKeyPoint* k2, const uint32_t* d1, const uint32_t* d2,
                                                    const float* ur1, const float* ur2, const int32_t* mp1,
                                                    const int32_t* mp2, const float* scale2, TriArgs a, int* cnt,
                                                    uint32_t* cand) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nitems) return;
    const int2 it = items[t];
    const unsigned i1 = idx1s[it.x];
    int nc = 0;
    const bool bStereo1 = !a.two1 && ur1 && ur1[i1] >= 0;
    if (mp1[i1] < 0 && !(a.bOnlyStereo && !bStereo1)) {
        uint32_t q[8];
#pragma unroll
        for (int w = 0; w < 8; w++) q[w] = d1[8 * i1 + w];
        uint32_t* out = cand + seg_off[t];
        const int base = off2[it.y];
        for (int ib = base; ib < off2[it.y + 1]; ib++) {
            const unsigned i2 = idx2s[ib];
            if (mp2[i2] >= 0) continue;
            const bool bStereo2 = !a.two2 && ur2 && ur2[i2] >= 0;
            if (a.bOnlyStereo && !bStereo2) continue;
            int dist = 0;
#pragma unroll
            for (int w = 0; w < 8; w++) dist += __popc(q[w] ^ d2[8 * i2 + w]);
            if (dist > MT_TH_LOW) continue;
            if (!bStereo1 && !bStereo2 && !a.two1) {
                const OrbKeyPoint kp2 = k2[i2];
                const float distex = a.ep[0] - kp2.x, distey = a.ep[1] - kp2.y;
                if (distex * distex + distey * distey < 100 * scale2[kp2.octave]) continue;
            }
            // (dist, reverse node position): ascending order = the test order
            const uint32_t key = ((uint32_t)dist << 20) | (0xFFFFFu - (uint32_t)(ib - base));
            int j = nc++;
            for (; j > 0 && out[j - 1] > key; j--) out[j] = out[j - 1];
            out[j] = key;
        }
        for (int j = 0; j < nc; j++) out[j] = idx2s[base + (int)(0xFFFFFu - (out[j] & 0xFFFFFu))];
    }
    cnt[t] = nc;
}

extern "C" {

int orbfe_search_by_bow_kf(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                           const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2, const uint8_t* desc2,
                           const int32_t* mp2, int32_t n2, const orbfe_feature_vector* fv2, int32_t* out12,
                           float nnratio, int32_t checkOri) {
    return orbfe_search_by_bow_kf2(keys1, desc1, mp1, n1, -1, fv1, keys2, desc2, mp2, n2, -1, fv2, out12, nnratio,
                                   checkOri);
}

int orbfe_search_by_bow_kf2(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                            int32_t nleft1, const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2,
                            const uint8_t* desc2, const int32_t* mp2, int32_t n2, int32_t nleft2,
                            const orbfe_feature_vector* fv2, int32_t* out12, float nnratio, int32_t checkOri) {
    if (n1 < 0 || n2 < 0 || !fv1 || !fv2 || (n1 > 0 && (!keys1 || !desc1 || !mp1 || !out12)) ||
        (n2 > 0 && (!keys2 || !desc2 || !mp2)) || nleft1 < -1 || nleft1 > n1 || nleft2 < -1 || nleft2 > n2)
        return ORBFE_E_ARG;
    const int lim1 = nleft1 >= 0 ? nleft1 : n1, lim2 = nleft2 >= 0 ? nleft2 : n2;
    for (int i = 0; i < n1; i++) out12[i] = -1;
    if (n1 == 0 || n2 == 0 || fv1->n_nodes <= 0 || fv2->n_nodes <= 0) return 0;
    for (const orbfe_feature_vector* fv : {fv1, fv2}) {
        if (!fv->node_ids || !fv->offsets || fv->offsets[0] != 0) return ORBFE_E_ARG;
        for (int i = 0; i < fv->n_nodes; i++)
            if (fv->offsets[i + 1] < fv->offsets[i] || (i > 0 && fv->node_ids[i] <= fv->node_ids[i - 1]))
                return ORBFE_E_ARG;
    }
    // each keypoint index belongs to one node of its FeatureVector (per-node threads rely on it)
    auto unique_in_range = [](const orbfe_feature_vector* fv, int n) {
        std::vector<uint8_t> seen(n, 0);
        for (int i = 0; i < fv->offsets[fv->n_nodes]; i++) {
            const uint32_t x = fv->indices[i];
            if (x >= (uint32_t)n || seen[x]) return false;
            seen[x] = 1;
        }
        return true;
    };
    if (!unique_in_range(fv1, n1) || !unique_in_range(fv2, n2)) return ORBFE_E_ARG;
    std::vector<int32_t> pairs;
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) { pairs.push_back(a); pairs.push_back(b); a++; b++; }
        else if (fv1->node_ids[a] < fv2->node_ids[b]) a++;
        else b++;
    }
    if (pairs.empty()) return 0;
    const int npairs = (int)pairs.size() / 2;
    const int m1 = fv1->offsets[fv1->n_nodes], m2 = fv2->offsets[fv2->n_nodes];
    Plan p;
    const size_t o_pairs = p.upload(pairs.data(), pairs.size() * 4);
    const size_t o_off1 = p.upload(fv1->offsets, (size_t)(fv1->n_nodes + 1) * 4);
    const size_t o_idx1 = p.upload(fv1->indices, (size_t)m1 * 4);
    const size_t o_off2 = p.upload(fv2->offsets, (size_t)(fv2->n_nodes + 1) * 4);
    const size_t o_idx2 = p.upload(fv2->indices, (size_t)m2 * 4);
    const size_t o_mp1 = p.upload(mp1, (size_t)n1 * 4), o_mp2 = p.upload(mp2, (size_t)n2 * 4);
    const size_t o_d1 = p.upload(desc1, (size_t)n1 * 32), o_d2 = p.upload(desc2, (size_t)n2 * 32);
    const size_t o_k1 = p.upload(keys1, (size_t)n1 * sizeof(orbfe_keypoint));
    const size_t o_k2 = p.upload(keys2, (size_t)n2 * sizeof(orbfe_keypoint));
    const size_t o_m2 = p.scratch((size_t)n2 * 4), o_oi = p.scratch((size_t)n1 * 4);
    const size_t o_out = p.scratch((size_t)n1 * 4), o_res = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    fill(ms_ptr<int>(o_m2), n2, 0);
    fill(ms_ptr<int>(o_oi), n1, -1);
    hipLaunchKernelGGL(k_bow_kfkf, dim3((npairs + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, ms_ptr<const int>(o_pairs),
                       npairs, ms_ptr<const int>(o_off1), ms_ptr<const uint32_t>(o_idx1), ms_ptr<const int>(o_off2),
                       ms_ptr<const uint32_t>(o_idx2), ms_ptr<const int32_t>(o_mp1), ms_ptr<const int32_t>(o_mp2),
                       ms_ptr<const uint32_t>(o_d1), ms_ptr<const uint32_t>(o_d2), nnratio, ms_ptr<int>(o_m2),
                       ms_ptr<int>(o_oi), lim1, lim2);
    hipLaunchKernelGGL(k_bow_kfkf_commit, dim3(1), dim3(1024), 0, s, ms_ptr<const OrbKeyPoint>(o_k1),
                       ms_ptr<const OrbKeyPoint>(o_k2), n1, ms_ptr<const int32_t>(o_mp2), checkOri,
                       ms_ptr<const int>(o_oi), ms_ptr<int>(o_out), ms_ptr<int>(o_res));
    HIPCHK(hipGetLastError());
    timer.end();
    int nm = 0;
    HIPCHK(hipMemcpyAsync(out12, ms_ptr<int>(o_out), (size_t)n1 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ms_ptr<int>(o_res), 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    nm = t_ms.hs[0];
    return nm;
}

int orbfe_distinctive_descriptors(const uint8_t* desc, const int32_t* offsets, int32_t n_points, int32_t* best) {
    if (n_points < 0 || (n_points > 0 && (!offsets || !best))) return ORBFE_E_ARG;
    if (n_points == 0) return 0;
    if (offsets[0] != 0) return ORBFE_E_ARG;
    for (int p = 0; p < n_points; p++)
        if (offsets[p + 1] < offsets[p] || offsets[p + 1] - offsets[p] > DD_MAXN) return ORBFE_E_ARG;
    const int total = offsets[n_points];
    if (total > 0 && !desc) return ORBFE_E_ARG;
    Plan p;
    const size_t o_d = p.upload(desc, (size_t)std::max(total, 1) * 32);
    const size_t o_off = p.upload(offsets, (size_t)(n_points + 1) * 4);
    const size_t o_best = p.scratch((size_t)n_points * 4);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    hipLaunchKernelGGL(k_distinctive, dim3((n_points + 3) / 4), dim3(256), 0, s, ms_ptr<const uint32_t>(o_d),
                       ms_ptr<const int>(o_off), n_points, ms_ptr<int>(o_best));
    HIPCHK(hipGetLastError());
    timer.end();
    HIPCHK(hipMemcpyAsync(best, ms_ptr<int>(o_best), (size_t)n_points * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return n_points;
}

}  // extern "C"

namespace {

KfGeom kf_geom(const orbfe_kf_camera* cam, const orbfe_frame* target, float logsf, int proj, int dist_cam, int view) {
    KfGeom g;
    memset(&g, 0, sizeof(g));
    g.T = cam->Tcw;
    memcpy(g.Ow, cam->Ow, sizeof(g.Ow));
    g.fx = cam->fx; g.fy = cam->fy; g.cx = cam->cx; g.cy = cam->cy;
    g.logsf = logsf;
    g.mbf = target->mbf;
    g.minx = target->min_x; g.maxx = target->max_x; g.miny = target->min_y; g.maxy = target->max_y;
    g.nlevels = target->nlevels;
    g.proj = proj;
    g.dist_cam = dist_cam;
    g.view = view;
    g.skip_flags = ORBFE_MP_BAD | ORBFE_MP_SKIP;
    return g;
}

// keypoint octaves index mvScaleFactors / mvInvLevelSigma2: reject out-of-range ones
bool octaves_ok(const orbfe_frame* F) {
    for (int i = 0; i < F->n; i++)
        if (F->keys[i].octave < 0 || F->keys[i].octave >= F->nlevels) return false;
    return true;
}

bool pose_ok(const orbfe_pose* p) { return p && (p->kind == ORBFE_SE3 || p->kind == ORBFE_SIM3); }

bool fv_ok(const orbfe_feature_vector* fv, int n) {
    if (!fv || fv->n_nodes < 0) return false;
    if (fv->n_nodes == 0) return true;
    if (!fv->node_ids || !fv->offsets || !fv->indices || fv->offsets[0] != 0) return false;
    for (int i = 0; i < fv->n_nodes; i++)
        if (fv->offsets[i + 1] < fv->offsets[i] || (i > 0 && fv->node_ids[i] <= fv->node_ids[i - 1])) return false;
    std::vector<uint8_t> seen(n > 0 ? n : 1, 0);
    for (int i = 0; i < fv->offsets[fv->n_nodes]; i++) {
        const uint32_t x = fv->indices[i];
        if (x >= (uint32_t)n || seen[x]) return false;
        seen[x] = 1;
    }
    return true;
}

}  // namespace

extern "C" {

int orbfe_search_for_triangulation(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                   const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                   const float* F12, const float* ep, const float* level_sigma2_2,
                                   int32_t bOnlyStereo, int32_t bCoarse, int32_t checkOri, int32_t* matches12) {
    // keyframes with a second camera (NLeft != -1): keys = mvKeys ++ mvKeysRight (the reference's kp1 /
    // kp2 selection, ORBmatcher.cc:979-1008); their epipolar test is KannalaBrandt8::TriangulateMatches
    // (an Eigen JacobiSVD), which stays with the camera model on the host: bCoarse only
    if (!frame_ok(KF1) || !frame_ok(KF2) || !F12 || !ep || !level_sigma2_2 || (KF1->n > 0 && (!mp1 || !matches12)) ||
        (KF2->n > 0 && !mp2) || ((KF1->two_cams || KF2->two_cams) && !bCoarse))
        return ORBFE_E_ARG;
    const int n1 = KF1->n, n2 = KF2->n;
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    if (!fv_ok(fv1, n1) || !fv_ok(fv2, n2)) return ORBFE_E_ARG;
    if (n1 == 0 || n2 == 0) return 0;
    if (!octaves_ok(KF2)) return ORBFE_E_ARG;
    std::vector<int2> items;
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            for (int ia = fv1->offsets[a]; ia < fv1->offsets[a + 1]; ia++) items.push_back(make_int2(ia, b));
            a++;
            b++;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) a++;
        else b++;
    }
    if (items.empty()) return 0;
    const int nitems = (int)items.size();
    const int m1 = fv1->offsets[fv1->n_nodes], m2 = fv2->offsets[fv2->n_nodes];
    Plan p;
    const size_t o_items = p.upload(items.data(), items.size() * sizeof(int2));
    const size_t o_idx1 = p.upload(fv1->indices, (size_t)m1 * 4);
    const size_t o_off2 = p.upload(fv2->offsets, (size_t)(fv2->n_nodes + 1) * 4);
    const size_t o_idx2 = p.upload(fv2->indices, (size_t)m2 * 4);
    const size_t o_k1 = p.upload(KF1->keys, (size_t)n1 * sizeof(orbfe_keypoint));
    const size_t o_k2 = p.upload(KF2->keys, (size_t)n2 * sizeof(orbfe_keypoint));
    const size_t o_d1 = p.upload(KF1->desc, (size_t)n1 * 32), o_d2 = p.upload(KF2->desc, (size_t)n2 * 32);
    const bool u1 = KF1->uright && !KF1->two_cams, u2 = KF2->uright && !KF2->two_cams;
    const size_t o_u1 = u1 ? p.upload(KF1->uright, (size_t)n1 * 4) : 0;
    const size_t o_u2 = u2 ? p.upload(KF2->uright, (size_t)n2 * 4) : 0;
    const size_t o_mp1 = p.upload(mp1, (size_t)n1 * 4), o_mp2 = p.upload(mp2, (size_t)n2 * 4);
    const size_t o_sc2 = p.upload(KF2->scale_factors, (size_t)KF2->nlevels * 4);
    const size_t o_sg2 = p.upload(level_sigma2_2, (size_t)KF2->nlevels * 4);
    const size_t o_oi = p.scratch((size_t)n1 * 4), o_out = p.scratch((size_t)n1 * 4), o_res = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    TriArgs ta;
    memcpy(ta.F, F12, sizeof(ta.F));
    ta.ep[0] = ep[0];
    ta.ep[1] = ep[1];
    ta.bOnlyStereo = bOnlyStereo != 0;
    ta.bCoarse = bCoarse != 0;
    ta.two1 = KF1->two_cams != 0;
    ta.two2 = KF2->two_cams != 0;
    fill(ms_ptr<int>(o_oi), n1, -1);
    hipLaunchKernelGGL(k_tri, dim3((nitems + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, ms_ptr<const int2>(o_items), nitems,
                       ms_ptr<const uint32_t>(o_idx1), ms_ptr<const int>(o_off2), ms_ptr<const uint32_t>(o_idx2),
                       ms_ptr<const OrbKeyPoint>(o_k1), ms_ptr<const OrbKeyPoint>(o_k2), ms_ptr<const uint32_t>(o_d1),
                       ms_ptr<const uint32_t>(o_d2), u1 ? ms_ptr<const float>(o_u1) : nullptr,
                       u2 ? ms_ptr<const float>(o_u2) : nullptr, ms_ptr<const int32_t>(o_mp1),
                       ms_ptr<const int32_t>(o_mp2), ms_ptr<const float>(o_sc2), ms_ptr<const float>(o_sg2), ta,
                       ms_ptr<int>(o_oi));
    hipLaunchKernelGGL(k_bow_kfkf_commit, dim3(1), dim3(1024), 0, s, ms_ptr<const OrbKeyPoint>(o_k1),
                       ms_ptr<const OrbKeyPoint>(o_k2), n1, (const int32_t*)nullptr, checkOri, ms_ptr<const int>(o_oi),
                       ms_ptr<int>(o_out), ms_ptr<int>(o_res));
    HIPCHK(hipGetLastError());
    timer.end();
    int nm = 0;
    HIPCHK(hipMemcpyAsync(matches12, ms_ptr<int>(o_out), (size_t)n1 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ms_ptr<int>(o_res), 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    nm = t_ms.hs[0];
    return nm;
}

static constexpr size_t kTriEpiMaxSlots = (size_t)1 << 24;

int orbfe_search_for_triangulation_epi(const orbfe_frame* KF1, const int32_t* mp1, const orbfe_feature_vector* fv1,
                                       const orbfe_frame* KF2, const int32_t* mp2, const orbfe_feature_vector* fv2,
                                       const float* ep, int32_t bOnlyStereo, int32_t checkOri,
                                       orbfe_epipolar_fn epipolar, void* ctx, int32_t* matches12) {
    if (!frame_ok(KF1) || !frame_ok(KF2) || !ep || !epipolar || (KF1->n > 0 && (!mp1 || !matches12)) ||
        (KF2->n > 0 && !mp2))
        return ORBFE_E_ARG;
    const int n1 = KF1->n, n2 = KF2->n;
    for (int i = 0; i < n1; i++) matches12[i] = -1;
    if (!fv_ok(fv1, n1) || !fv_ok(fv2, n2)) return ORBFE_E_ARG;
    if (n1 == 0 || n2 == 0) return 0;
    if (!octaves_ok(KF1) || !octaves_ok(KF2)) return ORBFE_E_ARG;
    // one item per KF1 entry of a shared node (:961-966), its candidate segment sized by the KF2 node
    std::vector<int2> items;
    std::vector<int> seg;
    size_t total = 0;
    int a = 0, b = 0;
    while (a < fv1->n_nodes && b < fv2->n_nodes) {
        if (fv1->node_ids[a] == fv2->node_ids[b]) {
            const int nb = fv2->offsets[b + 1] - fv2->offsets[b];
            if (nb >= (1 << 20)) return ORBFE_E_CAPACITY;   // k_tri_cand packs the node position in 20 bits
            for (int ia = fv1->offsets[a]; ia < fv1->offsets[a + 1]; ia++) {
                items.push_back(make_int2(ia, b));
                seg.push_back((int)total);
                total += (size_t)nb;
            }
            a++;
            b++;
        } else if (fv1->node_ids[a] < fv2->node_ids[b]) a++;
        else b++;
    }
    if (items.empty()) return 0;
    // candidate slots = sum over items of the KF2 node size: a pair of keyframes with very coarse
    // vocabulary nodes would need a large scratch (and k_tri_cand's per-item insertion is O(nb^2));
    // beyond 16 M slots (64 MB) the call reports capacity and the caller keeps its CPU body
    if (total > kTriEpiMaxSlots) return ORBFE_E_CAPACITY;
    const int nitems = (int)items.size();
    const int m1 = fv1->offsets[fv1->n_nodes], m2 = fv2->offsets[fv2->n_nodes];
    Plan p;
    const size_t o_items = p.upload(items.data(), items.size() * sizeof(int2));
    const size_t o_seg = p.upload(seg.data(), seg.size() * 4);
    const size_t o_idx1 = p.upload(fv1->indices, (size_t)m1 * 4);
    const size_t o_off2 = p.upload(fv2->offsets, (size_t)(fv2->n_nodes + 1) * 4);
    const size_t o_idx2 = p.upload(fv2->indices, (size_t)m2 * 4);
    const size_t o_k2 = p.upload(KF2->keys, (size_t)n2 * sizeof(orbfe_keypoint));
    const size_t o_d1 = p.upload(KF1->desc, (size_t)n1 * 32), o_d2 = p.upload(KF2->desc, (size_t)n2 * 32);
    const bool u1 = KF1->uright && !KF1->two_cams, u2 = KF2->uright && !KF2->two_cams;
    const size_t o_u1 = u1 ? p.upload(KF1->uright, (size_t)n1 * 4) : 0;
    const size_t o_u2 = u2 ? p.upload(KF2->uright, (size_t)n2 * 4) : 0;
    const size_t o_mp1 = p.upload(mp1, (size_t)n1 * 4), o_mp2 = p.upload(mp2, (size_t)n2 * 4);
    const size_t o_sc2 = p.upload(KF2->scale_factors, (size_t)KF2->nlevels * 4);
    const size_t o_cnt = p.scratch((size_t)nitems * 4), o_cand = p.scratch(std::max<size_t>(total, 1) * 4);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    TriArgs ta;
    memset(&ta, 0, sizeof(ta));
    ta.ep[0] = ep[0];
    ta.ep[1] = ep[1];
    ta.bOnlyStereo = bOnlyStereo != 0;
    ta.two1 = KF1->two_cams != 0;
    ta.two2 = KF2->two_cams != 0;
    hipLaunchKernelGGL(k_tri_cand, dim3((nitems + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, ms_ptr<const int2>(o_items),
                       nitems, ms_ptr<const int>(o_seg), ms_ptr<const uint32_t>(o_idx1), ms_ptr<const int>(o_off2),
                       ms_ptr<const uint32_t>(o_idx2), ms_ptr<const OrbKeyPoint>(o_k2), ms_ptr<const uint32_t>(o_d1),
                       ms_ptr<const uint32_t>(o_d2), u1 ? ms_ptr<const float>(o_u1) : nullptr,
                       u2 ? ms_ptr<const float>(o_u2) : nullptr, ms_ptr<const int32_t>(o_mp1),
                       ms_ptr<const int32_t>(o_mp2), ms_ptr<const float>(o_sc2), ta, ms_ptr<int>(o_cnt),
                       ms_ptr<uint32_t>(o_cand));
    HIPCHK(hipGetLastError());
    timer.end();
    std::vector<int> cnt(nitems);
    std::vector<uint32_t> cand(std::max<size_t>(total, 1));
    HIPCHK(hipMemcpyAsync(cnt.data(), ms_ptr<int>(o_cnt), (size_t)nitems * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cand.data(), ms_ptr<uint32_t>(o_cand), total * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    // the caller's test in the candidates' order; the first pass is the reference's bestIdx2
    int nmatches = 0;
    int hist[MT_HISTO] = {0};
    for (int t = 0; t < nitems; t++) {
        const int i1 = (int)fv1->indices[items[t].x];
        for (int j = 0; j < cnt[t]; j++) {
            const int i2 = (int)cand[(size_t)seg[t] + j];
            if (epipolar(ctx, i1, i2)) {
                matches12[i1] = i2;
                nmatches++;
                if (checkOri) hist[mt_rot_bin(KF1->keys[i1].angle, KF2->keys[i2].angle)]++;
                break;
            }
        }
    }
    // the rotation-histogram filter (:1114-1131): entries outside the three maxima are dropped
    if (checkOri && nmatches > 0) {
        const unsigned keep = mt_three_maxima_keep(hist);
        for (int i = 0; i < n1; i++) {
            const int i2 = matches12[i];
            if (i2 >= 0 && !((keep >> mt_rot_bin(KF1->keys[i].angle, KF2->keys[i2].angle)) & 1u)) {
                matches12[i] = -1;
                nmatches--;
            }
        }
    }
    return nmatches;
}

int orbfe_fuse(const orbfe_frame* KF, const orbfe_kf_camera* cam, const float* inv_level_sigma2,
               const orbfe_map_point_3d* pts, int32_t n, float th, int32_t sim3, int32_t* best_idx,
               int32_t* best_dist) {
    if (KF && KF->two_cams) return ORBFE_E_ARG;   // the pinhole API: no camera model / side
    return orbfe_fuse_rig(KF, cam, nullptr, inv_level_sigma2, pts, n, th, sim3, 0, best_idx, best_dist);
}

int orbfe_fuse_rig(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_camera_model* model,
                   const float* inv_level_sigma2, const orbfe_map_point_3d* pts, int32_t n, float th, int32_t sim3,
                   int32_t bRight, int32_t* best_idx, int32_t* best_dist) {
    if (!frame_ok(KF) || !cam || !pose_ok(&cam->Tcw) || n < 0 || (n > 0 && (!pts || !best_idx || !best_dist)) ||
        (!sim3 && !inv_level_sigma2) || (bRight && (sim3 || !KF->two_cams)) ||
        (model && model->type != ORBFE_CAM_PINHOLE && model->type != ORBFE_CAM_KANNALA_BRANDT8))
        return ORBFE_E_ARG;
    for (int i = 0; i < n; i++) best_idx[i] = best_dist[i] = -1;
    if (n == 0 || KF->n == 0) return 0;
    if (!octaves_ok(KF)) return ORBFE_E_ARG;
    Plan p;
    FramePlan fp;
    fp.plan(p, KF, true, !sim3);
    const size_t o_pts = p.upload(pts, (size_t)n * sizeof(orbfe_map_point_3d));
    const size_t o_sig = sim3 ? 0 : p.upload(inv_level_sigma2, (size_t)KF->nlevels * 4);
    fp.plan_grid(p, KF->nlevels + 1);
    const size_t o_pj = p.scratch((size_t)n * sizeof(KfProj));
    const size_t o_as = p.scratch((size_t)n * 4), o_ds = p.scratch((size_t)n * 4), o_cnt = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    const FrameDev fr = fp.view();
    fp.launch_grid(fr);
    KfGeom g = kf_geom(cam, KF, cam->log_scale_factor, BE_PRJ_PINHOLE, 0, 1);
    if (model) {   // pCamera->project: mpCamera, or mpCamera2 with bRight (ORBmatcher.cc:1154-1163)
        g.proj = BE_PRJ_MODEL;
        g.cam_type = model->type;
        g.fx = model->params[0]; g.fy = model->params[1]; g.cx = model->params[2]; g.cy = model->params[3];
        for (int k = 0; k < 4; k++) g.kb[k] = model->type == ORBFE_CAM_KANNALA_BRANDT8 ? model->params[4 + k] : 0.f;
    }
    const dim3 gq((n + MT_NT - 1) / MT_NT);
    hipLaunchKernelGGL(k_kf_geom, gq, dim3(MT_NT), 0, s, g, ms_ptr<const orbfe_map_point_3d>(o_pts), n,
                       (const uint8_t*)nullptr, ms_ptr<KfProj>(o_pj));
    fill(ms_ptr<int>(o_as), n, -1);
    hipLaunchKernelGGL(k_kf_search, gq, dim3(MT_NT), 0, s, fr, ms_ptr<const KfProj>(o_pj),
                       ms_ptr<const orbfe_map_point_3d>(o_pts), n, th, sim3 ? 0 : 1,
                       sim3 ? (const float*)nullptr : ms_ptr<const float>(o_sig), sim3 ? INT_MAX : 256,
                       (float)MT_TH_LOW, (const int*)nullptr, (const int*)nullptr, ms_ptr<int>(o_as), ms_ptr<int>(o_ds),
                       (int*)nullptr, bRight ? MT_NCELL : 0);
    HIPCHK(hipMemsetAsync(ms_ptr<int>(o_cnt), 0, 4, s));
    hipLaunchKernelGGL(k_count_ge0, gq, dim3(MT_NT), 0, s, ms_ptr<const int>(o_as), n, ms_ptr<int>(o_cnt));
    HIPCHK(hipGetLastError());
    timer.end();
    int nf = 0;
    HIPCHK(hipMemcpyAsync(best_idx, ms_ptr<int>(o_as), (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(best_dist, ms_ptr<int>(o_ds), (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ms_ptr<int>(o_cnt), 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    nf = t_ms.hs[0];
    return nf;
}

int orbfe_search_by_projection_sim3(const orbfe_frame* KF, const orbfe_kf_camera* cam, const orbfe_map_point_3d* pts,
                                    int32_t n, const int32_t* point_kfs, int32_t th, float ratioHamming,
                                    int32_t* matched, int32_t* matched_kf) {
    // the pinhole API: the first overload on a two-camera keyframe needs its camera model
    if (KF && KF->two_cams && !point_kfs) return ORBFE_E_ARG;
    return orbfe_search_by_projection_sim3_rig(KF, cam, nullptr, pts, n, point_kfs, th, ratioHamming, matched,
                                               matched_kf);
}

int orbfe_search_by_projection_sim3_rig(const orbfe_frame* KF, const orbfe_kf_camera* cam,
                                        const orbfe_camera_model* model, const orbfe_map_point_3d* pts, int32_t n,
                                        const int32_t* point_kfs, int32_t th, float ratioHamming, int32_t* matched,
                                        int32_t* matched_kf) {
    if (!frame_ok(KF) || !cam || !pose_ok(&cam->Tcw) || n < 0 || (n > 0 && !pts) || (KF->n > 0 && !matched) ||
        (point_kfs && KF->n > 0 && !matched_kf) ||
        (model && model->type != ORBFE_CAM_PINHOLE && model->type != ORBFE_CAM_KANNALA_BRANDT8))
        return ORBFE_E_ARG;
    if (n == 0 || KF->n == 0) return 0;
    if (n > (1 << 24)) return ORBFE_E_CAPACITY;
    if (!octaves_ok(KF)) return ORBFE_E_ARG;
    const int nk = KF->n;
    // spAlreadyFound: the handles already in vpMatched
    std::vector<int32_t> found;
    for (int k = 0; k < nk; k++)
        if (matched[k] >= 0) found.push_back(matched[k]);
    std::sort(found.begin(), found.end());
    std::vector<uint8_t> skip(n);
    for (int i = 0; i < n; i++) skip[i] = std::binary_search(found.begin(), found.end(), pts[i].id) ? 1 : 0;
    std::vector<int32_t> blocked0(nk);
    for (int k = 0; k < nk; k++) blocked0[k] = matched[k] >= 0;
    Plan p;
    FramePlan fp;
    fp.plan(p, KF, true, false);
    const size_t o_pts = p.upload(pts, (size_t)n * sizeof(orbfe_map_point_3d));
    const size_t o_skip = p.upload(skip.data(), (size_t)n);
    const size_t o_b0 = p.upload(blocked0.data(), (size_t)nk * 4);
    const size_t o_m = p.upload(matched, (size_t)nk * 4);
    const size_t o_mk = point_kfs ? p.upload(matched_kf, (size_t)nk * 4) : 0;
    const size_t o_pk = point_kfs ? p.upload(point_kfs, (size_t)n * 4) : 0;
    fp.plan_grid(p, KF->nlevels + 1);
    const size_t o_pj = p.scratch((size_t)n * sizeof(KfProj));
    const size_t o_as = p.scratch((size_t)n * 4), o_first = p.scratch((size_t)nk * 4);
    const size_t o_changed = p.scratch(MT_MAX_PASSES * 4), o_cnt = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    const FrameDev fr = fp.view();
    fp.launch_grid(fr);
    KfGeom g = kf_geom(cam, KF, cam->log_scale_factor, point_kfs ? BE_PRJ_INVZ_F : BE_PRJ_PINHOLE, 0, 1);
    if (model && !point_kfs) {   // pKF->mpCamera->project (ORBmatcher.cc:465)
        g.proj = BE_PRJ_MODEL;
        g.cam_type = model->type;
        g.fx = model->params[0]; g.fy = model->params[1]; g.cx = model->params[2]; g.cy = model->params[3];
        for (int k = 0; k < 4; k++) g.kb[k] = model->type == ORBFE_CAM_KANNALA_BRANDT8 ? model->params[4 + k] : 0.f;
    }
    g.skip_flags = ORBFE_MP_BAD;   // spAlreadyFound is the skip array
    const dim3 gq((n + MT_NT - 1) / MT_NT);
    hipLaunchKernelGGL(k_kf_geom, gq, dim3(MT_NT), 0, s, g, ms_ptr<const orbfe_map_point_3d>(o_pts), n,
                       ms_ptr<const uint8_t>(o_skip), ms_ptr<KfProj>(o_pj));
    int* assign = ms_ptr<int>(o_as);
    int* first = ms_ptr<int>(o_first);
    int* changed = ms_ptr<int>(o_changed);
    HIPCHK(hipMemsetAsync(changed, 0, MT_MAX_PASSES * 4, s));
    fill(assign, n, -1);
    const float max_acc = MT_TH_LOW * ratioHamming;
    int pass = 0;
    while (true) {
        for (int c = 0; c < 2; c++, pass++) {
            if (pass >= MT_MAX_PASSES) return ORBFE_E_CAPACITY;
            fill(first, nk, MT_INF);
            hipLaunchKernelGGL(k_mt_first_strided, gq, dim3(MT_NT), 0, s, assign, (const uint8_t*)assign, 4, n, 0,
                               first, 1);
            hipLaunchKernelGGL(k_kf_search, gq, dim3(MT_NT), 0, s, fr, ms_ptr<const KfProj>(o_pj),
                               ms_ptr<const orbfe_map_point_3d>(o_pts), n, (float)th, 0, (const float*)nullptr, 256,
                               max_acc, ms_ptr<const int>(o_b0), first, assign, (int*)nullptr, changed + pass);
        }
        int ch = 0;
        HIPCHK(hipMemcpyAsync(t_ms.hs, changed + pass - 1, 4, hipMemcpyDeviceToHost, s));   // pinned
        HIPCHK(hipStreamSynchronize(s));
        ch = t_ms.hs[0];
        if (ch == 0) break;
    }
    HIPCHK(hipMemsetAsync(ms_ptr<int>(o_cnt), 0, 4, s));
    hipLaunchKernelGGL(k_kf_commit, gq, dim3(MT_NT), 0, s, assign, n, ms_ptr<const orbfe_map_point_3d>(o_pts),
                       point_kfs ? ms_ptr<const int32_t>(o_pk) : nullptr, ms_ptr<int32_t>(o_m),
                       point_kfs ? ms_ptr<int32_t>(o_mk) : nullptr, ms_ptr<int>(o_cnt));
    HIPCHK(hipGetLastError());
    timer.end();
    int nm = 0;
    HIPCHK(hipMemcpyAsync(matched, ms_ptr<int32_t>(o_m), (size_t)nk * 4, hipMemcpyDeviceToHost, s));
    if (point_kfs) HIPCHK(hipMemcpyAsync(matched_kf, ms_ptr<int32_t>(o_mk), (size_t)nk * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ms_ptr<int>(o_cnt), 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    nm = t_ms.hs[0];
    return nm;
}

int orbfe_search_by_sim3(const orbfe_frame* KF1, const orbfe_frame* KF2, const orbfe_map_point_3d* pts1,
                         const orbfe_map_point_3d* pts2, const orbfe_kf_camera* cam1, const orbfe_kf_camera* cam2,
                         const orbfe_pose* S12, const orbfe_pose* S21, float th, int32_t* matches12,
                         const int32_t* matched_idx2) {
    // two-camera keyframes are searched on their left grids (mvKeys), every camera with the pinhole
    // expression on pKF1's intrinsics as the reference does (ORBmatcher.cc:1514-1519,1594-1599)
    if (!frame_ok(KF1) || !frame_ok(KF2) || !cam1 || !cam2 || !pose_ok(&cam1->Tcw) || !pose_ok(&cam2->Tcw) ||
        !pose_ok(S12) || !pose_ok(S21) || (KF1->n > 0 && (!pts1 || !matches12)) || (KF2->n > 0 && !pts2))
        return ORBFE_E_ARG;
    const int n1 = KF1->n, n2 = KF2->n;
    if (n1 == 0) return 0;
    std::vector<uint8_t> already1(n1, 0), already2(std::max(n2, 1), 0);
    for (int i = 0; i < n1; i++)
        if (matches12[i] >= 0) {
            already1[i] = 1;
            const int idx2 = matched_idx2 ? matched_idx2[i] : -1;
            if (idx2 >= 0 && idx2 < n2) already2[idx2] = 1;
        }
    if (n2 == 0) return 0;
    if (!octaves_ok(KF1) || !octaves_ok(KF2)) return ORBFE_E_ARG;
    Plan p;
    FramePlan f1, f2;
    f1.plan(p, KF1, true, false);
    f2.plan(p, KF2, true, false);
    const size_t o_p1 = p.upload(pts1, (size_t)n1 * sizeof(orbfe_map_point_3d));
    const size_t o_p2 = p.upload(pts2, (size_t)n2 * sizeof(orbfe_map_point_3d));
    const size_t o_a1 = p.upload(already1.data(), (size_t)n1), o_a2 = p.upload(already2.data(), (size_t)n2);
    const size_t o_m12 = p.upload(matches12, (size_t)n1 * 4);
    f1.plan_grid(p, KF1->nlevels + 1);
    f2.plan_grid(p, KF2->nlevels + 1);
    const size_t o_pj1 = p.scratch((size_t)n1 * sizeof(KfProj)), o_pj2 = p.scratch((size_t)n2 * sizeof(KfProj));
    const size_t o_v1 = p.scratch((size_t)n1 * 4), o_v2 = p.scratch((size_t)n2 * 4), o_cnt = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    const FrameDev v1 = f1.view(), v2 = f2.view();
    f1.launch_grid(v1);
    f2.launch_grid(v2);
    // KF1 points -> KF2 (T1w, then S21), searched in KF2; and KF2 points -> KF1 (T2w, S12). Both use
    // pKF1's intrinsics, each target's IsInImage / scale pyramid.
    KfGeom g1 = kf_geom(cam1, KF2, cam2->log_scale_factor, BE_PRJ_INVZ_D, 1, 0);
    g1.S = *S21;
    g1.two = 1;
    g1.skip_flags = ORBFE_MP_BAD;
    KfGeom g2 = kf_geom(cam1, KF1, cam1->log_scale_factor, BE_PRJ_INVZ_D, 1, 0);
    g2.T = cam2->Tcw;
    g2.S = *S12;
    g2.two = 1;
    g2.skip_flags = ORBFE_MP_BAD;
    const dim3 gq1((n1 + MT_NT - 1) / MT_NT), gq2((n2 + MT_NT - 1) / MT_NT);
    hipLaunchKernelGGL(k_kf_geom, gq1, dim3(MT_NT), 0, s, g1, ms_ptr<const orbfe_map_point_3d>(o_p1), n1,
                       ms_ptr<const uint8_t>(o_a1), ms_ptr<KfProj>(o_pj1));
    hipLaunchKernelGGL(k_kf_geom, gq2, dim3(MT_NT), 0, s, g2, ms_ptr<const orbfe_map_point_3d>(o_p2), n2,
                       ms_ptr<const uint8_t>(o_a2), ms_ptr<KfProj>(o_pj2));
    fill(ms_ptr<int>(o_v1), n1, -1);
    fill(ms_ptr<int>(o_v2), n2, -1);
    hipLaunchKernelGGL(k_kf_search, gq1, dim3(MT_NT), 0, s, v2, ms_ptr<const KfProj>(o_pj1),
                       ms_ptr<const orbfe_map_point_3d>(o_p1), n1, th, 0, (const float*)nullptr, INT_MAX,
                       (float)MT_TH_HIGH, (const int*)nullptr, (const int*)nullptr, ms_ptr<int>(o_v1), (int*)nullptr,
                       (int*)nullptr);
    hipLaunchKernelGGL(k_kf_search, gq2, dim3(MT_NT), 0, s, v1, ms_ptr<const KfProj>(o_pj2),
                       ms_ptr<const orbfe_map_point_3d>(o_p2), n2, th, 0, (const float*)nullptr, INT_MAX,
                       (float)MT_TH_HIGH, (const int*)nullptr, (const int*)nullptr, ms_ptr<int>(o_v2), (int*)nullptr,
                       (int*)nullptr);
    HIPCHK(hipMemsetAsync(ms_ptr<int>(o_cnt), 0, 4, s));
    hipLaunchKernelGGL(k_sim3_agree, gq1, dim3(MT_NT), 0, s, ms_ptr<const int>(o_v1), n1, ms_ptr<const int>(o_v2),
                       ms_ptr<const orbfe_map_point_3d>(o_p2), ms_ptr<int32_t>(o_m12), ms_ptr<int>(o_cnt));
    HIPCHK(hipGetLastError());
    timer.end();
    int nf = 0;
    HIPCHK(hipMemcpyAsync(matches12, ms_ptr<int32_t>(o_m12), (size_t)n1 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ms_ptr<int>(o_cnt), 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    nf = t_ms.hs[0];
    return nf;
}

}  // extern "C"
