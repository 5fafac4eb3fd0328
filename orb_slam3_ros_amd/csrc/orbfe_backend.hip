// Back-end ORBmatcher pieces on CDNA4; included into orbfe_engine.hip after the
// matcher (per-thread arena / stream helpers, rotation histogram helpers).
//  * SearchByBoW(KF1, KF2) (ORBmatcher.cc:765-903): like SearchByBoW(KF, F) one thread walks one
//    shared vocabulary node; vbMatched2 is node-local because a KF2 index lives in one node.
//  * MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:329-403): one wave per map point, the
//    point's descriptors staged in LDS, every row's median found by a wave-wide counting search.
#pragma once

__global__ __launch_bounds__(MT_NT) void k_bow_kfkf(const int* pairs, int npairs, const int* off1, const uint32_t* idx1s,
                                                    const int* off2, const uint32_t* idx2s, const int32_t* mp1,
                                                    const int32_t* mp2, const uint32_t* d1, const uint32_t* d2,
                                                    float nnratio, int* matched2, int* out_idx) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npairs) return;
    const int a = pairs[2 * t], b = pairs[2 * t + 1];
    for (int ia = off1[a]; ia < off1[a + 1]; ia++) {
        const unsigned i1 = idx1s[ia];
        if (mp1[i1] < 0) continue;
        uint32_t q[8];
#pragma unroll
        for (int w = 0; w < 8; w++) q[w] = d1[8 * i1 + w];
        int bestDist1 = 256, bestIdx2 = -1, bestDist2 = 256;
        for (int ib = off2[b]; ib < off2[b + 1]; ib++) {
            const unsigned i2 = idx2s[ib];
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
        if (j >= 0 && (!checkOri || ((s_keep >> mt_rot_bin(k1[i].angle, k2[j].angle)) & 1u))) o = mp2[j];
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

extern "C" {

int orbfe_search_by_bow_kf(const orbfe_keypoint* keys1, const uint8_t* desc1, const int32_t* mp1, int32_t n1,
                           const orbfe_feature_vector* fv1, const orbfe_keypoint* keys2, const uint8_t* desc2,
                           const int32_t* mp2, int32_t n2, const orbfe_feature_vector* fv2, int32_t* out12,
                           float nnratio, int32_t checkOri) {
    if (n1 < 0 || n2 < 0 || !fv1 || !fv2 || (n1 > 0 && (!keys1 || !desc1 || !mp1 || !out12)) ||
        (n2 > 0 && (!keys2 || !desc2 || !mp2)))
        return ORBFE_E_ARG;
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
                       ms_ptr<int>(o_oi));
    hipLaunchKernelGGL(k_bow_kfkf_commit, dim3(1), dim3(1024), 0, s, ms_ptr<const OrbKeyPoint>(o_k1),
                       ms_ptr<const OrbKeyPoint>(o_k2), n1, ms_ptr<const int32_t>(o_mp2), checkOri,
                       ms_ptr<const int>(o_oi), ms_ptr<int>(o_out), ms_ptr<int>(o_res));
    HIPCHK(hipGetLastError());
    timer.end();
    int nm = 0;
    HIPCHK(hipMemcpyAsync(out12, ms_ptr<int>(o_out), (size_t)n1 * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(&nm, ms_ptr<int>(o_res), 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
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
