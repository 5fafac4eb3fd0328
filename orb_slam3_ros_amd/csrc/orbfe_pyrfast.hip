// Fused pyramid + FAST pass for CDNA4 (gfx950), one launch per pyramid level (included into the
// engine's translation unit after orbfe_kernels.hip).
//
// Level l's launch runs ComputeKeyPointsOctTree's cell loop with cv::FAST 9/16 + NMS on every cell
// of level l (ORBextractor.cc:781-872) AND produces level l+1 (ComputePyramid's cv::resize
// INTER_LINEAR from level l, :1170-1195) from the same staged rows, so every level is read from
// HBM once and written once (the algorithmic bytes of SURVEY.md §8(d)).
//
// Work unit: ONE WAVE per (image, band, slice), fully independent (no workgroup barrier). A band is
// one row of FAST cells; a slice is a run of whole cells whose detection columns fit the wave's
// 64 lanes x 4 columns (lane L holds columns A0 + 4 L .. + 3 of every row; lanes 0 and 63 are
// halo), so NMS neighbourhoods, per-cell emission and the fallback never leave the wave. The wave
// also owns the output columns of level l+1 whose source columns start in its slice. It streams the
// band's source rows top to bottom in blocks of 7:
//   A  one dword load per lane and row (two blocks ahead), written to the wave's LDS image ring; a
//      7-row (left, centre, right)-dword window in registers (DPP neighbours) feeds FAST's exact
//      necessary test (every 9-arc holds one pixel of each opposite ring pair (k, k+8), k = 0, 2, 4,
//      6) at iniThFAST for 4 pixels per lane; 4-pixel groups with a candidate are queued;
//   B  exact scores (M - 1, corner iff M > th, packed f16) of each queued group, one group per lane,
//      into the LDS score ring; the groups holding corners are compacted; the H / V passes of
//      cv::resize for the output rows of level l+1 whose source rows are complete;
//   C  NMS of the corners whose neighbour rows are scored, with the reference's per-cell detection
//      rectangles (neighbours outside the corner's cell count as 0), into a survivor bitmap;
//   D  per (cell, row) emission of the survivors in FAST's row-major order into the cell's key
//      slots (x - minBorder | (y - minBorder) << 12 | score << 24), the layout k_octree reads.
// A cell without any survivor at iniThFAST is re-run at minThFAST after the band with the per-cell
// detector of k_fast (attempt 1 only): the reference's fallback (ORBextractor.cc:826-846).
//
// The host (build_bands) enables this path per handle only when every level's cell detection
// rectangles tile the level (no clipped interior cell) and the slices / bands fit the layout;
// otherwise the legacy k_resize + k_fast pair runs.
#pragma once

namespace orbfe {

#define PF_RING 16      // image / score / bitmap ring rows
#define PF_MIRROR 6     // image ring rows 0..5 mirrored after row 15: 7 consecutive rows are contiguous
#define PF_RS 256       // ring row bytes (64 lanes x 4 columns)
#define PF_BW 8         // survivor bitmap words per ring row
#define PF_QCAP 512     // queued group records: <= 62 carried + 7 x 62 new
#define PF_TYCAP 128    // owned output rows of the next level per band
#define PF_MAXC 8       // cells per slice
#ifndef PF_ABL
#define PF_ABL 0        // timing-only ablation builds (tools/build_variant.sh -DPF_ABL=bits); outputs invalid
#endif
#define PF_LDS_BYTES ((PF_RING + PF_MIRROR + PF_RING) * PF_RS + PF_RING * PF_BW * 4 + PF_TYCAP * 16 + PF_QCAP * 4 + PF_MAXC * 4 + 1024)

#ifdef PF_STATS
__device__ unsigned long long g_pf_stats[8 * 8];   // per level: groups, entry pairs, corners, blocks, chunks, -, fallback cells, units
#define PF_STAT(i, v) atomicAdd(&g_pf_stats[8 * l + (i)], (unsigned long long)(v))
#else
#define PF_STAT(i, v) do { } while (0)
#endif

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {   // lane i <- lane i - 1 (wave_shr:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t v) {   // lane i <- lane i + 1 (wave_shl:1)
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xf, 0xf, false);
}
// bytes o and o + 2 of {hi:lo} as an f16x2 of denormals byte * 2^-24
__device__ __forceinline__ orbfe_half2 pf_pair(uint32_t hi, uint32_t lo, uint32_t o) {
    return as_h2(__builtin_amdgcn_perm(hi, lo, 0x0c000c00u | o | ((o + 2u) << 16)));
}

// FAST's exact necessary test for the 4 pixels of a lane (byte k of the centre dword), from the
// (left, centre, right) dwords of rows y - 3, y - 2, y, y + 2, y + 3. Returns 8 flag bits: pixel k
// bit 2k + 1 = dark possible, 2k = bright possible (same encoding as k_fast's pass 1).
__device__ __forceinline__ uint32_t pf_pretest(uint32_t cM3, uint32_t lM2, uint32_t cM2, uint32_t rM2, uint32_t lY,
                                               uint32_t cY, uint32_t rY, uint32_t lP2, uint32_t cP2, uint32_t rP2,
                                               uint32_t cP3, orbfe_half2 tv) {
    uint32_t sd[2], sb[2];
#pragma unroll
    for (int par = 0; par < 2; par++) {
        const uint32_t p = (uint32_t)par;
        const orbfe_half2 v = pf_pair(cY, cY, p);
        // ring (k, k + 8) pairs: (0,3)/(0,-3), (2,2)/(-2,-2), (3,0)/(-3,0), (2,-2)/(-2,2) (dx, dy)
        const orbfe_half2 a0 = pf_pair(cP3, cP3, p), b0 = pf_pair(cM3, cM3, p);
        const orbfe_half2 a1 = pf_pair(rP2, cP2, 2 + p), b1 = pf_pair(cM2, lM2, 2 + p);
        const orbfe_half2 a2 = pf_pair(rY, cY, 3 + p), b2 = pf_pair(cY, lY, 1 + p);
        const orbfe_half2 a3 = pf_pair(rM2, cM2, 2 + p), b3 = pf_pair(cP2, lP2, 2 + p);
        const orbfe_half2 D = hmax(hmax(hmax(hmin(a0, b0), hmin(a1, b1)), hmin(a2, b2)), hmin(a3, b3));
        const orbfe_half2 B = hmin(hmin(hmin(hmax(a0, b0), hmax(a1, b1)), hmax(a2, b2)), hmax(a3, b3));
        sd[par] = h2_bits(D - (v - tv));   // sign bit set <=> dark possible
        sb[par] = h2_bits((v + tv) - B);   // sign bit set <=> bright possible
    }
    const uint32_t A = __builtin_amdgcn_perm(sd[1], sd[0], 0x07030501u);
    const uint32_t Bq = __builtin_amdgcn_perm(sb[1], sb[0], 0x07030501u);
    const uint32_t F = (A & 0x80808080u) | ((Bq >> 1) & 0x40404040u);
    return __builtin_amdgcn_udot4(F >> 6, 0x40100401u, 0u, false);
}

// Exact FAST score of two ring-pixel sets (entries e0 / e1 as sign + centre addresses) in packed
// f16: returns M for each (negative -> no corner), the k_fast pass-2 arithmetic.
__device__ __forceinline__ void pf_exact2(const uint8_t* q0, const uint8_t* q1, bool bright0, bool bright1, int RS,
                                          int* M0, int* M1) {
    const orbfe_half2 v2 = as_h2(__builtin_bit_cast(uint32_t, orbfe_ushort2{q0[0], q1[0]}));
    const uint32_t bmask = (bright0 ? 0x00008000u : 0u) | (bright1 ? 0x80000000u : 0u);
    const orbfe_half2 ns = as_h2(0xBC00BC00u ^ bmask);   // -s
    const orbfe_half2 sv = as_h2(h2_bits(v2) ^ bmask);   // s v
    const uint8_t* t0 = q0 - 3 * RS - 3;
    const uint8_t* t1 = q1 - 3 * RS - 3;
    orbfe_half2 P[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int o = (kRingDy[k] + 3) * RS + kRingDx[k] + 3;
        const orbfe_half2 x2 = as_h2(__builtin_bit_cast(uint32_t, orbfe_ushort2{t0[o], t1[o]}));
        P[k] = __builtin_elementwise_fma(x2, ns, sv);
    }
    orbfe_half2 m2[16], m4[16], m9[16];
#pragma unroll
    for (int k = 0; k < 16; k++) m2[k] = hmin(P[k], P[(k + 1) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) m4[k] = hmin(m2[k], m2[(k + 2) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) m9[k] = hmin(hmin(m4[k], m4[(k + 4) & 15]), P[(k + 8) & 15]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int k = 0; k < w; k++) m9[k] = hmax(m9[k], m9[k + w]);
    const uint32_t mb = h2_bits(m9[0]);
    *M0 = (mb & 0x8000u) ? -1 : (int)(mb & 0x7fffu);
    *M1 = (mb & 0x80000000u) ? -1 : (int)((mb >> 16) & 0x7fffu);
}

__global__ __launch_bounds__(64) void k_pyrfast(const uint8_t* const* imgs, int in_pitch, uint8_t* pyr,
                                                int pyr_stride, const int16_t* __restrict__ tab, OrbGeom g, int l,
                                                uint32_t* cellkeys, int* cellcnt, int* fb_list) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_pf[];
    const OrbLevel& L = g.lv[l];
    const int lane = threadIdx.x;
    const int nsl = L.pf_ns;
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int unit = lb % gridDim.x, b = lb / gridDim.x;
    const int band = small_div(unit, nsl), slice = unit - band * nsl;
    int spitch;
    const gptr_u8 src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l, &spitch);
    const int16_t* bt = tab + L.pf_band_tab + 4 * band;
    const int ry0 = bt[0], ry1 = bt[1], e_lo = bt[2], e_hi = bt[3];
    const int16_t* st = tab + L.pf_slice_tab + 4 * slice;
    const int A0 = st[0], j0 = st[1] & 255, j1 = st[1] >> 8, g0 = st[2], g1 = st[3];
    const int nrel = ry1 - ry0;
    const int ncols = L.n_cols, wc = L.w_cell;
    const int iniY = ORBFE_MINB + band * L.h_cell;
    const int roi_end = min(iniY + L.h_cell + 6, L.h - ORBFE_MINB);
    const int cy0 = iniY + 3 - ry0, cy1 = roi_end - 3 - ry0;   // centre rows [cy0, cy1), band-relative
    const int xdet0 = ORBFE_MINB + 3, xdet1 = L.w - ORBFE_MINB - 3;
    const int c_lo = xdet0 + j0 * wc, c_hi = j1 == ncols ? xdet1 : xdet0 + j1 * wc;   // the slice's centres
    // ---- LDS (per wave) ----
    uint8_t* s_img = smem_pf;                                        // (RING + MIRROR) x RS
    uint8_t* s_sc = s_img + (PF_RING + PF_MIRROR) * PF_RS;          // RING x RS scores
    uint32_t* s_bm = (uint32_t*)(s_sc + PF_RING * PF_RS);           // RING x BW survivor bits
    int4* s_ty = (int4*)(s_bm + PF_RING * PF_BW);                   // the band's output rows of level l+1
    uint32_t* s_q = (uint32_t*)(s_ty + PF_TYCAP);                   // group / corner records
    int* s_base = (int*)(s_q + PF_QCAP);                            // keypoints emitted per cell
    uint16_t* s_ent = (uint16_t*)(s_base + PF_MAXC);                // pass-2 entries of one chunk
    const int cb = 4 * lane;   // this lane's ring byte; image column A0 + cb
    for (int i = lane; i < PF_RING * PF_RS / 4; i += 64) ((uint32_t*)s_sc)[i] = 0u;
    for (int i = lane; i < PF_RING * PF_BW; i += 64) s_bm[i] = 0u;
    if (lane < PF_MAXC) s_base[lane] = 0;
    const bool col_ok = A0 + cb < L.w;
    uint32_t vmask = 0;
    if (lane >= 1 && lane <= 62) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (A0 + cb + k >= c_lo && A0 + cb + k < c_hi) vmask |= 3u << (2 * k);
    }
    const _Float16 tf = __builtin_bit_cast(_Float16, (unsigned short)g.ini_th);   // iniThFAST * 2^-24
    const orbfe_half2 tv = {tf, tf};
    // ---- next level: this lane's output group of 4 columns (resize source = this level) ----
    const bool has_next = l + 1 < g.nlevels;
    const OrbLevel& L1 = g.lv[has_next ? l + 1 : l];
    const int16_t* tx = tab + L1.tab_x;
    const int16_t* ty = tab + L1.tab_y;
    int rlo = 1 << 20, rhi = -1;   // band-relative source rows the band's output rows need
    if (has_next && e_lo < e_hi) {
        rlo = ty[4 * e_lo] - ry0;
        rhi = ty[4 * (e_hi - 1) + 1] - ry0;
    }
    const int gi = g0 + lane;
    const int dx0 = 4 * gi;
    const bool rz_act = has_next && gi < g1;
    uint32_t rz_sx[4], rz_a[4];   // ring byte of the source column, a0 | a1 << 16 (both << 4)
    bool rz_simd = true;
    bool rz_vec[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int dx = min(dx0 + q, (has_next ? L1.w : 1) - 1);
        const int sx = rz_act ? tx[3 * dx] : A0;
        const bool lin = dx < L1.xmax;
        const uint32_t a0 = lin ? (uint32_t)tx[3 * dx + 1] : 2048u, a1 = lin ? (uint32_t)tx[3 * dx + 2] : 0u;
        rz_sx[q] = (uint32_t)(sx - A0);
        rz_a[q] = (a0 << 4) | ((a1 << 4) << 16);
        rz_vec[q] = dx0 + q < L1.simd_end;
        rz_simd = rz_simd && rz_vec[q];
    }
    // stored H: H << 4, masked to (H >> 4) << 8 for the universal-intrinsic columns (k_resize's form);
    // a lane is either entirely in those columns or handles the scalar tail (per-column choice)
    uint32_t rz_m[4];
#pragma unroll
    for (int q = 0; q < 4; q++) rz_m[q] = rz_vec[q] ? 0xFFFF00u : 0xFFFFFFFFu;
    uint32_t hp[4] = {0u, 0u, 0u, 0u};
    int e_next = e_lo;
    uint8_t* dst1 = has_next ? pyr + (size_t)b * pyr_stride + L1.pyr_off : nullptr;
    for (int e = lane; has_next && e < e_hi - e_lo; e += 64) {
        const int16_t* t4 = ty + 4 * (e_lo + e);
        s_ty[e] = make_int4(t4[0] - ry0, t4[1] - ry0, (int)t4[2] << 8, (int)t4[3] << 8);
    }
    // ---- blocks of 7 rows ----
    const int kA = cy1 - 4 > 0 ? (cy1 - 4 + 6) / 7 : 0;
    const int kB = rhi - 6 > 0 ? (rhi - 6 + 6) / 7 : 0;
    const int nblk = max(kA, kB) + 1;
    const gptr_u8 colp = src + A0 + cb;
    auto ld = [&](int r) -> uint32_t {
        if (r < nrel && col_ok) return *(const ORBFE_GLOBAL uint32_t*)(colp + (size_t)(ry0 + r) * spitch);
        return 0u;
    };
    uint32_t pf[7], pf2[7], wl[7], wcen[7], wr[7];   // rows of the next block and the one after
#pragma unroll
    for (int u = 0; u < 7; u++) {
        pf[u] = ld(u);
        pf2[u] = ld(u + 7);
        wl[u] = wcen[u] = wr[u] = 0u;
    }
    int qn = 0;       // queued records: [0, qc) carried corner records, then new groups
    int nms_lo = 0;   // first centre row not yet emitted
    const int ncell = j1 - j0;
    WAVE_SYNC();
    for (int k = 0; k < nblk; k++) {
        // ===== A: zeroing, ring rows, register window, pass 1 =====
        if (!(PF_ABL & 8)) {
#pragma unroll
            for (int rr = 0; rr < 7; rr++) *(uint32_t*)(s_sc + ((7 * k - 3 + rr) & (PF_RING - 1)) * PF_RS + cb) = 0u;
            // bitmap rows [7k-4, 7k+3]: 8 rows x 8 words, one per lane
            s_bm[((7 * k - 4 + (lane >> 3)) & (PF_RING - 1)) * PF_BW + (lane & 7)] = 0u;
        }
        const int qc = qn;
#pragma unroll
        for (int u = 0; u < 7; u++) {
            const int r = 7 * k + u;
            const uint32_t c = pf[u];
            pf[u] = pf2[u];
            const int slot = r & (PF_RING - 1);
            *(uint32_t*)(s_img + slot * PF_RS + cb) = c;
            if (slot < PF_MIRROR) *(uint32_t*)(s_img + (slot + PF_RING) * PF_RS + cb) = c;
            pf2[u] = ld(r + 14);
            wcen[u] = c;
            wl[u] = dpp_shr1(c);
            wr[u] = dpp_shl1(c);
            const int y = r - 3;
            if (y >= cy0 && y < cy1) {
                const int sM3 = (u + 1) % 7, sM2 = (u + 2) % 7, sY = (u + 4) % 7, sP2 = (u + 6) % 7;
                const uint32_t m8 = pf_pretest(wcen[sM3], wl[sM2], wcen[sM2], wr[sM2], wl[sY], wcen[sY], wr[sY],
                                               wl[sP2], wcen[sP2], wr[sP2], wcen[u], tv) & vmask;
                const unsigned long long gm = __ballot(m8 != 0u);
                if (m8)
                    s_q[qn + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(gm >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)gm, 0u))] =
                        (uint32_t)(lane | (y << 6)) | (m8 << 16);
                qn += __popcll(gm);
                if (lane == 0) PF_STAT(0, __popcll(gm));
            }
        }
        if (lane == 0) PF_STAT(3, 1);
        WAVE_SYNC();
        // ===== B: exact scores of the queued groups' (pixel, sign) entries, two per lane (packed f16);
        //          groups holding a corner compacted after the carried corner records =====
        int ncor = qc;
        for (int g0r = qc; !(PF_ABL & 1) && g0r < qn; g0r += 64) {
            int nent = 0;
            {   // expansion: entry = group (in chunk) << 3 | pixel k << 1 | bright
                const int gq = g0r + lane;
                const uint32_t rec = gq < qn ? s_q[gq] : 0u;
                const int cnt = __popc((rec >> 16) & 0xFFu);
                const unsigned long long lt = (1ull << lane) - 1ull;
                const unsigned long long m0 = __ballot(cnt & 1), m1 = __ballot(cnt & 2), m2 = __ballot(cnt & 4),
                                         m3 = __ballot(cnt & 8);
                int pos = __popcll(m0 & lt) + 2 * __popcll(m1 & lt) + 4 * __popcll(m2 & lt) + 8 * __popcll(m3 & lt);
                for (int i = 0; i < 4; i++) {
                    const uint32_t di = (rec >> (17 + 2 * i)) & 1u, bi = (rec >> (16 + 2 * i)) & 1u;
                    if (di) s_ent[pos++] = (uint16_t)((lane << 3) | (i << 1));
                    if (bi) s_ent[pos++] = (uint16_t)((lane << 3) | (i << 1) | 1);
                }
                nent = __popcll(m0) + 2 * __popcll(m1) + 4 * __popcll(m2) + 8 * __popcll(m3);
            }
            if (lane == 0) { PF_STAT(1, nent); PF_STAT(4, 1); }
            WAVE_SYNC();
            for (int j0e = 0; j0e < nent; j0e += 128) {
                const int j = j0e + 2 * lane;
                const bool ok0 = j < nent, ok1 = j + 1 < nent;
                const uint32_t e2 = ok0 ? ((const uint32_t*)s_ent)[j >> 1] : 0u;
                const uint32_t e0 = e2 & 0xFFFFu, e1 = ok1 ? e2 >> 16 : e0;
                const uint32_t r0 = s_q[g0r + (e0 >> 3)], r1 = s_q[g0r + (e1 >> 3)];
                const int y0 = (r0 >> 6) & 255, x0 = 4 * (int)(r0 & 63) + ((e0 >> 1) & 3);
                const int y1 = (r1 >> 6) & 255, x1 = 4 * (int)(r1 & 63) + ((e1 >> 1) & 3);
                int M0, M1;
                pf_exact2(s_img + (((y0 - 3) & (PF_RING - 1)) + 3) * PF_RS + x0,
                          s_img + (((y1 - 3) & (PF_RING - 1)) + 3) * PF_RS + x1, e0 & 1u, e1 & 1u, PF_RS, &M0, &M1);
                const bool c0 = ok0 && M0 > g.ini_th, c1 = ok1 && M1 > g.ini_th;
                if (c0) {
                    s_sc[(y0 & (PF_RING - 1)) * PF_RS + x0] = (uint8_t)(M0 - 1);
                    atomicOr(&s_q[g0r + (e0 >> 3)], 1u << (24 + ((e0 >> 1) & 3)));
                }
                if (c1) {
                    s_sc[(y1 & (PF_RING - 1)) * PF_RS + x1] = (uint8_t)(M1 - 1);
                    atomicOr(&s_q[g0r + (e1 >> 3)], 1u << (24 + ((e1 >> 1) & 3)));
                }
            }
            WAVE_SYNC();
            {   // compaction: lane | y << 6 | corner mask << 16
                const int gq = g0r + lane;
                const uint32_t rec = gq < qn ? s_q[gq] : 0u;
                const uint32_t cm = (rec >> 24) & 0xFu;
                const unsigned long long m = __ballot(cm != 0u);
                if (cm) s_q[ncor + __popcll(m & ((1ull << lane) - 1ull))] = (rec & 0x3FFFu) | (cm << 16);
                ncor += __popcll(m);
                PF_STAT(2, __popc(cm));
            }
            WAVE_SYNC();
        }
        // ----- resize of level l+1: H of the block's source rows, V of the output rows they complete -----
        if (has_next && !(PF_ABL & 2) && 7 * k + 6 >= rlo && 7 * k <= rhi) {
#pragma unroll
            for (int u = 0; u < 7; u++) {
                const int r = 7 * k + u;
                if (r < rlo || r > rhi) continue;
                const int4 te = s_ty[min(e_next, e_hi - 1) - e_lo];
                uint32_t hc[4];
                const uint8_t* row = s_img + (r & (PF_RING - 1)) * PF_RS;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t p0 = row[rz_sx[q]], p1 = row[rz_sx[q] + 1];
                    hc[q] = (__umul24(p0, rz_a[q] & 0xFFFFu) + __umul24(p1, rz_a[q] >> 16)) & rz_m[q];
                }
                int4 t = te;
                while (e_next < e_hi && t.y == r) {   // sy1 == r: at most two rows (bottom clip)
                    const uint32_t b0s = (uint32_t)t.z, b1s = (uint32_t)t.w;
                    uint32_t packed = 0;
                    if (rz_simd) {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const uint32_t h0 = t.x == r ? hc[q] : hp[q];
                            packed |= ((mulhi_u24(h0, b0s) + mulhi_u24(hc[q], b1s) + 2) >> 2) << (8 * q);
                        }
                    } else {
#pragma unroll
                        for (int q = 0; q < 4; q++) {
                            const uint32_t h0 = t.x == r ? hc[q] : hp[q], h1 = hc[q];
                            const uint32_t vs = (mulhi_u24(h0, b0s) + mulhi_u24(h1, b1s) + 2) >> 2;
                            const uint32_t vl =
                                (__umul24(h0 >> 4, b0s >> 8) + __umul24(h1 >> 4, b1s >> 8) + (1u << 21)) >> 22;
                            packed |= (rz_vec[q] ? vs : vl) << (8 * q);
                        }
                    }
                    if (rz_act) {
                        uint8_t* dp = dst1 + (size_t)e_next * L1.pitch + dx0;
                        if (dx0 + 4 <= L1.w) *(uint32_t*)dp = packed;
                        else
                            for (int q = 0; q < 4 && dx0 + q < L1.w; q++) dp[q] = (uint8_t)(packed >> (8 * q));
                    }
                    e_next++;
                    if (e_next < e_hi) t = s_ty[e_next - e_lo];
                }
#pragma unroll
                for (int q = 0; q < 4; q++) hp[q] = hc[q];
            }
        }
        // ===== C: NMS of the corners whose neighbour rows are final =====
        const int nms_hi = (7 * k + 3 >= cy1 - 1) ? cy1 : 7 * k + 3;
        {
            int nkeep = 0;
            for (int i0 = 0; !(PF_ABL & 4) && i0 < ncor; i0 += 64) {
                const int i = i0 + lane;
                const uint32_t rec = i < ncor ? s_q[i] : 0u;
                const int y = (rec >> 6) & 255;
                const bool keep = i < ncor && y >= nms_hi;
                uint32_t todo = (i < ncor && y < nms_hi) ? (rec >> 16) & 0xFu : 0u;
                const int xb = 4 * (int)(rec & 63);
                const uint8_t* rm = s_sc + ((y - 1) & (PF_RING - 1)) * PF_RS;
                const uint8_t* rc = s_sc + (y & (PF_RING - 1)) * PF_RS;
                const uint8_t* rp = s_sc + ((y + 1) & (PF_RING - 1)) * PF_RS;
                const bool up = y - 1 >= cy0, dn = y + 1 < cy1;
                uint32_t bits = 0;
                while (__ballot(todo != 0u)) {
                    if (todo) {
                        const int kk = __builtin_ctz(todo);
                        todo &= todo - 1u;
                        const int x = xb + kk, xi = A0 + x;   // ring byte, image column
                        const int j = min(small_div(xi - xdet0, wc), ncols - 1);
                        const int xlo = xdet0 + j * wc, xhi = j == ncols - 1 ? xdet1 : xlo + wc;
                        const bool lf = xi - 1 >= xlo, rt = xi + 1 < xhi;
                        const int s = rc[x];
                        const int n0 = lf ? rc[x - 1] : 0, n1 = rt ? rc[x + 1] : 0;
                        const int n2 = up ? max(lf ? rm[x - 1] : 0, max((int)rm[x], rt ? rm[x + 1] : 0)) : 0;
                        const int n3 = dn ? max(lf ? rp[x - 1] : 0, max((int)rp[x], rt ? rp[x + 1] : 0)) : 0;
                        if (s > max(max(n0, n1), max(n2, n3))) bits |= 1u << kk;
                    }
                }
                if (bits) atomicOr(&s_bm[(y & (PF_RING - 1)) * PF_BW + (xb >> 5)], bits << (xb & 31));
                const unsigned long long m = __ballot(keep);
                if (keep) s_q[nkeep + __popcll(m & ((1ull << lane) - 1ull))] = rec;
                nkeep += __popcll(m);
            }
            qn = nkeep;
        }
        WAVE_SYNC();
        // ===== D: emission of rows [nms_lo, nms_hi), one (cell, row) pair per lane =====
        const int nrow = nms_hi - nms_lo;
        if (nrow > 0 && !(PF_ABL & 4)) {
            const int jc = small_div(lane, nrow), rr = lane - jc * nrow, y = nms_lo + rr;
            const bool act = jc < ncell;
            const int jl = j0 + min(jc, ncell - 1);
            const int xlo = xdet0 + jl * wc - A0, xhi = (jl == ncols - 1 ? xdet1 : xdet0 + jl * wc + wc) - A0;
            const uint32_t* bm = s_bm + (y & (PF_RING - 1)) * PF_BW;
            int c = 0;
            if (act) {
                for (int wd = xlo >> 5; wd <= (xhi - 1) >> 5; wd++) {
                    uint32_t m = bm[wd];
                    if (wd == xlo >> 5) m &= 0xFFFFFFFFu << (xlo & 31);
                    if (wd == (xhi - 1) >> 5 && ((xhi & 31) != 0)) m &= (1u << (xhi & 31)) - 1u;
                    c += __popc(m);
                }
            }
            // position = cell base + survivors of the cell's earlier rows (inclusive scan minus the
            // scan before the cell's first row)
            const int incl = wave_incl_scan(c);
            const int before = __shfl(incl - c, min(jc * nrow, 63), 64);
            const int pos0 = (act ? s_base[min(jc, PF_MAXC - 1)] : 0) + (incl - c) - before;
            WAVE_SYNC();
            if (act && rr == nrow - 1) s_base[jc] = pos0 + c;
            if (act && c) {
                int pos = pos0;
                const uint8_t* sr = s_sc + (y & (PF_RING - 1)) * PF_RS;
                uint32_t* out = cellkeys + (size_t)b * g.cellkeys_per_img + L.cellkey_off +
                                (size_t)(band * ncols + jl) * L.cell_cap;
                const uint32_t yk = (uint32_t)(ry0 + y - ORBFE_MINB) << 12;
                for (int wd = xlo >> 5; wd <= (xhi - 1) >> 5; wd++) {
                    uint32_t m = bm[wd];
                    if (wd == xlo >> 5) m &= 0xFFFFFFFFu << (xlo & 31);
                    if (wd == (xhi - 1) >> 5 && ((xhi & 31) != 0)) m &= (1u << (xhi & 31)) - 1u;
                    while (m) {
                        const int x = 32 * wd + __builtin_ctz(m);
                        m &= m - 1u;
                        out[pos++] = (uint32_t)(A0 + x - ORBFE_MINB) | yk | ((uint32_t)sr[x] << 24);
                    }
                }
            }
            nms_lo = nms_hi;
            WAVE_SYNC();
        }
    }
    // ===== counts; cells without a survivor at iniThFAST are listed for k_fallback (the reference's
    //       FAST(minThFAST) re-run, ORBextractor.cc:826-846), which runs after every level =====
    {
        const int nl = lane < ncell ? s_base[lane] : 1;
        int* cnt_out = cellcnt + (size_t)b * g.total_cells + L.cell_base + band * ncols + j0;
        if (lane < ncell) cnt_out[lane] = nl;
        const unsigned long long fb = __ballot(nl == 0);
        if (lane == 0) { PF_STAT(6, __popcll(fb)); PF_STAT(7, 1); }
        if (fb) {
            int at = 0;
            if (lane == 0) at = atomicAdd(fb_list, __popcll(fb));
            at = __shfl(at, 0, 64);
            if (nl == 0) fb_list[1 + at + __popcll(fb & ((1ull << lane) - 1ull))] =
                (b << 16) | (L.cell_base + band * ncols + j0 + lane);
        }
    }
}

// The reference's per-cell fallback (ORBextractor.cc:826-846) for the cells k_pyrfast listed:
// FAST at minThFAST on the cell's ROI with k_fast's per-cell detector (attempt 1 only). One wave per
// listed cell, 4 waves per block over a fixed grid (every wave exits when the list is done).
__global__ __launch_bounds__(256) void k_fallback(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                                  int pyr_stride, OrbGeom g, FastLds fl, uint32_t* cellkeys,
                                                  int* cellcnt, const int* fb_list) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_fb[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    uint8_t* f_img = smem_fb + wave * fl.wave_bytes;
    uint8_t* f_sc = f_img + fl.roi;
    uint16_t* f_cor = (uint16_t*)(f_sc + fl.sc);
    uint16_t* f_ent = (uint16_t*)((uint8_t*)f_cor + fl.cor);
    const int n = fb_list[0];
    for (int i = blockIdx.x * 4 + wave; i < n; i += gridDim.x * 4) {
        const int e = fb_list[1 + i];
        const int b = e >> 16, c = e & 0xFFFF;
        const FastCell me = fast_cell(imgs, in_pitch, pyr, pyr_stride, g, b, c);
        orbfe_u32x4 pf4[FAST_PF];
        fast_prefetch(me, lane, pf4);
        fast_stage_cell(me, pf4, f_img, f_sc, lane);
        int ng, nd, cpr, rpl;
        fast_geom(me, &ng, &nd, &cpr, &rpl);
        const int dw = me.cols - 6, dh = me.rows - 6;
        if (fast_rsd(nd) == 12)
            fast_cell_detect<12>(g, fl, me, ng, nd, dw, dh, f_img, f_sc, f_cor, f_ent, cellkeys, cellcnt, b, c, lane, 0, 1);
        else
            fast_cell_detect<0>(g, fl, me, ng, nd, dw, dh, f_img, f_sc, f_cor, f_ent, cellkeys, cellcnt, b, c, lane, 0, 1);
    }
}

// Level 0 with unaligned rows (e.g. a 1241-byte pitch) copied to a 16-byte pitch for the fused pass's
// dword row loads: 4 rows per block, 4 bytes per thread per pass.
__global__ __launch_bounds__(256) void k_repitch(const uint8_t* const* imgs, int pitch, uint8_t* dst, int p16, int w,
                                                 int h) {
    const int b = blockIdx.y;
    const uint8_t* src = imgs[b];
    uint8_t* d = dst + (size_t)b * h * p16;
    for (int r = blockIdx.x * 4; r < min(blockIdx.x * 4 + 4, h); r++) {
        const uint8_t* sr = src + (size_t)r * pitch;
        for (int x = 4 * threadIdx.x; x < w; x += 1024) {
            uint32_t v = 0;
            for (int k = 0; k < 4 && x + k < w; k++) v |= (uint32_t)sr[x + k] << (8 * k);
            *(uint32_t*)(d + (size_t)r * p16 + x) = v;
        }
    }
}

}  // namespace orbfe
