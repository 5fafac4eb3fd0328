// ORB front-end kernels for CDNA4 (gfx950). Batched: every kernel takes B images (y grid dim) so
// one launch covers a whole multi-camera / multi-frame batch. Integer work is bit-exact with the
// reference semantics; float work follows the reference expression order (contraction disabled).
//
//   k_resize     ORBextractor::ComputePyramid + cv::resize INTER_LINEAR (ORBextractor.cc:1170-1195)
//   k_blur       cv::GaussianBlur 7x7 sigma 2 REFLECT_101, fixed point (ORBextractor.cc:1132-1133)
//   k_fast       ComputeKeyPointsOctTree cell loop + cv::FAST 9/16 NMS (ORBextractor.cc:781-872)
//   k_octree     DistributeOctTree (ORBextractor.cc:555-779) + lapping ranks (:1153-1162)
//   k_describe   IC_Angle (:76-103) + computeOrbDescriptor (:107-146) + output assembly (:1106-1167)
//   k_stereo     Frame::ComputeStereoMatches (Frame.cc:811-981)
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include "brief_pattern.h"
#include "glibc_sincosf.h"
#include "orbfe_types.h"
#include "stl_sort.h"

namespace orbfe {

#define SYNC() __syncthreads()

__constant__ int c_umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
__constant__ signed char c_pattern[ORBFE_PATTERN_PAIRS * 4] = ORBFE_BRIEF_PATTERN_INIT;
__constant__ int c_ring_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_ring_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

__device__ __forceinline__ int wave_incl_scan(int v) {
    const int lane = lane_id();
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        int t = __shfl_up(v, d, 64);
        if (lane >= d) v += t;
    }
    return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    return v;
}

// In-place exclusive scan of arr[0..n) by ONE wave (the caller's block is that wave). Returns total.
__device__ int wave_excl_scan_lds(int* arr, int n) {
    const int lane = lane_id();
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const int v = i < n ? arr[i] : 0;
        const int incl = wave_incl_scan(v);
        if (i < n) arr[i] = carry + incl - v;
        carry += __shfl(incl, 63, 64);
    }
    SYNC();
    return carry;
}

__device__ __forceinline__ const uint8_t* level_base(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                                     int pyr_stride, const OrbGeom& g, int b, int l, int* pitch) {
    if (l == 0) { *pitch = in_pitch; return imgs[b]; }
    *pitch = g.lv[l].pitch;
    return pyr + (size_t)b * pyr_stride + g.lv[l].pyr_off;
}

__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// ---------------------------------------------------------------------------------------------
// K1: level l from level l-1 (chained pyramid). tab: per-level int16 coefficient tables computed
// on the host with OpenCV's exact float/double expressions. Vertical pass: columns < simd_end use
// the universal-intrinsic rounding ((H>>4)*b>>16 summed, +2 >>2), the rest the scalar >>22 form.
// ---------------------------------------------------------------------------------------------
#define RESIZE_ROWS 4
__global__ __launch_bounds__(256) void k_resize(const uint8_t* const* imgs, int in_pitch, uint8_t* pyr, int pyr_stride,
                                                const int16_t* __restrict__ tab, OrbGeom g, int l) {
    const OrbLevel& L = g.lv[l];
    const int b = blockIdx.y;
    int spitch;
    const uint8_t* src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l - 1, &spitch);
    uint8_t* dst = pyr + (size_t)b * pyr_stride + L.pyr_off;
    const int16_t* tx = tab + L.tab_x;
    const int16_t* ty = tab + L.tab_y;
    for (int r = 0; r < RESIZE_ROWS; r++) {
        const int dy = blockIdx.x * RESIZE_ROWS + r;
        if (dy >= L.h) break;
        const int sy0 = ty[4 * dy], sy1 = ty[4 * dy + 1], b0 = ty[4 * dy + 2], b1 = ty[4 * dy + 3];
        const uint8_t* S0 = src + (size_t)sy0 * spitch;
        const uint8_t* S1 = src + (size_t)sy1 * spitch;
        for (int dx = threadIdx.x; dx < L.w; dx += blockDim.x) {
            const int sx = tx[3 * dx], a0 = tx[3 * dx + 1], a1 = tx[3 * dx + 2];
            int h0, h1;
            if (dx < L.xmax) {
                h0 = S0[sx] * a0 + S0[sx + 1] * a1;
                h1 = S1[sx] * a0 + S1[sx + 1] * a1;
            } else {
                h0 = S0[sx] * 2048;
                h1 = S1[sx] * 2048;
            }
            int v;
            if (dx < L.simd_end) v = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
            else v = (h0 * b0 + h1 * b1 + (1 << 21)) >> 22;
            dst[(size_t)dy * L.pitch + dx] = sat_u8(v);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K2: 7x7 Gaussian, separable fixed point: row pass Q8 (exact), column pass Q16, (v+2^15)>>16.
// One 64x16 output tile per block; halo 3 with reflect-101 at the level edges.
// ---------------------------------------------------------------------------------------------
#define BT_W 64
#define BT_H 16
__device__ __forceinline__ int reflect101(int p, int n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
    return p;
}
struct BlurKernel { int k[7]; };
__global__ __launch_bounds__(256) void k_blur(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                              int pyr_stride, uint8_t* blur, int blur_stride, OrbGeom g,
                                              BlurKernel bk) {
    __shared__ uint8_t s_in[BT_H + 6][BT_W + 8];
    __shared__ uint32_t s_row[BT_H + 6][BT_W];
    const int b = blockIdx.y;
    int l = 0;
    while (l + 1 < g.nlevels && (int)blockIdx.x >= g.lv[l + 1].blur_tile_base) l++;
    const OrbLevel& L = g.lv[l];
    const int t = blockIdx.x - L.blur_tile_base;
    const int tx0 = (t % L.blur_tiles_x) * BT_W, ty0 = (t / L.blur_tiles_x) * BT_H;
    int pitch;
    const uint8_t* src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l, &pitch);
    for (int i = threadIdx.x; i < (BT_H + 6) * (BT_W + 6); i += blockDim.x) {
        const int r = i / (BT_W + 6), c = i % (BT_W + 6);
        const int y = reflect101(ty0 + r - 3, L.h), x = reflect101(tx0 + c - 3, L.w);
        s_in[r][c] = src[(size_t)y * pitch + x];
    }
    SYNC();
    for (int i = threadIdx.x; i < (BT_H + 6) * BT_W; i += blockDim.x) {
        const int r = i / BT_W, c = i % BT_W;
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < 7; k++) s += (uint32_t)bk.k[k] * s_in[r][c + k];
        s_row[r][c] = s;
    }
    SYNC();
    uint8_t* dst = blur + (size_t)b * blur_stride + L.blur_off;
    for (int i = threadIdx.x; i < BT_H * BT_W; i += blockDim.x) {
        const int r = i / BT_W, c = i % BT_W;
        const int y = ty0 + r, x = tx0 + c;
        if (y < L.h && x < L.w) {
            uint32_t s = 0;
#pragma unroll
            for (int k = 0; k < 7; k++) s += (uint32_t)bk.k[k] * s_row[r + k][c];
            const uint32_t v = (s + 32768u) >> 16;
            dst[(size_t)y * L.pitch + x] = (uint8_t)(v > 255 ? 255 : v);
        }
    }
}

// ---------------------------------------------------------------------------------------------
// K3: FAST-9/16 per cell. One wave per cell (4 cells per 256-thread block). The cell ROI
// (wCell+6)x(hCell+6) is staged in LDS; the score of every detection pixel is computed ONCE at
// minThFAST (score = M-1 where M = max over 9-arcs of the arc-min contrast, corner iff M > th), and
// per-cell NMS is exact because the ROI ring outside the detection rect is zero. A cell emits its
// survivors with score >= iniThFAST, or all survivors when there are none (the reference's
// FAST(iniTh) -> FAST(minTh) fallback, ORBextractor.cc:826-846). Keys are packed
// x_rel | y_rel<<12 | score<<24 in row-major order (FAST emission order).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int fast_M(const uint8_t* im, int cols, int x, int y) {
    const int v = im[y * cols + x];
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; k++) d[k] = v - (int)im[(y + c_ring_dy[k]) * cols + x + c_ring_dx[k]];
    int mn2[16], mx2[16];
#pragma unroll
    for (int k = 0; k < 16; k++) { mn2[k] = min(d[k], d[(k + 1) & 15]); mx2[k] = max(d[k], d[(k + 1) & 15]); }
    int mn4[16], mx4[16];
#pragma unroll
    for (int k = 0; k < 16; k++) { mn4[k] = min(mn2[k], mn2[(k + 2) & 15]); mx4[k] = max(mx2[k], mx2[(k + 2) & 15]); }
    int M = -1000;
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const int mn9 = min(min(mn4[k], mn4[(k + 4) & 15]), d[(k + 8) & 15]);
        const int mx9 = max(max(mx4[k], mx4[(k + 4) & 15]), d[(k + 8) & 15]);
        M = max(M, max(mn9, -mx9));
    }
    return M;
}

__global__ __launch_bounds__(256) void k_fast(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                              int pyr_stride, OrbGeom g, int roi_max, uint32_t* cellkeys,
                                              int* cellcnt) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_fast[];
    const int wave = threadIdx.x >> 6, lane = lane_id();
    const int c = blockIdx.x * 4 + wave;
    const int b = blockIdx.y;
    uint8_t* s_img = smem_fast + wave * 2 * roi_max;
    uint8_t* s_sc = s_img + roi_max;
    const bool active = c < g.total_cells;
    int l = 0;
    if (active)
        while (l + 1 < g.nlevels && c >= g.lv[l + 1].cell_base) l++;
    const OrbLevel& L = g.lv[l];
    const int local = c - L.cell_base;
    const int ci = active ? local / L.n_cols : 0, cj = active ? local % L.n_cols : 0;
    const int maxBX = L.w - ORBFE_MINB, maxBY = L.h - ORBFE_MINB;
    const int r0 = ORBFE_MINB + ci * L.h_cell, c0 = ORBFE_MINB + cj * L.w_cell;
    const int r1 = min(r0 + L.h_cell + 6, maxBY), c1 = min(c0 + L.w_cell + 6, maxBX);
    // the reference skips such cells (ORBextractor.cc:810,819); never true for its grid, kept for parity
    const bool skip = !active || (r0 >= maxBY - 3) || (c0 >= maxBX - 6);
    const int rows = skip ? 0 : r1 - r0, cols = skip ? 0 : c1 - c0;
    int pitch;
    const uint8_t* src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l, &pitch);
    for (int i = lane; i < rows * cols; i += 64) {
        const int y = i / cols, x = i - y * cols;
        s_img[i] = src[(size_t)(r0 + y) * pitch + c0 + x];
        s_sc[i] = 0;
    }
    SYNC();
    const int dw = cols - 6, dh = rows - 6;
    const int ndet = (dw > 0 && dh > 0) ? dw * dh : 0;
    for (int p = lane; p < ndet; p += 64) {
        const int dy = p / dw, dx = p - dy * dw;
        const int M = fast_M(s_img, cols, dx + 3, dy + 3);
        s_sc[(dy + 3) * cols + dx + 3] = (uint8_t)(M > g.min_th ? M - 1 : 0);
    }
    SYNC();
    // NMS: survivors written into s_img (the pixels are no longer needed)
    int nhi = 0;
    for (int p = lane; p < ndet; p += 64) {
        const int dy = p / dw, dx = p - dy * dw;
        const int y = dy + 3, x = dx + 3;
        const uint8_t* q = s_sc + y * cols + x;
        const int s = q[0];
        const bool surv = s > 0 && s > q[-1] && s > q[1] && s > q[-cols - 1] && s > q[-cols] && s > q[-cols + 1] &&
                          s > q[cols - 1] && s > q[cols] && s > q[cols + 1];
        nhi += (surv && s >= g.ini_th) ? 1 : 0;
        // s_img row y is read only through s_sc now; store survivor score in place
        s_img[y * cols + x] = surv ? (uint8_t)s : 0;
    }
    nhi = wave_sum(nhi);
    SYNC();
    const int thr = nhi > 0 ? g.ini_th : 1;
    int base = 0;
    uint32_t* out = cellkeys + (size_t)b * g.cellkeys_per_img + L.cellkey_off + (size_t)local * L.cell_cap;
    const int xr0 = c0 - ORBFE_MINB + 3, yr0 = r0 - ORBFE_MINB + 3;
    for (int dy = 0; dy < dh; dy++) {
        for (int dx0 = 0; dx0 < dw; dx0 += 64) {
            const int dx = dx0 + lane;
            int s = 0;
            if (dx < dw) s = s_img[(dy + 3) * cols + dx + 3];
            const bool f = s >= thr && s > 0;
            const unsigned long long m = __ballot(f);
            const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
            if (f) out[pos] = (uint32_t)(xr0 + dx) | ((uint32_t)(yr0 + dy) << 12) | ((uint32_t)s << 24);
            base += __popcll(m);
        }
    }
    if (active && lane == 0) cellcnt[(size_t)b * g.total_cells + c] = base;
}

// ---------------------------------------------------------------------------------------------
// K4: DistributeOctTree for one (image, level), one wave. Keys are swept in parallel (each key
// carries the list position of its node); the ordered list/sort logic of the reference runs on
// LDS tables: phase-1 rounds are rebuilt with scans (list order = push_front order), phase-2
// passes sort the expandable nodes with the libstdc++ introsort replica (tie order matters) and
// replay the reference's break-at-N walk. The per-node winner is the first max-response key in
// key order, i.e. max(score) then min(index) (ORBextractor.cc:757-776).
// ---------------------------------------------------------------------------------------------
struct ExpEnt { int size; int x0; int pos; };
struct ExpLess {
    __device__ bool operator()(const ExpEnt& a, const ExpEnt& b) const {   // compareNodes
        if (a.size < b.size) return true;
        if (a.size > b.size) return false;
        return a.x0 < b.x0;
    }
};
struct NodeTab {
    int16_t *x0, *x1, *y0, *y1;
    int* size;
};
__device__ __forceinline__ int quadrant(uint32_t key, int x0, int x1, int y0, int y1) {
    const int halfX = (int)ceilf((float)(x1 - x0) / 2.f);
    const int halfY = (int)ceilf((float)(y1 - y0) / 2.f);
    const float fx = (float)(key & 0xfff), fy = (float)((key >> 12) & 0xfff);
    const int q = (fx < (float)(x0 + halfX)) ? (fy < (float)(y0 + halfY) ? 0 : 2) : (fy < (float)(y0 + halfY) ? 1 : 3);
    return q;
}
__device__ __forceinline__ void child_rect(int q, int x0, int x1, int y0, int y1, int* cx0, int* cx1, int* cy0,
                                           int* cy1) {
    const int mx = x0 + (int)ceilf((float)(x1 - x0) / 2.f);
    const int my = y0 + (int)ceilf((float)(y1 - y0) / 2.f);
    *cx0 = (q & 1) ? mx : x0;
    *cx1 = (q & 1) ? x1 : mx;
    *cy0 = (q & 2) ? my : y0;
    *cy1 = (q & 2) ? y1 : my;
}

__global__ __launch_bounds__(64) void k_octree(OrbGeom g, const uint32_t* __restrict__ cellkeys,
                                               const int* __restrict__ cellcnt, uint32_t* lkeys, uint16_t* nodeof,
                                               uint32_t* outkeys, int* lvinfo, int* ranks, int lap0, int lap1) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_oct[];
    const int l = blockIdx.x, b = blockIdx.y, lane = lane_id();
    const OrbLevel& L = g.lv[l];
    const int NC = g.node_cap;
    const int ncell = L.n_cols * L.n_rows;
    // ---- LDS carve (all offsets multiples of 16 bytes) ----
    uint8_t* p = smem_oct;
    auto carve = [&](size_t bytes) { uint8_t* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    int* cellpre = (int*)carve(sizeof(int) * (g.max_cells_level + 1));
    NodeTab T[2];
    for (int k = 0; k < 2; k++) {
        T[k].x0 = (int16_t*)carve(2 * NC); T[k].x1 = (int16_t*)carve(2 * NC);
        T[k].y0 = (int16_t*)carve(2 * NC); T[k].y1 = (int16_t*)carve(2 * NC);
        T[k].size = (int*)carve(4 * NC);
    }
    int* cnt[2] = {(int*)carve(16 * NC), (int*)carve(16 * NC)};
    int16_t* childpos = (int16_t*)carve(8 * NC);
    int16_t* newpos = (int16_t*)carve(2 * NC);
    int* divorder = (int*)carve(4 * NC);
    int* tmpA = (int*)carve(4 * NC);
    int* tmpB = (int*)carve(4 * NC);
    int* tmpC = (int*)carve(4 * NC);
    int* procp = (int*)carve(4 * NC);
    ExpEnt* expv = (ExpEnt*)carve(sizeof(ExpEnt) * NC);
    unsigned long long* best = (unsigned long long*)carve(8 * NC);
    __shared__ int s_misc[8];

    // ---- gather this level's cell key lists in cell order (vToDistributeKeys order) ----
    const int* cc = cellcnt + (size_t)b * g.total_cells + L.cell_base;
    {
        int carry = 0;
        for (int base = 0; base < ncell; base += 64) {
            const int i = base + lane;
            const int v = i < ncell ? cc[i] : 0;
            const int incl = wave_incl_scan(v);
            if (i < ncell) cellpre[i + 1] = carry + incl;
            carry += __shfl(incl, 63, 64);
        }
        if (lane == 0) cellpre[0] = 0;
    }
    SYNC();
    const int K = cellpre[ncell];
    const size_t kbase = (size_t)b * g.cellkeys_per_img + L.cellkey_off;
    uint32_t* keys = lkeys + kbase;
    uint16_t* nof = nodeof + kbase;
    const uint32_t* ck = cellkeys + kbase;
    for (int k = lane; k < K; k += 64) {
        int lo = 0, hi = ncell - 1;   // largest c with cellpre[c] <= k
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (cellpre[mid] <= k) lo = mid; else hi = mid - 1;
        }
        keys[k] = ck[(size_t)lo * L.cell_cap + (k - cellpre[lo])];
    }
    // ---- initial nodes (ORBextractor.cc:559-601) ----
    const int nIni = L.n_ini;
    const float hX = L.hx;
    const int H = (L.h - ORBFE_MINB) - ORBFE_MINB;
    for (int i = lane; i < nIni; i += 64) tmpA[i] = 0;
    SYNC();
    for (int k = lane; k < K; k += 64) {
        const int r = (int)((float)(keys[k] & 0xfff) / hX);
        atomicAdd(&tmpA[r], 1);
    }
    SYNC();
    int cur = 0;
    for (int i = lane; i < nIni; i += 64) tmpB[i] = tmpA[i] > 0 ? 1 : 0;
    SYNC();
    int n = wave_excl_scan_lds(tmpB, nIni);   // position of each non-empty root
    for (int i = lane; i < nIni; i += 64) {
        if (tmpA[i] > 0) {
            const int q = tmpB[i];
            T[cur].x0[q] = (int16_t)(int)(hX * (float)i);
            T[cur].x1[q] = (int16_t)(int)(hX * (float)(i + 1));
            T[cur].y0[q] = 0;
            T[cur].y1[q] = (int16_t)H;
            T[cur].size[q] = tmpA[i];
        }
    }
    for (int i = lane; i < 4 * NC; i += 64) cnt[cur][i] = 0;
    SYNC();
    for (int k = lane; k < K; k += 64) {
        const uint32_t key = keys[k];
        const int r = (int)((float)(key & 0xfff) / hX);
        const int q = tmpB[r];
        nof[k] = (uint16_t)q;
        if (T[cur].size[q] > 1)
            atomicAdd(&cnt[cur][4 * q + quadrant(key, T[cur].x0[q], T[cur].x1[q], T[cur].y0[q], T[cur].y1[q])], 1);
    }
    SYNC();

    const int N = L.budget;
    bool phase2 = false, finish = false;
    int m = 0;   // expandable-node count of the last rebuild (vSizeAndPointerToNode)
    for (int i = lane; i < NC; i += 64) divorder[i] = -1;
    SYNC();
    int guard = 0;
    while (!finish && guard++ < 100000) {
        const int prevN = n;
        int T_div;   // number of divided nodes in this step
        if (!phase2) {
            // every node with >1 keys divides, in list order
            for (int i = lane; i < n; i += 64) {
                const bool dv = T[cur].size[i] > 1;
                divorder[i] = dv ? 1 : -1;
                tmpA[i] = dv ? 1 : 0;
            }
            SYNC();
            T_div = wave_excl_scan_lds(tmpA, n);   // tmpA[i] = divider rank t (list order)
            for (int i = lane; i < n; i += 64)
                if (divorder[i] >= 0) { divorder[i] = tmpA[i]; procp[tmpA[i]] = i; }
            SYNC();
        } else {
            if (lane == 0) {
                stl_sort(expv, m, ExpLess());
                int Lsz = n, t = 0;
                for (int j = m - 1; j >= 0; j--) {
                    const int q = expv[j].pos;
                    int c = 0;
                    for (int k = 0; k < 4; k++) c += cnt[cur][4 * q + k] > 0;
                    divorder[q] = t;
                    procp[t] = q;
                    t++;
                    Lsz += c - 1;
                    if (Lsz >= N) break;
                }
                s_misc[0] = t;
            }
            SYNC();
            T_div = s_misc[0];
        }
        // children counts per processed node (t order): tmpB = nonempty, tmpC = expandable (>1)
        for (int t = lane; t < T_div; t += 64) {
            const int q = procp[t];
            int c = 0, e = 0;
            for (int k = 0; k < 4; k++) { const int v = cnt[cur][4 * q + k]; c += v > 0; e += v > 1; }
            tmpB[t] = c;
            tmpC[t] = e;
        }
        SYNC();
        const int Ctot = wave_excl_scan_lds(tmpB, T_div);
        const int Etot = wave_excl_scan_lds(tmpC, T_div);
        const int nxt = cur ^ 1;
        // children: block of t starts at sum_{t'>t} c_t' = Ctot - (excl_t + c_t); order n4,n3,n2,n1
        for (int t = lane; t < T_div; t += 64) {
            const int q = procp[t];
            int c = 0;
            for (int k = 0; k < 4; k++) c += cnt[cur][4 * q + k] > 0;
            const int start = Ctot - (tmpB[t] + c);
            int kk = 0;
            const int px0 = T[cur].x0[q], px1 = T[cur].x1[q], py0 = T[cur].y0[q], py1 = T[cur].y1[q];
            for (int ch = 3; ch >= 0; ch--) {
                const int v = cnt[cur][4 * q + ch];
                if (v > 0) {
                    const int np = start + kk++;
                    childpos[4 * q + ch] = (int16_t)np;
                    int a0, a1, b0, b1;
                    child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                    T[nxt].x0[np] = (int16_t)a0; T[nxt].x1[np] = (int16_t)a1;
                    T[nxt].y0[np] = (int16_t)b0; T[nxt].y1[np] = (int16_t)b1;
                    T[nxt].size[np] = v;
                } else {
                    childpos[4 * q + ch] = -1;
                }
            }
            int e = tmpC[t];
            for (int ch = 0; ch < 4; ch++) {
                const int v = cnt[cur][4 * q + ch];
                if (v > 1) {
                    int a0, a1, b0, b1;
                    child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                    expv[e].size = v; expv[e].x0 = a0; expv[e].pos = childpos[4 * q + ch];
                    e++;
                }
            }
        }
        // undivided nodes keep their relative order after the pushed children
        for (int i = lane; i < n; i += 64) tmpA[i] = divorder[i] < 0 ? 1 : 0;
        SYNC();
        const int nKeep = wave_excl_scan_lds(tmpA, n);
        for (int i = lane; i < n; i += 64) {
            if (divorder[i] < 0) {
                const int np = Ctot + tmpA[i];
                newpos[i] = (int16_t)np;
                T[nxt].x0[np] = T[cur].x0[i]; T[nxt].x1[np] = T[cur].x1[i];
                T[nxt].y0[np] = T[cur].y0[i]; T[nxt].y1[np] = T[cur].y1[i];
                T[nxt].size[np] = T[cur].size[i];
            }
        }
        const int newN = Ctot + nKeep;
        for (int i = lane; i < 4 * newN; i += 64) cnt[nxt][i] = 0;
        SYNC();
        // key sweep: move keys to their new node positions and count the next split
        for (int k = lane; k < K; k += 64) {
            const uint32_t key = keys[k];
            const int q = nof[k];
            int np;
            if (divorder[q] >= 0) np = childpos[4 * q + quadrant(key, T[cur].x0[q], T[cur].x1[q], T[cur].y0[q], T[cur].y1[q])];
            else np = newpos[q];
            nof[k] = (uint16_t)np;
            if (T[nxt].size[np] > 1)
                atomicAdd(&cnt[nxt][4 * np + quadrant(key, T[nxt].x0[np], T[nxt].x1[np], T[nxt].y0[np], T[nxt].y1[np])], 1);
        }
        for (int i = lane; i < NC; i += 64) divorder[i] = -1;
        SYNC();
        cur = nxt;
        n = newN;
        m = Etot;
        if (n >= N || n == prevN) finish = true;
        else if (!phase2 && n + 3 * m > N) phase2 = true;
    }
    // ---- retain the best key per node ----
    for (int i = lane; i < n; i += 64) best[i] = 0ull;
    SYNC();
    for (int k = lane; k < K; k += 64) {
        const uint32_t key = keys[k];
        const unsigned long long v = ((unsigned long long)(key >> 24) << 32) | (0xFFFFFFFFull - (unsigned)k);
        atomicMax(&best[nof[k]], v);
    }
    SYNC();
    uint32_t* ok = outkeys + (size_t)b * g.out_per_img + L.out_off;
    int* rk = ranks + (size_t)b * g.out_per_img + L.out_off;
    int carry_lap = 0, carry_mono = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        bool lap = false;
        if (i < n) {
            const unsigned k = 0xFFFFFFFFu - (unsigned)(best[i] & 0xFFFFFFFFull);
            const uint32_t key = keys[k];
            const int x = (int)(key & 0xfff) + ORBFE_MINB, y = (int)((key >> 12) & 0xfff) + ORBFE_MINB;
            ok[i] = (uint32_t)x | ((uint32_t)y << 12) | (key & 0xff000000u);
            const float sx = (l == 0) ? (float)x : (float)x * L.scale;
            lap = sx >= (float)lap0 && sx <= (float)lap1;
        }
        const int il = wave_incl_scan(lap ? 1 : 0);
        const int im = wave_incl_scan((i < n && !lap) ? 1 : 0);
        if (i < n) rk[i] = lap ? (int)(0x40000000 | (carry_lap + il - 1)) : (carry_mono + im - 1);
        carry_lap += __shfl(il, 63, 64);
        carry_mono += __shfl(im, 63, 64);
    }
    if (lane == 0) {
        int* inf = lvinfo + ((size_t)b * g.nlevels + l) * 4;
        inf[0] = n; inf[1] = carry_lap; inf[2] = carry_mono; inf[3] = K;
    }
}

// ---------------------------------------------------------------------------------------------
// K5: orientation + rBRIEF + output assembly. One wave per keypoint, 4 per block.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float fast_atan2_dev(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

__global__ __launch_bounds__(256) void k_describe(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                                  int pyr_stride, const uint8_t* blur, int blur_stride, OrbGeom g,
                                                  const uint32_t* __restrict__ outkeys, const int* __restrict__ lvinfo,
                                                  const int* __restrict__ ranks, OrbKeyPoint* kps, uint8_t* desc,
                                                  int* counts) {
    const int wave = threadIdx.x >> 6, lane = lane_id();
    const int b = blockIdx.y;
    const int flat = blockIdx.x * 4 + wave;   // index over all levels' output slots
    if (flat >= g.out_per_img) return;
    int l = 0;
    while (l + 1 < g.nlevels && flat >= g.lv[l + 1].out_off) l++;
    const OrbLevel& L = g.lv[l];
    const int i = flat - L.out_off;
    const int* inf = lvinfo + (size_t)b * g.nlevels * 4;
    int ntot = 0, lap_before = 0, mono_before = 0, mono_tot = 0;
    for (int k = 0; k < g.nlevels; k++) {
        ntot += inf[4 * k];
        mono_tot += inf[4 * k + 2];
        if (k < l) { lap_before += inf[4 * k + 1]; mono_before += inf[4 * k + 2]; }
    }
    if (flat == 0 && lane == 0) { counts[2 * b] = ntot; counts[2 * b + 1] = mono_tot; }
    if (i >= inf[4 * l]) return;
    const uint32_t key = outkeys[(size_t)b * g.out_per_img + flat];
    const int x = key & 0xfff, y = (key >> 12) & 0xfff;
    // IC_Angle on the unblurred level
    int pitch;
    const uint8_t* im = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l, &pitch);
    const uint8_t* center = im + (size_t)y * pitch + x;
    const int u = (lane & 31) - 15;
    const bool ucol = (lane & 31) < 31;
    int m10 = 0, m01 = 0;
    if (ucol) {
        if (lane < 32) {
            m10 += u * (int)center[u];
            for (int v = 1; v <= 8; v++) {
                if (u >= -c_umax[v] && u <= c_umax[v]) {
                    const int vp = center[u + v * pitch], vm = center[u - v * pitch];
                    m10 += u * (vp + vm);
                    m01 += v * (vp - vm);
                }
            }
        } else {
            for (int v = 9; v <= 15; v++) {
                if (u >= -c_umax[v] && u <= c_umax[v]) {
                    const int vp = center[u + v * pitch], vm = center[u - v * pitch];
                    m10 += u * (vp + vm);
                    m01 += v * (vp - vm);
                }
            }
        }
    }
    m10 = wave_sum(m10);
    m01 = wave_sum(m01);
    const float angle = fast_atan2_dev((float)m01, (float)m10);
    // rBRIEF on the blurred level
    const float factorPI = (float)(M_PI / 180.f);
    const float ang = angle * factorPI;
    const float a = glibc_cosf(ang), bs = glibc_sinf(ang);
    const uint8_t* bl = blur + (size_t)b * blur_stride + L.blur_off;
    const uint8_t* bc = bl + (size_t)y * L.pitch + x;
    unsigned long long masks[4];
#pragma unroll
    for (int mm = 0; mm < 4; mm++) {
        const int pr = 64 * mm + lane;
        const float px0 = (float)c_pattern[4 * pr], py0 = (float)c_pattern[4 * pr + 1];
        const float px1 = (float)c_pattern[4 * pr + 2], py1 = (float)c_pattern[4 * pr + 3];
        const int t0 = bc[(int)rintf(px0 * bs + py0 * a) * L.pitch + (int)rintf(px0 * a - py0 * bs)];
        const int t1 = bc[(int)rintf(px1 * bs + py1 * a) * L.pitch + (int)rintf(px1 * a - py1 * bs)];
        masks[mm] = __ballot(t0 < t1);
    }
    const int rk = ranks[(size_t)b * g.out_per_img + flat];
    int slot;
    if (rk & 0x40000000) slot = ntot - 1 - (lap_before + (rk & 0x3fffffff));
    else slot = mono_before + rk;
    const size_t o = (size_t)b * g.kp_cap + slot;
    if (lane < 4) {
        unsigned long long mv = lane == 0 ? masks[0] : lane == 1 ? masks[1] : lane == 2 ? masks[2] : masks[3];
        ((unsigned long long*)(desc + o * 32))[lane] = mv;
    }
    if (lane == 0) {
        OrbKeyPoint kp;
        kp.x = (l == 0) ? (float)x : (float)x * L.scale;
        kp.y = (l == 0) ? (float)y : (float)y * L.scale;
        kp.size = (float)L.patch_size;
        kp.angle = angle;
        kp.response = (float)(key >> 24);
        kp.octave = l;
        kp.class_id = -1;
        kps[o] = kp;
    }
}

// ---------------------------------------------------------------------------------------------
// K6: Frame::ComputeStereoMatches for a batch of rectified frames. One block (4 waves) per frame;
// one wave per left keypoint. Candidate = right kps whose row band [floor(y-2s), ceil(y+2s)]
// contains (int)vL, octave within +-1, uR in [uL-maxD, uL]; the reference takes the FIRST best
// in iR order, i.e. min (dist, iR). Then 11x11 SAD over 11 shifts on the unblurred levels,
// parabola, and the median outlier cut over the frame.
// ---------------------------------------------------------------------------------------------
struct StereoArgs {
    float bf, fx;
    int max_kp;
};
// One side (left or right camera) of a batch of frames: image f of this side is image
// (base + f*step) of the extractor batch whose buffers are given here.
struct StereoSide {
    const uint8_t* const* imgs;
    int in_pitch;
    const uint8_t* pyr;
    int pyr_stride;
    const OrbKeyPoint* kps;
    const uint8_t* desc;
    const int* counts;
    int base, step;
};
__device__ __forceinline__ int hamming32(const uint32_t* a, const uint32_t* b) {
    int d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d += __popc(a[i] ^ b[i]);
    return d;
}
__global__ __launch_bounds__(256) void k_stereo(OrbGeom g, StereoSide SL, StereoSide SR, StereoArgs sa,
                                                float* uright, float* depth, int* nmatch) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_st[];
    const int f = blockIdx.x;
    const int bL = SL.base + f * SL.step, bR = SR.base + f * SR.step;
    const int wave = threadIdx.x >> 6, lane = lane_id();
    const int N = SL.counts[2 * bL], Nr = SR.counts[2 * bR];
    uint32_t* s_descR = (uint32_t*)smem_st;                               // Nr * 8 words
    float* s_xR = (float*)(s_descR + 8 * sa.max_kp);
    int* s_oct = (int*)(s_xR + sa.max_kp);
    int* s_minr = s_oct + sa.max_kp;
    int* s_maxr = s_minr + sa.max_kp;
    int* s_list = s_maxr + sa.max_kp;                                     // accepted (dist) per left kp
    int* s_idx = s_list + sa.max_kp;
    __shared__ int s_nacc;
    const OrbKeyPoint* kR = SR.kps + (size_t)bR * g.kp_cap;
    const OrbKeyPoint* kL = SL.kps + (size_t)bL * g.kp_cap;
    const uint32_t* dR = (const uint32_t*)(SR.desc + (size_t)bR * g.kp_cap * 32);
    const uint32_t* dL = (const uint32_t*)(SL.desc + (size_t)bL * g.kp_cap * 32);
    for (int i = threadIdx.x; i < Nr * 8; i += blockDim.x) s_descR[i] = dR[i];
    for (int i = threadIdx.x; i < Nr; i += blockDim.x) {
        const OrbKeyPoint kp = kR[i];
        const float r = 2.0f * g.lv[kp.octave].scale;
        s_xR[i] = kp.x;
        s_oct[i] = kp.octave;
        s_maxr[i] = (int)ceilf(kp.y + r);
        s_minr[i] = (int)floorf(kp.y - r);
    }
    if (threadIdx.x == 0) s_nacc = 0;
    float* uR_out = uright + (size_t)f * g.kp_cap;
    float* dp_out = depth + (size_t)f * g.kp_cap;
    for (int i = threadIdx.x; i < N; i += blockDim.x) { uR_out[i] = -1.0f; dp_out[i] = -1.0f; }
    SYNC();
    const float mb = sa.bf / sa.fx;
    const float minZ = mb, minD = 0.f, maxD = sa.bf / minZ;
    for (int iL = wave; iL < N; iL += 4) {
        const OrbKeyPoint kpL = kL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const int row = (int)vL;
        const float minU = uL - maxD, maxU = uL - minD;
        if (maxU < 0) continue;
        uint32_t dl[8];
#pragma unroll
        for (int k = 0; k < 8; k++) dl[k] = dL[(size_t)iL * 8 + k];
        int bestKey = 0x7fffffff;   // (dist << 16) | iR, min
        bool anyCand = false;
        for (int iR = lane; iR < Nr; iR += 64) {
            if (s_minr[iR] <= row && row <= s_maxr[iR]) {
                anyCand = true;
                const int o = s_oct[iR];
                if (o < levelL - 1 || o > levelL + 1) continue;
                const float uR = s_xR[iR];
                if (uR >= minU && uR <= maxU) {
                    const int dist = hamming32(dl, s_descR + 8 * iR);
                    const int kk = (dist << 16) | iR;
                    bestKey = min(bestKey, kk);
                }
            }
        }
        if (!__any(anyCand)) continue;   // vCandidates.empty()
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) bestKey = min(bestKey, __shfl_xor(bestKey, d, 64));
        const int bestDist = bestKey == 0x7fffffff ? 100 : min(100, bestKey >> 16);
        if (!(bestDist < 75)) continue;   // thOrbDist = (TH_HIGH+TH_LOW)/2
        const int bestIdxR = bestKey & 0xffff;
        const float uR0 = s_xR[bestIdxR];
        const float sf = g.lv[levelL].inv_scale;
        const float scaleduL = roundf(kpL.x * sf);
        const float scaledvL = roundf(kpL.y * sf);
        const float scaleduR0 = roundf(uR0 * sf);
        const int w = 5, Lr = 5;
        const float iniu = scaleduR0 + Lr - w;
        const float endu = scaleduR0 + Lr + w + 1;
        const OrbLevel& LV = g.lv[levelL];
        if (iniu < 0 || endu >= LV.w) continue;
        int pL, pR;
        const uint8_t* IL = level_base(SL.imgs, SL.in_pitch, SL.pyr, SL.pyr_stride, g, bL, levelL, &pL);
        const uint8_t* IR = level_base(SR.imgs, SR.in_pitch, SR.pyr, SR.pyr_stride, g, bR, levelL, &pR);
        const int r0 = (int)(scaledvL - w), c0L = (int)(scaleduL - w);
        // lanes: pixel (yy, xx) of the 11x11 window, 121 = 64 + 57
        float dists[11];
        int bestD = 0x7fffffff, bestinc = 0;
        for (int inc = -Lr; inc <= Lr; inc++) {
            const int c0R = (int)(scaleduR0 + inc - w);
            int s = 0;
            for (int pix = lane; pix < 121; pix += 64) {
                const int yy = pix / 11, xx = pix - yy * 11;
                s += abs((int)IL[(size_t)(r0 + yy) * pL + c0L + xx] - (int)IR[(size_t)(r0 + yy) * pR + c0R + xx]);
            }
            s = wave_sum(s);
            const float dist = (float)s;
            if (dist < (float)bestD) { bestD = (int)dist; bestinc = inc; }
            dists[Lr + inc] = dist;
        }
        if (bestinc == -Lr || bestinc == Lr) continue;
        const float dist1 = dists[Lr + bestinc - 1], dist2 = dists[Lr + bestinc], dist3 = dists[Lr + bestinc + 1];
        const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
        if (deltaR < -1 || deltaR > 1) continue;
        float bestuR = g.lv[levelL].scale * ((float)scaleduR0 + (float)bestinc + deltaR);
        float disparity = (uL - bestuR);
        if (disparity >= minD && disparity < maxD) {
            if (disparity <= 0) { disparity = (float)0.01; bestuR = (float)((double)uL - 0.01); }
            if (lane == 0) {
                dp_out[iL] = sa.bf / disparity;
                uR_out[iL] = bestuR;
                const int slot = atomicAdd(&s_nacc, 1);
                s_list[slot] = bestD;
                s_idx[slot] = iL;
            }
        }
    }
    SYNC();
    const int nacc = s_nacc;
    if (nacc == 0) { if (threadIdx.x == 0) nmatch[f] = 0; return; }
    // median of the (dist, iL)-sorted list = the (nacc/2)-th smallest dist: rank selection
    __shared__ int s_med;
    for (int i = threadIdx.x; i < nacc; i += blockDim.x) {
        const int di = s_list[i], ii = s_idx[i];
        int rank = 0;
        for (int j = 0; j < nacc; j++) {
            const int dj = s_list[j];
            rank += (dj < di) || (dj == di && s_idx[j] < ii);
        }
        if (rank == nacc / 2) s_med = di;
    }
    SYNC();
    const float median = (float)s_med;
    const float thDist = 1.5f * 1.4f * median;
    int kept = 0;
    for (int i = threadIdx.x; i < nacc; i += blockDim.x) {
        if (!((float)s_list[i] < thDist)) { uR_out[s_idx[i]] = -1; dp_out[s_idx[i]] = -1; }
        else kept++;
    }
    (void)kept;
    if (threadIdx.x == 0) nmatch[f] = nacc;
}

}  // namespace orbfe
