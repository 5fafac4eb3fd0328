// ORB front-end kernels for CDNA4 (gfx950). Batched: every kernel takes B images (y grid dim) so
// one launch covers a whole multi-camera / multi-frame batch. Integer work is bit-exact with the
// reference semantics; float work follows the reference expression order (contraction disabled).
//
//   k_resize     ORBextractor::ComputePyramid + cv::resize INTER_LINEAR (ORBextractor.cc:1170-1195)
//   k_fast       ComputeKeyPointsOctTree cell loop + cv::FAST 9/16 NMS (ORBextractor.cc:781-872)
//   k_octree     DistributeOctTree (ORBextractor.cc:555-779) + lapping ranks (:1153-1162)
//   k_describe   IC_Angle (:76-103) + GaussianBlur 7x7 (:1132-1133, only at the rBRIEF samples) +
//                computeOrbDescriptor (:107-146) + output assembly (:1106-1167)
//   k_stereo     Frame::ComputeStereoMatches (Frame.cc:811-981)
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>
#include <float.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "brief_pattern.h"
#include "glibc_sincosf.h"
#include "orbfe_types.h"
#include "stl_sort.h"

namespace orbfe {

#define SYNC() __syncthreads()
// Intra-wave LDS hand-off (producer and consumer lanes belong to one wave; other waves of the
// block may already have exited, so no workgroup barrier): order the LDS accesses for the
// compiler and wait for this wave's outstanding LDS operations.
#define WAVE_SYNC()                                               \
    do {                                                          \
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");    \
        __builtin_amdgcn_s_waitcnt(0xc07f);                       \
        __builtin_amdgcn_wave_barrier();                          \
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");    \
    } while (0)

__constant__ int c_umax[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
// IC_Angle disc as byte masks: row v = -15..15 of the 43x43 describe patch (centre column 21),
// dwords 1..9 of the 48-byte row (columns 4..39); byte = 0xFF iff |column - 21| <= umax[|v|]
// (ORBextractor.cc:451-468 umax, :76-103 disc). 12 dwords per row (16-byte aligned rows).
struct IcMaskTab { uint32_t m[31][12]; };
constexpr IcMaskTab make_ic_mask() {
    IcMaskTab t{};
    constexpr int um[16] = {15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3};
    for (int vi = 0; vi < 31; vi++) {
        const int d = um[vi < 15 ? 15 - vi : vi - 15];
        for (int j = 0; j < 9; j++) {
            uint32_t w = 0;
            for (int b = 0; b < 4; b++) {
                const int u = 4 * (j + 1) + b - 21;
                if (u >= -d && u <= d) w |= 0xFFu << (8 * b);
            }
            t.m[vi][j] = w;
        }
    }
    return t;
}
__constant__ IcMaskTab c_ic_mask = make_ic_mask();
__constant__ signed char c_pattern[ORBFE_PATTERN_PAIRS * 4] = ORBFE_BRIEF_PATTERN_INIT;
// the pattern as f16 (x0, y0), (x1, y1) pairs (pair i at 4 i): k_describe holds a lane's four pairs
// in 8 VGPRs (as f32 they took 16 and the kernel spilled 36 bytes per lane at 6 waves per SIMD)
struct PatternH { unsigned short v[ORBFE_PATTERN_PAIRS * 4]; };
constexpr unsigned short f16_bits_small_int(int v) {   // |v| <= 2048: exact
    if (v == 0) return 0;
    const unsigned short sgn = v < 0 ? 0x8000 : 0;
    unsigned a = (unsigned)(v < 0 ? -v : v);
    int e = 0;
    while ((a >> e) > 1) e++;
    const unsigned mant = (a << (10 - e)) & 0x3FFu;
    return (unsigned short)(sgn | ((unsigned)(e + 15) << 10) | mant);
}
constexpr PatternH make_pattern_h() {
    constexpr signed char p[ORBFE_PATTERN_PAIRS * 4] = ORBFE_BRIEF_PATTERN_INIT;
    PatternH t{};
    for (int i = 0; i < ORBFE_PATTERN_PAIRS * 4; i++) t.v[i] = f16_bits_small_int(p[i]);
    return t;
}
__constant__ PatternH c_pattern_h = make_pattern_h();
constexpr int kRingDx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
constexpr int kRingDy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
__constant__ int c_ring_dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
__constant__ int c_ring_dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Workgroups are dealt round-robin over the 8 XCDs (blocks b and b + 8 share one, each XCD has its
// own L2): remap the linear block id so every XCD walks one contiguous range of logical blocks and
// neighbouring tiles / cells / keypoints (which share halo rows and cache lines) share an L2.
__device__ __forceinline__ int xcd_logical(int bid, int total) {
    const int q = total >> 3, r = total & 7;
    const int x = bid & 7, sl = bid >> 3;
    return x * q + min(x, r) + sl;
}
__device__ __forceinline__ int block_linear() {
    return blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
}

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

// Wave-uniform sum with four DPP steps (row_shr 1, 2, 4, 8 leave each 16-lane row's sum in its
// lane 15) and four readlanes: 8 VALU instead of the bpermute butterfly's ~18. Every lane must be
// active.
__device__ __forceinline__ int wave_min_dpp(int v) {
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x111, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x112, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x114, 0xf, 0xf, false));
    v = min(v, __builtin_amdgcn_update_dpp(0x7fffffff, v, 0x118, 0xf, 0xf, false));
    return min(min(__builtin_amdgcn_readlane(v, 15), __builtin_amdgcn_readlane(v, 31)),
               min(__builtin_amdgcn_readlane(v, 47), __builtin_amdgcn_readlane(v, 63)));
}
__device__ __forceinline__ int wave_sum_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    return __builtin_amdgcn_readlane(v, 15) + __builtin_amdgcn_readlane(v, 31) + __builtin_amdgcn_readlane(v, 47) +
           __builtin_amdgcn_readlane(v, 63);
}

// Number of set bits of a wave mask below this lane (v_mbcnt_lo / v_mbcnt_hi: 2 VALU).
__device__ __forceinline__ int lanes_below(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Inclusive wave scan with six DPP adds: row_shr 1, 2, 4, 8 scan each 16-lane row, row_bcast 15 /
// 31 carry rows 0 -> 1, 2 -> 3 and row 1 -> 2, 3. Every lane must be active.
__device__ __forceinline__ int wave_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
    return v;
}

// In-place exclusive scan of arr[0..n) by ONE wave (the caller's block is that wave). Returns total.
__device__ int wave_excl_scan_lds(int* arr, int n) {
    const int lane = lane_id();
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const int v = i < n ? arr[i] : 0;
        const int incl = wave_incl_scan_dpp(v);
        if (i < n) arr[i] = carry + incl - v;
        carry += __builtin_amdgcn_readlane(incl, 63);
    }
    SYNC();
    return carry;
}

// Image pointers come from a pointer table, so the compiler cannot prove they are global memory
// and would emit flat_* loads (which also count against lgkmcnt and serialise with LDS traffic).
// Every image access goes through an explicit address_space(1) pointer instead.
#define ORBFE_GLOBAL __attribute__((address_space(1)))
typedef const ORBFE_GLOBAL uint8_t* gptr_u8;
typedef const ORBFE_GLOBAL uint32_t* gptr_u32;
__device__ __forceinline__ gptr_u8 as_global(const uint8_t* p) { return (gptr_u8)p; }
typedef uint32_t orbfe_u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ gptr_u8 level_base(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                              int pyr_stride, const OrbGeom& g, int b, int l, int* pitch) {
    if (l == 0) { *pitch = in_pitch; return as_global(imgs[b]); }
    *pitch = g.lv[l].pitch;
    return as_global(pyr + (size_t)b * pyr_stride + g.lv[l].pyr_off);
}

__device__ __forceinline__ int reflect101(int p, int n) {
    if (p < 0) p = -p;
    if (p >= n) p = 2 * n - 2 - p;
    return p;
}

// a / d for 0 <= a < 2^16 and 1 <= d <= 2^16 (d typically wave-uniform): (a + 0.5) / d is at least
// 1 / (2d) away from an integer, far above the error of v_rcp_f32, so the truncation is exact
__device__ __forceinline__ int small_div(int a, int d) {
    return (int)(((float)a + 0.5f) * __builtin_amdgcn_rcpf((float)d));
}

// bits 32..47 of the product of two 24-bit operands (v_mul_hi_u32_u24)
__device__ __forceinline__ uint32_t mulhi_u24(uint32_t a, uint32_t b) {
    return (uint32_t)(((uint64_t)(a & 0xFFFFFFu) * (uint64_t)(b & 0xFFFFFFu)) >> 32);
}

__device__ __forceinline__ uint8_t sat_u8(int v) { return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v)); }

// ---------------------------------------------------------------------------------------------
// K1: level l from level l-1 (chained pyramid, cv::resize INTER_LINEAR 8U fixed point).
// tab: per-level int16 coefficient tables computed on the host with OpenCV's exact float/double
// expressions. Vertical pass: columns < simd_end use the universal-intrinsic rounding
// ((H>>4)*b>>16 summed, +2 >>2), the rest the scalar >>22 form.
// One block = RZ_ROWS output rows x RZ_COLS output columns; the source rows it needs are staged
// in LDS with dword loads; each thread produces 4 adjacent output pixels (one dword store).
// ---------------------------------------------------------------------------------------------
// Tile = up to RZ_TR output rows x RZ_TC output columns (the host shrinks both per level so the
// source window fits): (A) the source window is loaded with one batch of 16-byte chunk loads,
// (B) the horizontal pass H = S[sx]*a0 + S[sx+1]*a1 (exact int) runs once per (source row,
// output column) into LDS, (C) every thread finishes 4 adjacent output pixels of a row from two
// 16-byte H reads and stores them with one dword store.
#define RZ_TR 24
#define RZ_SR 32              // source rows of a tile window (host-checked)
#define RZ_TC 128
#define RZ_SCB 176            // source bytes of a tile window row (host-checked)
#define RZ_LD ((RZ_SR * RZ_SCB / 16 + 255) / 256)  // window 16-byte chunks per thread
#define RZ_TPB 4              // vertically adjacent tiles per block: the next tile's window loads fly
                              // while this tile's passes run
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(7))) void k_resize(const uint8_t* const* imgs, int in_pitch, uint8_t* pyr, int pyr_stride,
                                                const int16_t* __restrict__ tab, OrbGeom g, int l) {
    __shared__ __attribute__((aligned(16))) uint8_t s_src[RZ_SR][RZ_SCB];
    __shared__ __attribute__((aligned(16))) int s_h[RZ_SR][RZ_TC];
    __shared__ int s_ty[RZ_TR][4];
    const OrbLevel& L = g.lv[l];
    const OrbLevel& Ps = g.lv[l - 1];
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y * gridDim.z);
    const int bx = lb % gridDim.x, by = (lb / gridDim.x) % gridDim.y;
    const int b = lb / (gridDim.x * gridDim.y), t = threadIdx.x;
    const int TR = L.rz_rows, TC = L.rz_cols;
    const int x0 = bx * TC, x1 = min(x0 + TC, L.w);
    const int tile0 = by * RZ_TPB, tile1 = min(tile0 + RZ_TPB, (L.h + TR - 1) / TR);
    int spitch;
    gptr_u8 src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l - 1, &spitch);
    uint8_t* dst = pyr + (size_t)b * pyr_stride + L.pyr_off;
    const int16_t* tx = tab + L.tab_x;
    const int16_t* ty = tab + L.tab_y;
    // source columns [sc0, sc1) of the column tile (the same for all of the block's tiles)
    const int sc0 = tx[3 * x0] & ~3;
    const int sc1 = min((int)tx[3 * (x1 - 1)] + 2, Ps.w);
    const int nsc16 = (sc1 - sc0 + 15) >> 4;
    const bool aligned = ((spitch & 3) == 0) && ((((uintptr_t)src) & 3) == 0);
    // this thread's output column for the horizontal pass and its coefficients
    const int hr0 = small_div(t, TC), hx = t - hr0 * TC, hstep = small_div(256, TC);
    const int hdx = min(x0 + hx, x1 - 1);
    const int hsx = tx[3 * hdx] - sc0, ha0 = tx[3 * hdx + 1], ha1 = tx[3 * hdx + 2];
    const bool hlin = hdx < L.xmax;
    // stored horizontal sums: Hs = H << 4 (exact: H < 2^20), for the universal-intrinsic columns
    // masked to (H >> 4) << 8, the operand the vertical pass feeds to v_mul_hi_u32_u24
    const uint32_t hmask = hdx < L.simd_end ? 0xFFFF00u : 0xFFFFFFFFu;
    // window items of this thread: 16-byte chunk i = (r, c) with r = i / nsc16 (reciprocal-exact for
    // i < 2^16); rows < 2^12 and pitches < 2^13, so the offsets are 24-bit products. A chunk that
    // would cross the row's pitch (the last one of a row, the source may be the caller's image) is
    // read as guarded bytes.
    int it_r[RZ_LD], it_off[RZ_LD], it_g[RZ_LD];
    bool it_al[RZ_LD];
#pragma unroll
    for (int u = 0; u < RZ_LD; u++) {
        const int i = t + 256 * u;
        const int r = small_div(i, nsc16), c = i - (int)__umul24((uint32_t)r, (uint32_t)nsc16);
        it_r[u] = r;
        it_off[u] = (int)__umul24((uint32_t)r, RZ_SCB) + 16 * c;
        it_g[u] = sc0 + 16 * c;
        it_al[u] = aligned && sc0 + 16 * c + 16 <= spitch;
    }
    // (A) window of the tile at output rows [y0, y1): source rows [sr0, sr0 + nsr)
    orbfe_u32x4 v[RZ_LD];
    int tyv = 0;
    auto fetch = [&](int y0, int y1, int sr0, int nsr) {
#pragma unroll
        for (int u = 0; u < RZ_LD; u++) {
            if (it_r[u] < nsr) {
                gptr_u8 sp = src + __umul24((uint32_t)(sr0 + it_r[u]), (uint32_t)spitch) + it_g[u];
                if (it_al[u]) {
                    v[u] = *(const ORBFE_GLOBAL orbfe_u32x4*)sp;
                } else {
                    orbfe_u32x4 x = {0u, 0u, 0u, 0u};
                    for (int k = 0; k < 16; k++)
                        if (it_g[u] + k < Ps.w) x[k >> 2] |= (uint32_t)sp[k] << (8 * (k & 3));
                    v[u] = x;
                }
            }
        }
        // (sy, sy + 1, b0 << 8, b1 << 8): the vertical pass multiplies the b's with v_mul_hi_u32_u24
        if (t < 4 * (y1 - y0)) tyv = (int)ty[4 * y0 + t] << ((t & 2) ? 8 : 0);
    };
    int y0 = tile0 * TR, y1 = min(y0 + TR, L.h);
    int sr0 = ty[4 * y0], nsr = ty[4 * (y1 - 1) + 1] - sr0 + 1;
    fetch(y0, y1, sr0, nsr);
    // (C) vertical pass mapping: thread -> (row lane, 4-column group)
    const int ng = TC >> 2, rl = small_div(t, ng), cg = t - rl * ng, rstep = small_div(256, ng);
    const int xq = x0 + 4 * cg;
    const bool vact = rl < rstep && xq < x1;
    // columns < simd_end take the universal-intrinsic rounding; a 4-column group is almost always
    // entirely on one side (one wave-uniform branch, no per-column divergence)
    const bool all_vec = xq + 3 < L.simd_end;
    bool vec[4];
#pragma unroll
    for (int q = 0; q < 4; q++) vec[q] = xq + q < L.simd_end;
    for (int tile = tile0; tile < tile1; tile++) {
#pragma unroll
        for (int u = 0; u < RZ_LD; u++)
            if (it_r[u] < nsr) *(orbfe_u32x4*)(&s_src[0][0] + it_off[u]) = v[u];
        if (t < 4 * (y1 - y0)) (&s_ty[0][0])[t] = tyv;
        SYNC();
        const int cy0 = y0, cy1 = y1, csr0 = sr0, cnsr = nsr;
        if (tile + 1 < tile1) {   // the next tile's window loads overlap this tile's passes
            y0 = y1;
            y1 = min(y0 + TR, L.h);
            sr0 = ty[4 * y0];
            nsr = ty[4 * (y1 - 1) + 1] - sr0 + 1;
            fetch(y0, y1, sr0, nsr);
        }
        // (B) horizontal pass
        if (hr0 < hstep) {
            // beyond xmax the reference takes S[sx] * 2048: a0 = 2048, a1 = 0 gives it branch-free
            // (the byte at sx + 1 is inside the LDS window and multiplied by 0); 24-bit multiplies
            // are exact (coefficients <= 2048). A plain loop: unrolling it measured slower.
            const uint32_t a0 = (hlin ? (uint32_t)ha0 : 2048u) << 4, a1 = (hlin ? (uint32_t)ha1 : 0u) << 4;
            for (int r = hr0; r < cnsr; r += hstep) {
                const uint32_t p0 = s_src[r][hsx], p1 = s_src[r][hsx + 1];
                s_h[r][hx] = (int)((__umul24(p0, a0) + __umul24(p1, a1)) & hmask);
            }
        }
        SYNC();
        // (C) vertical pass
        if (vact) {
            for (int dy = cy0 + rl; dy < cy1; dy += rstep) {
                const int* tyr = s_ty[dy - cy0];
                const int r0 = tyr[0] - csr0, r1 = tyr[1] - csr0;
                const uint32_t b0s = (uint32_t)tyr[2], b1s = (uint32_t)tyr[3];   // coefficients in [0, 2048], << 8
                const int4 H0 = *(const int4*)&s_h[r0][4 * cg];
                const int4 H1 = *(const int4*)&s_h[r1][4 * cg];
                const uint32_t h0[4] = {(uint32_t)H0.x, (uint32_t)H0.y, (uint32_t)H0.z, (uint32_t)H0.w};
                const uint32_t h1[4] = {(uint32_t)H1.x, (uint32_t)H1.y, (uint32_t)H1.z, (uint32_t)H1.w};
                // universal-intrinsic columns: ((H >> 4) * b) >> 16 = mul_hi_u24((H >> 4) << 8, b << 8).
                // No saturation is needed: a0 + a1 and b0 + b1 are at most 2049 (independently rounded
                // coefficients), so H >> 4 <= 32655 and both forms are <= 255 (1020 + 2 >> 2; and
                // (522495 * 2049 + 2^21) >> 22).
                uint32_t packed = 0;
                if (all_vec) {
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t vv = (mulhi_u24(h0[q], b0s) + mulhi_u24(h1[q], b1s) + 2) >> 2;
                        packed |= vv << (8 * q);
                    }
                } else {
                    const uint32_t b0 = b0s >> 8, b1 = b1s >> 8;
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const uint32_t vs = (mulhi_u24(h0[q], b0s) + mulhi_u24(h1[q], b1s) + 2) >> 2;
                        const uint32_t vl = (__umul24(h0[q] >> 4, b0) + __umul24(h1[q] >> 4, b1) + (1u << 21)) >> 22;
                        packed |= (vec[q] ? vs : vl) << (8 * q);
                    }
                }
                uint8_t* dp = dst + (size_t)dy * L.pitch + xq;
                if (xq + 4 <= x1) {
                    *(uint32_t*)dp = packed;
                } else {
                    for (int q = 0; q < 4 && xq + q < x1; q++) dp[q] = (uint8_t)(packed >> (8 * q));
                }
            }
        }
        SYNC();   // s_src / s_h / s_ty are refilled for the next tile
    }
}

// ---------------------------------------------------------------------------------------------
// K1b: the same level build as k_resize (same tables, xmax and simd_end rules, bit-identical
// output), streamed by rows with no LDS and no barrier. One wave owns a strip of 256 output
// columns (4 adjacent ones per lane) and a chunk of rs_rows output rows, and walks the chunk's
// source rows in order:
//  - a source row is 3 aligned dwords per lane from (sx_0 & ~3), the window holding the byte pairs
//    (S[sx_q], S[sx_q + 1]) of the lane's 4 columns; RS_D rows of loads are in flight;
//  - the horizontal sum of a column is one v_perm (the byte pair as u16x2) and one
//    v_dot2_u32_u16 with the packed coefficients (a0 << 4, a1 << 4): H << 4, as k_resize stores it;
//  - an output row is finished when its second source row is in (rows s - 1, s);
//  - every row step stores exactly one dword per lane, unconditionally (a step that finishes no
//    output row, and a lane past the width, store to the image's slack area): with a static store
//    count per step the compiler waits for a row's loads without draining later stores.
// Host-checked per level (OrbLevel::rs_ok): columns 0, 1 take their pair from bytes 0..7 of the
// window, columns 2, 3 from bytes 2..9; every output row reads rows (s - 1, s) for distinct s (the
// table never clips). Bytes at or past the source width only ever meet a zero coefficient, so a
// dword that would cross the row pitch is read from the row's last dword instead.
// ---------------------------------------------------------------------------------------------
#define RS_D 5               // rows of loads in flight per wave = RS_D - 1 (the loop body's unroll;
                             // with the dwordx3 loads: 2 / 3 / 5 / 7 -> 729 / 676 / 637 / 675 us per
                             // 1024 images, 7 costs a wave per SIMD)
#define RS_ROWS 48           // output rows per wave (<= 64: one table row per lane; 16 / 32 / 48 / 64
                             // with RS_D 5: 637 / 613 / 592 / 615 us per 1024 images)
#define RS_COLS 256          // output columns per wave strip
typedef unsigned short orbfe_ushort2_rs __attribute__((ext_vector_type(2)));
#define RS_WPB 4   // waves per block (1 / 2 / 4 measured equal: r03_kernel_ab.txt item 24)
// one wave's item of k_resize_s (image b, level l, item = chunk * nstrips + strip)
__device__ __forceinline__ void resize_s_item(const uint8_t* const* imgs, int in_pitch, uint8_t* pyr, int pyr_stride,
                                              const int16_t* __restrict__ tab, const OrbGeom& g, int l, int nstrips,
                                              int item, int b) {
    const OrbLevel& L = g.lv[l];
    const int lane = lane_id();
    const int chunk = item / nstrips, strip = item - chunk * nstrips;
    const int y0 = chunk * L.rs_rows, y1 = min(y0 + L.rs_rows, L.h);
    int spitch;
    gptr_u8 src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l - 1, &spitch);
    uint8_t* dst = pyr + (size_t)b * pyr_stride + L.pyr_off;
    const int16_t* tx = tab + L.tab_x;
    const int16_t* ty = tab + L.tab_y;
    const int xq = strip * RS_COLS + 4 * lane;
    const bool act = xq < L.w;
    // the lane's columns: v_perm selectors, packed coefficients, stored-sum masks
    const int base = tx[3 * min(xq, L.w - 1)] & ~3;
    uint32_t sel[4], coef[4], hmask[4];
    bool vec[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int x = min(xq + q, L.w - 1);
        const bool lin = x < L.xmax;
        const uint32_t a0 = lin ? (uint32_t)tx[3 * x + 1] : 2048u, a1 = lin ? (uint32_t)tx[3 * x + 2] : 0u;
        const uint32_t off = (uint32_t)(tx[3 * x] - base) - (q >= 2 ? 2u : 0u);
        sel[q] = 0x0c000c00u | (off & 7u) | (((off + 1u) & 7u) << 16);
        coef[q] = (a0 << 4) | (a1 << 20);
        vec[q] = x < L.simd_end;
        hmask[q] = vec[q] ? 0xFFFF00u : 0xFFFFFFFFu;
    }
    const bool lv_all = !act || (vec[0] && vec[1] && vec[2] && vec[3]);
    // the chunk's vertical table rows, one per lane: (sy + 1, b0 << 8, b1 << 8) of row y0 + lane
    int t_s0 = 0, t_r1 = 0, t_b0 = 0, t_b1 = 0;
    if (y0 + lane < y1) {
        const int16_t* tr = ty + 4 * (y0 + lane);
        t_s0 = tr[0];
        t_r1 = tr[1];
        t_b0 = (int)tr[2] << 8;
        t_b1 = (int)tr[3] << 8;
    }
    const int s_lo = __builtin_amdgcn_readfirstlane(t_s0);
    const int s_hi = ty[4 * (y1 - 1) + 1];
    int y = y0;
    int r1 = __builtin_amdgcn_readfirstlane(t_r1);
    uint32_t b0s = (uint32_t)__builtin_amdgcn_readfirstlane(t_b0), b1s = (uint32_t)__builtin_amdgcn_readfirstlane(t_b1);
    uint8_t* drow = dst + (size_t)y0 * L.pitch + xq;
    uint32_t* slack = (uint32_t*)(pyr + (size_t)b * pyr_stride + g.pyr_slack) + lane;
    uint32_t Hp[4] = {0u, 0u, 0u, 0u};
    // one source row s (window dwords w0..w2): its horizontal sums, then the output row whose
    // second source row is s, if any
    auto step = [&](int s, uint32_t w0, uint32_t w1, uint32_t w2) {
        // bytes 2..9 of the window for columns 2, 3
        const uint32_t c0 = __builtin_amdgcn_alignbyte(w1, w0, 2u), c1 = __builtin_amdgcn_alignbyte(w2, w1, 2u);
        uint32_t Hc[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t pr = q < 2 ? __builtin_amdgcn_perm(w1, w0, sel[q]) : __builtin_amdgcn_perm(c1, c0, sel[q]);
            Hc[q] = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2_rs, pr),
                                           __builtin_bit_cast(orbfe_ushort2_rs, coef[q]), 0u, false) &
                    hmask[q];
        }
        const bool fin = r1 == s;   // wave-uniform: a step that finishes no row skips the vertical pass
        uint32_t packed = 0;
        if (fin) {
#pragma unroll
            for (int q = 0; q < 4; q++)
                packed |= ((mulhi_u24(Hp[q], b0s) + mulhi_u24(Hc[q], b1s) + 2u) >> 2) << (8 * q);
            if (!lv_all) {   // the lane holding the level's scalar-tail columns (>= simd_end)
                // (H0 b0 + H1 b1 + 2^21) >> 22 on the stored 16 H (unmasked for these columns):
                // (16 H0 b0 + 16 H1 b1 + 2^25) >> 26 in 64 bits, the same floor
                const uint64_t b0 = b0s >> 8, b1 = b1s >> 8;
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const uint32_t vl = (uint32_t)(((uint64_t)Hp[q] * b0 + (uint64_t)Hc[q] * b1 + (1ull << 25)) >> 26);
                    const uint32_t m = vec[q] ? 0u : 0xFFu << (8 * q);
                    packed = (packed & ~m) | ((vl << (8 * q)) & m);
                }
            }
        }
        // a whole dword even for the level's last, partial group: the bytes past the width land
        // in the row's pitch padding, which nothing reads as pixels
        *(uint32_t*)(fin && act ? (uint32_t*)drow : slack) = packed;
        if (fin) {
            drow += L.pitch;
            if (++y == y1) {
                r1 = -1;
            } else {
                const int k = y - y0;
                r1 = __builtin_amdgcn_readlane(t_r1, k);
                b0s = (uint32_t)__builtin_amdgcn_readlane(t_b0, k);
                b1s = (uint32_t)__builtin_amdgcn_readlane(t_b1, k);
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) Hp[q] = Hc[q];
    };
    // dword loads: the host launches this kernel only on 4-byte aligned rows (the pyramid always;
    // level 0 when the caller's images are, else k_resize builds level 1). A loop over blocks of
    // RS_D rows, each unrolled (static buffer indices, small code). A row's buffer is reloaded right
    // after its step, RS_D rows ahead, unconditionally (clamped to the last row; the steps past the
    // last row finish no output row), so no buffer is copied. Row address = the scalar row base +
    // a 32-bit lane offset (the SGPR-base load form, no 64-bit address arithmetic per load). The
    // prologue issues the loop's (store, loads) pattern per row, in order, so the loop entry and
    // its back edge present the same outstanding counts.
    const uint32_t win = (uint32_t)min(base, spitch - 4);
    // buffer loads: descriptor over the source level (rows of spitch bytes, the same bytes the
    // clamped offsets always read), row offset s * spitch in soffset
    const uint64_t sp = (uint64_t)(uintptr_t)src;
    const uint32_t sp_lo = __builtin_amdgcn_readfirstlane((uint32_t)sp), sp_hi = __builtin_amdgcn_readfirstlane((uint32_t)(sp >> 32));
    const int sbytes = __builtin_amdgcn_readfirstlane(spitch * g.lv[l - 1].h);
    const __amdgpu_buffer_rsrc_t srd =
        __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)sp_hi << 32) | sp_lo), (short)0, sbytes, 0x00020000);
    auto ld = [&](int s, uint32_t (&w)[3]) {
        const int so = __builtin_amdgcn_readfirstlane(s * spitch);
        // one 12-byte load from the window's first dword; a window that runs past the row's pitch
        // reads the next row's first bytes (or zeros past the level: the descriptor's range
        // check), which only ever meet zero coefficients
        typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
        const u32x3 v = __builtin_bit_cast(u32x3, __builtin_amdgcn_raw_buffer_load_b96(srd, (int)win, so, 0));
        w[0] = v.x; w[1] = v.y; w[2] = v.z;
    };
    uint32_t buf[RS_D][3];
#pragma unroll
    for (int d = 0; d < RS_D; d++) {
        *slack = 0u;
        ld(min(s_lo + d, s_hi), buf[d]);
        __builtin_amdgcn_sched_barrier(0);
    }
    for (int sb = s_lo; sb <= s_hi; sb += RS_D) {
#pragma unroll
        for (int d = 0; d < RS_D; d++) {
            step(sb + d, buf[d][0], buf[d][1], buf[d][2]);
            ld(min(sb + RS_D + d, s_hi), buf[d]);
            // keep the loads here: the scheduler would otherwise sink them next to their use
            __builtin_amdgcn_sched_barrier(0);
        }
    }
}
__global__ __launch_bounds__(64 * RS_WPB) void k_resize_s(const uint8_t* const* imgs, int in_pitch, uint8_t* pyr,
                                                  int pyr_stride, const int16_t* __restrict__ tab, OrbGeom g, int l,
                                                  int nstrips, int nitems) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int bx = lb % gridDim.x, b = lb / gridDim.x;
    const int item = bx * RS_WPB + wave;
    if (item >= nitems) return;
    resize_s_item(imgs, in_pitch, pyr, pyr_stride, tab, g, l, nstrips, item, b);
}

// ---------------------------------------------------------------------------------------------
// K1c: the whole pyramid (levels 1 .. nlevels-1) in ONE launch for small batches, where the chain
// of per-level launches is latency-bound (each ~5 us for a few thousand pixels). One block per
// (tile, image): a tile owns a rectangle of every level (the same fraction of each level, columns
// on multiples of 4) and builds the rectangle it NEEDS at each level (what it owns plus the source
// cone of its higher levels, computed on the host from the same coefficient tables), level by
// level in LDS; only owned dwords are stored. Per pixel the arithmetic is k_resize's (H = S[sx]
// a0 + S[sx+1] a1, a0 = 2048 / a1 = 0 past xmax; the universal-intrinsic rounding below simd_end,
// the >> 22 form above), so the levels are bit-identical to the chained launches. The block reads
// its tile record (header + relative column / row tables) and its level-0 window in one batch of
// loads, then touches global memory only to store.
// Record (dwords): per level l a 5-dword header {ax0 | ax1 << 16, ny0 | ny1 << 16, ox0 | ox1 << 16,
// oy0 | oy1 << 16, coloff | rowoff << 16}; per level >= 1 the needed columns (sx - ax0(l-1) |
// min(sx + 1, last) - ax0(l-1) << 15 | simd << 30, a0 | a1 << 16) and rows (s0 - ny0(l-1) |
// s1 - ny0(l-1) << 16, b0 | b1 << 16).
// ---------------------------------------------------------------------------------------------
#ifndef PYR_NT
#define PYR_NT 1024   // threads per tile block (512 / 256: +7 % / +29 % at 48x40 tiles, tools/gpu_pyr_ab.sh)
#endif
#define PYR_RU 2     // record 16-byte chunks per thread
#ifndef PYR_U0
#define PYR_U0 4     // level-0 window dwords per thread
#endif
__global__ __launch_bounds__(PYR_NT) void k_pyramid(const uint8_t* const* imgs, int in_pitch, uint8_t* pyr, int pyr_stride,
                                                    OrbGeom g, const uint32_t* __restrict__ ptile, int pt_stride, int cap,
                                                    int al0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_pyr[];
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int tile = lb % gridDim.x, b = lb / gridDim.x;
    const int tid = threadIdx.x;
    uint32_t* srec = (uint32_t*)smem_pyr;
    uint8_t* buf0 = smem_pyr + (size_t)pt_stride * 4;
    uint8_t* buf1 = buf0 + cap;
    const uint32_t* rec = ptile + (size_t)tile * pt_stride;
    const uint32_t hx = rec[0], hy = rec[1];
    const int ax0 = (int)(hx & 0xffff), ax1 = (int)(hx >> 16), ny0 = (int)(hy & 0xffff), ny1 = (int)(hy >> 16);
    const int dpr = (ax1 - ax0) >> 2, items0 = dpr * (ny1 - ny0);
    const int W0 = g.lv[0].w;
    gptr_u8 src = as_global(imgs[b]);
    // every load of the block issued before any store
    orbfe_u32x4 rv[PYR_RU];
#pragma unroll
    for (int u = 0; u < PYR_RU; u++) {
        const int i = tid + PYR_NT * u;
        if (i < (pt_stride >> 2)) rv[u] = ((const ORBFE_GLOBAL orbfe_u32x4*)rec)[i];
    }
    uint32_t wv[PYR_U0];
#pragma unroll
    for (int u = 0; u < PYR_U0; u++) {
        const int i = tid + PYR_NT * u;
        wv[u] = 0u;
        if (i < items0) {
            const int r = small_div(i, dpr), c = i - r * dpr;
            const int x = ax0 + 4 * c;
            gptr_u8 sp = src + (size_t)(ny0 + r) * in_pitch + x;
            if (al0 && x + 4 <= W0) {
                wv[u] = *(const ORBFE_GLOBAL uint32_t*)sp;
            } else {
                uint32_t w = 0u;
                for (int k = 0; k < 4; k++)
                    if (x + k < W0) w |= (uint32_t)sp[k] << (8 * k);
                wv[u] = w;
            }
        }
    }
#pragma unroll
    for (int u = 0; u < PYR_RU; u++) {
        const int i = tid + PYR_NT * u;
        if (i < (pt_stride >> 2)) ((orbfe_u32x4*)srec)[i] = rv[u];
    }
#pragma unroll
    for (int u = 0; u < PYR_U0; u++) {
        const int i = tid + PYR_NT * u;
        if (i < items0) ((uint32_t*)buf0)[i] = wv[u];   // rows of (ax1 - ax0) bytes, dword-packed
    }
    SYNC();
    for (int l = 1; l < g.nlevels; l++) {
        const OrbLevel& L = g.lv[l];
        const uint32_t* hp = srec + 5 * (l - 1);
        const uint32_t* hl = srec + 5 * l;
        const int sw = (int)(hp[0] >> 16) - (int)(hp[0] & 0xffff);
        const int dx0 = (int)(hl[0] & 0xffff), dw = (int)(hl[0] >> 16) - dx0;
        const int dy0 = (int)(hl[1] & 0xffff), drows = (int)(hl[1] >> 16) - dy0;
        const int ox0 = (int)(hl[2] & 0xffff), ox1 = (int)(hl[2] >> 16);
        const int oy0 = (int)(hl[3] & 0xffff), oy1 = (int)(hl[3] >> 16);
        const uint2* cols = (const uint2*)(srec + (hl[4] & 0xffff));
        const uint2* rows = (const uint2*)(srec + (hl[4] >> 16));
        const uint8_t* sb = (l & 1) ? buf0 : buf1;   // level l - 1
        uint8_t* db = (l & 1) ? buf1 : buf0;
        uint8_t* gdst = pyr + (size_t)b * pyr_stride + L.pyr_off;
        const int ngr = dw >> 2, items = ngr * drows;
        for (int i = tid; i < items; i += PYR_NT) {
            const int r = small_div(i, ngr), gi = i - r * ngr;
            const uint2 rw = rows[r];
            const uint8_t* s0 = sb + (int)(rw.x & 0xffff) * sw;
            const uint8_t* s1 = sb + (int)(rw.x >> 16) * sw;
            const uint32_t b0 = rw.y & 0xffff, b1 = rw.y >> 16;
            uint32_t packed = 0;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint2 cw = cols[4 * gi + q];
                const int x0 = (int)(cw.x & 0x7fff), x1 = (int)((cw.x >> 15) & 0x7fff);
                const uint32_t a0 = cw.y & 0xffff, a1 = cw.y >> 16;
                const uint32_t H0 = (uint32_t)s0[x0] * a0 + (uint32_t)s0[x1] * a1;
                const uint32_t H1 = (uint32_t)s1[x0] * a0 + (uint32_t)s1[x1] * a1;
                const uint32_t v = (cw.x >> 30)
                                       ? (mulhi_u24((H0 << 4) & 0xFFFF00u, b0 << 8) + mulhi_u24((H1 << 4) & 0xFFFF00u, b1 << 8) + 2u) >> 2
                                       : (H0 * b0 + H1 * b1 + (1u << 21)) >> 22;
                packed |= v << (8 * q);
            }
            *(uint32_t*)(db + r * dw + 4 * gi) = packed;
            const int x = dx0 + 4 * gi, y = dy0 + r;
            if (x >= ox0 && x < ox1 && y >= oy0 && y < oy1) *(uint32_t*)(gdst + (size_t)y * L.pitch + x) = packed;
        }
        SYNC();
    }
}

// Gaussian 7x7 quantised kernel taps (the blur itself is fused into k_describe, K5).
struct BlurKernel { int k[7]; };

// ---------------------------------------------------------------------------------------------
// K3: FAST-9/16 per cell. One wave per cell, single-wave blocks (FAST_WPB). The cell ROI
// (wCell+6)x(hCell+6) is staged in LDS; the score of every detection pixel is computed ONCE at
// minThFAST (score = M-1 where M = max over 9-arcs of the arc-min contrast, corner iff M > th),
// and per-cell NMS is exact because the ROI ring outside the detection rect is zero. A cell
// emits its survivors with score >= iniThFAST, or all survivors when there are none (the
// reference's FAST(iniTh) -> FAST(minTh) fallback, ORBextractor.cc:826-846). Keys are packed
// x_rel | y_rel<<12 | score<<24 in row-major order (FAST emission order).
// Pass 1 runs FAST's exact necessary test (every 9-arc holds one pixel of each opposite pair
// (k, k+8), k = 0,2,4,6) on all pixels and compacts the candidates; pass 2 scores candidates only.
// ---------------------------------------------------------------------------------------------
typedef short orbfe_short2 __attribute__((ext_vector_type(2)));
// Pixels as f16 denormals v * 2^-24 (the u16 bit pattern of the byte; the kernels keep f16
// denormals, float_denorm_mode_16_64 = 3): every value, threshold offset and difference FAST forms
// is an integer multiple of 2^-24 below 2048 * 2^-24, exact in f16, and gfx950's 3-input
// v_pk_minimum3_f16 / v_pk_maximum3_f16 halve the min/max networks.
typedef _Float16 orbfe_half2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ orbfe_half2 as_h2(uint32_t w) { return __builtin_bit_cast(orbfe_half2, w); }
__device__ __forceinline__ uint32_t h2_bits(orbfe_half2 h) { return __builtin_bit_cast(uint32_t, h); }
__device__ __forceinline__ orbfe_half2 hmin(orbfe_half2 a, orbfe_half2 b) { return __builtin_elementwise_minimum(a, b); }
__device__ __forceinline__ orbfe_half2 hmax(orbfe_half2 a, orbfe_half2 b) { return __builtin_elementwise_maximum(a, b); }
// bytes 0 and 2 (sel 0x0c020c00) or 1 and 3 (sel 0x0c030c01) of w as f16 byte * 2^-24
__device__ __forceinline__ orbfe_half2 px_h2(uint32_t w, uint32_t sel) {
    return as_h2(__builtin_amdgcn_perm(0u, w, sel));
}

typedef unsigned short orbfe_ushort2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ orbfe_ushort2 as_us2(uint32_t w) { return __builtin_bit_cast(orbfe_ushort2, w); }
// M = max over the 16 arcs of 9 contiguous ring pixels of max(min d, min -d), d_k = v - ring_k.
// Both signs ride in one packed int16x2 lane so every min/max is one v_pk_{min,max}_i16.
__device__ __forceinline__ int fast_M(const uint8_t* im, int stride, int x, int y) {
    const uint8_t* q = im + y * stride + x;
    const int v = q[0];
    orbfe_short2 P[16];
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const short d = (short)(v - (int)q[c_ring_dy[k] * stride + c_ring_dx[k]]);
        P[k] = orbfe_short2{d, (short)-d};
    }
    orbfe_short2 m2[16], m4[16];
#pragma unroll
    for (int k = 0; k < 16; k++) m2[k] = __builtin_elementwise_min(P[k], P[(k + 1) & 15]);
#pragma unroll
    for (int k = 0; k < 16; k++) m4[k] = __builtin_elementwise_min(m2[k], m2[(k + 2) & 15]);
    orbfe_short2 best = orbfe_short2{(short)-1000, (short)-1000};
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const orbfe_short2 m9 = __builtin_elementwise_min(__builtin_elementwise_min(m4[k], m4[(k + 4) & 15]), P[(k + 8) & 15]);
        best = __builtin_elementwise_max(best, m9);
    }
    return max((int)best.x, (int)best.y);
}

#define FAST_PF 4
//             prefetched 16-byte chunks per lane (rows / rows-per-load: 2 at W = 35)
struct FastCell {
    int l, local, ci, cj, r0, c0, rows, cols, pitch;
    gptr_u8 src;
};
__device__ __forceinline__ void fast_cell_rect(FastCell& f, const OrbLevel& L) {
    const int maxBX = L.w - ORBFE_MINB, maxBY = L.h - ORBFE_MINB;
    f.r0 = ORBFE_MINB + f.ci * L.h_cell;
    f.c0 = ORBFE_MINB + f.cj * L.w_cell;
    const int r1 = min(f.r0 + L.h_cell + 6, maxBY), c1 = min(f.c0 + L.w_cell + 6, maxBX);
    // the reference skips such cells (ORBextractor.cc:810,819); never true for its grid, kept for parity
    const bool skip = (f.r0 >= maxBY - 3) || (f.c0 >= maxBX - 6);
    f.rows = skip ? 0 : r1 - f.r0;
    f.cols = skip ? 0 : c1 - f.c0;
}
__device__ __forceinline__ FastCell fast_cell(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                              int pyr_stride, const OrbGeom& g, int b, int c) {
    FastCell f;
    int l = 0;
    while (l + 1 < g.nlevels && c >= g.lv[l + 1].cell_base) l++;
    const OrbLevel& L = g.lv[l];
    f.l = l;
    f.local = c - L.cell_base;
    f.ci = f.local / L.n_cols;
    f.cj = f.local - f.ci * L.n_cols;
    fast_cell_rect(f, L);
    f.src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l, &f.pitch);
    return f;
}
// the cell after f in cell order (no divisions: the wave walks consecutive cells)
__device__ __forceinline__ FastCell fast_cell_next(const FastCell& f, const uint8_t* const* imgs, int in_pitch,
                                                   const uint8_t* pyr, int pyr_stride, const OrbGeom& g, int b) {
    FastCell n = f;
    n.local++;
    if (++n.cj == g.lv[n.l].n_cols) {
        n.cj = 0;
        if (++n.ci == g.lv[n.l].n_rows) {
            n.l++;
            n.local = n.ci = 0;
            n.src = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, n.l, &n.pitch);
        }
    }
    fast_cell_rect(n, g.lv[n.l]);
    return n;
}
// LDS layout of a cell: rows of RS = 16 * ceil(nd / 4) bytes (nd = ng + 2 dwords are read, ng =
// ceil(dw / 4) pixel groups; the rest of a row is padding), byte j of a row = ROI column j - 1, so
// every row starts 16-byte aligned and a realigned chunk is one ds_write_b128. A row is loaded as
// cpr 16-byte chunks from the aligned dword A0 = (c0 - 1) & ~3 (cpr = ceil((nd + 1) / 4): the
// written chunks plus the dword the realignment takes from the next one), one chunk per lane, rpl
// rows per load; the realigned fourth dword of a chunk takes the next lane's first dword (a DPP
// wave_shl; for the last chunk of a row that is padding). Reads end at most 20 bytes past c1 <=
// w - 16, inside the next row (ROI rows end 17 rows above the last image row).
__device__ __forceinline__ void fast_geom(const FastCell& f, int* ng, int* nd, int* cpr, int* rpl) {
    const int dw = f.cols - 6, dh = f.rows - 6;
    *ng = (dw > 0 && dh > 0) ? (dw + 3) >> 2 : 0;
    *nd = *ng + 2;
    *cpr = (*nd + 4) >> 2;
    *rpl = small_div(64, *cpr);
}
// row stride of the cell's LDS image and score map in dwords
__device__ __forceinline__ int fast_rsd(int nd) { return 4 * ((nd + 3) >> 2); }
__device__ __forceinline__ orbfe_u32x4 fast_chunk(gptr_u8 rp, bool al) {
    if (al) return *(const ORBFE_GLOBAL orbfe_u32x4*)rp;
    orbfe_u32x4 q = {0u, 0u, 0u, 0u};
    for (int k = 0; k < 16; k++) q[k >> 2] |= (uint32_t)rp[k] << (8 * (k & 3));
    return q;
}
__device__ __forceinline__ void fast_prefetch(const FastCell& f, int lane, orbfe_u32x4 (&pf)[FAST_PF]) {
    int ng, nd, cpr, rpl;
    fast_geom(f, &ng, &nd, &cpr, &rpl);
    if (!ng) return;
    const int sy = small_div(lane, cpr), st = lane - sy * cpr;
    if (sy >= rpl) return;
    const int A0 = (f.c0 - 1) & ~3;
    const bool al = (f.pitch & 3) == 0 && ((((uintptr_t)f.src) & 3) == 0);
    gptr_u8 base = f.src + (size_t)f.r0 * f.pitch + A0 + 16 * st;
#pragma unroll
    for (int u = 0; u < FAST_PF; u++) {
        const int y = sy + u * rpl;
        if (y < f.rows) pf[u] = fast_chunk(base + (size_t)y * f.pitch, al);
    }
}
// realign a chunk by sal bytes (the DPP needs every lane) and store it as row y's chunk st
__device__ __forceinline__ void fast_stage_chunk(uint8_t* s_img, const orbfe_u32x4& q, int sal, int y, int st,
                                                 int rs, bool ok) {
    const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q.x, 0x130, 0xf, 0xf, false);
    const orbfe_u32x4 w = {__builtin_amdgcn_alignbyte(q.y, q.x, (uint32_t)sal), __builtin_amdgcn_alignbyte(q.z, q.y, (uint32_t)sal),
                           __builtin_amdgcn_alignbyte(q.w, q.z, (uint32_t)sal), __builtin_amdgcn_alignbyte(nx, q.w, (uint32_t)sal)};
    if (ok) *(orbfe_u32x4*)(s_img + y * rs + 16 * st) = w;
}

// Stage a prefetched cell ROI into the wave's LDS image and zero the score map (rows < dh + 2);
// ends with WAVE_SYNC.
__device__ __forceinline__ void fast_stage_cell(const FastCell& cur, const orbfe_u32x4 (&pf)[FAST_PF], uint8_t* s_img,
                                                uint8_t* s_sc, int lane) {
    int ng, nd, cpr, rpl;
    fast_geom(cur, &ng, &nd, &cpr, &rpl);
    const int dh = cur.rows - 6;
    if (ng) {
        const int sy = small_div(lane, cpr), st = lane - sy * cpr, sal = (cur.c0 - 1) & 3;
        const int rs = 4 * fast_rsd(nd), nw = (nd + 3) >> 2;
        const bool wr = sy < rpl && st < nw;
#pragma unroll
        for (int u = 0; u < FAST_PF; u++) {
            const int y = sy + u * rpl;
            fast_stage_chunk(s_img, pf[u], sal, y, st, rs, wr && y < cur.rows);
        }
        // rows beyond the prefetch window (only very tall cells of tiny levels): direct loads with a
        // wave-uniform trip count (the DPP needs every lane)
        if (FAST_PF * rpl < cur.rows) {
            const bool al = (cur.pitch & 3) == 0 && ((((uintptr_t)cur.src) & 3) == 0);
            gptr_u8 base = cur.src + (size_t)cur.r0 * cur.pitch + ((cur.c0 - 1) & ~3) + 16 * st;
            for (int y0 = FAST_PF * rpl; y0 < cur.rows; y0 += rpl) {
                const int y = y0 + sy;
                const bool ok = sy < rpl && y < cur.rows;
                orbfe_u32x4 q = {0u, 0u, 0u, 0u};
                if (ok) q = fast_chunk(base + (size_t)y * cur.pitch, al);
                fast_stage_chunk(s_img, q, sal, y, st, rs, ok && st < nw);
            }
        }
        const orbfe_u32x4 z = {0u, 0u, 0u, 0u};
        const int nz = (dh + 2) * (rs >> 4);
        for (int i = lane; i < nz; i += 64) ((orbfe_u32x4*)s_sc)[i] = z;
    }
    WAVE_SYNC();
}

struct FastLds {
    int roi, sc, cor, wave_bytes;   // bytes per wave: ROI image, score map, corner list (+ entries)
};
#define FAST_ENT_BYTES 1024     // entry chunk: 64 groups x <= 8 entries x 2 B

// Detection of one staged cell (both attempts, NMS, emission). NDC = the LDS row stride in dwords
// when known at compile time (0: runtime): every LDS offset of the ring / neighbour reads is then
// an immediate instead of a per-read VALU add.
template <int NDC>
__device__ __forceinline__ void fast_cell_detect(const OrbGeom& g, const FastLds& fl, const FastCell& me, int ng,
                                                 int nd_rt, int dw, int dh, uint8_t* s_img, uint8_t* s_sc,
                                                 uint16_t* s_cor, uint16_t* s_ent, uint32_t* cellkeys, int* cellcnt,
                                                 int b, int c, int lane, int first_attempt = 0) {
    const int nd = NDC ? NDC : fast_rsd(nd_rt);   // row stride in dwords (>= the nd_rt dwords read)
    const int RS = 4 * nd;
    const OrbLevel& L = g.lv[me.l];
    const uint8_t* s_px = s_img + 1;   // ROI pixel (y, x) = s_px[y * RS + x]
    // attempt 0 = FAST at iniThFAST; attempt 1 (only when attempt 0 leaves no NMS survivor) =
    // FAST at minThFAST over a cleared score map: the reference's per-cell fallback
    // (ORBextractor.cc:826-846). Most cells stop after attempt 0, whose candidate set is a
    // fraction of minThFAST's.
    int nsurv = 0;
    uint32_t* out = cellkeys + (size_t)b * g.cellkeys_per_img + L.cellkey_off + (size_t)me.local * L.cell_cap;
    const int xr0 = me.c0 - ORBFE_MINB + 3, yr0 = me.r0 - ORBFE_MINB + 3;
    for (int attempt = first_attempt; attempt < 2; attempt++) {
        const int th = attempt == 0 ? g.ini_th : g.min_th;
        if (attempt) {
            uint32_t* s32z = (uint32_t*)s_sc;
            for (int i = lane; i < (dh + 2) * nd; i += 64) s32z[i] = 0u;
            WAVE_SYNC();
        }
        // pass 1: FAST's exact necessary test (each 9-arc contains one pixel of every opposite
        // pair (k, k+8), k = 0, 2, 4, 6, all of one sign) for 4 pixels per lane in packed u16x2
        // arithmetic (even bytes / odd bytes); candidates compacted row-major as (dy << 8 | dx).
        int ngrp = 0;
        // group records at the tail of the corner list: <= ng * dh of them
        uint32_t* s_grp = (uint32_t*)((uint8_t*)s_cor + fl.cor) - ng * dh;
        if (ng) {
            const int rpi = 64 / ng;
            const int ly = small_div(lane, ng), lg = lane - ly * ng;
            const _Float16 tf = __builtin_bit_cast(_Float16, (unsigned short)th);   // th * 2^-24
            const orbfe_half2 tv = {tf, tf};
            const int valid4 = min(4, dw - 4 * lg);
            // flag bits of pixel k: 2k + 1 = dark possible, 2k = bright possible
            const uint32_t vmask = ly < rpi && valid4 > 0 ? (1u << (2 * valid4)) - 1u : 0u;
            // the test for the lane's 4 pixels of ROI row y + 3
            auto pretest = [&](int y) -> uint32_t {
                if (!(vmask && y < dh)) return 0u;
                // centre pixels k = 0..3 at ROI (y + 3, 4 lg + 3 + k) = byte 4 lg + 4 + k of the row
                const uint8_t* cp = s_img + (y + 3) * RS + 4 * lg + 4;
                const uint32_t cw = *(const uint32_t*)cp;
                // aligned dwords + v_alignbyte: unaligned ds_read_b32 measured 40 % slower for the kernel
                const uint32_t* r0p = (const uint32_t*)cp - 1;   // dword of ROI columns 4 lg - 1 ..
                const uint32_t c0w = r0p[0], c2w = r0p[2];
                // ring samples as (hi, lo, byte shift): the 4 bytes of sample k are bytes s .. s + 3 of
                // hi:lo, so one v_perm per parity picks its even / odd pixels as f16 halves directly
                const uint32_t ph[8] = {0u, 0u, c2w, cw, r0p[2 * nd + 2], r0p[-2 * nd + 1], r0p[-2 * nd + 2], r0p[2 * nd + 1]};
                const uint32_t pl[8] = {r0p[3 * nd + 1], r0p[-3 * nd + 1], cw, c0w,          // (0, 3), (0, -3), (3, 0), (-3, 0)
                                        r0p[2 * nd + 1], r0p[-2 * nd], r0p[-2 * nd + 1], r0p[2 * nd]};   // (2, 2), (-2, -2), (2, -2), (-2, 2)
                constexpr uint32_t psh[8] = {0, 0, 3, 1, 2, 2, 2, 2};
                uint32_t sd[2], sb[2];
#pragma unroll
                for (int par = 0; par < 2; par++) {
                    const uint32_t sel = par ? 0x0c030c01u : 0x0c020c00u;
                    const orbfe_half2 v = px_h2(cw, sel);
                    // dark possible  <=> every pair has a member < v - t <=> max_k min(pair k) < v - t
                    // bright possible <=> every pair has a member > v + t <=> min_k max(pair k) > v + t
                    orbfe_half2 mn[4], mx[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const uint32_t sa = 0x0c000c00u | (psh[2 * k] + par) | ((psh[2 * k] + par + 2) << 16);
                        const uint32_t sb2 = 0x0c000c00u | (psh[2 * k + 1] + par) | ((psh[2 * k + 1] + par + 2) << 16);
                        const orbfe_half2 xa = as_h2(__builtin_amdgcn_perm(ph[2 * k], pl[2 * k], sa));
                        const orbfe_half2 xb = as_h2(__builtin_amdgcn_perm(ph[2 * k + 1], pl[2 * k + 1], sb2));
                        mn[k] = hmin(xa, xb);
                        mx[k] = hmax(xa, xb);
                    }
                    const orbfe_half2 D = hmax(hmax(hmax(mn[0], mn[1]), mn[2]), mn[3]);
                    const orbfe_half2 B = hmin(hmin(hmin(mx[0], mx[1]), mx[2]), mx[3]);
                    // exact differences: the sign bit of each half is the flag
                    sd[par] = h2_bits(D - (v - tv));
                    sb[par] = h2_bits((v + tv) - B);
                }
                // sign bytes -> pixel order (byte k = pixel k), dark at bit 7, bright at bit 6,
                // then gathered into bits 2k + 1 / 2k by one dot product
                const uint32_t A = __builtin_amdgcn_perm(sd[1], sd[0], 0x07030501u);
                const uint32_t Bq = __builtin_amdgcn_perm(sb[1], sb[0], 0x07030501u);
                const uint32_t F = (A & 0x80808080u) | ((Bq >> 1) & 0x40404040u);
                return __builtin_amdgcn_udot4(F >> 6, 0x40100401u, 0u, false) & vmask;
            };
            // 4-pixel groups with any candidate, compacted row-major (iteration-major, then lane
            // order): dy << 7 | dx0 in bits 0-13, flags in bits 16-23 (pixel k: bit 17 + 2k dark,
            // 16 + 2k bright)
            auto compact = [&](int y, uint32_t m8) {
                const unsigned long long gm = __ballot(m8 != 0u);
                if (m8)
                    s_grp[ngrp + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(gm >> 32),
                                                                __builtin_amdgcn_mbcnt_lo((uint32_t)gm, 0u))] =
                        (uint32_t)((y << 7) | (4 * lg)) | (m8 << 16);
                ngrp += __popcll(gm);
            };
            // two row blocks per iteration: both blocks' LDS reads issue before either's compute
            for (int y0 = 0; y0 < dh; y0 += 2 * rpi) {
                const uint32_t ma = pretest(y0 + ly), mb = pretest(y0 + rpi + ly);
                compact(y0 + ly, ma);
                if (y0 + rpi < dh) compact(y0 + rpi + ly, mb);
            }
        }
        WAVE_SYNC();
        // per chunk of 64 groups: expand into entries, one per (pixel, possible sign): dy << 7 |
        // dx, bit 14 = bright, bit 15 = second entry of a pixel (both signs passed; at most one
        // can be a corner); then the exact score of the chunk's entries. Corners are appended in
        // pixel order to the corner list, whose tail holds the group records still to come
        // (cor_bytes >= 8 * groups + 256 keeps the two apart).
        int ncorner = 0;
        for (int g0 = 0; g0 < ngrp; g0 += 64) {
            int nent = 0;
            {
                const int gi = g0 + lane;
                const uint32_t rec = gi < ngrp ? s_grp[gi] : 0u;
                const int cnt = __popc(rec >> 16);   // <= 8 entries per group
                const int incl = wave_incl_scan_dpp(cnt);
                int pos = incl - cnt;
                const int packed = (int)(rec & 0x3FFFu);
                // branch-free per entry: every potential entry is stored, the absent ones to this
                // lane's own (already read) group record slot, which nothing reads again
                uint16_t* trash = (uint16_t*)(s_grp + gi);
                if (rec != 0u)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint32_t di = (rec >> (17 + 2 * i)) & 1u, bi = (rec >> (16 + 2 * i)) & 1u;
                    *(di ? s_ent + pos : trash) = (uint16_t)(packed + i);
                    pos += (int)di;
                    *(bi ? s_ent + pos : trash) = (uint16_t)((packed + i) | 0x4000 | (di << 15));
                    pos += (int)bi;
                }
                nent = __builtin_amdgcn_readlane(incl, 63);
            }
            WAVE_SYNC();
            // pass 2: exact score M - 1 (corner iff M > th) of each entry for its sign only, two
            // entries per lane in packed f16 (pixels as 1024 + v, exact signed differences)
            for (int j0 = 0; j0 < nent; j0 += 128) {
                const int j = j0 + 2 * lane;
                const uint32_t e2 = j < nent ? ((const uint32_t*)s_ent)[j >> 1] : 0u;
                const bool ok0 = j < nent, ok1 = j + 1 < nent;
                const uint32_t e0 = e2 & 0xFFFFu, e1 = ok1 ? e2 >> 16 : e0;
                const uint8_t* q0 = s_px + (((e0 >> 7) & 127) + 3) * RS + (e0 & 127) + 3;
                const uint8_t* q1 = s_px + (((e1 >> 7) & 127) + 3) * RS + (e1 & 127) + 3;
                // the two entries' pixels as one u16x2 = f16 denormals v * 2^-24 (f16 denormals are
                // kept, float_denorm_mode_16_64 = 3; every sum / difference here is exact)
                const orbfe_half2 v2 = as_h2(__builtin_bit_cast(uint32_t, orbfe_ushort2{q0[0], q1[0]}));
                // d = s (v - x) with s = +1 (dark) / -1 (bright) per half, one exact fma per ring pixel
                const uint32_t bmask = ((e0 & 0x4000u) ? 0x00008000u : 0u) | ((e1 & 0x4000u) ? 0x80000000u : 0u);
                const orbfe_half2 ns = as_h2(0xBC00BC00u ^ bmask);   // -s
                const orbfe_half2 sv = as_h2(h2_bits(v2) ^ bmask);   // s v
                // ring reads from the top-left corner of the 7x7 box: non-negative immediate offsets
                const uint8_t* t0 = q0 - 3 * RS - 3;
                const uint8_t* t1 = q1 - 3 * RS - 3;
                orbfe_half2 P[16];
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int o = (kRingDy[k] + 3) * RS + kRingDx[k] + 3;
                    const orbfe_half2 x2 = as_h2(__builtin_bit_cast(uint32_t, orbfe_ushort2{t0[o], t1[o]}));
                    P[k] = __builtin_elementwise_fma(x2, ns, sv);
                }
                // M = max over the 16 arcs of the arc minimum (signed: an arc with a minimum <= 0
                // never makes a corner, th >= 0): arc k = runs k, k + 3, k + 6 of three, each
                // minimum one v_pk_minimum3_f16
                orbfe_half2 m3[16], m9[16];
#pragma unroll
                for (int k = 0; k < 16; k++) m3[k] = hmin(hmin(P[k], P[(k + 1) & 15]), P[(k + 2) & 15]);
#pragma unroll
                for (int k = 0; k < 16; k++) m9[k] = hmin(hmin(m3[k], m3[(k + 3) & 15]), m3[(k + 6) & 15]);
                // maximum of the 16 arc minima as a tree of v_pk_maximum3_f16 (8 instead of 15)
                orbfe_half2 r[6];
#pragma unroll
                for (int k = 0; k < 5; k++) r[k] = hmax(hmax(m9[3 * k], m9[3 * k + 1]), m9[3 * k + 2]);
                r[5] = m9[15];
                const orbfe_half2 mx = hmax(hmax(hmax(r[0], r[1]), r[2]), hmax(hmax(r[3], r[4]), r[5]));
                // M as an integer: the bits of a non-negative denormal; negative -> no corner
                const uint32_t mb = h2_bits(mx);
                const int bx = (mb & 0x8000u) ? -1 : (int)(mb & 0x7fffu);
                const int by = (mb & 0x80000000u) ? -1 : (int)((mb >> 16) & 0x7fffu);
                const bool c0 = ok0 && bx > th, c1 = ok1 && by > th;
                if (c0) s_sc[(((e0 >> 7) & 127) + 1) * RS + (e0 & 127) + 1] = (uint8_t)(bx - 1);
                if (c1) s_sc[(((e1 >> 7) & 127) + 1) * RS + (e1 & 127) + 1] = (uint8_t)(by - 1);
                const int cc = (int)c0 + (int)c1;
                const unsigned long long b0 = __ballot(cc & 1), b1 = __ballot(cc & 2);
                int pos = ncorner + lanes_below(b0) + 2 * lanes_below(b1);
                if (c0) s_cor[pos++] = (uint16_t)(e0 & 0x3FFFu);
                if (c1) s_cor[pos] = (uint16_t)(e1 & 0x3FFFu);
                ncorner += __popcll(b0) + 2 * __popcll(b1);
            }
            WAVE_SYNC();   // s_ent is refilled by the next chunk
        }
        // NMS over corners (every other pixel has score 0), fused with the emission: the corner list
        // is in pixel order, so each chunk's survivors go straight to the cell's key list in FAST's
        // row-major emission order. A cell whose attempt leaves no survivor has emitted nothing.
        nsurv = 0;
        for (int i0 = 0; i0 < ncorner; i0 += 64) {
            const int i = i0 + lane;
            bool surv = false;
            int p = 0, sc = 0;
            if (i < ncorner) {
                p = s_cor[i];
                const uint8_t* q = s_sc + ((p >> 7) + 1) * RS + (p & 127) + 1;
                // all nine reads issued together (a short-circuit && chain compiles to eight
                // dependent LDS round trips with an exec-mask branch each)
                const int n0 = q[-RS - 1], n1 = q[-RS], n2 = q[-RS + 1], n3 = q[-1], n4 = q[1];
                const int n5 = q[RS - 1], n6 = q[RS], n7 = q[RS + 1];
                sc = q[0];
                const int mx = max(max(max(n0, n1), max(n2, n3)), max(max(n4, n5), max(n6, n7)));
                surv = sc > mx;
            }
            const unsigned long long m = __ballot(surv);
            if (surv)
                out[nsurv + lanes_below(m)] = (uint32_t)(xr0 + (p & 127)) | ((uint32_t)(yr0 + (p >> 7)) << 12) |
                                              ((uint32_t)sc << 24);
            nsurv += __popcll(m);
        }
        if (nsurv > 0) break;
        WAVE_SYNC();   // the fallback attempt clears the score map
    }   // attempt
    if (lane == 0) cellcnt[(size_t)b * g.total_cells + c] = nsurv;
    WAVE_SYNC();   // LDS is restaged for the next cell
}

#define FAST_WPB 1   // waves per block: a block's LDS is held until its last wave retires, and the cells
                     // of one block finish at different times; single-wave blocks return each wave's LDS
                     // at once: 1.60 -> 1.45 ms per 1024 images against 4 (2: 1.51; r03_kernel_ab.txt item 24)
__global__ __launch_bounds__(64 * FAST_WPB) void k_fast(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                              int pyr_stride, OrbGeom g, FastLds fl, uint32_t* cellkeys,
                                              int* cellcnt, int c_lo, int c_hi, int cpw) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_fast[];
    // wave-uniform in an SGPR: the cell geometry (level search, cell row / column division, ROI
    // bounds, row bases) is then scalar code instead of per-lane VALU divisions
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int bx = lb % gridDim.x, b = lb / gridDim.x;
    // per wave: ROI image (rows of RS bytes) | score map of the detection rect + 1-pixel ring
    // (same RS, origin at ROI (2, 2)) | corner list (2 B per pixel; its tail holds the pass-1
    // group records) | entry chunk (<= 8 entries for each of 64 groups)
    uint8_t* s_img = smem_fast + wave * fl.wave_bytes;
    uint8_t* s_sc = s_img + fl.roi;
    uint16_t* s_cor = (uint16_t*)(s_sc + fl.sc);
    uint16_t* s_ent = (uint16_t*)((uint8_t*)s_cor + fl.cor);
    // the launch covers cells [c_lo, c_hi), cpw consecutive cells per wave (the next cell's ROI is
    // prefetched into registers while this one is processed)
    const int cbeg = c_lo + (bx * FAST_WPB + wave) * cpw;
    if (cbeg >= c_hi) return;
    const int cend = min(cbeg + cpw, c_hi);
    orbfe_u32x4 pf[FAST_PF];
    FastCell cur = fast_cell(imgs, in_pitch, pyr, pyr_stride, g, b, cbeg);
    fast_prefetch(cur, lane, pf);
    for (int c = cbeg; c < cend; c++) {
        int ng, nd, cpr, rpl;
        fast_geom(cur, &ng, &nd, &cpr, &rpl);
        const int dw = cur.cols - 6, dh = cur.rows - 6;
        fast_stage_cell(cur, pf, s_img, s_sc, lane);
        const FastCell me = cur;
        if (c + 1 < cend) {   // prefetch the next cell while this one is processed
            cur = fast_cell_next(cur, imgs, in_pitch, pyr, pyr_stride, g, b);
            fast_prefetch(cur, lane, pf);
        }
        if (fast_rsd(nd) == 12)
            fast_cell_detect<12>(g, fl, me, ng, nd, dw, dh, s_img, s_sc, s_cor, s_ent, cellkeys, cellcnt, b, c, lane);
        else
            fast_cell_detect<0>(g, fl, me, ng, nd, dw, dh, s_img, s_sc, s_cor, s_ent, cellkeys, cellcnt, b, c, lane);
    }
}

// ---------------------------------------------------------------------------------------------
// K4: DistributeOctTree for one (image, level) per 256-thread block. Keys are swept in parallel
// (each key carries the list position of its node, loads batched 4 deep); the ordered list/sort
// logic of the reference runs on LDS tables: phase-1 rounds are rebuilt with block scans (list
// order = push_front order), phase-2 passes sort the expandable nodes with the libstdc++
// introsort replica (tie order matters) and replay the reference's break-at-N walk. The per-node
// winner is the first max-response key in key order, i.e. max(score) then min(index)
// (ORBextractor.cc:757-776).
// ---------------------------------------------------------------------------------------------
#define OCT_NT 256
#define OCT_U 4
// expandable node: (size << 44) | (UL.x << 32) | list position; compareNodes orders by the high 32 bits
struct ExpLess64 {
    __device__ bool operator()(const unsigned long long& a, const unsigned long long& b) const {
        return (a >> 32) < (b >> 32);
    }
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
// Block-wide (NT threads) in-place exclusive scan of arr[0..n); returns the total.
template <int NT>
__device__ __forceinline__ int block_excl_scan(int* arr, int n, int* s_ws) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    int carry = 0;
    for (int base = 0; base < n; base += NT) {
        const int i = base + threadIdx.x;
        const int v = i < n ? arr[i] : 0;
        const int incl = wave_incl_scan_dpp(v);
        if (lane == 63) s_ws[wave] = incl;
        SYNC();
        int woff = 0, tot = 0;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) {
            const int t = s_ws[w];
            woff += w < wave ? t : 0;
            tot += t;
        }
        if (i < n) arr[i] = carry + woff + incl - v;
        carry += tot;
        SYNC();
    }
    return carry;
}

// Block-wide exclusive scan of two per-thread values (thread = element, one element per thread):
// one barrier. s_w2 must not be reused before the caller's next barrier.
template <int NT>
__device__ __forceinline__ void block_scan2(int a, int b, int2* s_w2, int& exa, int& exb, int& tota, int& totb) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int ia = wave_incl_scan_dpp(a), ib = wave_incl_scan_dpp(b);
    if (lane == 63) s_w2[wave] = make_int2(ia, ib);
    SYNC();
    int oa = 0, ob = 0, ta = 0, tb = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; w++) {
        const int2 t = s_w2[w];
        oa += w < wave ? t.x : 0;
        ob += w < wave ? t.y : 0;
        ta += t.x;
        tb += t.y;
    }
    exa = oa + ia - a;
    exb = ob + ib - b;
    tota = ta;
    totb = tb;
}

// Block-parallel, element-for-element replica of libstdc++ std::sort on u64 elements ordered by
// their high 32 bits (see stl_sort.h "Data-parallel formulation"): every wave of the block
// partitions its own segments (median-of-three, then the unguarded partition as stop pairing by
// ballots); leaves (<= 16 elements) are stably sorted by rank as soon as they are cut;
// depth-exhausted leaves fall back to the serial heapsort replica. block_introsort below.
// In-place exclusive scan of arr[0..n) by the calling wave only (no workgroup barrier).
__device__ __forceinline__ int wave_scan_lds(int* arr, int n) {
    const int lane = lane_id();
    int carry = 0;
    for (int base = 0; base < n; base += 64) {
        const int i = base + lane;
        const int v = i < n ? arr[i] : 0;
        const int incl = wave_incl_scan_dpp(v);
        if (i < n) arr[i] = carry + incl - v;
        carry += __builtin_amdgcn_readlane(incl, 63);
    }
    WAVE_SYNC();
    return carry;
}

// Wave-aggregated LDS increment: every active lane adds 1 to base[t]. The keys of a wave arrive in
// cell order, so adjacent lanes mostly share a node (and quadrant); each run of equal targets adds
// its length once from its first lane, instead of up to 64 same-address atomics serialised in the
// LDS. Needs every lane of the wave (DPP + ballot): callers keep the trip counts wave-uniform.
__device__ __forceinline__ void atomic_inc_runs(int* base, int t, bool act) {
    const int lane = lane_id();
    const int key = act ? t : -1 - lane;   // inactive lanes: distinct keys, never in a run
    const int prev = __builtin_amdgcn_update_dpp(INT_MIN, key, 0x138, 0xf, 0xf, false);   // wave_shr:1
    const bool head = key != prev;   // lane 0 reads INT_MIN
    const unsigned long long hm = __ballot(head);
    const unsigned long long above = hm & ~((2ull << lane) - 1ull);   // heads after this lane
    const int next = above ? (int)__builtin_ctzll(above) : 64;
    if (head && act) atomicAdd(&base[t], next - lane);
}

// One unguarded partition of a[lo, hi) by the calling wave (hi - lo > 16): __move_median_to_first
// then __unguarded_partition (stl_sort.h). Returns the cut. The stops are ranked by ballots; the k-th
// left / right stop of the segment lands at lpos[lo + k] / rpos[lo + k] (segments are disjoint, so
// waves partitioning different segments share the scratch).
__device__ __forceinline__ int wave_partition(unsigned long long* a, int lo, int hi, int* lpos, int* rpos) {
    const int tid = lane_id();
    const unsigned long long lt = (1ull << tid) - 1ull;
    // __move_median_to_first(first, first + 1, mid, last - 1): every lane evaluates the
    // comparison tree on the same four values, lane 0 performs the one swap
    unsigned long long xpiv;
    {
        const int ia = lo + 1, ib = lo + (hi - lo) / 2, ic = hi - 1;
        const unsigned long long x0 = a[lo], xa = a[ia], xb = a[ib], xc = a[ic];
        const ExpLess64 comp;
        int pick;
        if (comp(xa, xb)) pick = comp(xb, xc) ? ib : (comp(xa, xc) ? ic : ia);
        else pick = comp(xa, xc) ? ia : (comp(xb, xc) ? ic : ib);
        xpiv = pick == ia ? xa : (pick == ib ? xb : xc);
        if (tid == 0) {
            a[lo] = xpiv;
            a[pick] = x0;
        }
    }
    WAVE_SYNC();
    const unsigned P = (unsigned)(xpiv >> 32);   // the pivot every lane already holds
    const int m = hi - lo - 1;
    int* lp = lpos + lo;
    int* rp = rpos + lo;
    // left stops (scan rightwards over [lo+1, hi)): !(x < P); right stops (leftwards from hi-1): !(P < x)
    int nl = 0, nr = 0;
    for (int b0 = 0; b0 < m; b0 += 64) {
        const int i = b0 + tid;
        bool lf = false, rf = false;
        if (i < m) {
            lf = !((unsigned)(a[lo + 1 + i] >> 32) < P);
            rf = !(P < (unsigned)(a[hi - 1 - i] >> 32));
        }
        const unsigned long long lm = __ballot(lf), rm = __ballot(rf);
        if (lf) lp[nl + __popcll(lm & lt)] = lo + 1 + i;
        if (rf) rp[nr + __popcll(rm & lt)] = hi - 1 - i;
        nl += __popcll(lm);
        nr += __popcll(rm);
    }
    WAVE_SYNC();
    // lpos increasing, rpos decreasing: the pairs that swap (lpos[k] < rpos[k]) are a prefix
    const int kmax = min(nl, nr);
    int sw = 0;
    for (int b0 = 0; b0 < kmax; b0 += 64) {
        const int k = b0 + tid;
        sw += __popcll(__ballot(k < kmax && lp[k] < rp[k]));
    }
    for (int k = tid; k < sw; k += 64) {
        const unsigned long long x = a[lp[k]];
        a[lp[k]] = a[rp[k]];
        a[rp[k]] = x;
    }
    int cut;
    if (sw == 0) cut = lp[0];
    else cut = (sw < nl && lp[sw] < rp[sw - 1]) ? lp[sw] : rp[sw - 1];
    WAVE_SYNC();
    return cut;
}

// A finished introsort leaf a[lo, hi), sorted at once by the wave that cut it: the final insertion
// sort never moves an element across a partition boundary, so it equals a stable sort of each leaf
// (<= 16 elements: ranks from the keys broadcast by readlane); a depth-exhausted leaf (> 16) is the
// serial heapsort replica (__partial_sort) on lane 0.
__device__ __forceinline__ void wave_leaf(unsigned long long* a, int lo, int hi) {
    const int lane = lane_id();
    const int len = hi - lo;
    if (len <= 1) return;
    if (len > 16) {
        if (lane == 0) st_heap_sort(a + lo, len, ExpLess64());
        WAVE_SYNC();
        return;
    }
    const unsigned long long x = a[lo + min(lane, len - 1)];
    const unsigned kx = (unsigned)(x >> 32);
    int r = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const unsigned ku = (unsigned)__builtin_amdgcn_readlane((int)kx, u);
        r += (u < len && (ku < kx || (ku == kx && u < lane))) ? 1 : 0;
    }
    WAVE_SYNC();
    if (lane < len) a[lo + r] = x;
    WAVE_SYNC();
}

#if ORBFE_OCT_STAMPS
// diagnostic builds: per-wave phase stamps of the last block sort of block (0, 0) (16 waves x 16)
// and of wave 0's last register sort (16 more), buffered in LDS (a global store would make the
// next barrier wait for it) and flushed at the end of the sort
__device__ unsigned long long g_sort_ts[16 * 16 + 16];
__shared__ unsigned long long s_dbg_ts[16 * 16 + 16];
#endif
__device__ __forceinline__ unsigned long long rl64(unsigned long long x, int l) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)x, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(x >> 32), l);
    return ((unsigned long long)hi << 32) | lo;
}
// gather: lane i gets x of lane src(i)
__device__ __forceinline__ unsigned long long bp64(unsigned long long x, int src) {
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)x);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_bpermute(src << 2, (int)(unsigned)(x >> 32));
    return ((unsigned long long)hi << 32) | lo;
}
// scatter: lane dst(i) gets x of lane i
__device__ __forceinline__ unsigned long long pm64(unsigned long long x, int dst) {
    const unsigned lo = (unsigned)__builtin_amdgcn_ds_permute(dst << 2, (int)(unsigned)x);
    const unsigned hi = (unsigned)__builtin_amdgcn_ds_permute(dst << 2, (int)(unsigned)(x >> 32));
    return ((unsigned long long)hi << 32) | lo;
}

// __introsort_loop of a segment a[lo0, lo0 + len) of <= 64 elements in the calling wave's registers
// (element i in lane i), then the final insertion sort of all its leaves at once; the same
// partitions as wave_partition. Per partition: the median of three by readlane; left stops
// !(x < P) and right stops !(P < x) by ballot, ranked by popcount (left ascending, right
// descending); the k-th left stop swaps with the k-th right stop iff it lies below it, i.e. iff
// more than k right stops lie above it, so the swap count is one more ballot; the pairs exchange
// values through two crossbar scatters (ds_permute) and gathers (ds_bpermute). No LDS round trip.
__device__ __forceinline__ void wave_sort64(unsigned long long* a, int lo0, int len, int d0) {
    const int lane = lane_id();
#if ORBFE_OCT_STAMPS
    int s64i = 0;
#define S64_STAMP() do { if (lane == 0 && s64i < 15 && (threadIdx.x >> 6) == 0 && blockIdx.x == 0 && blockIdx.y == 0) s_dbg_ts[256 + s64i] = __builtin_amdgcn_s_memtime(); s64i++; } while (0)
#else
#define S64_STAMP() do { } while (0)
#endif
    S64_STAMP();
    unsigned long long x = a[lo0 + min(lane, len - 1)];
    const unsigned long long below = (1ull << lane) - 1ull;
    const unsigned long long above = lane == 63 ? 0ull : (~0ull << (lane + 1));
    unsigned long long leafm = 0, heapm = 0;   // leaf starts (wave-uniform); depth-exhausted leaves
    int sg_lo = 0, sg_hi = lane == 0 ? len : 0, sg_dp = lane == 0 ? d0 : 0;
    int sp = 1;
    while (sp > 0) {
        --sp;
        const int lo = __builtin_amdgcn_readlane(sg_lo, sp), hi = __builtin_amdgcn_readlane(sg_hi, sp);
        const int dp = __builtin_amdgcn_readlane(sg_dp, sp);
        if (hi - lo <= 16 || dp == 0) {
            leafm |= 1ull << lo;
            if (hi - lo > 16) heapm |= 1ull << lo;
            continue;
        }
        // __move_median_to_first(first, first + 1, mid, last - 1)
        const int ia = lo + 1, ib = lo + (hi - lo) / 2, ic = hi - 1;
        const unsigned kx = (unsigned)(x >> 32);
        const unsigned ka = (unsigned)__builtin_amdgcn_readlane((int)kx, ia);
        const unsigned kb = (unsigned)__builtin_amdgcn_readlane((int)kx, ib);
        const unsigned kc = (unsigned)__builtin_amdgcn_readlane((int)kx, ic);
        int pick;
        if (ka < kb) pick = kb < kc ? ib : (ka < kc ? ic : ia);
        else pick = ka < kc ? ia : (kb < kc ? ic : ib);
        const unsigned long long x0 = rl64(x, lo), xp = rl64(x, pick);
        if (lane == lo) x = xp;
        else if (lane == pick) x = x0;
        const unsigned P = (unsigned)(xp >> 32);
        // __unguarded_partition(first + 1, last, first)
        const unsigned k = (unsigned)(x >> 32);
        const bool inr = lane > lo && lane < hi;
        const bool lf = inr && !(k < P), rf = inr && !(P < k);
        const unsigned long long LM = __ballot(lf), RM = __ballot(rf);
        const int rl = __popcll(LM & below), rr = __popcll(RM & above);
        const bool sL = lf && __popcll(RM & above) > rl;
        const int sw = __popcll(__ballot(sL));
        const bool sR = rf && rr < sw;
        int cut;
        if (sw == 0) {
            cut = __builtin_ctzll(LM);
        } else {
            const int rp = __builtin_ctzll(__ballot(rf && rr == sw - 1));
            const int lp = sw < __popcll(LM) ? __builtin_ctzll(__ballot(lf && rl == sw)) : 64;
            cut = lp < rp ? lp : rp;
            // lane k of vR / vL holds the k-th right / left stop's value (other lanes park on 63,
            // never read: sw <= 31)
            const unsigned long long vR = pm64(x, sR ? rr : 63);
            const unsigned long long vL = pm64(x, sL ? rl : 63);
            const unsigned long long fromR = bp64(vR, rl & 63), fromL = bp64(vL, rr & 63);
            if (sL) x = fromR;
            else if (sR) x = fromL;
        }
        if (lane == sp) { sg_lo = cut; sg_hi = hi; sg_dp = dp - 1; }
        if (lane == sp + 1) { sg_lo = lo; sg_hi = cut; sg_dp = dp - 1; }
        sp += 2;
        S64_STAMP();
    }
    S64_STAMP();
    // final insertion sort = a stable sort of each ordinary leaf: rank among the leaf's keys, scatter
    const unsigned long long upto = leafm & ~above;
    const int ls = 63 - __builtin_clzll(upto | 1ull);
    const unsigned long long after = leafm & above;
    const int le = after ? __builtin_ctzll(after) : len;
    const bool heap = (heapm >> ls) & 1ull;
    const unsigned kx = (unsigned)(x >> 32);
    // the 16 gathers issued back to back, then the compares (branch-free)
    unsigned kj[16];
#pragma unroll
    for (int u = 0; u < 16; u++) kj[u] = (unsigned)__builtin_amdgcn_ds_bpermute(min(ls + u, 63) << 2, (int)kx);
    int r = 0;
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int j = ls + u;
        r += (int)((j < le) & ((kj[u] < kx) | ((kj[u] == kx) & (j < lane))));
    }
    x = pm64(x, (lane < len && !heap) ? ls + r : lane);
    if (lane < len) a[lo0 + lane] = x;
    if (heapm) {
        WAVE_SYNC();
        if (lane == 0) {
            unsigned long long hm = heapm;
            while (hm) {
                const int hs = __builtin_ctzll(hm);
                hm &= hm - 1ull;
                const unsigned long long nx = leafm & (hs == 63 ? 0ull : (~0ull << (hs + 1)));
                const int he = nx ? __builtin_ctzll(nx) : len;
                st_heap_sort(a + lo0 + hs, he - hs, ExpLess64());
            }
        }
    }
    WAVE_SYNC();
    S64_STAMP();
#if ORBFE_OCT_STAMPS
    if (lane == 0 && (threadIdx.x >> 6) == 0 && blockIdx.x == 0 && blockIdx.y == 0) s_dbg_ts[256 + 15] = s64i;
#endif
#undef S64_STAMP
}

// __introsort_loop of one segment by the calling wave, depth first. The segment stack lives in
// registers, entry k in lane k (ORBFE_SORT_STACK = 64 = the wave; pop = three readlanes).
__device__ __forceinline__ void wave_sort_seg(unsigned long long* a, int lo0, int hi0, int dp0, int* lpos, int* rpos) {
    const int tid = lane_id();
    int sg_lo = lo0, sg_hi = tid == 0 ? hi0 : 0, sg_dp = tid == 0 ? dp0 : 0;
    int sp = 1;
    while (sp > 0) {
        --sp;
        const int lo = __builtin_amdgcn_readlane(sg_lo, sp), hi = __builtin_amdgcn_readlane(sg_hi, sp);
        const int depth = __builtin_amdgcn_readlane(sg_dp, sp);
        if (hi - lo <= 64 && depth > 0) {
            if (hi - lo > 1) wave_sort64(a, lo, hi - lo, depth);
            continue;
        }
        if (depth == 0) {
            wave_leaf(a, lo, hi);
            continue;
        }
        const int cut = wave_partition(a, lo, hi, lpos, rpos);
        if (tid == sp) { sg_lo = cut; sg_hi = hi; sg_dp = depth - 1; }
        if (tid == sp + 1) { sg_lo = lo; sg_hi = cut; sg_dp = depth - 1; }
        sp += 2;
    }
}

// segment list entry: lo | hi << 16 | depth << 32
__device__ __forceinline__ unsigned long long seg_pack(int lo, int hi, int d) {
    return (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 16) | ((unsigned long long)d << 32);
}

// Block entry: every wave of the block sorts. Partitions of disjoint segments are independent, so
// the order they run in does not change the result: breadth-first rounds (wave w takes list entries
// w, w + nw, ...; an entry's two children go to entries 2s and 2s + 1 of the next list, empty when
// the child was a leaf and sorted at once; block barrier between rounds) until the list has at least
// as many entries as there are waves, then each wave finishes its entries depth first. No atomics:
// the compiler's lane-serial expansion of a wave's LDS atomic cost ~5 k cycles per push or pop.
// Scratch: lpos, rpos int[n]; tmp u64[n] (two segment lists); s_ctl[8] (non-empty flags).
// fl, leaves, segs, s_ws unused.
__device__ __forceinline__ void block_introsort(unsigned long long* a, int n, int* fl, int* lpos, int* rpos, int* leaves,
                                unsigned long long* tmp, int4* segs, int* s_ws, int* s_ctl) {
    (void)fl; (void)leaves; (void)segs; (void)s_ws;
    const int lane = lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
#if ORBFE_OCT_STAMPS
    int sti = 0;
#define SORT_STAMP() do { if (lane == 0 && sti < 15 && blockIdx.x == 0 && blockIdx.y == 0) s_dbg_ts[wave * 16 + sti] = __builtin_amdgcn_s_memtime(); sti++; } while (0)
#else
#define SORT_STAMP() do { } while (0)
#endif
    SORT_STAMP();
    if (threadIdx.x == 0) {
        tmp[0] = seg_pack(0, n, 2 * st_lg(n));
#pragma unroll
        for (int k = 0; k < 8; k++) s_ctl[k] = 0;
    }
    SYNC();
    SORT_STAMP();
    if (n <= 1) return;
    // a list holds at most 2 * nw - 2 entries (it doubles while below nw): tmp needs 4 * nw entries
    // (k_octree: the 2 * NC of the next-count table; the debug entry: its LDS tail)
    unsigned long long* cur = tmp;
    unsigned long long* nxt = tmp + 2 * nw;
    int S = 1, r = 0;
    while (S > 0 && S < nw && r < 7) {
        bool any = false;
        for (int s = wave; s < S; s += nw) {
            const unsigned long long e = cur[s];
            const int lo = (int)(e & 0xffff), hi = (int)((e >> 16) & 0xffff), d = (int)(e >> 32);
            unsigned long long c0 = 0, c1 = 0;
            if (hi - lo <= 16 || d == 0) {
                wave_leaf(a, lo, hi);
            } else if (hi - lo <= 64) {
                wave_sort64(a, lo, hi - lo, d);
            } else {
                const int cut = wave_partition(a, lo, hi, lpos, rpos);
                if (hi - cut <= 16 || d == 1) wave_leaf(a, cut, hi);
                else c0 = seg_pack(cut, hi, d - 1);
                if (cut - lo <= 16 || d == 1) wave_leaf(a, lo, cut);
                else c1 = seg_pack(lo, cut, d - 1);
            }
            if (lane == 0) {
                nxt[2 * s] = c0;
                nxt[2 * s + 1] = c1;
            }
            any = any || c0 != 0 || c1 != 0;
        }
        if (any && lane == 0) s_ctl[r] = 1;   // plain stores of one value: no atomic needed
        SYNC();
        SORT_STAMP();
        S = s_ctl[r] ? 2 * S : 0;
        r++;
        unsigned long long* t = cur; cur = nxt; nxt = t;
    }
    for (int s = wave; s < S; s += nw) {
        const unsigned long long e = cur[s];
        if (e) wave_sort_seg(a, (int)(e & 0xffff), (int)((e >> 16) & 0xffff), (int)(e >> 32), lpos, rpos);
    }
    SORT_STAMP();
    SYNC();
    SORT_STAMP();
#if ORBFE_OCT_STAMPS
    if (lane == 0 && blockIdx.x == 0 && blockIdx.y == 0) s_dbg_ts[wave * 16 + 15] = sti;
    SYNC();
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < 16 * 16 + 16; i += blockDim.x) g_sort_ts[i] = s_dbg_ts[i];
#endif
#undef SORT_STAMP
}

// Debug/test entry: sort one array with the block sort (single block).
__global__ __launch_bounds__(OCT_NT) void k_debug_block_sort(unsigned long long* a, int n) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_dbs[];
    unsigned long long* la = (unsigned long long*)smem_dbs;
    unsigned long long* tmp = la + n;
    int* fl = (int*)(tmp + n);
    int* lpos = fl + n;
    int* rpos = lpos + n;
    int* leaves = rpos + n;
    int4* segs = (int4*)(((uintptr_t)(leaves + n) + 15) & ~(uintptr_t)15);
    __shared__ int s_ws[OCT_NT / 64];
    __shared__ int s_ctl[8];
    for (int i = threadIdx.x; i < n; i += OCT_NT) la[i] = a[i];
    SYNC();
    block_introsort(la, n, fl, lpos, rpos, leaves, tmp, segs, s_ws, s_ctl);
    for (int i = threadIdx.x; i < n; i += OCT_NT) a[i] = la[i];
}

// NT = 256 threads per (image, level) for batches; a small batch (the host API's single image,
// where the level-0 and level-1 blocks are the frame's long pole and nothing else competes for
// the CUs) takes NT = 1024: the key sweeps and scans run in a quarter of the iterations.
template <int NT>
__global__ __launch_bounds__(NT, NT <= 256 ? 6 : 1) void k_octree(OrbGeom g, const uint32_t* __restrict__ cellkeys,
                                                   const int* __restrict__ cellcnt, uint32_t* lkeys,
                                                   uint16_t* nodeof, uint32_t* outkeys, int* lvinfo, int* ranks,
                                                   const int2* __restrict__ laps, unsigned long long* tstamp,
                                                   int lv0) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_oct[];
    // grid (B, levels from lv0): level-0 blocks (the longest) are dispatched first
    const int b = blockIdx.x, l = lv0 + (int)blockIdx.y, tid = threadIdx.x;
    const int lap0 = laps[b].x, lap1 = laps[b].y;   // this image's vLappingArea
    const OrbLevel& L = g.lv[l];
    const int NC = g.node_cap;
    const int ncell = L.n_cols * L.n_rows;
    // ---- LDS carve (all offsets multiples of 16 bytes) ----
    uint8_t* p = smem_oct;
    auto carve = [&](size_t bytes) { uint8_t* r = p; p += (bytes + 15) & ~(size_t)15; return r; };
    int* cellpre = (int*)carve(sizeof(int) * (g.max_cells_level + 1));
    // current (C*) and next (X*) node tables; swapped by pointer after each rebuild
    int16_t *Cx0 = (int16_t*)carve(2 * NC), *Cx1 = (int16_t*)carve(2 * NC);
    int16_t *Cy0 = (int16_t*)carve(2 * NC), *Cy1 = (int16_t*)carve(2 * NC);
    int* Csz = (int*)carve(4 * NC);
    int16_t *Xx0 = (int16_t*)carve(2 * NC), *Xx1 = (int16_t*)carve(2 * NC);
    int16_t *Xy0 = (int16_t*)carve(2 * NC), *Xy1 = (int16_t*)carve(2 * NC);
    int* Xsz = (int*)carve(4 * NC);
    int* Ccnt = (int*)carve(16 * NC);
    int* Xcnt = (int*)carve(16 * NC);
    int16_t* childpos = (int16_t*)carve(8 * NC);
    int16_t* newpos = (int16_t*)carve(2 * NC);
    int* divorder = (int*)carve(4 * NC);
    int* tmpA = (int*)carve(4 * NC);
    int* tmpB = (int*)carve(4 * NC);
    int* tmpC = (int*)carve(4 * NC);
    int* procp = (int*)carve(4 * NC);
    unsigned long long* expv = (unsigned long long*)carve(8 * NC);
    // the introsort's u64 / int scratch and the final best-key table live in the next-count table
    // (16 * NC bytes), dead from the top of a step until its zeroing before the key sweep and after
    // the last step: 12 * NC bytes less LDS (7 blocks per CU instead of 6 at EuRoC geometry; the
    // kernel time is set by the level-0 blocks' serial steps, so this measured only -0.6 %)
    int4* segs = (int4*)carve(sizeof(int4) * ORBFE_SORT_STACK);
    __shared__ int s_ws[NT / 64];
    __shared__ int s_misc[8];
    __shared__ int2 s_ws2[NT / 64];

    // diagnostic phase stamps (image 0 of the batch, every level), tstamp == nullptr in normal runs
    unsigned long long* ts = (tstamp && b == 0) ? tstamp + 64 * l : nullptr;
    int tsi = 0;
    (void)ts;
    (void)tsi;
#if ORBFE_OCT_STAMPS
    __shared__ unsigned long long s_octts[64];
#define OCT_STAMP() do { if (ts && tid == 0 && tsi < 62) s_octts[tsi] = __builtin_amdgcn_s_memtime(); tsi++; } while (0)
#else
#define OCT_STAMP() do { } while (0)
#endif
    OCT_STAMP();
    // ---- gather this level's cell key lists in cell order (vToDistributeKeys order) ----
    const int* cc = cellcnt + (size_t)b * g.total_cells + L.cell_base;
    for (int i = tid; i < ncell; i += NT) cellpre[i] = cc[i];
    SYNC();
    const int K = block_excl_scan<NT>(cellpre, ncell, s_ws);
    if (tid == 0) cellpre[ncell] = K;
    const int nIni = L.n_ini;
    const float hX = L.hx;
    const int H = (L.h - ORBFE_MINB) - ORBFE_MINB;
    // registers hold the keys (below) and the initial columns fit one per thread: the gather also
    // counts each key's root quadrant by column (a root's rectangle is its column's), so the
    // initial nodes need no second pass over the keys
    const bool fini = NT >= 1024 && K <= NT * (NT >= 1024 ? 8 : OCT_U) && nIni <= NT;
    for (int i = tid; i < nIni; i += NT) tmpA[i] = 0;
    if (fini)
        for (int i = tid; i < 4 * nIni; i += NT) tmpC[i] = 0;
    for (int i = tid; i < 4 * NC; i += NT) Ccnt[i] = 0;
    SYNC();
    const size_t kbase = (size_t)b * g.cellkeys_per_img + L.cellkey_off;
    uint32_t* keys = lkeys + kbase;
    uint16_t* nof = nodeof + kbase;
    const uint32_t* ck = cellkeys + kbase;
    // Keys of this level held in registers for the whole kernel when they fit (key k = tid + NT * u
    // in rkv[u], its node in rq[u]): no key / node-index round trips through global memory, and no
    // barrier waiting on their stores. Otherwise the global lists (lkeys, nodeof) carry them.
    constexpr int OU = NT >= 1024 ? 8 : OCT_U;
    // (the 1024-thread small-batch instance only: at 256 threads the batch fills the CUs, and the
    // registers would cost resident blocks)
    const bool regk = NT >= 1024 && K <= NT * OU;
    uint32_t rkv[OU];
    int rq[OU];
    // the gather also counts the keys of each initial node (ORBextractor.cc:559-601's root columns;
    // wave-uniform trip counts: the aggregated increments need every lane)
    for (int kb = 0; kb < K; kb += NT * OU) {
        const int k0 = kb + tid;
        uint32_t v[OU];
#pragma unroll
        for (int u = 0; u < OU; u++) {
            if ((u & 3) == 0 && kb + NT * u >= K) break;   // block-uniform, per group of 4 slots (the
                                                             // group's chains interleave)
            const int k = min(k0 + NT * u, K - 1);
            int lo = 0, hi = ncell - 1;   // largest c with cellpre[c] <= k
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (cellpre[mid] <= k) lo = mid; else hi = mid - 1;
            }
            v[u] = ck[(size_t)lo * L.cell_cap + (k - cellpre[lo])];
        }
#pragma unroll
        for (int u = 0; u < OU; u++) {
            if ((u & 3) == 0 && kb + NT * u >= K) break;
            if (regk) rkv[u] = v[u];   // regk: this loop runs once
            else if (k0 + NT * u < K) keys[k0 + NT * u] = v[u];
            const int col = (int)((float)(v[u] & 0xfff) / hX);
            atomic_inc_runs(tmpA, col, k0 + NT * u < K);
            if (fini) {
                rq[u] = col;   // remapped to the root's list position below
                atomic_inc_runs(tmpC, 4 * col + quadrant(v[u], (int)(hX * (float)col), (int)(hX * (float)(col + 1)), 0, H),
                                k0 + NT * u < K);
            }
        }
    }
    OCT_STAMP();
    // ---- initial nodes (ORBextractor.cc:559-601) ----
    SYNC();
    int n;
    if (fini) {
        // one thread per column: the non-empty columns in order are the initial list; their counts
        // and quadrant counts come from the gather; each key's column becomes its node position
        const int i = tid;
        const bool f = i < nIni && tmpA[i] > 0;
        int ex, exZ, totZ;
        block_scan2<NT>(f ? 1 : 0, 0, s_ws2, ex, exZ, n, totZ);
        (void)exZ;
        (void)totZ;
        if (f) {
            Cx0[ex] = (int16_t)(int)(hX * (float)i);
            Cx1[ex] = (int16_t)(int)(hX * (float)(i + 1));
            Cy0[ex] = 0;
            Cy1[ex] = (int16_t)H;
            Csz[ex] = tmpA[i];
            *(int4*)&Ccnt[4 * ex] = *(const int4*)&tmpC[4 * i];
        }
        if (i < nIni) tmpB[i] = ex;
        for (int j = tid; j < NC; j += NT) divorder[j] = -1;
        SYNC();
#pragma unroll
        for (int u = 0; u < (NT >= 1024 ? 8 : OCT_U); u++) {
            if ((u & 3) == 0 && NT * u >= K) break;   // the slots the gather filled
            rq[u] = tmpB[rq[u]];
        }
        OCT_STAMP();
    } else {
    for (int i = tid; i < nIni; i += NT) tmpB[i] = tmpA[i] > 0 ? 1 : 0;
    SYNC();
    n = block_excl_scan<NT>(tmpB, nIni, s_ws);   // position of each non-empty root
    for (int i = tid; i < nIni; i += NT) {
        if (tmpA[i] > 0) {
            const int q = tmpB[i];
            Cx0[q] = (int16_t)(int)(hX * (float)i);
            Cx1[q] = (int16_t)(int)(hX * (float)(i + 1));
            Cy0[q] = 0;
            Cy1[q] = (int16_t)H;
            Csz[q] = tmpA[i];
        }
    }
    SYNC();
    for (int kb = 0; kb < K; kb += NT * OU) {
        const int k0 = kb + tid;
        uint32_t v[OU];
#pragma unroll
        for (int u = 0; u < OU; u++) v[u] = regk ? rkv[u] : keys[min(k0 + NT * u, K - 1)];
#pragma unroll
        for (int u = 0; u < OU; u++) {
            if ((u & 3) == 0 && kb + NT * u >= K) break;
            const int k = k0 + NT * u;
            const uint32_t key = v[u];
            const int q = tmpB[(int)((float)(key & 0xfff) / hX)];
            if (regk) rq[u] = q;
            else if (k < K) nof[k] = (uint16_t)q;
            atomic_inc_runs(Ccnt, 4 * q + quadrant(key, Cx0[q], Cx1[q], Cy0[q], Cy1[q]), k < K && Csz[q] > 1);
        }
    }
    for (int i = tid; i < NC; i += NT) divorder[i] = -1;
    SYNC();
    OCT_STAMP();
    }

    const int N = L.budget;
    bool phase2 = false, finish = false;
    int m = 0;   // expandable-node count of the last rebuild (vSizeAndPointerToNode)
    int guard = 0;
    while (!finish && guard++ < 100000) {
        const int prevN = n;
        int newN, Etot;
        if (!phase2 && n <= NT) {
            // Phase-1 step fused (one node per thread): every node with > 1 keys divides, in list order,
            // so the divider rank t, the children / expandable-children offsets and the kept-node rank
            // are one packed two-value block scan over the list (counts < 2^16: n <= NT <= 1024)
            const int i = tid;
            const bool live = i < n;
            const int csz = live ? Csz[i] : 0;
            const bool div = csz > 1;
            int4 cq = make_int4(0, 0, 0, 0);
            if (div) cq = *(const int4*)&Ccnt[4 * i];
            const int cv[4] = {cq.x, cq.y, cq.z, cq.w};
            int c = 0, e = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) { c += cv[k] > 0; e += cv[k] > 1; }
            int exA, exB, totA, totB;
            block_scan2<NT>(live ? (div ? 1 : 0x10000) : 0, c | (e << 16), s_ws2, exA, exB, totA, totB);
            const int Ctot = totB & 0xffff;
            Etot = totB >> 16;
            newN = Ctot + (totA >> 16);
            if (div) {
                divorder[i] = exA & 0xffff;
                // children: block of t starts at sum_{t'>t} c_t'; order n4,n3,n2,n1 (push_front)
                const int start = Ctot - ((exB & 0xffff) + c);
                int kk = 0;
                const int px0 = Cx0[i], px1 = Cx1[i], py0 = Cy0[i], py1 = Cy1[i];
                int cpos[4];
#pragma unroll
                for (int ch = 3; ch >= 0; ch--) {
                    const int v = cv[ch];
                    cpos[ch] = -1;
                    if (v > 0) {
                        const int np = start + kk++;
                        cpos[ch] = np;
                        childpos[4 * i + ch] = (int16_t)np;
                        int a0, a1, b0, b1;
                        child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                        Xx0[np] = (int16_t)a0; Xx1[np] = (int16_t)a1;
                        Xy0[np] = (int16_t)b0; Xy1[np] = (int16_t)b1;
                        Xsz[np] = v;
                    } else {
                        childpos[4 * i + ch] = -1;
                    }
                }
                int ei = exB >> 16;
#pragma unroll
                for (int ch = 0; ch < 4; ch++) {
                    const int v = cv[ch];
                    if (v > 1) {
                        int a0, a1, b0, b1;
                        child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                        expv[ei] = ((unsigned long long)v << 44) | ((unsigned long long)(a0 & 0xfff) << 32) |
                                   (unsigned long long)(uint16_t)cpos[ch];
                        ei++;
                    }
                }
            } else if (live) {
                // undivided nodes keep their relative order after the pushed children
                divorder[i] = -1;
                const int np = Ctot + (exA >> 16);
                newpos[i] = (int16_t)np;
                Xx0[np] = Cx0[i]; Xx1[np] = Cx1[i];
                Xy0[np] = Cy0[i]; Xy1[np] = Cy1[i];
                Xsz[np] = csz;
            }
            for (int j = tid; j < 4 * newN; j += NT) Xcnt[j] = 0;
            SYNC();
            OCT_STAMP();
        } else if (phase2 && m <= NT && n <= NT) {
            // Phase-2 step fused: std::sort(vPrevSizeAndPointerToNode, compareNodes) (ORBextractor.cc:700),
            // exact replica, then the walk from the back (ORBextractor.cc:701-748) and the rebuild with
            // three scans in two packed block scans: sorted position t = thread (node expv[m-1-t])
#if ORBFE_OCT_STAMPS
            if (ts && tid == 0) s_octts[62] = (unsigned long long)m | ((unsigned long long)n << 16) | ((unsigned long long)K << 32);
#endif
            block_introsort(expv, m, tmpC, tmpA, tmpB, Xcnt + 2 * NC, (unsigned long long*)Xcnt, segs, s_ws,
                            s_misc);
            OCT_STAMP();
            const int t = tid;
            const bool live = t < m;
            int q = 0;
            int4 cq = make_int4(0, 0, 0, 0);
            if (live) {
                q = (int)(expv[m - 1 - t] & 0xffffffffull);
                cq = *(const int4*)&Ccnt[4 * q];
            }
            const int cv[4] = {cq.x, cq.y, cq.z, cq.w};
            int c = 0, e = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) { c += cv[k] > 0; e += cv[k] > 1; }
            const int grow = live ? c - 1 : 0;   // the list grows by (children - 1) per division
            if (tid == 0) s_misc[6] = m;
            int exG, exCE, totG, totCE;
            block_scan2<NT>(grow, c | (e << 16), s_ws2, exG, exCE, totG, totCE);
            // first t at which the list reaches N: nodes [0, T_div) of the walk divide
            if (live && n + exG + grow >= N) atomicMin(&s_misc[6], t + 1);
            if (live) tmpB[t] = exCE + (c | (e << 16));   // inclusive (children | expandable << 16)
            SYNC();
            const int T_div = s_misc[6];
            const int tot = T_div > 0 ? tmpB[T_div - 1] : 0;
            const int Ctot = tot & 0xffff;
            Etot = tot >> 16;
            if (t < T_div) {
                divorder[q] = t;
                // children: block of t starts at sum_{t'>t} c_t'; order n4,n3,n2,n1 (push_front)
                const int start = Ctot - ((exCE & 0xffff) + c);
                int kk = 0;
                const int px0 = Cx0[q], px1 = Cx1[q], py0 = Cy0[q], py1 = Cy1[q];
                int cpos[4];
#pragma unroll
                for (int ch = 3; ch >= 0; ch--) {
                    const int v = cv[ch];
                    cpos[ch] = -1;
                    if (v > 0) {
                        const int np = start + kk++;
                        cpos[ch] = np;
                        childpos[4 * q + ch] = (int16_t)np;
                        int a0, a1, b0, b1;
                        child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                        Xx0[np] = (int16_t)a0; Xx1[np] = (int16_t)a1;
                        Xy0[np] = (int16_t)b0; Xy1[np] = (int16_t)b1;
                        Xsz[np] = v;
                    } else {
                        childpos[4 * q + ch] = -1;
                    }
                }
                int ei = exCE >> 16;
#pragma unroll
                for (int ch = 0; ch < 4; ch++) {
                    const int v = cv[ch];
                    if (v > 1) {
                        int a0, a1, b0, b1;
                        child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                        expv[ei] = ((unsigned long long)v << 44) | ((unsigned long long)(a0 & 0xfff) << 32) |
                                   (unsigned long long)(uint16_t)cpos[ch];
                        ei++;
                    }
                }
            }
            SYNC();
            // undivided nodes keep their relative order after the pushed children
            const int i = tid;
            const bool keep = i < n && divorder[i] < 0;
            int exK, exZ, nKeep, totZ;
            block_scan2<NT>(keep ? 1 : 0, 0, s_ws2, exK, exZ, nKeep, totZ);
            (void)exZ;
            (void)totZ;
            if (keep) {
                const int np = Ctot + exK;
                newpos[i] = (int16_t)np;
                Xx0[np] = Cx0[i]; Xx1[np] = Cx1[i];
                Xy0[np] = Cy0[i]; Xy1[np] = Cy1[i];
                Xsz[np] = Csz[i];
            }
            newN = Ctot + nKeep;
            for (int j = tid; j < 4 * newN; j += NT) Xcnt[j] = 0;
            SYNC();
            OCT_STAMP();
        } else {
            int T_div;   // number of divided nodes in this step
            if (!phase2) {
                // every node with >1 keys divides, in list order
                for (int i = tid; i < n; i += NT) tmpA[i] = Csz[i] > 1 ? 1 : 0;
                SYNC();
                for (int i = tid; i < n; i += NT) divorder[i] = Csz[i] > 1 ? 1 : -1;
                T_div = block_excl_scan<NT>(tmpA, n, s_ws);   // tmpA[i] = divider rank t (list order)
                for (int i = tid; i < n; i += NT)
                    if (divorder[i] >= 0) { divorder[i] = tmpA[i]; procp[tmpA[i]] = i; }
                SYNC();
            } else {
                // std::sort(vPrevSizeAndPointerToNode, compareNodes) (ORBextractor.cc:700), exact replica
#if ORBFE_OCT_STAMPS
                if (ts && tid == 0) s_octts[62] = (unsigned long long)m | ((unsigned long long)n << 16) | ((unsigned long long)K << 32);
#endif
                block_introsort(expv, m, tmpC, tmpA, tmpB, Xcnt + 2 * NC, (unsigned long long*)Xcnt, segs, s_ws,
                                s_misc);
                OCT_STAMP();
                // walk from the back until the list reaches N (ORBextractor.cc:701-748): processed node t is
                // expv[m-1-t]; the list grows by (children - 1) per division -> first t where it reaches N
                for (int t = tid; t < m; t += NT) {
                    const int q = (int)(expv[m - 1 - t] & 0xffffffffull);
                    const int4 cq = *(const int4*)&Ccnt[4 * q];
                    tmpA[t] = (cq.x > 0) + (cq.y > 0) + (cq.z > 0) + (cq.w > 0) - 1;
                    procp[t] = q;
                }
                if (tid == 0) s_misc[6] = m;
                SYNC();
                (void)block_excl_scan<NT>(tmpA, m, s_ws);   // tmpA[t] = growth before processing t
                for (int t = tid; t < m; t += NT) {
                    const int q = procp[t];
                    const int4 cq = *(const int4*)&Ccnt[4 * q];
                    const int grow = (cq.x > 0) + (cq.y > 0) + (cq.z > 0) + (cq.w > 0) - 1;
                    if (n + tmpA[t] + grow >= N) atomicMin(&s_misc[6], t + 1);
                }
                SYNC();
                T_div = s_misc[6];
                for (int t = tid; t < T_div; t += NT) divorder[procp[t]] = t;
                SYNC();
            }
            OCT_STAMP();
            // children counts per processed node (t order): tmpB = nonempty, tmpC = expandable (>1)
            for (int t = tid; t < T_div; t += NT) {
                const int q = procp[t];
                int c = 0, e = 0;
                const int4 cq = *(const int4*)&Ccnt[4 * q];
                const int cv[4] = {cq.x, cq.y, cq.z, cq.w};
    #pragma unroll
                for (int k = 0; k < 4; k++) { c += cv[k] > 0; e += cv[k] > 1; }
                tmpB[t] = c;
                tmpC[t] = e;
            }
            SYNC();
            const int Ctot = block_excl_scan<NT>(tmpB, T_div, s_ws);
            Etot = block_excl_scan<NT>(tmpC, T_div, s_ws);
            // children: block of t starts at sum_{t'>t} c_t' = Ctot - (excl_t + c_t); order n4,n3,n2,n1
            for (int t = tid; t < T_div; t += NT) {
                const int q = procp[t];
                // the four counts in one read: the child writes below may alias them for the compiler,
                // which would otherwise re-read each count behind the previous child's stores
                const int4 cq = *(const int4*)&Ccnt[4 * q];
                const int cv[4] = {cq.x, cq.y, cq.z, cq.w};
                int c = 0;
    #pragma unroll
                for (int k = 0; k < 4; k++) c += cv[k] > 0;
                const int start = Ctot - (tmpB[t] + c);
                int kk = 0;
                const int px0 = Cx0[q], px1 = Cx1[q], py0 = Cy0[q], py1 = Cy1[q];
                int cpos[4];
    #pragma unroll
                for (int ch = 3; ch >= 0; ch--) {
                    const int v = cv[ch];
                    cpos[ch] = -1;
                    if (v > 0) {
                        const int np = start + kk++;
                        cpos[ch] = np;
                        childpos[4 * q + ch] = (int16_t)np;
                        int a0, a1, b0, b1;
                        child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                        Xx0[np] = (int16_t)a0; Xx1[np] = (int16_t)a1;
                        Xy0[np] = (int16_t)b0; Xy1[np] = (int16_t)b1;
                        Xsz[np] = v;
                    } else {
                        childpos[4 * q + ch] = -1;
                    }
                }
                int e = tmpC[t];
    #pragma unroll
                for (int ch = 0; ch < 4; ch++) {
                    const int v = cv[ch];
                    if (v > 1) {
                        int a0, a1, b0, b1;
                        child_rect(ch, px0, px1, py0, py1, &a0, &a1, &b0, &b1);
                        expv[e] = ((unsigned long long)v << 44) | ((unsigned long long)(a0 & 0xfff) << 32) |
                                  (unsigned long long)(uint16_t)cpos[ch];
                        e++;
                    }
                }
            }
            // undivided nodes keep their relative order after the pushed children
            for (int i = tid; i < n; i += NT) tmpA[i] = divorder[i] < 0 ? 1 : 0;
            SYNC();
            const int nKeep = block_excl_scan<NT>(tmpA, n, s_ws);
            for (int i = tid; i < n; i += NT) {
                if (divorder[i] < 0) {
                    const int np = Ctot + tmpA[i];
                    newpos[i] = (int16_t)np;
                    Xx0[np] = Cx0[i]; Xx1[np] = Cx1[i];
                    Xy0[np] = Cy0[i]; Xy1[np] = Cy1[i];
                    Xsz[np] = Csz[i];
                }
            }
            newN = Ctot + nKeep;
            for (int i = tid; i < 4 * newN; i += NT) Xcnt[i] = 0;
            SYNC();
            OCT_STAMP();
        }
        // key sweep: move keys to their new node positions and count the next split
        for (int kb = 0; kb < K; kb += NT * OU) {
            const int k0 = kb + tid;
            uint32_t v[OU];
            int qv[OU];
#pragma unroll
            for (int u = 0; u < OU; u++) {
                const int k = min(k0 + NT * u, K - 1);
                v[u] = regk ? rkv[u] : keys[k];
                qv[u] = regk ? rq[u] : nof[k];
            }
#pragma unroll
            for (int u = 0; u < OU; u++) {
                if ((u & 3) == 0 && kb + NT * u >= K) break;
                const int k = k0 + NT * u;
                const uint32_t key = v[u];
                const int q = qv[u];
                int np;
                if (divorder[q] >= 0) np = childpos[4 * q + quadrant(key, Cx0[q], Cx1[q], Cy0[q], Cy1[q])];
                else np = newpos[q];
                if (regk) rq[u] = np;
                else if (k < K) nof[k] = (uint16_t)np;
                atomic_inc_runs(Xcnt, 4 * np + quadrant(key, Xx0[np], Xx1[np], Xy0[np], Xy1[np]), k < K && Xsz[np] > 1);
            }
        }
        SYNC();
        // no barrier after the reset: the next step touches divorder only behind its own barriers
        // (the fused step's scan, the sort's entry), and nothing else here is shared
        for (int i = tid; i < NC; i += NT) divorder[i] = -1;
        {
            int16_t* t;
            int* ti;
            t = Cx0; Cx0 = Xx0; Xx0 = t; t = Cx1; Cx1 = Xx1; Xx1 = t;
            t = Cy0; Cy0 = Xy0; Xy0 = t; t = Cy1; Cy1 = Xy1; Xy1 = t;
            ti = Csz; Csz = Xsz; Xsz = ti; ti = Ccnt; Ccnt = Xcnt; Xcnt = ti;
        }
        n = newN;
        m = Etot;
        if (n > NC - 4) { n = NC - 4; finish = true; }   // capacity guard (bound: n <= max(N+2, 4*nIni) = NC-8-1)
        if (n >= N || n == prevN) finish = true;
        else if (!phase2 && n + 3 * m > N) phase2 = true;
    }
    OCT_STAMP();
    // ---- retain the best key per node ----
    unsigned long long* best = (unsigned long long*)Xcnt;
    for (int i = tid; i < n; i += NT) best[i] = 0ull;
    SYNC();
    for (int k0 = tid; k0 < K; k0 += NT * OU) {
        uint32_t v[OU];
        int qv[OU];
#pragma unroll
        for (int u = 0; u < OU; u++) {
            const int k = min(k0 + NT * u, K - 1);
            v[u] = regk ? rkv[u] : keys[k];
            qv[u] = regk ? rq[u] : nof[k];
        }
#pragma unroll
        for (int u = 0; u < OU; u++) {
            const int k = k0 + NT * u;
            if ((u & 3) == 0 && k0 - tid + NT * u >= K) break;
            if (k < K)
                atomicMax(&best[qv[u]], ((unsigned long long)(v[u] >> 24) << 32) | (0xFFFFFFFFull - (unsigned)k));
        }
    }
    SYNC();
    uint32_t* ok = outkeys + (size_t)b * g.out_per_img + L.out_off;
    int* rk = ranks + (size_t)b * g.out_per_img + L.out_off;
    // the output key of each node and its lapping flag: written by the thread holding the node's
    // winning key (registers), or read back from the global key list
    auto emit = [&](int i, uint32_t key) {
        const int x = (int)(key & 0xfff) + ORBFE_MINB, y = (int)((key >> 12) & 0xfff) + ORBFE_MINB;
        ok[i] = (uint32_t)x | ((uint32_t)y << 12) | (key & 0xff000000u);
        const float sx = (l == 0) ? (float)x : (float)x * L.scale;
        tmpA[i] = (sx >= (float)lap0 && sx <= (float)lap1) ? 1 : 0;
    };
    if (regk) {
#pragma unroll
        for (int u = 0; u < OU; u++) {
            const int k = tid + NT * u;
            if ((u & 3) == 0 && NT * u >= K) break;
            if (k < K && best[rq[u]] == (((unsigned long long)(rkv[u] >> 24) << 32) | (0xFFFFFFFFull - (unsigned)k)))
                emit(rq[u], rkv[u]);
        }
    } else {
        for (int i = tid; i < n; i += NT) emit(i, keys[0xFFFFFFFFu - (unsigned)(best[i] & 0xFFFFFFFFull)]);
    }
    SYNC();
    // ranks among lapping / non-lapping keys
    int nlap, nmono;
    if (n <= NT) {
        const int f = tid < n ? tmpA[tid] : 0;
        int exl, exm;
        block_scan2<NT>(f, tid < n ? 1 - f : 0, s_ws2, exl, exm, nlap, nmono);
        if (tid < n) rk[tid] = f ? (int)(0x40000000 | exl) : exm;
    } else {
        for (int i = tid; i < n; i += NT) tmpB[i] = 1 - tmpA[i];
        SYNC();
        nlap = block_excl_scan<NT>(tmpA, n, s_ws);
        nmono = block_excl_scan<NT>(tmpB, n, s_ws);
        for (int i = tid; i < n; i += NT) {
            const bool lap = (i + 1 < n ? tmpA[i + 1] : nlap) != tmpA[i];
            rk[i] = lap ? (int)(0x40000000 | tmpA[i]) : tmpB[i];
        }
    }
    OCT_STAMP();
#if ORBFE_OCT_STAMPS
    if (ts && tid == 0) {
        for (int i = 0; i < min(tsi, 62); i++) ts[i] = s_octts[i];
        ts[62] = s_octts[62];
        ts[63] = (unsigned long long)tsi;
    }
#endif
#undef OCT_STAMP
    if (tid == 0) {
        int* inf = lvinfo + ((size_t)b * g.nlevels + l) * 4;
        inf[0] = n; inf[1] = nlap; inf[2] = nmono; inf[3] = K;
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

// Fused per-keypoint pipeline, one wave per keypoint (several keypoints per wave with the next
// patch prefetched into registers measured slower: the loop raised the kernel to 123-129 VGPRs,
// 3-4 waves per SIMD, against 7 with one keypoint): the 43x43 patch of the UNBLURRED level
// around the keypoint (reflect-101 outside the level) is staged in LDS once; IC_Angle reads it
// directly; the 7x7 Gaussian of the level is evaluated on the 37x37 window the descriptor can
// sample (|offset| <= 18) with the exact separable fixed-point arithmetic of the reference's GaussianBlur
// semantics (GaussianBlur of the whole level, ORBextractor.cc:1132-1133, restricted to the pixels
// the descriptor reads); rBRIEF samples that window. No blurred level ever touches HBM.
#define DP_R 21                      // patch radius: 18 (pattern) + 3 (blur)
#define DP_N (2 * DP_R + 1)          // 43
#define DP_RAW_S 48                  // raw row stride (bytes)
#define DP_NP 22                     // row pairs of the Q8 row pass (row 43 is padding)
#define DP_P_S 40                    // row-pair stride (dwords: one (row 2p, row 2p+1) u16 pair per column)
#define DP_WAVE_LDS 5600   // >= 43*48 + 22*40*4, multiple of 16
#define DP_ND (DP_N * (DP_RAW_S / 4))   // 516 patch dwords
// One output slot of an image (wave-uniform): level, key, output index and the patch geometry.
struct DescSlot {
    int valid, l, x, y, interior, pitch, gx0, sh;
    uint32_t key;
    size_t o;
    gptr_u8 im;
};
// Per-image level table of one wave (k_octree's lvinfo): lane l < nlevels holds level l's
// (n, nlap, nmono, K); the lapping / non-lapping keys of the levels before l (exclusive prefixes)
// and the image totals come from DPP scans over the first 16 lanes (nlevels <= 12), no scalar loops.
struct DescImg {
    int n, lap_before, mono_before;   // per lane (level = lane)
    int ntot, mono_tot;               // wave-uniform
};
__device__ __forceinline__ int row_incl_scan_dpp(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
    return v;
}
__device__ __forceinline__ DescImg desc_img(const OrbGeom& g, const int* __restrict__ inf, int lane) {
    int4 li = make_int4(0, 0, 0, 0);
    if (lane < g.nlevels) li = ((const int4*)inf)[lane];
    DescImg di;
    di.n = li.x;
    const int lapi = row_incl_scan_dpp(li.y), monoi = row_incl_scan_dpp(li.z), ni = row_incl_scan_dpp(li.x);
    di.lap_before = lapi - li.y;
    di.mono_before = monoi - li.z;
    di.ntot = __builtin_amdgcn_readlane(ni, 15);
    di.mono_tot = __builtin_amdgcn_readlane(monoi, 15);
    return di;
}
// Slot `flat` of an image: its level (searched upwards from *lvl: a wave's slots ascend), key and
// rank (lane j of kv / rv holds those of the wave's slot j).
__device__ __forceinline__ DescSlot desc_slot(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                              int pyr_stride, const OrbGeom& g, const DescImg& di, uint32_t kv,
                                              int rv, int j, int* lvl, int b, int flat) {
    DescSlot d;
    d.valid = 0;
    if (flat >= g.out_per_img) return d;
    int l = *lvl;
    while (l + 1 < g.nlevels && flat >= g.lv[l + 1].out_off) l++;
    *lvl = l;
    const OrbLevel& L = g.lv[l];
    if (flat - L.out_off >= __builtin_amdgcn_readlane(di.n, l)) return d;
    d.valid = 1;
    d.l = l;
    d.key = (uint32_t)__builtin_amdgcn_readlane((int)kv, j);
    d.x = d.key & 0xfff;
    d.y = (d.key >> 12) & 0xfff;
    // output slot: lapping reorder (ORBextractor.cc:1153-1162)
    const int rk = __builtin_amdgcn_readlane(rv, j);
    const int slot = (rk & 0x40000000) ? di.ntot - 1 - (__builtin_amdgcn_readlane(di.lap_before, l) + (rk & 0x3fffffff))
                                       : __builtin_amdgcn_readlane(di.mono_before, l) + rk;
    d.o = (size_t)b * g.kp_cap + slot;
    d.im = level_base(imgs, in_pitch, pyr, pyr_stride, g, b, l, &d.pitch);
    const int px0 = d.x - DP_R, py0 = d.y - DP_R;
    d.gx0 = px0 & ~3;
    d.sh = px0 - d.gx0;
    d.interior = px0 >= 0 && py0 >= 0 && py0 + DP_N <= L.h && d.gx0 + DP_RAW_S + 4 <= L.w && (d.pitch & 3) == 0 &&
                 ((((uintptr_t)d.im) & 3) == 0);
    return d;
}
// Patch of an interior slot as 16-byte chunks of the 48-byte rows from gx0: lane = 3 r + k (k =
// chunk of the row), load u covers rows 21 u .. 21 u + 20 (lane 63 idle; rows past 42 re-read row
// 42, not stored). Three dwordx4 loads per lane instead of 18 dword loads.
__device__ __forceinline__ void desc_load(const DescSlot& d, int lane, orbfe_u32x4 (&q)[3]) {
    const int r0 = small_div(lane, 3), k = lane - 3 * r0;
    gptr_u8 b0 = d.im + (size_t)(d.y - DP_R) * d.pitch + d.gx0 + 16 * k;
#pragma unroll
    for (int u = 0; u < 3; u++) {
        const uint32_t row = (uint32_t)min(r0 + 21 * u, DP_N - 1);
        q[u] = *(const ORBFE_GLOBAL orbfe_u32x4*)(b0 + __umul24(row, (uint32_t)d.pitch));
    }
}
// Realign the chunks to the patch origin (byte shift sh; the fourth dword takes the next lane's
// first, a DPP wave_shl) and store them as 16-byte rows pieces. The last chunk of a row only needs
// bytes up to column 42 < 48 - 3, so its neighbour (the next row's chunk) is never used.
__device__ __forceinline__ void desc_stage(uint8_t* raw, int lane, const orbfe_u32x4 (&q)[3], int sh) {
    const int r0 = small_div(lane, 3), k = lane - 3 * r0;
#pragma unroll
    for (int u = 0; u < 3; u++) {
        const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q[u].x, 0x130, 0xf, 0xf, false);
        uint4 w;
        w.x = __builtin_amdgcn_alignbyte(q[u].y, q[u].x, (uint32_t)sh);
        w.y = __builtin_amdgcn_alignbyte(q[u].z, q[u].y, (uint32_t)sh);
        w.z = __builtin_amdgcn_alignbyte(q[u].w, q[u].z, (uint32_t)sh);
        w.w = __builtin_amdgcn_alignbyte(nx, q[u].w, (uint32_t)sh);
        if (lane < 63 && r0 + 21 * u < DP_N) *(uint4*)(raw + (r0 + 21 * u) * DP_RAW_S + 16 * k) = w;
    }
}
// IC_Angle + Gaussian + rBRIEF of one slot whose raw patch is staged in `raw`; writes the
// keypoint record and the descriptor row.
__device__ __forceinline__ void describe_one(const DescSlot& d, const OrbGeom& g, const uint8_t* raw, uint32_t* rowp,
                                             const uint2 (&pat)[4], int lane, OrbKeyPoint* kps, uint8_t* desc,
                                             const BlurKernel& bk, const uint4 (*icm)[3]) {
    const OrbLevel& L = g.lv[d.l];
    const int l = d.l, x = d.x, y = d.y;
    const uint32_t key = d.key;
    const size_t o = d.o;
    auto emit_kp = [&](float angle) {
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
    };
    // ---- IC_Angle on the unblurred patch, centre (21, 21): lane v + 15 sums disc row v with
    // two v_dot4 per dword: m10 = sum (u + 16) I - 16 sum I, m01 = sum v * sum I (exact integers,
    // the reference's sums in another order) ----
    int m10 = 0, m01 = 0;
    if (lane < 31) {
        const uint4* rowp = (const uint4*)(raw + (lane + DP_R - 15) * DP_RAW_S);
        const uint4* mk = icm[lane];   // the block's LDS copy of c_ic_mask
        const uint4 q0 = rowp[0], q1 = rowp[1], q2 = rowp[2];
        const uint4 k0 = mk[0], k1 = mk[1], k2 = mk[2];
        const uint32_t I[9] = {q0.y & k0.x, q0.z & k0.y, q0.w & k0.z, q1.x & k0.w, q1.y & k1.x,
                               q1.z & k1.y, q1.w & k1.z, q2.x & k1.w, q2.y & k2.x};
        uint32_t s1 = 0, su = 0;
#pragma unroll
        for (int j = 0; j < 9; j++) {
            // byte b of dword j is column 4 (j + 1) + b: weight u + 16 = 4 j + b - 1 (0 for the
            // never-in-disc column 4)
            const uint32_t w = (j == 0 ? 0u : (uint32_t)(4 * j - 1)) | ((uint32_t)(4 * j) << 8) |
                               ((uint32_t)(4 * j + 1) << 16) | ((uint32_t)(4 * j + 2) << 24);
            s1 = __builtin_amdgcn_udot4(I[j], 0x01010101u, s1, false);
            su = __builtin_amdgcn_udot4(I[j], w, su, false);
        }
        m10 = (int)su - 16 * (int)s1;
        m01 = (lane - 15) * (int)s1;
    }
    m10 = wave_sum_dpp(m10);
    m01 = wave_sum_dpp(m01);
    const float angle = fast_atan2_dev((float)m01, (float)m10);
    // ---- 7x7 Gaussian: row pass (Q8, exact) over the 43x37 region in packed u16x2 (every
    // partial sum fits 16 bits: sum(k) * 255 <= 65535); the column pass (Q16, rounded) runs only
    // at the 512 points rBRIEF samples. Both passes are exact integer sums before the final
    // rounding, so this equals blurring the whole level. ----
    const uint32_t k0 = bk.k[0], k1 = bk.k[1], k2 = bk.k[2], k3 = bk.k[3];
    {
        // output j of a 4-column group = bytes j .. j + 6 of the 12-byte run w0 w1 w2 times the taps
        // (k0 k1 k2 k3 k2 k1 k0): v_dot4_u32_u8 of each dword with the kernel shifted by j bytes, no
        // realignment (2 + 2 + 3 + 3 dot products per group; exact: <= 65280)
        const uint32_t KLO = k0 | (k1 << 8) | (k2 << 16) | (k3 << 24), KHI = k2 | (k1 << 8) | (k0 << 16);
        const uint32_t K10 = (k0 << 8) | (k1 << 16) | (k2 << 24), K11 = k3 | (k2 << 8) | (k1 << 16) | (k0 << 24);
        const uint32_t K20 = (k0 << 16) | (k1 << 24), K21 = k2 | (k3 << 8) | (k2 << 16) | (k1 << 24), K22 = k0;
        const uint32_t K30 = k0 << 24, K31 = k1 | (k2 << 8) | (k3 << 16) | (k2 << 24), K32 = k1 | (k0 << 8);
        // row pairs (2 p, 2 p + 1) x 10 groups of 4 output columns: lanes 0..59 = 6 pairs x 10 groups,
        // pairs p0 + 6 i; the pair is stored as one dword per column (row 2 p low, 2 p + 1 high), one
        // 16-byte store per group. Row 43 does not exist: its half is 0 (never weighted).
        const int p0 = small_div(lane, 10), gq = lane - 10 * p0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int pr = p0 + 6 * i;
            if (lane >= 60 || pr >= DP_NP) break;
            uint32_t h[2][4];
#pragma unroll
            for (int e = 0; e < 2; e++) {
                const uint32_t* rp = (const uint32_t*)(raw + (2 * pr + e) * DP_RAW_S) + gq;
                const uint32_t w0 = rp[0], w1 = rp[1], w2 = rp[2];
                h[e][0] = __builtin_amdgcn_udot4(w1, KHI, __builtin_amdgcn_udot4(w0, KLO, 0u, false), false);
                h[e][1] = __builtin_amdgcn_udot4(w1, K11, __builtin_amdgcn_udot4(w0, K10, 0u, false), false);
                h[e][2] = __builtin_amdgcn_udot4(w2, K22, __builtin_amdgcn_udot4(w1, K21, __builtin_amdgcn_udot4(w0, K20, 0u, false), false), false);
                h[e][3] = __builtin_amdgcn_udot4(w2, K32, __builtin_amdgcn_udot4(w1, K31, __builtin_amdgcn_udot4(w0, K30, 0u, false), false), false);
            }
            const bool last = 2 * pr + 1 >= DP_N;
            uint4 pk;
            pk.x = h[0][0] | (last ? 0u : h[1][0] << 16);
            pk.y = h[0][1] | (last ? 0u : h[1][1] << 16);
            pk.z = h[0][2] | (last ? 0u : h[1][2] << 16);
            pk.w = h[0][3] | (last ? 0u : h[1][3] << 16);
            *(uint4*)(rowp + pr * DP_P_S + 4 * gq) = pk;
        }
    }
    WAVE_SYNC();
    // ---- rBRIEF, centre (18, 18) of the blurred window ----
    const float factorPI = (float)(M_PI / 180.f);
    const float ang = angle * factorPI;
    const float a = glibc_cosf(ang), bs = glibc_sinf(ang);
    // sample (px, py) -> row cvRound(px b + py a), column cvRound(px a - py b) (ORBextractor.cc:117-119):
    // products in packed f32, then (px b, px a) + (py a, py b) * (1, -1) as one packed fma (the
    // product with +-1 is exact, so this rounds like the reference's separate add / subtract), then
    // + (1.5 * 2^23 + 18) rounds each sum half-even to an integer (|sum| < 2^22) in the low mantissa
    // bits: the row bits are 0x4B400000 + R, R = 18 + row the top tap of the column pass, the column
    // bits 0x4B400000 + C, C = 18 + column. Pair row R >> 1 of rowp holds rows (R & ~1, R | 1), so
    // pair rows R >> 1 .. (R >> 1) + 3 hold every tap; a byte shift of 2 (R odd) or 0 realigns them
    // to (R, R+1), (R+2, R+3), (R+4, R+5), (R+6, -) and one v_dot2_u32_u16 per dword sums the taps
    // with (k0, k1), (k2, k3), (k2, k1), (k0, 0). The LDS byte address (R >> 1) * S + 4 C is one
    // shift, one 24-bit multiply-add and one shift-add: the 24-bit multiply sees
    // (0x4B400000 + R) >> 1 as 0xA00000 + (R >> 1), and the constant offsets fold into KC (mod 2^32).
    // (__float_as_uint, not __builtin_bit_cast, on the vector elements: this clang folds a bit_cast
    // of rc.y to rc.x.)
    typedef float orbfe_f2 __attribute__((ext_vector_type(2)));
    typedef const __attribute__((address_space(3))) uint32_t* lds_u32p;
    const orbfe_f2 cs = {bs, a}, sn = {a, bs}, sg = {1.0f, -1.0f}, mag = {12582930.0f, 12582930.0f};
    const uint32_t S = 4 * DP_P_S;
    const uint32_t KC = (uint32_t)(uintptr_t)(lds_u32p)rowp - 0xA00000u * S - 4u * 0x4B400000u;
    struct Samp { uint32_t ad, sh; };
    auto sample_at = [&](float px, float py) -> Samp {
        const orbfe_f2 u = orbfe_f2{px, px} * cs;   // (px b, px a)
        const orbfe_f2 v = orbfe_f2{py, py} * sn;   // (py a, py b)
        const orbfe_f2 rc = __builtin_elementwise_fma(v, sg, u) + mag;
        const uint32_t rb = __float_as_uint(rc.x), cb = __float_as_uint(rc.y);
        return Samp{__umul24(rb >> 1, S) + 4u * cb + KC, rb << 1};
    };
    const uint32_t C01 = k0 | (k1 << 16), C23 = k2 | (k3 << 16), C21 = k2 | (k1 << 16), C0 = k0;
    // blurred value at a sample (exact: every partial sum < 2^32)
    auto blurred_at = [&](Samp sp) -> uint32_t {
        const lds_u32p q = (lds_u32p)(size_t)sp.ad;
        const uint32_t d0 = q[0], d1 = q[DP_P_S], d2 = q[2 * DP_P_S], d3 = q[3 * DP_P_S];
        // v_alignbyte uses the low 2 bits of the shift: rb << 1 is 2 for odd R, 0 for even
        const uint32_t a0 = __builtin_amdgcn_alignbyte(d1, d0, sp.sh), a1 = __builtin_amdgcn_alignbyte(d2, d1, sp.sh);
        const uint32_t a2 = __builtin_amdgcn_alignbyte(d3, d2, sp.sh), a3 = __builtin_amdgcn_alignbyte(0u, d3, sp.sh);
        uint32_t sum = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2, a0), __builtin_bit_cast(orbfe_ushort2, C01), 32768u, false);
        sum = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2, a1), __builtin_bit_cast(orbfe_ushort2, C23), sum, false);
        sum = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2, a2), __builtin_bit_cast(orbfe_ushort2, C21), sum, false);
        sum = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2, a3), __builtin_bit_cast(orbfe_ushort2, C0), sum, false);
        const uint32_t v = sum >> 16;
        return v > 255u ? 255u : v;
    };
    unsigned long long masks[4];
#pragma unroll
    for (int mm = 0; mm < 4; mm++) {
        // pair 64 * mm + lane: (x0, y0), (x1, y1) as f16 halves (the pattern's small integers are
        // exact in f16; one v_cvt_f32_f16 per coordinate)
        const orbfe_half2 p0 = __builtin_bit_cast(orbfe_half2, pat[mm].x), p1 = __builtin_bit_cast(orbfe_half2, pat[mm].y);
        const uint32_t t0 = blurred_at(sample_at((float)p0.x, (float)p0.y));
        const uint32_t t1 = blurred_at(sample_at((float)p1.x, (float)p1.y));
        masks[mm] = __ballot(t0 < t1);
    }
    if (lane < 4) {
        unsigned long long mv = lane == 0 ? masks[0] : lane == 1 ? masks[1] : lane == 2 ? masks[2] : masks[3];
        ((unsigned long long*)(desc + o * 32))[lane] = mv;
    }
    emit_kp(angle);
}

// DP_KPW: slots per wave: the next slot's patch loads overlap this slot's compute (a wave alone is
// two dependent memory round trips per slot: keys, then the patch). 8 slots (an 8-byte spill with
// the f16 pattern) ran the kernel alone 1.07 -> 1.04 ms but doubled its HBM reads (twice the images
// resident per XCD overflow its L2: hit rate 0.84 -> 0.70) and left the full step unchanged
// (r03_kernel_ab.txt item 19)
#define DP_KPW 4
// 6 waves per SIMD: 79 VGPRs, no spill since the pattern is held as f16 (at 5 waves without a spill
// or 6 with one the kernel measured slower or equal: 1 slot / 4 slots at 5, 6, 7 waves, 2, 3 and 8
// slots, tools/gpu_variants_trace.sh; DESIGN.md §7d, profiles/r03_kernel_ab.txt items 18-19)
#ifndef DP_WAVES
#define DP_WAVES 6
#endif
#define DP_ATTR __attribute__((amdgpu_waves_per_eu(DP_WAVES)))
// DP_WPB: waves per block: 2 / 4 / 8 measured 1.04 / 1.06 / 1.11 ms (r03_kernel_ab.txt item 23); 12
// blocks of 12.7 KB per CU give the same 6 waves per SIMD with finer-grained refill
#define DP_WPB 2
template <int KPW>
__global__ __launch_bounds__(64 * DP_WPB) DP_ATTR void k_describe(const uint8_t* const* imgs, int in_pitch, const uint8_t* pyr,
                                                  int pyr_stride, OrbGeom g, const uint32_t* __restrict__ outkeys,
                                                  const int* __restrict__ lvinfo, const int* __restrict__ ranks,
                                                  OrbKeyPoint* kps, uint8_t* desc, int* counts, BlurKernel bk) {
    __shared__ __attribute__((aligned(16))) uint8_t s_dp[DP_WPB][DP_WAVE_LDS];
    // the IC_Angle disc masks (31 rows x 12 dwords) in LDS: per slot three ds_read_b128 instead of
    // three vector loads from constant memory
    __shared__ uint4 s_icm[31][3];
    for (int i = threadIdx.x; i < 31 * 3; i += blockDim.x)
        (&s_icm[0][0])[i] = ((const uint4*)&c_ic_mask.m[0][0])[i];
    __syncthreads();
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int b = lb / gridDim.x;
    const int flat0 = ((lb % gridDim.x) * DP_WPB + wave) * KPW;   // first of this wave's output slots
    if (flat0 >= g.out_per_img) return;
    // the rBRIEF pairs of this lane (pair 64 * mm + lane: x0, y0, x1, y1), issued first
    uint2 pat[4];
#pragma unroll
    for (int mm = 0; mm < 4; mm++) pat[mm] = ((const uint2*)c_pattern_h.v)[64 * mm + lane];
    // keys and ranks of the wave's slots (lane j: slot flat0 + j), one load each
    uint32_t kv = 0;
    int rv = 0;
    if (lane < KPW && flat0 + lane < g.out_per_img) {
        kv = outkeys[(size_t)b * g.out_per_img + flat0 + lane];
        rv = ranks[(size_t)b * g.out_per_img + flat0 + lane];
    }
    const DescImg di = desc_img(g, lvinfo + (size_t)b * g.nlevels * 4, lane);
    if (flat0 == 0 && lane == 0) { counts[2 * b] = di.ntot; counts[2 * b + 1] = di.mono_tot; }
    uint8_t* raw = s_dp[wave];
    uint32_t* rowp = (uint32_t*)(raw + DP_N * DP_RAW_S);
    int lvl = 0;
    DescSlot cur = desc_slot(imgs, in_pitch, pyr, pyr_stride, g, di, kv, rv, 0, &lvl, b, flat0);
    orbfe_u32x4 pq[3];
    if (cur.valid && cur.interior) desc_load(cur, lane, pq);
#pragma unroll
    for (int j = 0; j < KPW; j++) {
        // ---- stage the raw patch: raw[r][c] = level(y - 21 + r, x - 21 + c), reflect-101 outside ----
        if (cur.valid) {
            if (cur.interior) {
                desc_stage(raw, lane, pq, cur.sh);
            } else {
                const OrbLevel& L = g.lv[cur.l];
                const int px0 = cur.x - DP_R, py0 = cur.y - DP_R;
                for (int it = lane; it < DP_N * DP_N; it += 64) {
                    const int r = it / DP_N, c = it - r * DP_N;
                    raw[r * DP_RAW_S + c] = cur.im[(size_t)reflect101(py0 + r, L.h) * cur.pitch + reflect101(px0 + c, L.w)];
                }
            }
        }
        WAVE_SYNC();
        // the next slot's patch loads fly while this one is described
        DescSlot nxt;
        nxt.valid = 0;
        if (j + 1 < KPW) {
            nxt = desc_slot(imgs, in_pitch, pyr, pyr_stride, g, di, kv, rv, j + 1, &lvl, b, flat0 + j + 1);
            if (nxt.valid && nxt.interior) desc_load(nxt, lane, pq);
        }
        if (cur.valid) describe_one(cur, g, raw, rowp, pat, lane, kps, desc, bk, s_icm);
        WAVE_SYNC();   // the patch area is restaged for the next slot
        cur = nxt;
    }
}
#undef DP_ND

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
    int sort_cap;   // LDS sort keys: >= max_kp, a power of two for the bitonic fallback
    int lk;         // left keypoints per block (ST_LK; fewer for a small batch of frames)
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
// Stage 1: one wave per left keypoint at a time (16 waves per block, keypoints taken from a block
// counter), ST_LK left keypoints per block; the right
// keypoints (x, row band, octave) and descriptors of the frame are staged in LDS once per block
// and the records are sorted by the first row of their band, so a left keypoint on row v scans
// only the records with minr in [v - maxspan, v] (the reference's vRowIndices[v] superset; the
// first-best-in-iR-order rule is kept by the (dist, iR) key).
// Writes per left kp: uRight, depth (-1 = none) and the SAD distance of an accepted match (-1).
#define ST_LK 512   // left keypoints per block (2 blocks per frame: 256 measured 10 % slower, 1024 20 %)
#define ST_NT 1024
#define ST_ROFF 32    // row-start table margin (rows -32 .. height + 32)
struct RightRec { float x; int minr, maxr, oct; };
__global__ __launch_bounds__(ST_NT) void k_stereo(OrbGeom g, StereoSide SL, StereoSide SR, StereoArgs sa,
                                                  float* uright, float* depth, int* sdist) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem_st[];
    __shared__ int s_maxspan;
    __shared__ int s_next;   // next left keypoint of the block (waves take them dynamically)
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int f = lb / gridDim.x;
    const int bL = SL.base + f * SL.step, bR = SR.base + f * SR.step;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = lane_id();
    const int N = SL.counts[2 * bL], Nr = SR.counts[2 * bR];
    const int i0 = (lb % gridDim.x) * sa.lk;
    if (i0 >= N) return;
    // right records ordered by a counting sort over band rows when the row table fits (every image
    // up to 1983 rows), else by a bitonic sort of P = pow2 >= Nr keys (sa.sort_cap is sized to match)
    const int nrow = g.height + 2 * ST_ROFF;
    const bool csort = nrow + 1 <= (ST_NT / 64) * 128;
    int P = 1;
    while (P < Nr) P <<= 1;
    if (csort) P = Nr;
    uint32_t* s_descR = (uint32_t*)smem_st;                        // sa.max_kp * 8 words
    RightRec* s_rec = (RightRec*)(s_descR + 8 * sa.max_kp);        // sa.max_kp records
    uint32_t* s_key = (uint32_t*)(s_rec + sa.max_kp);              // sort keys, sa.sort_cap entries
    uint8_t* s_win = (uint8_t*)(s_key + sa.sort_cap) + wave * 512; // per wave: IL 11x11 @0, IR 11x21 @128
    int* s_part = (int*)((uint8_t*)(s_key + sa.sort_cap) + (ST_NT / 64) * 512) + wave * 128;
    const OrbKeyPoint* kR = SR.kps + (size_t)bR * g.kp_cap;
    const OrbKeyPoint* kL = SL.kps + (size_t)bL * g.kp_cap;
    const uint4* dR = (const uint4*)(SR.desc + (size_t)bR * g.kp_cap * 32);
    const uint32_t* dL = (const uint32_t*)(SL.desc + (size_t)bL * g.kp_cap * 32);
    if (threadIdx.x == 0) { s_maxspan = 0; s_next = ST_NT / 64; }
    SYNC();
    for (int i = threadIdx.x; i < Nr * 2; i += blockDim.x) ((uint4*)s_descR)[i] = dR[i];
    int span = 0;
    for (int i = threadIdx.x; i < P; i += blockDim.x) {
        uint32_t key = 0xFFFFFFFFu;
        if (i < Nr) {
            const OrbKeyPoint kp = kR[i];
            const float r = 2.0f * g.lv[kp.octave].scale;
            RightRec rr;
            rr.x = kp.x;
            rr.oct = kp.octave;
            rr.maxr = (int)ceilf(kp.y + r);
            rr.minr = (int)floorf(kp.y - r);
            s_rec[i] = rr;
            span = max(span, rr.maxr - rr.minr);
            key = ((uint32_t)(rr.minr + 1024) << 16) | (uint32_t)i;
        }
        s_key[i] = key;
    }
    atomicMax(&s_maxspan, span);
    SYNC();
    // row -> first sorted record with minr >= row (rows -ST_ROFF .. height + ST_ROFF): the candidate
    // scan of a left keypoint reads one table entry per bound instead of a binary search
    uint16_t* s_rowst = (uint16_t*)((uint8_t*)(s_key + sa.sort_cap) + (ST_NT / 64) * (512 + 128 * 4));
    if (csort) {
        // counting sort by the first row of the band (clamped into the table; a clamped record only
        // moves towards the rows that can hold it, and the band test filters it): the order within
        // a row is immaterial, the scan keeps the first best in iR order through its (dist, iR) key.
        // Counts and cursors in the waves' SAD scratch, free until the keypoint loop.
        int* s_cnt = (int*)((uint8_t*)(s_key + sa.sort_cap) + (ST_NT / 64) * 512);
        for (int r = threadIdx.x; r <= nrow; r += blockDim.x) s_cnt[r] = 0;
        SYNC();
        for (int i = threadIdx.x; i < Nr; i += blockDim.x)
            atomicAdd(&s_cnt[min(max(s_rec[i].minr + ST_ROFF, 0), nrow - 1)], 1);
        SYNC();
        if (wave == 0) (void)wave_scan_lds(s_cnt, nrow + 1);
        SYNC();
        for (int r = threadIdx.x; r < nrow; r += blockDim.x) s_rowst[r] = (uint16_t)s_cnt[r];
        for (int i = threadIdx.x; i < Nr; i += blockDim.x) {
            const int bin = min(max(s_rec[i].minr + ST_ROFF, 0), nrow - 1);
            s_key[atomicAdd(&s_cnt[bin], 1)] = ((uint32_t)(bin - ST_ROFF + 1024) << 16) | (uint32_t)i;
        }
        SYNC();
    } else {
        for (int k = 2; k <= P; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = threadIdx.x; i < P; i += blockDim.x) {
                    const int ixj = i ^ j;
                    if (ixj > i) {
                        const uint32_t a = s_key[i], c = s_key[ixj];
                        if ((a > c) == ((i & k) == 0)) { s_key[i] = c; s_key[ixj] = a; }
                    }
                }
                SYNC();
            }
        for (int r = threadIdx.x; r < nrow; r += blockDim.x) {
            const uint32_t t = (uint32_t)max(r - ST_ROFF + 1024, 0) << 16;
            int lo = 0, hi = Nr;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_key[mid] < t) lo = mid + 1; else hi = mid;
            }
            s_rowst[r] = (uint16_t)lo;
        }
        SYNC();
    }
    const int maxspan = s_maxspan;
    float* uR_out = uright + (size_t)f * g.kp_cap;
    float* dp_out = depth + (size_t)f * g.kp_cap;
    int* sd_out = sdist + (size_t)f * g.kp_cap;
    const float mb = sa.bf / sa.fx;   // intended mb = mbf/fx (the reference reads it uninitialised)
    const float minZ = mb, minD = 0.f, maxD = sa.bf / minZ;
    const int iend = min(N, i0 + sa.lk);
    // the first keypoint of each wave is static; later ones come from a block counter, so waves whose
    // keypoints scan few candidates take more of them and the block ends with its work, not with its
    // slowest wave's fixed share (253 -> 236 us per 512 frames; r03_kernel_ab.txt item 29)
    for (int iL = i0 + wave; iL < iend;) {
        float outU = -1.0f, outD = -1.0f;
        int outS = -1;
        const OrbKeyPoint kpL = kL[iL];
        const int levelL = kpL.octave;
        const float vL = kpL.y, uL = kpL.x;
        const int row = (int)vL;
        const float minU = uL - maxD, maxU = uL - minD;
        uint32_t dl[8];
#pragma unroll
        for (int k = 0; k < 8; k++) dl[k] = dL[(size_t)iL * 8 + k];
        int bestKey = 0x7fffffff;   // (dist << 16) | iR: the first best in iR order
        bool anyCand = false;
        // records whose band can contain `row`: minr in [row - maxspan, row]
        auto lower = [&](uint32_t t) {
            int lo = 0, hi = Nr;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (s_key[mid] < t) lo = mid + 1; else hi = mid;
            }
            return lo;
        };
        const bool tab = row - maxspan >= -ST_ROFF && row + 1 < g.height + ST_ROFF;   // wave-uniform
        const int jlo = tab ? (int)s_rowst[row - maxspan + ST_ROFF] : lower((uint32_t)max(row - maxspan + 1024, 0) << 16);
        const int jhi = tab ? (int)s_rowst[row + 1 + ST_ROFF] : lower((uint32_t)max(row + 1 + 1024, 0) << 16);
        for (int j = jlo + lane; j < jhi; j += 64) {
            const int iR = (int)(s_key[j] & 0xFFFFu);
            const RightRec rr = s_rec[iR];
            if (rr.minr <= row && row <= rr.maxr) {
                anyCand = true;
                if (rr.oct >= levelL - 1 && rr.oct <= levelL + 1 && rr.x >= minU && rr.x <= maxU) {
                    const int dist = hamming32(dl, s_descR + 8 * iR);
                    bestKey = min(bestKey, (dist << 16) | iR);
                }
            }
        }
        bestKey = wave_min_dpp(bestKey);
        const bool cand = __any(anyCand) && !(maxU < 0);
        const int bestDist = bestKey == 0x7fffffff ? 100 : min(100, bestKey >> 16);
        if (cand && bestDist < 75) {   // thOrbDist = (TH_HIGH + TH_LOW) / 2
            const int bestIdxR = bestKey & 0xffff;
            const float uR0 = s_rec[bestIdxR].x;
            const float sf = g.lv[levelL].inv_scale;
            const float scaleduL = roundf(kpL.x * sf);
            const float scaledvL = roundf(kpL.y * sf);
            const float scaleduR0 = roundf(uR0 * sf);
            const int w = 5, Lr = 5;
            const float iniu = scaleduR0 + Lr - w;
            const float endu = scaleduR0 + Lr + w + 1;
            const OrbLevel& LV = g.lv[levelL];
            if (!(iniu < 0 || endu >= LV.w)) {
                int pL, pR;
                gptr_u8 IL = level_base(SL.imgs, SL.in_pitch, SL.pyr, SL.pyr_stride, g, bL, levelL, &pL);
                gptr_u8 IR = level_base(SR.imgs, SR.in_pitch, SR.pyr, SR.pyr_stride, g, bR, levelL, &pR);
                const int r0 = (int)(scaledvL - w), c0L = (int)(scaleduL - w), c0R = (int)(scaleduR0 - Lr - w);
                // stage the IL 11x11 and IR 11x21 windows as dword rows (IL: 3 dwords, byte 11
                // zeroed; IR: 6 dwords): lanes 0-10 load a left row, 11-21 a right row with aligned
                // dword loads (the windows lie >= 6 px inside the level, so the <= 3-byte over-reads
                // stay inside the image) realigned by v_alignbyte
                uint32_t* s_wl = (uint32_t*)s_win;          // [11][3]
                uint32_t* s_wr = (uint32_t*)s_win + 33;     // [11][6]
                if (lane < 22) {
                    const bool left = lane < 11;
                    const int yy = left ? lane : lane - 11;
                    gptr_u8 rp = left ? IL + (size_t)(r0 + yy) * pL + c0L : IR + (size_t)(r0 + yy) * pR + c0R;
                    const uint32_t sh = (uint32_t)((uintptr_t)rp & 3);
                    gptr_u32 ap = (gptr_u32)(rp - sh);
                    uint32_t w[7];
#pragma unroll
                    for (int k = 0; k < 7; k++) w[k] = (left && k >= 4) ? 0u : ap[k];
                    if (left) {
#pragma unroll
                        for (int k = 0; k < 3; k++) {
                            uint32_t o = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
                            if (k == 2) o &= 0x00FFFFFFu;
                            s_wl[yy * 3 + k] = o;
                        }
                    } else {
#pragma unroll
                        for (int k = 0; k < 6; k++) s_wr[yy * 6 + k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
                    }
                }
                // lanes: (shift inc, window row) pairs -> row SAD over 11 columns, 3 v_sad_u8
                for (int pidx = lane; pidx < 121; pidx += 64) {
                    const int inc = pidx / 11, yy = pidx - inc * 11;
                    const uint32_t* rr = s_wr + yy * 6 + (inc >> 2);
                    const uint32_t ish = (uint32_t)(inc & 3);
                    const uint32_t r0w = __builtin_amdgcn_alignbyte(rr[1], rr[0], ish);
                    const uint32_t r1w = __builtin_amdgcn_alignbyte(rr[2], rr[1], ish);
                    const uint32_t r2w = __builtin_amdgcn_alignbyte(rr[3], rr[2], ish) & 0x00FFFFFFu;
                    const uint32_t* ll = s_wl + yy * 3;
                    s_part[pidx] = (int)__builtin_amdgcn_sad_u8(
                        ll[2], r2w, __builtin_amdgcn_sad_u8(ll[1], r1w, __builtin_amdgcn_sad_u8(ll[0], r0w, 0u)));
                }
                int dsum = 0;
                if (lane < 11)
                    for (int yy = 0; yy < 11; yy++) dsum += s_part[lane * 11 + yy];
                float dists[11];
                int bestD = 0x7fffffff, bestinc = 0;
#pragma unroll
                for (int k = 0; k < 11; k++) {
                    const float dist = (float)__builtin_amdgcn_readlane(dsum, k);   // cv::norm(NORM_L1) of shift k - Lr
                    dists[k] = dist;
                    if (dist < (float)bestD) { bestD = (int)dist; bestinc = k - Lr; }
                }
                if (!(bestinc == -Lr || bestinc == Lr)) {
                    const float dist1 = dists[Lr + bestinc - 1], dist2 = dists[Lr + bestinc], dist3 = dists[Lr + bestinc + 1];
                    const float deltaR = (dist1 - dist3) / (2.0f * (dist1 + dist3 - 2.0f * dist2));
                    if (!(deltaR < -1 || deltaR > 1)) {
                        float bestuR = LV.scale * ((float)scaleduR0 + (float)bestinc + deltaR);
                        float disparity = (uL - bestuR);
                        if (disparity >= minD && disparity < maxD) {
                            if (disparity <= 0) { disparity = (float)0.01; bestuR = (float)((double)uL - 0.01); }
                            outD = sa.bf / disparity;
                            outU = bestuR;
                            outS = bestD;
                        }
                    }
                }
            }
        }
        if (lane == 0) { uR_out[iL] = outU; dp_out[iL] = outD; sd_out[iL] = outS; }
        int nx = 0;
        if (lane == 0) nx = atomicAdd(&s_next, 1);
        iL = i0 + __builtin_amdgcn_readfirstlane(nx);
    }
}

// Stage 2 (one block per frame): the median outlier cut of ComputeStereoMatches (Frame.cc:966-980):
// median = the (n/2)-th smallest accepted SAD distance (vDistIdx sorted, index size/2), then every
// match with dist >= 1.5f*1.4f*median is dropped. The median is selected by two histogram passes
// (distances are < 2^16: 121 window bytes x 255), high byte then low byte, instead of a sort.
__device__ __forceinline__ int block256_excl_scan(int v, int* s_ws, int* total) {
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    const int incl = wave_incl_scan(v);
    if (lane == 63) s_ws[wave] = incl;
    SYNC();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; w++) {
        const int t = s_ws[w];
        off += w < wave ? t : 0;
        tot += t;
    }
    *total = tot;
    return off + incl - v;
}
__global__ __launch_bounds__(256) void k_stereo_cut(OrbGeom g, StereoSide SL, StereoArgs sa, float* uright,
                                                    float* depth, const int* sdist, int* nmatch) {
    __shared__ int s_h[256];
    __shared__ int s_ws[4];
    __shared__ int s_sel[2];
    const int f = blockIdx.x, t = threadIdx.x;
    const int bL = SL.base + f * SL.step;
    const int N = SL.counts[2 * bL];
    const int* sd = sdist + (size_t)f * g.kp_cap;
    // pass 1: histogram of the high byte
    s_h[t] = 0;
    SYNC();
    for (int i = t; i < N; i += blockDim.x) {
        const int d = sd[i];
        if (d >= 0) atomicAdd(&s_h[min(d, 65535) >> 8], 1);
    }
    SYNC();
    int n;
    {
        const int c = s_h[t];
        const int ex = block256_excl_scan(c, s_ws, &n);
        const int k = n / 2;
        if (ex <= k && k < ex + c) { s_sel[0] = t; s_sel[1] = k - ex; }
    }
    if (t == 0) nmatch[f] = n;
    if (n == 0) return;   // the reference indexes vDistIdx[size/2] unguarded here (block-uniform)
    SYNC();
    const int hb = s_sel[0], k2 = s_sel[1];
    // pass 2: histogram of the low byte among the distances whose high byte is hb
    s_h[t] = 0;
    SYNC();
    for (int i = t; i < N; i += blockDim.x) {
        const int d = sd[i];
        if (d >= 0 && (min(d, 65535) >> 8) == hb) atomicAdd(&s_h[d & 255], 1);
    }
    SYNC();
    {
        int n2;
        const int c = s_h[t];
        SYNC();   // s_ws is reused by the second scan
        const int ex = block256_excl_scan(c, s_ws, &n2);
        if (ex <= k2 && k2 < ex + c) s_sel[0] = (hb << 8) | t;
    }
    SYNC();
    const float median = (float)s_sel[0];
    const float thDist = 1.5f * 1.4f * median;
    float* uR = uright + (size_t)f * g.kp_cap;
    float* dp = depth + (size_t)f * g.kp_cap;
    for (int i = t; i < N; i += blockDim.x) {
        const int d = sd[i];
        if (d >= 0 && !((float)d < thDist)) { uR[i] = -1; dp[i] = -1; }
    }
}

}  // namespace orbfe
