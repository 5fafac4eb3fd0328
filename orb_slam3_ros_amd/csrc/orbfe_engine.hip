// Host engine + C-ABI of liborbfe.so (declared in include/orbfe.h).
// Owns the device buffers of one extractor handle (sized for the largest batch seen so far),
// derives the per-level geometry with the reference's exact expressions, and launches the
// kernel sequence of orbfe_kernels.hip on one HIP stream.
#pragma clang fp contract(off)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cstddef>
#include <mutex>
#include <vector>

#include "../../include/orbfe.h"
#include "orbfe_types.h"

// Single translation unit: the kernels are compiled together with their launchers.
#include "orbfe_kernels.hip"

using namespace orbfe;

#define HIPCHK(x)                                                                                 \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            fprintf(stderr, "orbfe: HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return ORBFE_E_DEVICE;                                                                \
        }                                                                                         \
    } while (0)

namespace {

inline int cv_round(float v) { return (int)std::lrintf(v); }
inline int cv_floor(float v) { int i = (int)v; return i - (i > v); }
inline short sat_s16(float v) {
    int iv = cv_round(v);
    return (short)std::min(32767, std::max(-32768, iv));
}
inline int round_up(int v, int a) { return (v + a - 1) / a * a; }

// blur kernel quantisation (see oracle header): 0 = OpenCV >= 3.4.6 error-diffusion (default)
const int kBlurED[7] = {18, 34, 48, 56, 48, 34, 18};
const int kBlurRound[7] = {18, 34, 49, 55, 49, 34, 18};

size_t octree_lds_bytes(const OrbGeom& g) {
    auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    const size_t NC = g.node_cap;
    size_t s = a16(sizeof(int) * (g.max_cells_level + 1));
    s += 2 * (4 * a16(2 * NC) + a16(4 * NC));
    s += 2 * a16(16 * NC);
    s += a16(8 * NC) + a16(2 * NC) + a16(4 * NC) * 5;
    s += a16(8 * NC);   // expv (the sort scratch and the best keys alias the next-count table)
    s += a16(16 * ORBFE_SORT_STACK);
    return s;
}

// Output block of a batch of B images with kp_cap slots each: counts (2 ints per image) at 0,
// keypoints from *kps, descriptors from *desc (16-byte aligned), *end bytes in all.
void out_layout(int B, int kp_cap, size_t* kps, size_t* desc, size_t* end) {
    auto a16 = [](size_t b) { return (b + 15) & ~(size_t)15; };
    *kps = a16((size_t)B * 8);
    *desc = a16(*kps + (size_t)B * kp_cap * sizeof(OrbKeyPoint));
    *end = *desc + (size_t)B * kp_cap * 32;
}

// A/B switches (tools/gpu_pyr_ab.sh) are read from the environment only by a diagnostic build
// (tools/build_variant.sh NAME -DORBFE_AB_KNOBS=1); the product library's kernels, launch shapes
// and transfer paths never depend on the caller's environment.
#ifndef ORBFE_AB_KNOBS
#define ORBFE_AB_KNOBS 0
#endif
inline bool ab_knob(const char* name) {
#if ORBFE_AB_KNOBS
    return getenv(name) != nullptr;
#else
    (void)name;
    return false;
#endif
}

}  // namespace

struct orbfe_extractor {
    int nfeatures, nlevels, ini_th, min_th;
    float scale_factor_f;
    double scale_factor;
    int resize_simd_lanes = 16;
    bool no_fused_pyramid = ab_knob("ORBFE_NO_FUSED_PYRAMID");   // A/B: the chained launches
    bool fused_pyramid_batch = ab_knob("ORBFE_FUSED_PYR_BATCH");  // A/B: k_pyramid for large batches too
    bool no_pull = ab_knob("ORBFE_NO_PULL");   // A/B: the frame call's results by DMA copies
    bool no_push = ab_knob("ORBFE_NO_PUSH");   // A/B: the frame call's images by a DMA copy
    int blur_variant = 0;
    std::vector<float> scale, inv_scale, sigma2, inv_sigma2;
    std::vector<int> per_level;
    int device = 0;
    hipStream_t own_stream = nullptr;
    // split path: FAST of level 0 runs on side_stream while the resize chain runs on the batch
    // stream (fork / join events)
    hipStream_t side_stream = nullptr;
    hipEvent_t ev_fork[ORBFE_MAX_LEVELS + 1] = {};
    // geometry of the current allocation
    int W = 0, H = 0, cap_b = 0;
    OrbGeom g{};
    std::vector<int16_t> tab;
    FastLds fast_lds{};   // k_fast per-wave LDS layout (max over levels)
    FastLds fast_lds_lv[ORBFE_MAX_LEVELS] = {};   // per level: a launch over levels [a, b] sizes its LDS by their max
    size_t oct_lds = 0;
    // k_pyramid tile records (small batches); pt_n = 0 when the geometry does not fit its limits
    std::vector<uint32_t> ptile;
    int pt_n = 0, pt_stride = 0, pt_cap = 0;
    size_t pt_lds = 0;
    // device buffers
    int16_t* d_tab = nullptr;
    uint32_t* d_ptile = nullptr;
    uint8_t* d_pyr = nullptr;
    uint32_t* d_cellkeys = nullptr;
    int* d_cellcnt = nullptr;
    uint32_t* d_lkeys = nullptr;
    uint16_t* d_nodeof = nullptr;
    uint32_t* d_outkeys = nullptr;
    int* d_lvinfo = nullptr;
    int* d_ranks = nullptr;
    uint8_t* d_out = nullptr;      // one allocation: d_counts | d_kps | d_desc (out_layout)
    OrbKeyPoint* d_kps = nullptr;
    uint8_t* d_desc = nullptr;
    int* d_counts = nullptr;
    const uint8_t** d_ptrs = nullptr;
    uint8_t* d_stage = nullptr;    // host-API input staging (one image)
    size_t stage_bytes = 0;
    // host-API pinned staging: the image going up, then {counts, keypoints [kp_cap], descriptors
    // [kp_cap]} coming back in one round trip (DMA from / to pinned memory, no runtime bounce)
    uint8_t* h_pin = nullptr;
    size_t pin_bytes = 0;
    // host-API stereo results in one allocation {nmatch (16 B) | uR [stereo_kp] | depth [stereo_kp]}
    uint8_t* d_st = nullptr;
    float* d_uright = nullptr;
    float* d_depth = nullptr;
    int* d_nmatch = nullptr;
    int* d_sdist = nullptr;       // per left kp SAD distance of accepted stereo matches
    int sdist_frames = 0, sdist_kp = 0;   // d_sdist holds sdist_frames x sdist_kp entries
    int stereo_kp = 0;            // d_uright / d_depth (host-API stereo) hold stereo_kp entries
    std::mutex mu_stereo;
    // last batch description
    int last_nimg = 0, last_pitch = 0;
    // extraction counter (every run_batch) and the matcher view of the last orbfe_frame_stereo call:
    // its id, left keypoint count, and the scale factors on the device (orbfe_frame_device_view)
    uint64_t frame_id = 0, fs_id = 0;
    int fs_n = 0;
    float* d_scale = nullptr;
    std::vector<const uint8_t*> last_ptrs;
    std::vector<int> last_laps;   // vLappingArea {lap0, lap1} per image of the last batch
    // stage timing
    bool timing = false;
    hipEvent_t ev[ORBFE_NUM_STAGES + 1] = {};   // spare set (host API)
    // host-API call timing (orbfe_get_call_timing): events around the upload, the kernels and the
    // result copies of the last orbfe_extract / orbfe_stereo_match on this handle
    hipEvent_t call_ev[7] = {};
    float call_ms[5] = {};
    std::vector<std::vector<hipEvent_t>> ev_ring;  // one event set per timed batch, read lazily
    int ev_used = 0;
    float stage_ms[ORBFE_NUM_STAGES] = {};
    // optional caller-owned outputs (orbfe_set_batch_outputs)
    OrbKeyPoint* ext_kps = nullptr;
    uint8_t* ext_desc = nullptr;
    int* ext_counts = nullptr;
    int ext_cap_images = 0;
    OrbKeyPoint* last_kps = nullptr;
    uint8_t* last_desc = nullptr;
    int* last_counts = nullptr;
    std::mutex mu;
    unsigned long long* d_oct_ts = nullptr;   // -DORBFE_OCT_STAMPS builds: per-phase s_memtime of the octree (image 0)
};

static void free_buffers(orbfe_extractor* h) {
    void** bufs[] = {(void**)&h->d_tab, (void**)&h->d_ptile, (void**)&h->d_pyr, (void**)&h->d_cellkeys,
                     (void**)&h->d_cellcnt, (void**)&h->d_lkeys, (void**)&h->d_nodeof, (void**)&h->d_outkeys,
                     (void**)&h->d_lvinfo, (void**)&h->d_ranks, (void**)&h->d_out, (void**)&h->d_ptrs};
    for (void** p : bufs) {
        if (*p) (void)hipFree(*p);
        *p = nullptr;
    }
    h->d_kps = nullptr;   // inside d_out
    h->d_desc = nullptr;
    h->d_counts = nullptr;
    h->cap_b = 0;
    h->last_nimg = 0;   // the previous batch's intermediates are gone
    h->last_kps = nullptr;
    h->last_desc = nullptr;
    h->last_counts = nullptr;
    h->last_ptrs.clear();
    h->last_laps.clear();
}

// Per-level geometry with the reference's expressions (see orbfe_types.h), derived into the
// caller's locals: the handle's current geometry stays untouched when the size is rejected.
static int build_geom(const orbfe_extractor* h, int W, int H, OrbGeom& g, std::vector<int16_t>& tab,
                      FastLds& fast_lds, FastLds* fast_lds_lv, size_t& oct_lds) {
    memset(&g, 0, sizeof(g));
    g.nlevels = h->nlevels;
    g.width = W;
    g.height = H;
    g.ini_th = std::min(std::max(h->ini_th, 0), 255);
    g.min_th = std::min(std::max(h->min_th, 0), 255);
    tab.clear();
    int cell_base = 0, cellkey_off = 0, out_off = 0, pyr_off = 0;
    int max_cells = 0, node_cap = 0;
    FastLds fl{0, 0, 0, 0};
    int pw = W, ph = H;
    for (int l = 0; l < h->nlevels; l++) {
        OrbLevel& L = g.lv[l];
        L.w = cv_round((float)W * h->inv_scale[l]);
        L.h = cv_round((float)H * h->inv_scale[l]);
        if (L.w < 2 * ORBFE_MINB + ORBFE_CELL + 6 || L.h < 2 * ORBFE_MINB + ORBFE_CELL + 6 || L.w > 4096 + 32 ||
            L.h > 4096 + 32)
            return ORBFE_E_ARG;
        L.scale = h->scale[l];
        L.inv_scale = h->inv_scale[l];
        L.patch_size = (int)(31 * h->scale[l]);
        L.pitch = round_up(L.w, 16);
        L.pyr_off = l == 0 ? 0 : pyr_off;
        if (l > 0) pyr_off += round_up(L.pitch * L.h, 256);
        // FAST cell grid (ORBextractor.cc:789-803)
        const int minB = ORBFE_MINB, maxBX = L.w - ORBFE_MINB, maxBY = L.h - ORBFE_MINB;
        const float width = (float)(maxBX - minB), height = (float)(maxBY - minB);
        const float Wc = ORBFE_CELL;
        L.n_cols = (int)(width / Wc);
        L.n_rows = (int)(height / Wc);
        L.w_cell = (int)std::ceil(width / L.n_cols);
        L.h_cell = (int)std::ceil(height / L.n_rows);
        L.cell_base = cell_base;
        const int ncell = L.n_cols * L.n_rows;
        cell_base += ncell;
        max_cells = std::max(max_cells, ncell);
        L.cell_cap = ((L.w_cell + 1) / 2) * ((L.h_cell + 1) / 2);
        L.cellkey_off = cellkey_off;
        cellkey_off += ncell * L.cell_cap;
        {   // k_fast: RS = 16 * ceil((ceil(dw / 4) + 2) / 4) with dw <= w_cell; ROI rows <= h_cell + 6, score
            // map rows <= h_cell + 2; corner list 2 B per pixel and >= 8 B per 4-pixel group + 256
            const int rs = 16 * (((L.w_cell + 3) / 4 + 2 + 3) / 4), grp = ((L.w_cell + 3) / 4) * L.h_cell;
            FastLds& f = fast_lds_lv[l];
            f.roi = round_up(rs * (L.h_cell + 6), 16);
            f.sc = round_up(rs * (L.h_cell + 2), 16);
            f.cor = round_up(std::max(2 * L.w_cell * L.h_cell, 8 * grp + 256), 16);
            f.wave_bytes = f.roi + f.sc + f.cor + FAST_ENT_BYTES;
            fl.roi = std::max(fl.roi, f.roi);
            fl.sc = std::max(fl.sc, f.sc);
            fl.cor = std::max(fl.cor, f.cor);
        }
        if (L.w_cell > 127 || L.h_cell > 127) return ORBFE_E_ARG;   // k_fast packs dx, dy in 7 bits
        // octree
        L.budget = h->per_level[l];
        L.n_ini = (int)std::round((float)(maxBX - minB) / (maxBY - minB));
        if (L.n_ini < 1) return ORBFE_E_ARG;   // the reference indexes an empty node vector here
        L.hx = (float)(maxBX - minB) / L.n_ini;
        L.out_cap = std::max(L.budget + 3, 4 * L.n_ini);
        L.out_off = out_off;
        out_off += L.out_cap;
        node_cap = std::max(node_cap, L.out_cap + 8);
        // resize tables (cv::resize INTER_LINEAR, dsize given, from level l-1)
        if (l > 0) {
            const double inv_x = (double)L.w / pw, inv_y = (double)L.h / ph;
            const double scale_x = 1. / inv_x, scale_y = 1. / inv_y;
            L.tab_x = (int)tab.size();
            int xmax = L.w;
            for (int dx = 0; dx < L.w; dx++) {
                float fx = (float)((dx + 0.5) * scale_x - 0.5);
                int sx = cv_floor(fx);
                fx -= sx;
                if (sx < 0) { fx = 0; sx = 0; }
                if (sx + 1 >= pw) {
                    xmax = std::min(xmax, dx);
                    if (sx >= pw - 1) { fx = 0; sx = pw - 1; }
                }
                tab.push_back((int16_t)sx);
                tab.push_back(sat_s16((1.f - fx) * 2048));
                tab.push_back(sat_s16(fx * 2048));
            }
            L.xmax = xmax;
            L.tab_y = (int)tab.size();
            for (int dy = 0; dy < L.h; dy++) {
                float fy = (float)((dy + 0.5) * scale_y - 0.5);
                int sy = cv_floor(fy);
                fy -= sy;
                auto clip = [&](int v) { return v < 0 ? 0 : (v >= ph ? ph - 1 : v); };
                tab.push_back((int16_t)clip(sy));
                tab.push_back((int16_t)clip(sy + 1));
                tab.push_back(sat_s16((1.f - fy) * 2048));
                tab.push_back(sat_s16(fy * 2048));
            }
            int x = 0;
            const int lanes = h->resize_simd_lanes;
            if (lanes > 0) {
                for (; x <= L.w - lanes; x += lanes) {}
                for (; x < L.w - lanes / 2; x += lanes / 2) {}
            }
            L.simd_end = x;
            // tile geometry: the largest tile whose source window fits s_src[RZ_SR][RZ_SCB] for
            // every tile of the level (checked exactly on the coefficient tables)
            (void)scale_x;
            (void)scale_y;
            const int16_t* tx = tab.data() + L.tab_x;
            const int16_t* ty = tab.data() + L.tab_y;
            auto rows_fit = [&](int tr) {
                for (int y0 = 0; y0 < L.h; y0 += tr) {
                    const int y1 = std::min(y0 + tr, L.h);
                    if (ty[4 * (y1 - 1) + 1] - ty[4 * y0] + 1 > RZ_SR) return false;
                }
                return true;
            };
            auto cols_fit = [&](int tc) {
                for (int x0 = 0; x0 < L.w; x0 += tc) {
                    const int x1 = std::min(x0 + tc, L.w);
                    const int sc0 = tx[3 * x0] & ~3, sc1 = std::min((int)tx[3 * (x1 - 1)] + 2, pw);
                    if (round_up(sc1 - sc0, 16) > RZ_SCB) return false;   // k_resize stores 16-byte chunks
                }
                return true;
            };
            int tr = RZ_TR, tc = RZ_TC;
            while (tr > 1 && !rows_fit(tr)) tr--;
            while (tc > 4 && !cols_fit(tc)) tc -= 4;
            if (!rows_fit(tr) || !cols_fit(tc)) return ORBFE_E_ARG;
            L.rz_rows = tr;
            L.rz_cols = tc;
            // k_resize_s rules: in every lane group of 4 output columns, columns 0, 1 take their
            // byte pair at sx - (sx_0 & ~3) in [0, 6], columns 2, 3 at that offset - 2 in [0, 6];
            // every output row reads rows (s - 1, s), the table never clipping, for distinct s
            L.rs_ok = 1;
            for (int xq = 0; xq < L.w && L.rs_ok; xq += 4) {
                const int base = tx[3 * xq] & ~3;
                for (int q = 0; q < 4 && xq + q < L.w; q++) {
                    const int off = tx[3 * (xq + q)] - base - (q >= 2 ? 2 : 0);
                    if (off < 0 || off > 6) L.rs_ok = 0;
                }
            }
            for (int y = 0; y < L.h && L.rs_ok; y++)
                if (ty[4 * y + 1] != ty[4 * y] + 1 || (y > 0 && ty[4 * y + 1] == ty[4 * (y - 1) + 1])) L.rs_ok = 0;
            L.rs_rows = std::min(RS_ROWS, 64);
        }
        pw = L.w;
        ph = L.h;
    }
    g.total_cells = cell_base;
    g.cellkeys_per_img = cellkey_off;
    g.out_per_img = out_off;
    g.kp_cap = out_off;
    g.pyr_slack = pyr_off;
    g.pyr_bytes = round_up(pyr_off + 256, 256);
    g.max_cells_level = max_cells;
    g.node_cap = node_cap;
    fl.wave_bytes = fl.roi + fl.sc + fl.cor + FAST_ENT_BYTES;
    fast_lds = fl;
    oct_lds = octree_lds_bytes(g);
    if (oct_lds > 160 * 1024) return ORBFE_E_ARG;
    if ((size_t)FAST_WPB * fast_lds.wave_bytes > 160 * 1024) return ORBFE_E_ARG;   // k_fast: FAST_WPB waves per block
    return ORBFE_OK;
}

// k_pyramid tiles (orbfe_kernels.hip K1c): TX x TY tiles, tile (i, j) owning columns
// [4 floor(i W_l / 4 TX), ...) and rows [floor(j H_l / TY), ...) of every level l >= 1, and the
// rectangle it needs at each level: its own plus the source cone of its needs one level up
// (columns sx, sx + 1 and rows s0, s1 of the level's tables), from the top level down to the
// level-0 window. Returns false when a limit of the kernel is exceeded (then the chained launches run).
static bool build_pyr_tiles(const OrbGeom& g, const std::vector<int16_t>& tab, std::vector<uint32_t>& out, int& ntiles,
                            int& stride, int& cap, size_t& lds) {
    const int nl = g.nlevels;
    out.clear();
    ntiles = stride = cap = 0;
    lds = 0;
    if (nl < 2) return false;
    const int W1 = g.lv[1].w, H1 = g.lv[1].h;
    // level-1 tile target (ORBFE_PYR_TILE=WxH overrides it in an -DORBFE_AB_KNOBS=1 build): 56x40 at 752x480 makes
    // 12 x 10 tiles; k_pyramid at B=2, 1024 threads: 32x32 14.0 us, 48x40 11.7-12.1, 56x40 10.6,
    // 56x48 10.6-10.7, 64x48 10.9-11.0, 72x56 11.4 (r05_kernel_ab.txt item 12)
    int tw = 56, th = 40;
#if ORBFE_AB_KNOBS
    if (const char* e = getenv("ORBFE_PYR_TILE")) {
        int a = 0, c = 0;
        if (sscanf(e, "%dx%d", &a, &c) == 2 && a >= 8 && c >= 8) { tw = a; th = c; }
    }
#endif
    int TX = std::max(1, (W1 + tw - 1) / tw), TY = std::max(1, (H1 + th - 1) / th);
    struct R { int x0, x1, y0, y1; };
    auto own = [&](int l, int i, int j, int TXn, int TYn) {
        const OrbLevel& L = g.lv[l];
        R r;
        r.x0 = i == 0 ? 0 : (int)((long long)i * L.w / TXn) & ~3;
        r.x1 = i + 1 == TXn ? L.w : (int)((long long)(i + 1) * L.w / TXn) & ~3;
        r.y0 = (int)((long long)j * L.h / TYn);
        r.y1 = j + 1 == TYn ? L.h : (int)((long long)(j + 1) * L.h / TYn);
        return r;
    };
    for (;;) {   // every tile must own a non-empty rectangle of every level
        bool ok = true;
        for (int l = 1; l < nl && ok; l++)
            for (int i = 0; i < TX && ok; i++) {
                const R r = own(l, i, 0, TX, TY);
                if (r.x1 <= r.x0) ok = false;
            }
        for (int l = 1; l < nl && ok; l++)
            for (int j = 0; j < TY && ok; j++) {
                const R r = own(l, 0, j, TX, TY);
                if (r.y1 <= r.y0) ok = false;
            }
        if (ok) break;
        if (TX == 1 && TY == 1) return false;
        if (TX >= TY && TX > 1) TX--; else TY--;
    }
    std::vector<std::vector<uint32_t>> recs;
    for (int j = 0; j < TY; j++)
        for (int i = 0; i < TX; i++) {
            std::vector<R> need(nl), ow(nl);
            for (int l = 1; l < nl; l++) ow[l] = own(l, i, j, TX, TY);
            // top level: its own rectangle, columns rounded out to whole dwords
            need[nl - 1] = {ow[nl - 1].x0, round_up(ow[nl - 1].x1, 4), ow[nl - 1].y0, ow[nl - 1].y1};
            for (int l = nl - 1; l >= 1; l--) {
                const OrbLevel& L = g.lv[l];
                const OrbLevel& P = g.lv[l - 1];
                const int16_t* tx = tab.data() + L.tab_x;
                const int16_t* ty = tab.data() + L.tab_y;
                int c0 = 1 << 30, c1 = -1, r0 = 1 << 30, r1 = -1;
                for (int x = need[l].x0; x < need[l].x1; x++) {
                    const int xi = std::min(x, L.w - 1), sx = tx[3 * xi];
                    c0 = std::min(c0, sx);
                    c1 = std::max(c1, std::min(sx + 1, P.w - 1));
                }
                for (int y = need[l].y0; y < need[l].y1; y++) {
                    r0 = std::min(r0, (int)ty[4 * y]);
                    r1 = std::max(r1, (int)ty[4 * y + 1]);
                }
                R n{c0 & ~3, round_up(c1 + 1, 4), r0, r1 + 1};
                if (l - 1 >= 1) {
                    const R& o = ow[l - 1];
                    n.x0 = std::min(n.x0, o.x0);
                    n.x1 = std::max(n.x1, round_up(o.x1, 4));
                    n.y0 = std::min(n.y0, o.y0);
                    n.y1 = std::max(n.y1, o.y1);
                    n.x1 = std::min(n.x1, round_up(P.w, 4));
                }
                need[l - 1] = n;
            }
            std::vector<uint32_t> rc(5 * nl + (nl & 1 ? 1 : 0), 0u);   // header (body starts on an even dword)
            for (int l = 0; l < nl; l++) {
                const R& n = need[l];
                if (n.x1 > 65535 || n.y1 > 65535) return false;
                cap = std::max(cap, (n.x1 - n.x0) * (n.y1 - n.y0));
                rc[5 * l + 0] = (uint32_t)n.x0 | ((uint32_t)n.x1 << 16);
                rc[5 * l + 1] = (uint32_t)n.y0 | ((uint32_t)n.y1 << 16);
                if (l >= 1) {
                    rc[5 * l + 2] = (uint32_t)ow[l].x0 | ((uint32_t)ow[l].x1 << 16);
                    rc[5 * l + 3] = (uint32_t)ow[l].y0 | ((uint32_t)ow[l].y1 << 16);
                }
            }
            for (int l = 1; l < nl; l++) {
                const OrbLevel& L = g.lv[l];
                const R& n = need[l];
                const R& p = need[l - 1];
                const int16_t* tx = tab.data() + L.tab_x;
                const int16_t* ty = tab.data() + L.tab_y;
                const size_t coloff = rc.size();
                for (int x = n.x0; x < n.x1; x++) {
                    const int xi = std::min(x, L.w - 1);
                    const int sx = tx[3 * xi];
                    const bool lin = xi < L.xmax;
                    const int a0 = lin ? tx[3 * xi + 1] : 2048, a1 = lin ? tx[3 * xi + 2] : 0;
                    const int s0 = sx - p.x0, s1 = std::min(sx + 1, p.x1 - 1) - p.x0;
                    if (s0 < 0 || s1 >= p.x1 - p.x0 || s0 > 0x7fff || a0 < 0 || a1 < 0) return false;
                    rc.push_back((uint32_t)s0 | ((uint32_t)s1 << 15) | ((x < L.simd_end ? 1u : 0u) << 30));
                    rc.push_back((uint32_t)a0 | ((uint32_t)a1 << 16));
                }
                const size_t rowoff = rc.size();
                for (int y = n.y0; y < n.y1; y++) {
                    const int s0 = ty[4 * y] - p.y0, s1 = ty[4 * y + 1] - p.y0;
                    const int b0 = ty[4 * y + 2], b1 = ty[4 * y + 3];
                    if (s0 < 0 || s1 >= p.y1 - p.y0 || b0 < 0 || b1 < 0) return false;
                    rc.push_back((uint32_t)s0 | ((uint32_t)s1 << 16));
                    rc.push_back((uint32_t)b0 | ((uint32_t)b1 << 16));
                }
                if (rowoff > 65535) return false;
                rc[5 * l + 4] = (uint32_t)coloff | ((uint32_t)rowoff << 16);
            }
            const R& w0 = need[0];
            if (((w0.x1 - w0.x0) >> 2) * (w0.y1 - w0.y0) > PYR_NT * PYR_U0) return false;
            recs.push_back(std::move(rc));
        }
    for (auto& r : recs) stride = std::max(stride, round_up((int)r.size(), 4));
    if (stride / 4 > PYR_NT * PYR_RU) return false;
    cap = round_up(cap, 16);
    lds = (size_t)stride * 4 + 2 * (size_t)cap;
    if (lds > 64 * 1024) return false;
    ntiles = (int)recs.size();
    out.assign((size_t)ntiles * stride, 0u);
    for (int t = 0; t < ntiles; t++) std::copy(recs[t].begin(), recs[t].end(), out.begin() + (size_t)t * stride);
    return true;
}

static int ensure(orbfe_extractor* h, int W, int H, int B) {
    if (W == h->W && H == h->H && B <= h->cap_b) return ORBFE_OK;
    HIPCHK(hipSetDevice(h->device));
    if (W != h->W || H != h->H) {
        // a rejected size leaves the handle exactly as it was (geometry, tables and buffers)
        OrbGeom g;
        std::vector<int16_t> tab;
        FastLds fl{}, fl_lv[ORBFE_MAX_LEVELS] = {};
        size_t oct = 0;
        int rc = build_geom(h, W, H, g, tab, fl, fl_lv, oct);
        if (rc) return rc;
        free_buffers(h);
        h->g = g;
        h->tab.swap(tab);
        h->fast_lds = fl;
        memcpy(h->fast_lds_lv, fl_lv, sizeof(fl_lv));
        h->oct_lds = oct;
        if (!build_pyr_tiles(h->g, h->tab, h->ptile, h->pt_n, h->pt_stride, h->pt_cap, h->pt_lds)) h->pt_n = 0;
        h->W = W;
        h->H = H;
    } else {
        free_buffers(h);
    }
    B = std::max(B, 1);
    const OrbGeom& g = h->g;
    HIPCHK(hipMalloc(&h->d_tab, std::max<size_t>(2, h->tab.size() * 2)));
    HIPCHK(hipMemcpy(h->d_tab, h->tab.data(), h->tab.size() * 2, hipMemcpyHostToDevice));
    if (h->pt_n > 0) {
        HIPCHK(hipMalloc(&h->d_ptile, h->ptile.size() * 4));
        HIPCHK(hipMemcpy(h->d_ptile, h->ptile.data(), h->ptile.size() * 4, hipMemcpyHostToDevice));
    }
    HIPCHK(hipMalloc(&h->d_pyr, (size_t)B * g.pyr_bytes));
    HIPCHK(hipMalloc(&h->d_cellkeys, (size_t)B * g.cellkeys_per_img * 4));
    HIPCHK(hipMalloc(&h->d_cellcnt, (size_t)B * g.total_cells * 4));
    HIPCHK(hipMalloc(&h->d_lkeys, (size_t)B * g.cellkeys_per_img * 4));
    HIPCHK(hipMalloc(&h->d_nodeof, (size_t)B * g.cellkeys_per_img * 2));
    HIPCHK(hipMalloc(&h->d_outkeys, (size_t)B * g.out_per_img * 4));
    HIPCHK(hipMalloc(&h->d_lvinfo, (size_t)B * g.nlevels * 4 * 4));
    HIPCHK(hipMalloc(&h->d_ranks, (size_t)B * g.out_per_img * 4));
    // outputs in one block, {counts | keypoints | descriptors} (out_layout): for one image it is the
    // host API's pinned result layout, so orbfe_extract brings it back in a single copy
    size_t o_kps, o_desc, o_end;
    out_layout(B, g.kp_cap, &o_kps, &o_desc, &o_end);
    HIPCHK(hipMalloc(&h->d_out, o_end));
    h->d_counts = (int*)h->d_out;
    h->d_kps = (OrbKeyPoint*)(h->d_out + o_kps);
    h->d_desc = h->d_out + o_desc;
    HIPCHK(hipMalloc(&h->d_ptrs, (size_t)B * (sizeof(void*) + 2 * sizeof(int))));   // image pointers, then laps
    h->cap_b = B;
    h->last_ptrs.clear();
    h->last_laps.clear();
    return ORBFE_OK;
}

// Launch shapes for small batches (the drop-in host API extracts one image per call): below
// kSmallBatch images (or stereo frames) the kernels trade per-wave work for more, shorter waves,
// since one image cannot fill the GPU and the frame's latency is its longest chain of dependent steps.
constexpr int kSmallBatch = 16;
constexpr int kSmallRsRows = 4;       // k_resize_s output rows per wave (48 for large batches)
constexpr int kSmallStereoLk = 16;    // k_stereo left keypoints per block (ST_LK = 512)
constexpr int kSmallOctNt = 1024;     // k_octree threads per (image, level) block (OCT_NT = 256)

static int run_batch(orbfe_extractor* h, int B, const uint8_t* const* host_ptrs, int pitch, const int* laps,
                     hipStream_t s, bool use_ext) {
    const OrbGeom& g = h->g;
    // caller-owned outputs (orbfe_set_batch_outputs) too small for this batch: refuse rather than
    // silently writing the handle's own buffers
    if (use_ext && h->ext_kps && B > h->ext_cap_images) return ORBFE_E_CAPACITY;
    bool same = (int)h->last_ptrs.size() == B;
    for (int i = 0; same && i < B; i++) same = h->last_ptrs[i] == host_ptrs[i];
    for (int i = 0; same && i < 2 * B; i++) same = h->last_laps[i] == laps[i];
    int2* d_laps = (int2*)((uint8_t*)h->d_ptrs + (size_t)B * sizeof(void*));
    if (!same) {
        h->last_ptrs.assign(host_ptrs, host_ptrs + B);
        h->last_laps.assign(laps, laps + 2 * B);
        std::vector<uint8_t> pk((size_t)B * (sizeof(void*) + 2 * sizeof(int)));
        memcpy(pk.data(), h->last_ptrs.data(), (size_t)B * sizeof(void*));
        memcpy(pk.data() + (size_t)B * sizeof(void*), h->last_laps.data(), (size_t)B * 2 * sizeof(int));
        // synchronous w.r.t. the host buffer (pageable source), ordered on s for the device
        HIPCHK(hipMemcpyAsync(h->d_ptrs, pk.data(), pk.size(), hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    h->last_nimg = B;
    h->frame_id++;
    h->last_pitch = pitch;
    const uint8_t* const* P = h->d_ptrs;
    const bool tm = h->timing;
    hipEvent_t* ev = nullptr;
    if (tm) {
        if (h->ev_used == (int)h->ev_ring.size()) {
            if (h->ev_ring.size() >= 1024) return ORBFE_E_CAPACITY;
            std::vector<hipEvent_t> set(ORBFE_NUM_STAGES + 1);
            for (auto& e : set) HIPCHK(hipEventCreate(&e));
            h->ev_ring.push_back(set);
        }
        ev = h->ev_ring[h->ev_used++].data();
        HIPCHK(hipEventRecord(ev[0], s));
    }
    const bool ext = use_ext && h->ext_kps;
    const bool small = B < kSmallBatch;   // single-image launch shapes (kSmallBatch above)
    OrbKeyPoint* o_kps = ext ? h->ext_kps : h->d_kps;
    uint8_t* o_desc = ext ? h->ext_desc : h->d_desc;
    int* o_counts = ext ? h->ext_counts : h->d_counts;
    {
        // ComputePyramid's chain (level l from level l - 1) is a sequence of dependent k_resize
        // launches on the batch stream; k_fast launches (level l's cells are [lv[l].cell_base,
        // lv[l + 1].cell_base)) run beside it on the low-priority side stream as their levels
        // become ready. Measured: the launches share one saturated machine, so the
        // pass costs about the sum of the kernels' isolated times whatever the overlap; this
        // order is marginally the best of those tried.
        hipStream_t s2 = h->side_stream;
        // each launch sizes its per-wave LDS by the levels it covers (level 0's cells need less than
        // the tall cells of the top levels: more resident waves per CU)
        auto fast_range = [&](hipStream_t st, int l0, int l1) {
            // cells per wave: 4 for levels 0-3 (3 / 2 measured 0-2 % slower), 2 for the top levels'
            // smaller grids (4: +5 %, 1: +3 %; tools/gpu_variants_trace.sh, round 3)
            // small batches (the host API's single image): one cell per wave, so the launch is as
            // many short chains as there are cells instead of a quarter as many long ones
            const int cpw = B < kSmallBatch ? 1 : l0 >= 4 ? 2 : 4;
            FastLds fl{0, 0, 0, 0};
            for (int l = l0; l < l1; l++) {
                fl.roi = std::max(fl.roi, h->fast_lds_lv[l].roi);
                fl.sc = std::max(fl.sc, h->fast_lds_lv[l].sc);
                fl.cor = std::max(fl.cor, h->fast_lds_lv[l].cor);
            }
            const int c0 = g.lv[l0].cell_base, c1 = l1 < g.nlevels ? g.lv[l1].cell_base : g.total_cells;
            fl.wave_bytes = fl.roi + fl.sc + fl.cor + FAST_ENT_BYTES;
            hipLaunchKernelGGL(k_fast, dim3((c1 - c0 + FAST_WPB * cpw - 1) / (FAST_WPB * cpw), B), dim3(64 * FAST_WPB),
                               (size_t)FAST_WPB * fl.wave_bytes, st, P, pitch, h->d_pyr, g.pyr_bytes, g, fl, h->d_cellkeys,
                               h->d_cellcnt, c0, c1, cpw);
        };
#ifdef FAST_NO_OVERLAP
        s2 = s;   // profiling builds: every launch in stream order (isolated kernel times)
#endif
        // a small batch runs every launch in stream order: at one image the device has room for all
        // of them anyway, and a cross-stream event wait costs more than the overlap it buys (a stereo
        // frame through the host API: 0.43 -> 0.33 ms, profiles/r04_kernel_ab.txt item 13)
        if (small) s2 = s;
        constexpr int kFastMid = 4;   // FAST of levels [1, kFastMid) runs on the side stream once resize has built them
        // the pyramid chain: a small batch takes short row chunks per wave (more, shorter waves: the
        // chain of 7 launches is the frame's critical path at batch 1)
        OrbGeom gr = g;
        if (B < kSmallBatch)
            for (int l = 1; l < g.nlevels; l++) gr.lv[l].rs_rows = std::min(g.lv[l].rs_rows, kSmallRsRows);
        // side stream: FAST of level 0 at once, then of levels [1, lmid) when the chain has built
        // them (beside the chain's short, latency-bound top-level launches); batch stream: the
        // chain, then FAST of levels [lmid, nlevels)
        const int lmid = std::min(std::max(kFastMid, 1), g.nlevels);
        const bool fork = s2 != s;   // (profiling / one-stream builds: no fork or join)
        if (fork) {
            HIPCHK(hipEventRecord(h->ev_fork[0], s));
            HIPCHK(hipStreamWaitEvent(s2, h->ev_fork[0], 0));
        }
        // a small batch: the chain first, then FAST of every level in one launch (in one stream, a
        // FAST launch ahead of or inside the chain would only lengthen it)
        if (!small) fast_range(s2, 0, 1);
        // k_resize_s reads dwords: level 0 must be 4-byte aligned (else k_resize builds level 1)
        bool al0 = (pitch & 3) == 0;
        for (int i = 0; al0 && i < B; i++) al0 = (((uintptr_t)host_ptrs[i]) & 3) == 0;
        // ComputePyramid: one launch per level (level l from level l - 1); the row-streamed k_resize_s
        // unless the level's column windows break its rules (then the LDS-tiled k_resize)
        // a small batch: the whole pyramid in one launch (k_pyramid) when the tiles fit its limits
        const bool fused_pyr = h->pt_n > 0 && !h->no_fused_pyramid && (small || h->fused_pyramid_batch);
        if (fused_pyr)
            hipLaunchKernelGGL(k_pyramid, dim3(h->pt_n, B), dim3(PYR_NT), h->pt_lds, s, P, pitch, h->d_pyr, g.pyr_bytes, g,
                               h->d_ptile, h->pt_stride, h->pt_cap, al0 ? 1 : 0);
        for (int l = 1; l < g.nlevels && !fused_pyr; l++) {
            const OrbLevel& L = g.lv[l];
            if (L.rs_ok && (l > 1 || al0)) {
                const int rows = gr.lv[l].rs_rows;
                const int nstrips = (L.w + RS_COLS - 1) / RS_COLS, nitems = nstrips * ((L.h + rows - 1) / rows);
                hipLaunchKernelGGL(k_resize_s, dim3((nitems + RS_WPB - 1) / RS_WPB, B), dim3(64 * RS_WPB), 0, s, P, pitch, h->d_pyr,
                                   g.pyr_bytes, h->d_tab, gr, l, nstrips, nitems);
            } else {
                const int tiles_y = (L.h + L.rz_rows - 1) / L.rz_rows;
                dim3 grid((L.w + L.rz_cols - 1) / L.rz_cols, (tiles_y + RZ_TPB - 1) / RZ_TPB, B);
                hipLaunchKernelGGL(k_resize, grid, dim3(256), 0, s, P, pitch, h->d_pyr, g.pyr_bytes, h->d_tab, g, l);
            }
            if (l + 1 == lmid && !small) {
                if (fork) {
                    HIPCHK(hipEventRecord(h->ev_fork[2], s));
                    HIPCHK(hipStreamWaitEvent(s2, h->ev_fork[2], 0));
                }
                fast_range(s2, 1, lmid);
            }
        }
        if (small) {
            fast_range(s, 0, g.nlevels);
        } else {
            if (fork) HIPCHK(hipEventRecord(h->ev_fork[1], s2));
            if (fused_pyr) fast_range(s, 1, g.nlevels);   // level 0's FAST ran beside the pyramid
            else if (lmid < g.nlevels) fast_range(s, lmid, g.nlevels);
            if (fork) HIPCHK(hipStreamWaitEvent(s, h->ev_fork[1], 0));
        }
    }
    BlurKernel bk;   // the Gaussian blur is fused into k_describe
    memcpy(bk.k, h->blur_variant == 1 ? kBlurRound : kBlurED, sizeof(bk.k));
    if (tm) HIPCHK(hipEventRecord(ev[1], s));
    if (small) {
        hipLaunchKernelGGL(k_octree<kSmallOctNt>, dim3(B, g.nlevels), dim3(kSmallOctNt), h->oct_lds, s, g,
                           h->d_cellkeys, h->d_cellcnt, h->d_lkeys, h->d_nodeof, h->d_outkeys, h->d_lvinfo,
                           h->d_ranks, d_laps, h->d_oct_ts, 0);
    } else {
        hipLaunchKernelGGL(k_octree<OCT_NT>, dim3(B, g.nlevels), dim3(OCT_NT), h->oct_lds, s, g, h->d_cellkeys, h->d_cellcnt,
                           h->d_lkeys, h->d_nodeof, h->d_outkeys, h->d_lvinfo, h->d_ranks, d_laps, h->d_oct_ts, 0);
    }
    if (tm) HIPCHK(hipEventRecord(ev[2], s));
    if (B < kSmallBatch)   // one keypoint per wave: short chains for the single-image host API
        hipLaunchKernelGGL(k_describe<1>, dim3((g.out_per_img + DP_WPB - 1) / DP_WPB, B), dim3(64 * DP_WPB), 0, s, P,
                           pitch, h->d_pyr, g.pyr_bytes, g, h->d_outkeys, h->d_lvinfo, h->d_ranks, o_kps, o_desc,
                           o_counts, bk);
    else
        hipLaunchKernelGGL(k_describe<DP_KPW>, dim3((g.out_per_img + DP_WPB * DP_KPW - 1) / (DP_WPB * DP_KPW), B),
                           dim3(64 * DP_WPB), 0, s, P, pitch, h->d_pyr, g.pyr_bytes, g, h->d_outkeys, h->d_lvinfo,
                           h->d_ranks, o_kps, o_desc, o_counts, bk);
    if (tm) HIPCHK(hipEventRecord(ev[3], s));
    HIPCHK(hipGetLastError());
    h->last_kps = o_kps;
    h->last_desc = o_desc;
    h->last_counts = o_counts;
    return ORBFE_OK;
}

// The batched entry points run on the caller's stream; NULL is the legacy default (null) stream, as
// for every other stream argument of the C-ABI, so a caller's default-stream work (torch's default
// stream, a collective ordered after it) is ordered with the batch. (Until round 6 NULL selected the
// handle's own non-blocking stream, which nothing of the caller's waited for: a slab all-gather on
// the default stream could read the outputs before the kernels wrote them.)
static hipStream_t pick_stream(orbfe_extractor* h, void* stream) {
    (void)h;
    return (hipStream_t)stream;
}

typedef unsigned int orbfe_u32x4 __attribute__((ext_vector_type(4)));
// Streaming copy used by bench.py as the measured HBM ceiling: CP_U independent 16-byte loads in
// flight per lane (a block moves CP_U x 4 KB per round), non-temporal so the copy does not keep
// either buffer in L2 / the Infinity Cache.
#define CP_U 4
__global__ __launch_bounds__(256) void k_copy16(const orbfe_u32x4* __restrict__ src, orbfe_u32x4* __restrict__ dst,
                                                size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x * CP_U;
    size_t i = (size_t)blockIdx.x * blockDim.x * CP_U + threadIdx.x;
    for (; i + (CP_U - 1) * blockDim.x < n; i += stride) {
        orbfe_u32x4 v[CP_U];
#pragma unroll
        for (int u = 0; u < CP_U; u++) v[u] = __builtin_nontemporal_load(src + i + u * blockDim.x);
#pragma unroll
        for (int u = 0; u < CP_U; u++) __builtin_nontemporal_store(v[u], dst + i + u * blockDim.x);
    }
    for (; i < n; i += blockDim.x) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

// The stereo frame call's results written straight into the caller-side pinned block (mapped,
// coherent) by the launch stream: no copy-engine start-up between the last kernel and the results
// (a DMA started ~13 us after the stereo kernels in the drop-in trace). 16-byte items.
__global__ __launch_bounds__(256) void k_pull2(const orbfe_u32x4* __restrict__ s0, orbfe_u32x4* d0, int n0,
                                               const orbfe_u32x4* __restrict__ s1, orbfe_u32x4* d1, int n1) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < n0) d0[i] = s0[i];
    else if (i - n0 < n1) d1[i - n0] = s1[i - n0];
}

// The stereo frame call's two images read from the mapped pinned staging block by the launch
// stream (16-byte items, then a byte tail): the host-to-device copy without a copy-engine start-up.
__global__ __launch_bounds__(256) void k_push(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t bytes) {
    const size_t n16 = bytes / 16;
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n16) ((orbfe_u32x4*)dst)[i] = ((const orbfe_u32x4*)src)[i];
    else if (i == n16)
        for (size_t k = n16 * 16; k < bytes; k++) dst[k] = src[k];
}

extern "C" {

const char* orbfe_version(void) { return "orbfe 0.1 (gfx950, HIP)"; }

int orbfe_copy_stream(const void* d_src, void* d_dst, size_t bytes, void* stream) {
    if (!d_src || !d_dst || (bytes & 15) || (((uintptr_t)d_src | (uintptr_t)d_dst) & 15)) return ORBFE_E_ARG;
    const size_t n = bytes / 16;
    if (!n) return ORBFE_OK;
#define CP_BLOCKS (256 * 16)
    const unsigned blocks = (unsigned)std::min<size_t>((n + 256 * CP_U - 1) / (256 * CP_U), CP_BLOCKS);
    hipLaunchKernelGGL(k_copy16, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (const orbfe_u32x4*)d_src, (orbfe_u32x4*)d_dst, n);
    HIPCHK(hipGetLastError());
    return ORBFE_OK;
}

int orbfe_extractor_create(int nfeatures, float scaleFactor, int nlevels, int iniThFAST, int minThFAST,
                           orbfe_extractor** out) {
    if (!out || nfeatures <= 0 || nlevels <= 0 || nlevels > ORBFE_MAX_LEVELS || !(scaleFactor > 1.0f))
        return ORBFE_E_ARG;
    orbfe_extractor* h = new orbfe_extractor();
    h->nfeatures = nfeatures;
    h->nlevels = nlevels;
    h->ini_th = iniThFAST;
    h->min_th = minThFAST;
    h->scale_factor_f = scaleFactor;
    h->scale_factor = scaleFactor;   // double member initialised from the float argument (ORBextractor.h:96)
#if ORBFE_OCT_STAMPS
    if (hipMalloc(&h->d_oct_ts, 64 * 8 * ORBFE_MAX_LEVELS) != hipSuccess) { delete h; return ORBFE_E_DEVICE; }
    (void)hipMemset(h->d_oct_ts, 0, 64 * 8 * ORBFE_MAX_LEVELS);
#endif
    // ORBextractor.cc:414-445
    h->scale.resize(nlevels);
    h->sigma2.resize(nlevels);
    h->scale[0] = 1.0f;
    h->sigma2[0] = 1.0f;
    for (int i = 1; i < nlevels; i++) {
        h->scale[i] = (float)(h->scale[i - 1] * h->scale_factor);
        h->sigma2[i] = h->scale[i] * h->scale[i];
    }
    h->inv_scale.resize(nlevels);
    h->inv_sigma2.resize(nlevels);
    for (int i = 0; i < nlevels; i++) {
        h->inv_scale[i] = 1.0f / h->scale[i];
        h->inv_sigma2[i] = 1.0f / h->sigma2[i];
    }
    h->per_level.resize(nlevels);
    const float factor = (float)(1.0f / h->scale_factor);
    float nDesired = nfeatures * (1 - factor) / (1 - (float)std::pow((double)factor, (double)nlevels));
    int sum = 0;
    for (int l = 0; l < nlevels - 1; l++) {
        h->per_level[l] = cv_round(nDesired);
        sum += h->per_level[l];
        nDesired *= factor;
    }
    h->per_level[nlevels - 1] = std::max(nfeatures - sum, 0);
    hipError_t e = hipGetDevice(&h->device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&h->own_stream, hipStreamNonBlocking);
    int prio_lo = 0, prio_hi = 0;   // the side stream yields to the batch stream's critical path
    if (e == hipSuccess) e = hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (e == hipSuccess) e = hipStreamCreateWithPriority(&h->side_stream, hipStreamNonBlocking, prio_lo);
    for (int i = 0; e == hipSuccess && i <= ORBFE_MAX_LEVELS; i++)
        e = hipEventCreateWithFlags(&h->ev_fork[i], hipEventDisableTiming);
    for (int i = 0; e == hipSuccess && i <= ORBFE_NUM_STAGES; i++) e = hipEventCreate(&h->ev[i]);
    if (e != hipSuccess) {
        fprintf(stderr, "orbfe: extractor_create: HIP error %s\n", hipGetErrorString(e));
        delete h;
        return ORBFE_E_DEVICE;
    }
    *out = h;
    return ORBFE_OK;
}

void orbfe_extractor_destroy(orbfe_extractor* h) {
    if (!h) return;
    (void)hipSetDevice(h->device);
    (void)hipDeviceSynchronize();
    free_buffers(h);
    if (h->d_stage) (void)hipFree(h->d_stage);
    if (h->h_pin) (void)hipHostFree(h->h_pin);
    if (h->d_st) (void)hipFree(h->d_st);
    if (h->d_scale) (void)hipFree(h->d_scale);
    if (h->d_sdist) (void)hipFree(h->d_sdist);
    for (int i = 0; i <= ORBFE_NUM_STAGES; i++)
        if (h->ev[i]) (void)hipEventDestroy(h->ev[i]);
    for (int i = 0; i <= ORBFE_MAX_LEVELS; i++)
        if (h->ev_fork[i]) (void)hipEventDestroy(h->ev_fork[i]);
    if (h->side_stream) (void)hipStreamDestroy(h->side_stream);
    if (h->own_stream) (void)hipStreamDestroy(h->own_stream);
    delete h;
}

int orbfe_extractor_levels(const orbfe_extractor* h) { return h ? h->nlevels : ORBFE_E_ARG; }

int orbfe_extractor_scale_info(const orbfe_extractor* h, float* scale, float* inv_scale, float* sigma2,
                               float* inv_sigma2, int* per_level) {
    if (!h) return ORBFE_E_ARG;
    for (int l = 0; l < h->nlevels; l++) {
        if (scale) scale[l] = h->scale[l];
        if (inv_scale) inv_scale[l] = h->inv_scale[l];
        if (sigma2) sigma2[l] = h->sigma2[l];
        if (inv_sigma2) inv_sigma2[l] = h->inv_sigma2[l];
        if (per_level) per_level[l] = h->per_level[l];
    }
    return ORBFE_OK;
}

int orbfe_extractor_capacity(orbfe_extractor* h, int width, int height) {
    if (!h) return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    if (width != h->W || height != h->H) {
        int rc = ensure(h, width, height, std::max(h->cap_b, 1));
        if (rc) return rc;
    }
    return h->g.kp_cap;
}

int orbfe_extract_batch(orbfe_extractor* h, int nimg, const uint8_t* const* d_imgs, int width, int height, int pitch,
                        int lap0, int lap1, void* stream) {
    if (!h || nimg <= 0 || !d_imgs || pitch < width) return ORBFE_E_ARG;
    if (width <= 0 || height <= 0) return ORBFE_E_EMPTY;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure(h, width, height, nimg);
    if (rc) return rc;
    std::vector<int> laps(2 * (size_t)nimg);
    for (int i = 0; i < nimg; i++) { laps[2 * i] = lap0; laps[2 * i + 1] = lap1; }
    return run_batch(h, nimg, d_imgs, pitch, laps.data(), pick_stream(h, stream), true);
}

int orbfe_extract_batch_laps(orbfe_extractor* h, int nimg, const uint8_t* const* d_imgs, int width, int height,
                             int pitch, const int32_t* laps, void* stream) {
    if (!h || nimg <= 0 || !d_imgs || !laps || pitch < width) return ORBFE_E_ARG;
    if (width <= 0 || height <= 0) return ORBFE_E_EMPTY;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure(h, width, height, nimg);
    if (rc) return rc;
    return run_batch(h, nimg, d_imgs, pitch, laps, pick_stream(h, stream), true);
}

int orbfe_batch_outputs(orbfe_extractor* h, orbfe_keypoint** d_kps, uint8_t** d_desc, int** d_counts, int* cap) {
    if (!h || !h->cap_b) return ORBFE_E_ARG;
    if (d_kps) *d_kps = (orbfe_keypoint*)(h->last_kps ? h->last_kps : h->d_kps);
    if (d_desc) *d_desc = h->last_desc ? h->last_desc : h->d_desc;
    if (d_counts) *d_counts = h->last_counts ? h->last_counts : h->d_counts;
    if (cap) *cap = h->g.kp_cap;
    return ORBFE_OK;
}

int orbfe_extractor_set_opencv_model(orbfe_extractor* h, int resize_simd_lanes, int blur_variant) {
    if (!h || blur_variant < 0 || blur_variant > 1) return ORBFE_E_ARG;
    if (resize_simd_lanes != 0 && resize_simd_lanes != 8 && resize_simd_lanes != 16 && resize_simd_lanes != 32 &&
        resize_simd_lanes != 64)
        return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    std::lock_guard<std::mutex> lk2(h->mu_stereo);   // the batch buffers the stereo calls read are released
    if (h->resize_simd_lanes == resize_simd_lanes && h->blur_variant == blur_variant) return ORBFE_OK;
    HIPCHK(hipSetDevice(h->device));
    HIPCHK(hipDeviceSynchronize());   // in-flight batches read the handle's tables
    h->resize_simd_lanes = resize_simd_lanes;
    h->blur_variant = blur_variant;
    // the resize tables (simd_end per level) depend on the lane count: the next batch rebuilds the
    // geometry and its buffers
    free_buffers(h);
    h->W = h->H = 0;
    return ORBFE_OK;
}

int orbfe_extractor_get_opencv_model(const orbfe_extractor* h, int* resize_simd_lanes, int* blur_variant) {
    if (!h) return ORBFE_E_ARG;
    if (resize_simd_lanes) *resize_simd_lanes = h->resize_simd_lanes;
    if (blur_variant) *blur_variant = h->blur_variant;
    return ORBFE_OK;
}

int orbfe_set_stage_timing(orbfe_extractor* h, int enable) {
    if (!h) return ORBFE_E_ARG;
    h->timing = enable != 0;
    return ORBFE_OK;
}
int orbfe_get_stage_timing(orbfe_extractor* h, float* ms) {
    if (!h || !ms) return ORBFE_E_ARG;
    const int n = h->ev_used;
    for (int i = 0; i < ORBFE_NUM_STAGES; i++) ms[i] = 0.f;
    for (int r = 0; r < n; r++) {
        HIPCHK(hipEventSynchronize(h->ev_ring[r][ORBFE_NUM_STAGES]));
        for (int i = 0; i < ORBFE_NUM_STAGES; i++) {
            float t = 0.f;
            HIPCHK(hipEventElapsedTime(&t, h->ev_ring[r][i], h->ev_ring[r][i + 1]));
            ms[i] += t;
        }
    }
    if (n) for (int i = 0; i < ORBFE_NUM_STAGES; i++) ms[i] /= n;
    h->ev_used = 0;
    return n;
}

int orbfe_set_batch_outputs(orbfe_extractor* h, orbfe_keypoint* d_kps, uint8_t* d_desc, int* d_counts,
                            int cap_images) {
    if (!h) return ORBFE_E_ARG;
    h->ext_kps = (OrbKeyPoint*)d_kps;
    h->ext_desc = d_desc;
    h->ext_counts = d_counts;
    h->ext_cap_images = (d_kps && d_desc && d_counts) ? cap_images : 0;
    return ORBFE_OK;
}

int orbfe_extract(orbfe_extractor* h, const uint8_t* img, int width, int height, int stride, int lap0, int lap1,
                  orbfe_keypoint* kps, uint8_t* desc, int cap, int* n) {
    if (!h || !n) return ORBFE_E_ARG;
    *n = 0;
    if (!img || width <= 0 || height <= 0) return ORBFE_E_EMPTY;
    if (stride < width) return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure(h, width, height, 1);
    if (rc) return rc;
    hipStream_t s = h->own_stream;
    const size_t bytes = (size_t)width * height;
    if (h->stage_bytes < bytes) {
        if (h->d_stage) HIPCHK(hipFree(h->d_stage));
        HIPCHK(hipMalloc(&h->d_stage, bytes));
        h->stage_bytes = bytes;
    }
    const bool tm = h->timing;
    if (tm && !h->call_ev[0])
        for (auto& e : h->call_ev) HIPCHK(hipEventCreate(&e));
    // the pinned result layout is a one-image output block (out_layout)
    size_t o_kps, o_desc, o_end;
    out_layout(1, h->g.kp_cap, &o_kps, &o_desc, &o_end);
    const size_t kpb = (size_t)h->g.kp_cap * sizeof(OrbKeyPoint), db = (size_t)h->g.kp_cap * 32;
    const size_t pin_need = std::max(bytes, o_end);
    if (h->pin_bytes < pin_need) {
        if (h->h_pin) HIPCHK(hipHostFree(h->h_pin));
        h->h_pin = nullptr;
        h->pin_bytes = 0;
        HIPCHK(hipHostMalloc((void**)&h->h_pin, pin_need, hipHostMallocMapped | hipHostMallocCoherent));
        h->pin_bytes = pin_need;
    }
    // the previous call's result copies out of h_pin have completed (that call synchronised)
    if (stride == width) memcpy(h->h_pin, img, bytes);
    else
        for (int y = 0; y < height; y++) memcpy(h->h_pin + (size_t)y * width, img + (size_t)y * stride, width);
    const uint8_t* ptrs[1] = {h->d_stage};
    const int laps[2] = {lap0, lap1};
    uint8_t* hp = h->h_pin;
    // the whole call as stream work: upload, the batch launches, and counts plus the whole keypoint /
    // descriptor capacity back in one round trip (61 KB at 1000 features: one transfer costs less
    // than a second synchronisation)
    // (the mapped pinned block read / written by kernels on the stream, as in orbfe_frame_stereo)
    uint8_t* hpd = nullptr;
    if (!h->no_push || !h->no_pull) HIPCHK(hipHostGetDevicePointer((void**)&hpd, hp, 0));
    auto enqueue = [&]() -> int {
        if (tm) HIPCHK(hipEventRecord(h->call_ev[0], s));
        if (!h->no_push) {
            hipLaunchKernelGGL(k_push, dim3((unsigned)((bytes / 16 + 1 + 255) / 256)), dim3(256), 0, s,
                               (const uint8_t*)hpd, h->d_stage, bytes);
            HIPCHK(hipGetLastError());
        } else {
            HIPCHK(hipMemcpyAsync(h->d_stage, h->h_pin, bytes, hipMemcpyHostToDevice, s));
        }
        if (tm) HIPCHK(hipEventRecord(h->call_ev[1], s));
        h->timing = false;   // the call's own events bracket the kernels (the stage ring is for batches)
        const int r = run_batch(h, 1, ptrs, width, laps, s, false);
        h->timing = tm;
        if (r) return r;
        if (tm) HIPCHK(hipEventRecord(h->call_ev[2], s));
        if (h->cap_b == 1 && kps && desc && !h->no_pull) {   // the one-image output block, by one kernel
            const int n0 = (int)(o_end / 16);
            hipLaunchKernelGGL(k_pull2, dim3((n0 + 255) / 256), dim3(256), 0, s, (const orbfe_u32x4*)h->d_out,
                               (orbfe_u32x4*)hpd, n0, (const orbfe_u32x4*)nullptr, (orbfe_u32x4*)nullptr, 0);
            HIPCHK(hipGetLastError());
        } else if (h->cap_b == 1 && kps && desc) {   // the handle's one-image output block: one copy
            HIPCHK(hipMemcpyAsync(hp, h->d_out, o_end, hipMemcpyDeviceToHost, s));
        } else {
            HIPCHK(hipMemcpyAsync(hp, h->last_counts, 8, hipMemcpyDeviceToHost, s));
            if (kps) HIPCHK(hipMemcpyAsync(hp + o_kps, h->last_kps, kpb, hipMemcpyDeviceToHost, s));
            if (desc) HIPCHK(hipMemcpyAsync(hp + o_desc, h->last_desc, db, hipMemcpyDeviceToHost, s));
        }
        if (tm) HIPCHK(hipEventRecord(h->call_ev[3], s));
        return ORBFE_OK;
    };
    rc = enqueue();
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(s));
    int cnt[2];
    memcpy(cnt, hp, 8);
    *n = cnt[0];
    if (cnt[0] > cap) return ORBFE_E_CAPACITY;
    if (cnt[0] > 0) {
        if (kps) memcpy(kps, hp + o_kps, (size_t)cnt[0] * sizeof(OrbKeyPoint));
        if (desc) memcpy(desc, hp + o_desc, (size_t)cnt[0] * 32);
    }
    if (tm) {   // {upload, kernels, result copies}
        HIPCHK(hipEventElapsedTime(&h->call_ms[0], h->call_ev[0], h->call_ev[1]));
        HIPCHK(hipEventElapsedTime(&h->call_ms[1], h->call_ev[1], h->call_ev[2]));
        HIPCHK(hipEventElapsedTime(&h->call_ms[2], h->call_ev[2], h->call_ev[3]));
    }
    return cnt[1];
}

int orbfe_get_call_timing(orbfe_extractor* h, float* ms) {
    if (!h || !ms) return ORBFE_E_ARG;
    // the calls write call_ms and toggle `timing` under the handle's mutex
    std::lock_guard<std::mutex> lk(h->mu);
    for (int i = 0; i < 5; i++) ms[i] = h->call_ms[i];
    return h->timing ? 5 : 0;
}

int orbfe_pyramid_level(orbfe_extractor* h, int image, int level, uint8_t* dst, int dst_pitch, int* width,
                        int* height) {
    if (!h || level < 0 || level >= h->nlevels || !h->cap_b || image < 0 || image >= h->last_nimg) return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(h->mu);
    const OrbLevel& L = h->g.lv[level];
    if (width) *width = L.w;
    if (height) *height = L.h;
    if (!dst) return ORBFE_OK;
    if (dst_pitch < L.w) return ORBFE_E_CAPACITY;
    HIPCHK(hipStreamSynchronize(h->own_stream));
    HIPCHK(hipDeviceSynchronize());
    const uint8_t* src;
    int sp;
    if (level == 0) { src = h->last_ptrs[image]; sp = h->last_pitch; }
    else { src = h->d_pyr + (size_t)image * h->g.pyr_bytes + L.pyr_off; sp = L.pitch; }
    HIPCHK(hipMemcpy2D(dst, dst_pitch, src, sp, L.w, L.h, hipMemcpyDeviceToHost));
    return ORBFE_OK;
}

int orbfe_stereo_match_batch(orbfe_extractor* left, int lbase, int lstep, orbfe_extractor* right, int rbase,
                             int rstep, int nframes, float bf, float fx, float* d_uright, float* d_depth,
                             int* d_nmatch, void* stream) {
    if (!left || !right || nframes <= 0 || !left->cap_b || !right->cap_b) return ORBFE_E_ARG;
    if (left->W != right->W || left->H != right->H || left->nlevels != right->nlevels ||
        left->nfeatures != right->nfeatures || left->scale_factor_f != right->scale_factor_f)
        return ORBFE_E_ARG;
    if (lbase + (nframes - 1) * lstep >= left->last_nimg || rbase + (nframes - 1) * rstep >= right->last_nimg)
        return ORBFE_E_ARG;
    const OrbGeom& g = left->g;
    StereoSide SL{left->d_ptrs, left->last_pitch, left->d_pyr, g.pyr_bytes, left->last_kps, left->last_desc,
                  left->last_counts, lbase, lstep};
    StereoSide SR{right->d_ptrs, right->last_pitch, right->d_pyr, right->g.pyr_bytes, right->last_kps,
                  right->last_desc, right->last_counts, rbase, rstep};
    // sort keys: kp_cap for the counting sort (k_stereo's csort rule), a power of two for the
    // bitonic fallback of images taller than 1983 rows
    int sort_cap = 1;
    while (sort_cap < g.kp_cap) sort_cap <<= 1;
    if (g.height + 2 * ST_ROFF + 1 <= (ST_NT / 64) * 128) sort_cap = (g.kp_cap + 3) & ~3;   // 16-byte aligned tail
    // a small batch of frames splits each frame's left keypoints over more blocks (each restages the
    // right side: redundant work, but the frame's chain of keypoints per wave is what bounds batch 1)
    const int lkpb = nframes < kSmallBatch ? kSmallStereoLk : ST_LK;
    StereoArgs sa{bf, fx, g.kp_cap, sort_cap, lkpb};
    const size_t lds = (size_t)g.kp_cap * (32 + sizeof(RightRec)) + (size_t)sort_cap * 4 + (ST_NT / 64) * (512 + 128 * 4) +
                       (size_t)round_up(2 * (g.height + 2 * ST_ROFF), 16);
    if (lds > 160 * 1024 - 64 || g.kp_cap > 65535) return ORBFE_E_ARG;   // LDS: about 2700 keypoints per image
    hipStream_t s = pick_stream(left, stream);
    std::lock_guard<std::mutex> lk(left->mu_stereo);
    if (left->sdist_frames < nframes || left->sdist_kp < g.kp_cap) {
        if (left->d_sdist) HIPCHK(hipFree(left->d_sdist));
        left->d_sdist = nullptr;
        left->sdist_frames = left->sdist_kp = 0;
        HIPCHK(hipMalloc(&left->d_sdist, (size_t)nframes * g.kp_cap * 4));
        left->sdist_frames = nframes;
        left->sdist_kp = g.kp_cap;
    }
    hipLaunchKernelGGL(k_stereo, dim3((g.kp_cap + lkpb - 1) / lkpb, nframes), dim3(ST_NT), lds, s, g, SL, SR, sa,
                       d_uright, d_depth, left->d_sdist);
    hipLaunchKernelGGL(k_stereo_cut, dim3(nframes), dim3(256), 0, s, g, SL, sa, d_uright, d_depth, left->d_sdist,
                       d_nmatch);
    HIPCHK(hipGetLastError());
    return ORBFE_OK;
}

int orbfe_stereo_match(orbfe_extractor* left, orbfe_extractor* right, float bf, float fx, float* uright,
                       float* depth) {
    if (!left || !right) return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(left->mu);
    if (!left->d_st || left->stereo_kp < left->g.kp_cap) {   // (re)size for the current geometry
        if (left->d_st) HIPCHK(hipFree(left->d_st));
        left->d_st = nullptr;
        left->d_uright = left->d_depth = nullptr;
        left->d_nmatch = nullptr;
        left->stereo_kp = 0;
        HIPCHK(hipMalloc(&left->d_st, 16 + (size_t)left->g.kp_cap * 8));
        left->d_nmatch = (int*)left->d_st;
        left->d_uright = (float*)(left->d_st + 16);
        left->d_depth = left->d_uright + left->g.kp_cap;
        left->stereo_kp = left->g.kp_cap;
    }
    HIPCHK(hipStreamSynchronize(right->own_stream));
    hipStream_t s = left->own_stream;
    const bool tm = left->timing && left->call_ev[0];
    if (tm) HIPCHK(hipEventRecord(left->call_ev[4], s));
    int rc = orbfe_stereo_match_batch(left, 0, 1, right, 0, 1, 1, bf, fx, left->d_uright, left->d_depth,
                                      left->d_nmatch, s);
    if (rc) return rc;
    if (tm) HIPCHK(hipEventRecord(left->call_ev[5], s));
    // counts, then {nmatch | the whole uR / depth capacity} in one copy, one round trip through
    // pinned memory
    const size_t kc = (size_t)left->stereo_kp;
    const size_t need = 32 + 8 * kc;
    if (left->pin_bytes < need) {
        if (left->h_pin) HIPCHK(hipHostFree(left->h_pin));
        left->h_pin = nullptr;
        left->pin_bytes = 0;
        HIPCHK(hipHostMalloc((void**)&left->h_pin, need, hipHostMallocMapped | hipHostMallocCoherent));
        left->pin_bytes = need;
    }
    uint8_t* hp = left->h_pin;
    HIPCHK(hipMemcpyAsync(hp, left->last_counts, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(hp + 16, left->d_st, 16 + 8 * kc, hipMemcpyDeviceToHost, s));
    if (tm) HIPCHK(hipEventRecord(left->call_ev[6], s));
    HIPCHK(hipStreamSynchronize(s));
    int cnt[2], nm = 0;
    memcpy(cnt, hp, 8);
    memcpy(&nm, hp + 16, 4);
    if (cnt[0] > 0) {
        memcpy(uright, hp + 32, (size_t)cnt[0] * 4);
        memcpy(depth, hp + 32 + 4 * kc, (size_t)cnt[0] * 4);
    }
    if (tm) {   // {kernels, result copies}
        HIPCHK(hipEventElapsedTime(&left->call_ms[3], left->call_ev[4], left->call_ev[5]));
        HIPCHK(hipEventElapsedTime(&left->call_ms[4], left->call_ev[5], left->call_ev[6]));
    }
    return nm;
}

// Frame::Frame(stereo) in one call (Frame.cc:120-141): both ExtractORB calls (:122-125) as ONE
// two-image batch on the left handle (left image 0, right image 1), ComputeStereoMatches (:141) on
// the same stream, one pinned upload of both images and one synchronisation for all results. The
// right handle only supplies (and must equal) the extractor parameters, as Tracking constructs both
// extractors from the same settings (Tracking.cc:637-645); it is not written.
// The two-image frame call behind orbfe_frame_stereo (pinhole: vLappingArea {0, 0}, then
// ComputeStereoMatches) and orbfe_frame_fisheye (KannalaBrandt8: the caller's vLappingArea, then the
// kNN + ratio stage): one upload through a mapped pinned block, one launch chain, one result pull.
// The per-left-keypoint results (uR / depth floats, or l2r / dist ints) share the d_st region.
static int frame_pair(orbfe_extractor* left, orbfe_extractor* right, const uint8_t* img_left, const uint8_t* img_right,
                      int width, int height, int stride, bool fisheye, int lap0, int lap1, float bf, float fx,
                      float ratio, orbfe_keypoint* kps_left, uint8_t* desc_left, int cap_left, int* n_left,
                      int* mono_left, orbfe_keypoint* kps_right, uint8_t* desc_right, int cap_right, int* n_right,
                      int* mono_right, void* res_a, void* res_b) {
    if (!left || !right || !n_left || !n_right || !mono_left || !mono_right) return ORBFE_E_ARG;
    *n_left = *n_right = 0;
    *mono_left = *mono_right = -1;
    if (!img_left || !img_right || width <= 0 || height <= 0) return ORBFE_E_EMPTY;
    if (stride < width || !kps_left || !desc_left || !kps_right || !desc_right || !res_a || !res_b) return ORBFE_E_ARG;
    if (left != right && (left->nfeatures != right->nfeatures || left->nlevels != right->nlevels ||
                          left->scale_factor_f != right->scale_factor_f || left->ini_th != right->ini_th ||
                          left->min_th != right->min_th || left->resize_simd_lanes != right->resize_simd_lanes ||
                          left->blur_variant != right->blur_variant))
        return ORBFE_E_ARG;
    orbfe_extractor* h = left;
    std::lock_guard<std::mutex> lk(h->mu);
    int rc = ensure(h, width, height, 2);
    if (rc) return rc;
    hipStream_t s = h->own_stream;
    const size_t bytes = (size_t)width * height;
    if (h->stage_bytes < 2 * bytes) {
        if (h->d_stage) HIPCHK(hipFree(h->d_stage));
        h->d_stage = nullptr;
        h->stage_bytes = 0;
        HIPCHK(hipMalloc(&h->d_stage, 2 * bytes));
        h->stage_bytes = 2 * bytes;
    }
    const int kc = h->g.kp_cap;
    if (!h->d_st || h->stereo_kp < kc) {   // {nmatch (16 B) | uR [kc] | depth [kc]}
        if (h->d_st) HIPCHK(hipFree(h->d_st));
        h->d_st = nullptr;
        h->d_uright = h->d_depth = nullptr;
        h->d_nmatch = nullptr;
        h->stereo_kp = 0;
        HIPCHK(hipMalloc(&h->d_st, (16 + (size_t)kc * 8 + 15) & ~(size_t)15));   // whole 16-byte items (k_pull2)
        h->d_nmatch = (int*)h->d_st;
        h->d_uright = (float*)(h->d_st + 16);
        h->d_depth = h->d_uright + kc;
        h->stereo_kp = kc;
    }
    // pinned: both images going up; coming back {counts [2][2] | keypoints [2][kc] | descriptors
    // [2][kc]} (the two-image output block) then {nmatch | uR | depth}
    size_t o_kps, o_desc, o_end;
    out_layout(2, kc, &o_kps, &o_desc, &o_end);
    const size_t o_st = (o_end + 15) & ~(size_t)15, st_bytes = 16 + (size_t)h->stereo_kp * 8;
    const size_t st16 = (st_bytes + 15) & ~(size_t)15;
    const size_t pin_need = std::max(2 * bytes, o_st + st16);
    if (h->pin_bytes < pin_need) {
        if (h->h_pin) HIPCHK(hipHostFree(h->h_pin));
        h->h_pin = nullptr;
        h->pin_bytes = 0;
        HIPCHK(hipHostMalloc((void**)&h->h_pin, pin_need, hipHostMallocMapped | hipHostMallocCoherent));
        h->pin_bytes = pin_need;
    }
    uint8_t* hp = h->h_pin;
    const uint8_t* src[2] = {img_left, img_right};
    const bool tm = h->timing;
    if (tm && !h->call_ev[0])
        for (auto& e : h->call_ev) HIPCHK(hipEventCreate(&e));
    uint8_t* hpd = nullptr;
    if (!h->no_push) HIPCHK(hipHostGetDevicePointer((void**)&hpd, hp, 0));
    // whole 16-byte items per image: the left image's push runs while the right one is packed
    const bool split = !h->no_push && (bytes % 16) == 0;
    for (int i = 0; i < 2; i++) {
        if (stride == width) memcpy(hp + i * bytes, src[i], bytes);
        else
            for (int y = 0; y < height; y++)
                memcpy(hp + i * bytes + (size_t)y * width, src[i] + (size_t)y * stride, width);
        if (split) {
            if (i == 0 && tm) HIPCHK(hipEventRecord(h->call_ev[0], s));
            hipLaunchKernelGGL(k_push, dim3((unsigned)((bytes / 16 + 1 + 255) / 256)), dim3(256), 0, s,
                               (const uint8_t*)hpd + i * bytes, h->d_stage + i * bytes, bytes);
            HIPCHK(hipGetLastError());
        }
    }
    const uint8_t* ptrs[2] = {h->d_stage, h->d_stage + bytes};
    // the pinhole stereo Frame passes vLappingArea {0, 0} (Frame.cc:122-123), the KB8 one its
    // overlapping area (:1059-1060)
    const int laps[4] = {fisheye ? lap0 : 0, fisheye ? lap1 : 0, fisheye ? lap0 : 0, fisheye ? lap1 : 0};
    if (!split) {   // both images in one push (an image size that is not whole 16-byte items), or by DMA
        if (tm) HIPCHK(hipEventRecord(h->call_ev[0], s));
        if (!h->no_push) {
            hipLaunchKernelGGL(k_push, dim3((unsigned)((2 * bytes / 16 + 1 + 255) / 256)), dim3(256), 0, s,
                               (const uint8_t*)hpd, h->d_stage, 2 * bytes);
            HIPCHK(hipGetLastError());
        } else {
            HIPCHK(hipMemcpyAsync(h->d_stage, hp, 2 * bytes, hipMemcpyHostToDevice, s));
        }
    }
    if (tm) HIPCHK(hipEventRecord(h->call_ev[1], s));
    h->timing = false;   // the call's own events bracket the kernels (the stage ring is for batches)
    rc = run_batch(h, 2, ptrs, width, laps, s, false);
    h->timing = tm;
    if (rc) return rc;
    if (tm) HIPCHK(hipEventRecord(h->call_ev[2], s));
    if (fisheye)   // ComputeStereoFishEyeMatches' descriptor stage (Frame.cc:1126-1151): l2r / dist in d_st
        rc = orbfe_stereo_knn_batch(h, 0, 1, h, 1, 1, 1, ratio, (int32_t*)h->d_uright, (int32_t*)h->d_depth,
                                    h->d_nmatch, s);
    else
        rc = orbfe_stereo_match_batch(h, 0, 1, h, 1, 1, 1, bf, fx, h->d_uright, h->d_depth, h->d_nmatch, s);
    if (rc) return rc;
    if (tm) HIPCHK(hipEventRecord(h->call_ev[4], s));
    if (h->cap_b == 2 && !h->no_pull) {   // the two-image output block and the stereo results: one kernel
        uint8_t* hpd = nullptr;
        HIPCHK(hipHostGetDevicePointer((void**)&hpd, hp, 0));
        const int n0 = (int)(o_end / 16), n1 = (int)(st16 / 16);
        hipLaunchKernelGGL(k_pull2, dim3((n0 + n1 + 255) / 256), dim3(256), 0, s, (const orbfe_u32x4*)h->d_out,
                           (orbfe_u32x4*)hpd, n0, (const orbfe_u32x4*)h->d_st, (orbfe_u32x4*)(hpd + o_st), n1);
        HIPCHK(hipGetLastError());
    } else {
        if (h->cap_b == 2) {   // the handle's two-image output block: one copy
            HIPCHK(hipMemcpyAsync(hp, h->d_out, o_end, hipMemcpyDeviceToHost, s));
        } else {
            HIPCHK(hipMemcpyAsync(hp, h->last_counts, 16, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(hp + o_kps, h->last_kps, (size_t)2 * kc * sizeof(OrbKeyPoint), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(hp + o_desc, h->last_desc, (size_t)2 * kc * 32, hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipMemcpyAsync(hp + o_st, h->d_st, st_bytes, hipMemcpyDeviceToHost, s));
    }
    if (tm) HIPCHK(hipEventRecord(h->call_ev[5], s));
    HIPCHK(hipStreamSynchronize(s));
    int cnt[4], nm = 0;
    memcpy(cnt, hp, 16);
    memcpy(&nm, hp + o_st, 4);
    *n_left = cnt[0];
    *n_right = cnt[2];
    *mono_left = cnt[1];
    *mono_right = cnt[3];
    if (cnt[0] > cap_left || cnt[2] > cap_right) return ORBFE_E_CAPACITY;
    if (!fisheye) {   // the left image's records stay in the handle's output block (orbfe_frame_device_view)
        h->fs_id = h->frame_id;
        h->fs_n = cnt[0];
    }
    const OrbKeyPoint* hk = (const OrbKeyPoint*)(hp + o_kps);
    const uint8_t* hd = hp + o_desc;
    memcpy(kps_left, hk, (size_t)cnt[0] * sizeof(OrbKeyPoint));
    memcpy(desc_left, hd, (size_t)cnt[0] * 32);
    memcpy(kps_right, hk + kc, (size_t)cnt[2] * sizeof(OrbKeyPoint));
    memcpy(desc_right, hd + (size_t)kc * 32, (size_t)cnt[2] * 32);
    memcpy(res_a, hp + o_st + 16, (size_t)cnt[0] * 4);   // uR or l2r
    memcpy(res_b, hp + o_st + 16 + (size_t)h->stereo_kp * 4, (size_t)cnt[0] * 4);   // depth or dist
    // slots as the header documents: {upload, extraction kernels, result copies, stereo kernels}. On the
    // split path the upload slot starts at the left image's push and so also counts the host packing
    // of the right image (the GPU waits for it): it is push + packing, not a pure transfer time.
    if (tm) {
        HIPCHK(hipEventElapsedTime(&h->call_ms[0], h->call_ev[0], h->call_ev[1]));
        HIPCHK(hipEventElapsedTime(&h->call_ms[1], h->call_ev[1], h->call_ev[2]));
        HIPCHK(hipEventElapsedTime(&h->call_ms[3], h->call_ev[2], h->call_ev[4]));
        HIPCHK(hipEventElapsedTime(&h->call_ms[2], h->call_ev[4], h->call_ev[5]));
        h->call_ms[4] = 0.f;
    }
    return nm;
}

int orbfe_frame_stereo(orbfe_extractor* left, orbfe_extractor* right, const uint8_t* img_left,
                       const uint8_t* img_right, int width, int height, int stride, float bf, float fx,
                       orbfe_keypoint* kps_left, uint8_t* desc_left, int cap_left, int* n_left, int* mono_left,
                       orbfe_keypoint* kps_right, uint8_t* desc_right, int cap_right, int* n_right,
                       int* mono_right, float* uright, float* depth) {
    return frame_pair(left, right, img_left, img_right, width, height, stride, false, 0, 0, bf, fx, 0.f, kps_left,
                      desc_left, cap_left, n_left, mono_left, kps_right, desc_right, cap_right, n_right, mono_right,
                      uright, depth);
}

int orbfe_frame_fisheye(orbfe_extractor* left, orbfe_extractor* right, const uint8_t* img_left,
                        const uint8_t* img_right, int width, int height, int stride, int lap0, int lap1, float ratio,
                        orbfe_keypoint* kps_left, uint8_t* desc_left, int cap_left, int* n_left, int* mono_left,
                        orbfe_keypoint* kps_right, uint8_t* desc_right, int cap_right, int* n_right,
                        int* mono_right, int32_t* l2r, int32_t* dist) {
    return frame_pair(left, right, img_left, img_right, width, height, stride, true, lap0, lap1, 0.f, 1.f, ratio,
                      kps_left, desc_left, cap_left, n_left, mono_left, kps_right, desc_right, cap_right, n_right,
                      mono_right, l2r, dist);
}

uint64_t orbfe_extractor_frame_id(orbfe_extractor* h) { return h ? h->frame_id : 0; }

int orbfe_frame_device_view(orbfe_extractor* left, uint64_t frame_id, orbfe_frame* F) {
    if (!left || !F) return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(left->mu);
    if (frame_id == 0 || left->fs_id != frame_id || left->frame_id != frame_id || !left->last_kps || !left->d_st)
        return ORBFE_E_ARG;   // no frame call, or the handle has extracted since
    if (!left->d_scale) {
        HIPCHK(hipSetDevice(left->device));
        HIPCHK(hipMalloc(&left->d_scale, ORBFE_MAX_LEVELS * sizeof(float)));
        HIPCHK(hipMemcpy(left->d_scale, left->scale.data(), left->nlevels * sizeof(float), hipMemcpyHostToDevice));
    }
    F->n = left->fs_n;
    F->keys = (const orbfe_keypoint*)left->last_kps;   // image 0 of the last batch = the left image
    F->desc = left->last_desc;
    F->uright = left->d_uright;
    F->nlevels = left->nlevels;
    F->scale_factors = left->d_scale;
    F->two_cams = 0;
    F->nleft = 0;
    F->l2r = F->r2l = nullptr;
    F->device = 1;
    return ORBFE_OK;
}

int orbfe_debug_copy(orbfe_extractor* h, int what, int image, int level, void* dst, int cap_bytes) {
    if (!h || !h->cap_b || image < 0 || image >= h->last_nimg || level < 0 || level >= h->nlevels) return ORBFE_E_ARG;
    HIPCHK(hipDeviceSynchronize());
    const OrbGeom& g = h->g;
    const OrbLevel& L = g.lv[level];
    const int ncell = L.n_cols * L.n_rows;
    const void* src = nullptr;
    size_t bytes = 0;
    int count = 0;
    int info[4];
    HIPCHK(hipMemcpy(info, h->d_lvinfo + ((size_t)image * g.nlevels + level) * 4, 16, hipMemcpyDeviceToHost));
    if (what == 0) { src = h->d_cellcnt + (size_t)image * g.total_cells + L.cell_base; count = ncell; bytes = 4 * count; }
    else if (what == 1) { src = h->d_cellkeys + (size_t)image * g.cellkeys_per_img + L.cellkey_off; count = ncell * L.cell_cap; bytes = 4 * (size_t)count; }
    else if (what == 2) { src = h->d_outkeys + (size_t)image * g.out_per_img + L.out_off; count = info[0]; bytes = 4 * (size_t)count; }
    else if (what == 3) { if (cap_bytes < 16) return ORBFE_E_CAPACITY; memcpy(dst, info, 16); return 4; }
    else if (what == 4) {
        if (!h->d_oct_ts) return 0;
        src = h->d_oct_ts + 64 * level; count = 64; bytes = 64 * 8;
    }
    else return ORBFE_E_ARG;
    if (!dst) return count;
    if ((size_t)cap_bytes < bytes) return ORBFE_E_CAPACITY;
    if (bytes) HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return count;
}

#if ORBFE_OCT_STAMPS
// diagnostic builds: the per-wave stamps of the last block sort of block (0, 0)
int orbfe_debug_sort_stamps(uint64_t* out) {
    HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sort_ts), (16 * 16 + 16) * 8));
    return 272;
}
#endif
int orbfe_debug_block_sort(uint64_t* data, int n) {
    if (!data || n < 0 || n > 4096) return ORBFE_E_ARG;
    if (n == 0) return 0;
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc(&d, (size_t)n * 8));
    HIPCHK(hipMemcpy(d, data, (size_t)n * 8, hipMemcpyHostToDevice));
    const size_t lds = (size_t)n * 16 + (size_t)n * 16 + 16 + 16 * ORBFE_SORT_STACK;
    hipLaunchKernelGGL(k_debug_block_sort, dim3(1), dim3(OCT_NT), lds, 0, d, n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(data, d, (size_t)n * 8, hipMemcpyDeviceToHost));
    HIPCHK(hipFree(d));
#if ORBFE_OCT_STAMPS
    {
        unsigned long long ts[16 * 16 + 16];
        HIPCHK(hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_sort_ts), sizeof(ts)));
        fprintf(stderr, "sortts n=%d", n);
        for (int w = 0; w < OCT_NT / 64; w++) {
            fprintf(stderr, " | w%d:", w);
            for (int k = 1; k < (int)ts[w * 16 + 15] && k < 15; k++) fprintf(stderr, " %lld", (long long)(ts[w * 16 + k] - ts[0]));
        }
        fprintf(stderr, " | s64:");
        for (int k = 1; k < (int)ts[256 + 15] && k < 15; k++) fprintf(stderr, " %lld", (long long)(ts[256 + k] - ts[256 + k - 1]));
        fprintf(stderr, "\n");
    }
#endif
    return n;
}


int orbfe_descriptor_distance(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 8; i++) {
        uint32_t x, y;
        memcpy(&x, a + 4 * i, 4);
        memcpy(&y, b + 4 * i, 4);
        d += __builtin_popcount(x ^ y);
    }
    return d;
}

}  // extern "C"

// ORBmatcher methods (kernels + host wrappers; uses HIPCHK above).
#include "orbfe_matcher.hip"

// Back-end matcher pieces (SearchByBoW(KF, KF), ComputeDistinctiveDescriptors).
#include "orbfe_backend.hip"

// DBoW2 vocabulary transform (uses the matcher's per-thread arena).
#include "orbfe_bow.hip"

// cv::remap INTER_LINEAR (stereo rectification before extraction).
#include "orbfe_remap.hip"
