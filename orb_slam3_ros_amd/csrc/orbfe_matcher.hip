// ORBmatcher Tracking-thread methods on CDNA4 (included into orbfe_engine.hip's translation unit).
//
// The reference processes its queries strictly in order and later queries see earlier
// assignments (a keypoint taken by a point with Observations() > 0 is skipped, a keypoint
// "stolen" in SearchForInitialization, ...). Every such dependency is TRIANGULAR: query q only
// reads state written by queries j < q. The kernels therefore evaluate all queries in parallel
// against the state implied by the current assignment vector, recompute that state, and repeat
// until no assignment changes. After iteration t the first t queries are exactly the sequential
// result, so the loop reaches the reference's answer (in practice in 2-4 passes); no iteration
// cap below n_queries + 1 is needed for correctness.
//
// Each query scans its candidates in Frame::GetFeaturesInArea order (cell ix outer, iy inner,
// keypoint index inside a cell: the grid is rebuilt with a stable (cell, index) sort), so the
// reference's strict-< "first best wins" and best/second-best bookkeeping are reproduced verbatim.
#pragma once
#include "glibc_atan2f.h"
#include "glibc_logf.h"

#define MT_NT 256
#define MT_TH_HIGH 100
#define MT_TH_LOW 50
#define MT_HISTO 30
#define MT_NCELL (ORBFE_GRID_COLS * ORBFE_GRID_ROWS)
#define MT_INF 0x7fffffff

struct FrameDev {
    int n;
    const OrbKeyPoint* keys;
    const uint32_t* desc;   // n x 8 words
    const float* uright;    // may be null
    float minx, maxx, miny, maxy, invw, invh, mbf;
    const float* scale;
    const int* cstart;      // MT_NCELL + 1 offsets, cell = ix * ORBFE_GRID_ROWS + iy
    const int* cidx;        // keypoint indices sorted by (cell, index)
    // level-restricted grids (same layout): grid l holds the keypoints with octave in [l-1, l],
    // the candidate set of a level-l SearchByProjection query (grid 0 = octave 0 only)
    const int* pcstart;
    const int* pcidx;
    int gstride_c, gstride_i;
    int nlevels;            // scale_level / octave of a query must lie in [0, nlevels)
    // two-camera frame (Nleft != -1): rows [0, nleft) are mvKeys, [nleft, n) mvKeysRight; every
    // grid holds the left cells first and the right cells (mGridRight) at cell + MT_NCELL
    int nleft;              // -1: single camera
    const int* l2r;         // mvLeftToRightMatch [nleft]
    const int* r2l;         // mvRightToLeftMatch [n - nleft]
};

__device__ __forceinline__ int mt_hamming(const uint8_t* a, const uint32_t* b) {
    uint32_t w[8];
    memcpy(w, a, 32);
    int d = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d += __popc(w[i] ^ b[i]);
    return d;
}

// Frame::GetFeaturesInArea (Frame.cc:657-723), calling f(idx) in the reference's order.
template <typename Fn>
__device__ __forceinline__ void mt_for_area(const FrameDev& fr, const int* cs, const int* ci, float x, float y, float r,
                                            int minLevel, int maxLevel, Fn&& f) {
    const int nMinCellX = max(0, (int)floorf((x - fr.minx - r) * fr.invw));
    if (nMinCellX >= ORBFE_GRID_COLS) return;
    const int nMaxCellX = min(ORBFE_GRID_COLS - 1, (int)ceilf((x - fr.minx + r) * fr.invw));
    if (nMaxCellX < 0) return;
    const int nMinCellY = max(0, (int)floorf((y - fr.miny - r) * fr.invh));
    if (nMinCellY >= ORBFE_GRID_ROWS) return;
    const int nMaxCellY = min(ORBFE_GRID_ROWS - 1, (int)ceilf((y - fr.miny + r) * fr.invh));
    if (nMaxCellY < 0) return;
    const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
    // cells (ix, nMinCellY..nMaxCellY) are consecutive in the (cell, index)-sorted CSR, so each
    // grid column of the window is ONE contiguous run already in the reference's iy-inner order
    for (int ix = nMinCellX; ix <= nMaxCellX; ix++) {
        const int j1 = cs[ix * ORBFE_GRID_ROWS + nMaxCellY + 1];
        for (int j = cs[ix * ORBFE_GRID_ROWS + nMinCellY]; j < j1; j++) {
            const int idx = ci[j];
            const OrbKeyPoint kp = fr.keys[idx];
            if (bCheckLevels) {
                if (kp.octave < minLevel) continue;
                if (maxLevel >= 0 && kp.octave > maxLevel) continue;
            }
            if (fabsf(kp.x - x) < r && fabsf(kp.y - y) < r) f(idx, kp);
        }
    }
}

// Every per-search initialisation of sbp_run, run by the extra blocks of the grid launch (each used
// to be its own fill / memset / kernel call): initial blocked flags of a device-resident search
// (b0d != nullptr), the pass states of the all -1 assignment, the assignment, the change flags, the
// rotation histogram and the commit result (resb[0] = change-flag copy, resb[1..2] = counts,
// resb[3 + k] = -1). n == 0 and nassign == 0 with null pointers: nothing to initialise.
#define MT_MAX_PASSES 4096
struct SbpInit {
    const int32_t* mvp;
    const int32_t* obs;
    int any_slot;
    int* b0d;
    int* fb0;
    int* fb1;
    int* assign;
    int nassign;
    int* changed;
    int* hist;
    int* resb;
    int n;
};
__device__ __forceinline__ void sbp_init_elem(const SbpInit& a, int k) {
    if (k < a.n) {
        if (a.b0d) a.b0d[k] = a.any_slot ? (a.mvp[k] >= 0) : (a.mvp[k] >= 0 && a.obs[k] > 0);
        a.fb0[k] = MT_INF;
        a.fb1[k] = MT_INF;
    }
    if (k < a.nassign) a.assign[k] = -1;
    if (a.changed && k < MT_MAX_PASSES) a.changed[k] = 0;
    if (a.hist && k < MT_HISTO + 1) a.hist[k] = 0;   // + the commit's block-completion counter
    if (a.resb && k < a.n + 3) a.resb[k] = k < 3 ? 0 : -1;
}
inline int sbp_init_extent(const SbpInit& a) {
    return a.resb ? std::max(std::max(a.n + 3, a.nassign), MT_MAX_PASSES) : 0;
}

// AssignFeaturesToGrid (Frame.cc:385-416): stable (cell, index) order. One block per grid,
// n <= MT_GRID_MAXN. Normally a counting sort by cell (see below); crowded cells fall back to a
// bitonic sort of (cell << 16 | index) keys (unique, so any sorting network gives the same order):
// each thread holds the keys i = tid + 1024 r in registers, the compare-exchange stages with partner
// distance j < 64 stay inside a wave (lane shuffles, no barrier) and only the j >= 64 stages go
// through LDS.
// Two-camera frames (nleft >= 0): rows >= nleft go to the right grid, cells MT_NCELL..
// (Frame.cc:408-411). Blocks >= ngrids run the search initialisation (SbpInit) instead.
#define MT_GRID_MAXN 8192
#define MT_GRID_R (MT_GRID_MAXN / 1024)
__device__ __forceinline__ uint32_t bitonic_keep(uint32_t a, uint32_t c, int i, int j, int k) {
    const bool keep_min = ((i & j) == 0) == ((i & k) == 0);   // lower of the pair == ascending
    return keep_min ? min(a, c) : max(a, c);
}
// The band index of k_sbp_band (single-camera local-map search): keypoints in (octave, 8-row band of
// y) buckets, index order inside a bucket; bucket = octave * NB + min(max(floor(y / 8), 0), NB - 1),
// octaves outside [0, nlev) in no bucket. bstart == nullptr: not built.
#define MT_BAND_ROWS 8
struct BandGrid {
    int* bstart;   // nlev * NB + 1 bucket starts
    int* bidx;     // keypoint indices sorted by (bucket, index)
    int NB, nlev;
};
__device__ __forceinline__ int mt_band_of(float y, int NB) {
    return min(max((int)floorf(y * (1.0f / MT_BAND_ROWS)), 0), NB - 1);
}
__global__ __launch_bounds__(1024) void k_mt_grid(const OrbKeyPoint* keys, int n, int nleft, float minx, float miny,
                                                  float invw, float invh, int* cstart, int* cidx, int gstride_c,
                                                  int gstride_i, int ngrids, SbpInit ia, BandGrid band, int gfirst) {
    __shared__ uint32_t s_k[MT_GRID_MAXN];
    __shared__ int s_m;
    // blocks: grids gfirst .. ngrids - 1 (a search that reads only level grids skips the full one), the
    // band index, then the search initialisation
    const int nbg = ngrids - gfirst;
    const int gi = (int)blockIdx.x < nbg ? (int)blockIdx.x + gfirst : (int)blockIdx.x - nbg + ngrids;
    const int tid = threadIdx.x;
    const int nband = band.bstart ? 1 : 0;
    if (gi >= ngrids + nband) {
        sbp_init_elem(ia, (gi - ngrids - nband) * blockDim.x + tid);
        return;
    }
    const bool is_band = gi == ngrids;
    // block 0: full grid; block g >= 1: keypoints with octave in [g-2, g-1] (level-(g-1) candidates)
    const int lvlo = gi == 0 ? INT_MIN : gi - 2, lvhi = gi == 0 ? INT_MAX : gi - 1;
    if (is_band) {
        cstart = band.bstart;
        cidx = band.bidx;
    } else {
        cstart += (size_t)gi * gstride_c;
        cidx += (size_t)gi * gstride_i;
    }
    const int ncells = is_band ? band.nlev * band.NB : nleft >= 0 ? 2 * MT_NCELL : MT_NCELL;
    // cell of keypoint i (ncells: outside the grid, never a candidate: PosInGrid false)
    auto cell_of = [&](int i) -> uint32_t {
        const OrbKeyPoint kp = keys[i];
        uint32_t cell = (uint32_t)ncells;
        if (is_band) {
            // a two-camera frame's single-camera searches (SearchByProjection(CurrentFrame, pKF))
            // read its left grid only: the right rows [nleft, n) are in no bucket
            if (kp.octave >= 0 && kp.octave < band.nlev && (nleft < 0 || i < nleft))
                cell = (uint32_t)(kp.octave * band.NB + mt_band_of(kp.y, band.NB));
        } else {
            const int px = (int)roundf((kp.x - minx) * invw);
            const int py = (int)roundf((kp.y - miny) * invh);
            if (!(px < 0 || px >= ORBFE_GRID_COLS || py < 0 || py >= ORBFE_GRID_ROWS) && kp.octave >= lvlo &&
                kp.octave <= lvhi)
                cell = (uint32_t)(px * ORBFE_GRID_ROWS + py + (nleft >= 0 && i >= nleft ? MT_NCELL : 0));
        }
        return cell;
    };
    // Stable counting sort by cell when the cells fit in LDS and none is crowded: counts, an exclusive
    // scan (the cell starts), atomic placement, then each cell's few indices put back in index order
    // by one thread (insertion sort). The bitonic network below (about 40 barrier stages at 2,048
    // keys) stays for crowded cells and very many buckets.
    constexpr int CS_MAX = 2 * MT_NCELL;
    __shared__ int s_cnt[CS_MAX + 1];
    __shared__ int s_ws[16], s_maxc;
    uint32_t cr[MT_GRID_R];
#pragma unroll
    for (int r = 0; r < MT_GRID_R; r++) {
        const int i = tid + (r << 10);
        cr[r] = i < n ? cell_of(i) : 0xFFFFFFFFu;
    }
    if (ncells <= CS_MAX) {
        const int nb = ncells + 1;   // + the outside cell (its keys go last)
        for (int c = tid; c < nb; c += blockDim.x) s_cnt[c] = 0;
        if (tid == 0) s_maxc = 0;
        SYNC();
#pragma unroll
        for (int r = 0; r < MT_GRID_R; r++)
            if (cr[r] != 0xFFFFFFFFu) atomicAdd(&s_cnt[cr[r]], 1);
        SYNC();
        const int per = (nb + (int)blockDim.x - 1) / (int)blockDim.x, c0 = tid * per;
        int sum = 0, mx = 0;
        for (int u = 0; u < per; u++) {
            const int c = c0 + u;
            const int v = c < nb ? s_cnt[c] : 0;
            sum += v;
            if (c < ncells) mx = max(mx, v);
        }
        const int incl = wave_incl_scan_dpp(sum);
        if ((tid & 63) == 63) s_ws[tid >> 6] = incl;
        if (mx > 32) atomicMax(&s_maxc, mx);
        SYNC();
        if (s_maxc <= 32) {   // block-uniform
            int run = incl - sum;
            for (int w = 0; w < (int)(blockDim.x >> 6); w++) run += w < (tid >> 6) ? s_ws[w] : 0;
            for (int u = 0; u < per; u++) {
                const int c = c0 + u;
                if (c >= nb) break;
                const int v = s_cnt[c];
                s_cnt[c] = run;   // cursor of the placement
                if (c <= ncells) cstart[c] = run;
                run += v;
            }
            SYNC();
#pragma unroll
            for (int r = 0; r < MT_GRID_R; r++)
                if (cr[r] != 0xFFFFFFFFu) s_k[atomicAdd(&s_cnt[cr[r]], 1)] = (uint32_t)(tid + (r << 10));
            SYNC();
            // s_cnt[c] is now the end of cell c: restore index order inside each cell
            for (int c = tid; c < ncells; c += blockDim.x) {
                const int a = c ? s_cnt[c - 1] : 0, b = s_cnt[c];
                for (int x = a + 1; x < b; x++) {
                    const uint32_t v = s_k[x];
                    int y = x - 1;
                    while (y >= a && s_k[y] > v) { s_k[y + 1] = s_k[y]; y--; }
                    s_k[y + 1] = v;
                }
            }
            SYNC();
            // positions past cstart[ncells] (the outside cell) are never read by a search; the band
            // index keeps them as k_sbp_band stages all n positions
            for (int p = tid; p < n; p += blockDim.x) cidx[p] = (int)s_k[p];
            return;
        }
    }
    // the keys of the grid's keypoints, appended in any order (the (cell, index) sort restores it);
    // a level grid holds a fraction of the frame, so it sorts fewer keys. The band index keeps every
    // keypoint (k_sbp_band stages all n positions).
    if (tid == 0) s_m = 0;
    SYNC();
    // wave-aggregated appends (one LDS atomic per wave and round, positions by mbcnt)
#pragma unroll
    for (int r = 0; r < MT_GRID_R; r++) {
        const int i = tid + (r << 10);
        const uint32_t cell = cr[r];
        const bool keep = i < n && (is_band || cell < (uint32_t)ncells);
        const unsigned long long bm = __ballot(keep);
        const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(bm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bm, 0u));
        int base = 0;
        if ((threadIdx.x & 63) == 0 && bm) base = atomicAdd(&s_m, __popcll(bm));
        base = __shfl(base, 0, 64);
        if (keep) s_k[base + below] = (cell << 16) | (uint32_t)i;
    }
    SYNC();
    const int m = s_m;
    int P = 64;
    while (P < m) P <<= 1;
    const int R = (P + 1023) >> 10;
    uint32_t v[MT_GRID_R];
#pragma unroll
    for (int r = 0; r < MT_GRID_R; r++) {
        const int i = tid + (r << 10);
        v[r] = (r < R && i < m) ? s_k[i] : 0xFFFFFFFFu;
    }
    SYNC();   // every key is in registers before the sort's first LDS round overwrites s_k
    // the intra-wave stages j = min(k/2, 32) .. 1 of one k, on registers (elements >= P pair only
    // among themselves: j < P keeps i ^ j on the same side of P)
    auto wave_stages = [&](int k) {
        for (int j = min(k >> 1, 32); j > 0; j >>= 1)
#pragma unroll
            for (int r = 0; r < MT_GRID_R; r++)
                if (r < R) v[r] = bitonic_keep(v[r], (uint32_t)__shfl_xor((int)v[r], j), tid + (r << 10), j, k);
    };
    for (int k = 2; k <= 64; k <<= 1) wave_stages(k);
    for (int k = 128; k <= P; k <<= 1) {
#pragma unroll
        for (int r = 0; r < MT_GRID_R; r++)
            if (r < R) s_k[tid + (r << 10)] = v[r];
        SYNC();
        for (int j = k >> 1; j >= 64; j >>= 1) {
            for (int i = tid; i < P; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const uint32_t a = s_k[i], c = s_k[ixj];
                    if ((a > c) == ((i & k) == 0)) { s_k[i] = c; s_k[ixj] = a; }
                }
            }
            SYNC();
        }
#pragma unroll
        for (int r = 0; r < MT_GRID_R; r++)
            if (r < R) v[r] = s_k[tid + (r << 10)];
        wave_stages(k);
        SYNC();   // every wave has read s_k before the next k (or the final copy) overwrites it
    }
#pragma unroll
    for (int r = 0; r < MT_GRID_R; r++)
        if (r < R) s_k[tid + (r << 10)] = v[r];
    SYNC();
    for (int i = tid; i < m; i += blockDim.x) cidx[i] = (int)(s_k[i] & 0xFFFFu);
    for (int c = tid; c <= ncells; c += blockDim.x) {
        int lo = 0, hi = m;   // first position with cell >= c
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((int)(s_k[mid] >> 16) < c) lo = mid + 1; else hi = mid;
        }
        cstart[c] = lo;
    }
}

// first[k] = min entry index j with assign[j] == k (and Observations > 0 of its query when
// need_obs); the observation count is read from the query records (byte stride) in place. A query
// writes W consecutive entries (its slot writes in the reference's order), so entry j belongs to
// query j / W and entry order is the reference's write order.
__global__ void k_mt_first_strided(const int* assign, const uint8_t* qobs, int stride, int nent, int need_obs,
                                   int* first, int W) {
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nent) return;
    const int a = assign[j];
    if (a >= 0 && (!need_obs || *(const int*)(qobs + (size_t)(j / W) * stride) > 0)) atomicMin(&first[a], j);
}
__global__ void k_mt_fill(int* p, int n, int v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// Device-side convergence of the single-camera passes: ONE kernel per pass. Pass p reads the
// state first_p (built during pass p - 1), adds its own assignments to first_{p+1} (atomicMin of
// the query index; Observations() > 0 when need_obs) and clears first_{p+2} for the pass after
// (three rotating buffers). A pass whose predecessor changed nothing returns at once (gate), so
// the host enqueues a batch of passes plus the gated commit and synchronises once per call.
struct PassIO {
    const int* gate;     // changed count of the previous pass (nullptr: pass 0 always runs)
    int* first_next;     // first_{p+1}
    int* first_fill;     // first_{p+2}, cleared here
    int n;               // slots
    int need_obs;        // the slot blocks later queries only if the point has observations
    // orbfe_matcher_set_stats: [0] window candidates enumerated (grid cells of the window, octave
    // range), [1] candidate pairs whose Hamming distance is computed; nullptr: no counting
    unsigned long long* stats = nullptr;
};
__device__ __forceinline__ void pass_stats(const PassIO& io, unsigned nwin, unsigned npair) {
    if (io.stats && (nwin | npair)) {
        atomicAdd(&io.stats[0], (unsigned long long)nwin);
        atomicAdd(&io.stats[1], (unsigned long long)npair);
    }
}
__device__ __forceinline__ bool pass_gated(const PassIO& io) { return io.gate && *io.gate == 0; }
// A pass's change word is only ever tested against zero (the next pass's gate, the commit, the host):
// one plain store of 1 per wave that changed something. A counting atomicAdd from every changing
// query put tens of thousands of same-address atomics into one pass (one per wave of four queries
// in the wave-per-four-queries kernels) and serialised them at the memory side. Call from the lanes
// that changed (a ballot over the active lanes picks one writer).
__device__ __forceinline__ void mt_flag_changed(int* changed) {
    const unsigned long long m = __ballot(true);
    if ((int)(threadIdx.x & 63) == __ffsll((long long)m) - 1) *changed = 1;
}
__device__ __forceinline__ void pass_fill(const PassIO& io) {
    const int nt = gridDim.x * blockDim.x;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < io.n; i += nt) io.first_fill[i] = MT_INF;
}
__device__ __forceinline__ void pass_publish(const PassIO& io, int q, int result, int obs) {
    // first_next only decreases during the pass: a query that already sees a smaller index skips its
    // atomic (most of the queries that pick one keypoint come after its first picker)
    if (result >= 0 && (!io.need_obs || obs > 0) && q < __atomic_load_n(&io.first_next[result], __ATOMIC_RELAXED))
        atomicMin(&io.first_next[result], q);
}

// ---- SearchByProjection(Frame&, vector<MapPoint*>, th, bFarPoints, thFar) (ORBmatcher.cc:43-213) ----
__global__ __launch_bounds__(MT_NT) void k_sbp_local(FrameDev fr, const orbfe_map_point* mps, int nq, float th,
                                                     int bFar, float thFar, float nnratio, const int* blocked0,
                                                     const int* first, int* assign, int* changed, PassIO io) {
    if (pass_gated(io)) return;
    pass_fill(io);
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const orbfe_map_point& mp = mps[q];
    int result = -1;
    const bool bFactor = th != 1.0f;
    if ((mp.flags & ORBFE_MP_IN_VIEW) && !(bFar && mp.depth > thFar) && !(mp.flags & ORBFE_MP_BAD) &&
        mp.scale_level >= 0 && mp.scale_level < fr.nlevels) {   // level range: host-checked, device-guarded
        const int lvl = mp.scale_level;
        float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos (ORBmatcher.cc:215-221)
        if (bFactor) r *= th;
        const float R = r * fr.scale[lvl];
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        unsigned nwin = 0, npair = 0;
        mt_for_area(fr, fr.pcstart + lvl * fr.gstride_c, fr.pcidx + lvl * fr.gstride_i, mp.proj_x, mp.proj_y, R,
                    lvl - 1, lvl, [&](int idx, const OrbKeyPoint& kp) {
            nwin++;
            if (blocked0[idx] || first[idx] < q) return;
            if (fr.uright && fr.uright[idx] > 0) {
                const float er = fabsf(mp.proj_xr - fr.uright[idx]);
                if (er > R) return;
            }
            npair++;
            const int dist = mt_hamming(mp.desc, fr.desc + 8 * idx);
            if (dist < bestDist) {
                bestDist2 = bestDist; bestDist = dist;
                bestLevel2 = bestLevel; bestLevel = kp.octave;
                bestIdx = idx;
            } else if (dist < bestDist2) {
                bestLevel2 = kp.octave;
                bestDist2 = dist;
            }
        });
        if (bestDist <= MT_TH_HIGH) {
            if (!(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2)) result = bestIdx;
        }
        pass_stats(io, nwin, npair);
    }
    pass_publish(io, q, result, mp.observations);
    if (result != assign[q]) {
        assign[q] = result;
        mt_flag_changed(changed);
    }
}

// Wide search windows (th >= MT_WAVE_TH): four queries per wave, one per DPP row of 16 lanes. A row
// enumerates its query's candidates in GetFeaturesInArea order (cells ix-outer / iy-inner, 16 grid
// columns at a time flattened with a row prefix sum) and keeps the two smallest (dist, enumeration
// index) keys, exactly the reference's sequential best / second-best (a later equal distance never
// displaces an earlier one). Four query chains per wave in flight: one query per wave ran 0.77 ms at
// config 5 th = 15 against 0.51 (profiles/r04_kernel_ab.txt items 10-11), its time being the
// per-query chain (record -> grid columns -> candidates), not the window. Persistent blocks stage the
// frame's keypoints, descriptors and per-keypoint gates in LDS (a frame beyond MT_STAGE_MAX: keypoints
// and gates only). Frames of <= 2048 keypoints use the LDS-indexed forms instead (k_sbp_block /
// k_sbp_multi / k_sbp_band), so the threshold only splits larger frames: config 5 at N = 5000 measured
// th 3 / 5 at 0.192 / 0.267 ms here against 0.273 / 0.58 one thread per query, th 1 at 0.141 against
// 0.118 (r06_kernel_ab.txt item 20).
#ifndef MT_WAVE_TH
#define MT_WAVE_TH 2.5f
#endif
#define MT_STAGE_MAX 1536
#define MT_WNT 1024   // 16 waves per block share one staged copy of the frame
#define MT_QPW 4      // queries per wave: one per row of 16 lanes
// 64-bit minimum by DPP moves inside each row of 16 lanes (quad swaps, then half-row and row
// mirrors: every lane of a row ends with the row minimum), no LDS round trip
template <int CTRL>
__device__ __forceinline__ unsigned long long mt_min64_dpp_step(unsigned long long v) {
    const unsigned hi = (unsigned)(v >> 32), lo = (unsigned)v;
    const unsigned oh = (unsigned)__builtin_amdgcn_update_dpp((int)hi, (int)hi, CTRL, 0xf, 0xf, false);
    const unsigned ol = (unsigned)__builtin_amdgcn_update_dpp((int)lo, (int)lo, CTRL, 0xf, 0xf, false);
    const unsigned long long o = ((unsigned long long)oh << 32) | ol;
    return o < v ? o : v;
}
__device__ __forceinline__ int mt_row_incl_scan(int v) {   // inclusive scan within each row of 16 lanes
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    return v;
}
__device__ __forceinline__ unsigned long long mt_row_min64(unsigned long long v) {   // every lane: its row's min
    v = mt_min64_dpp_step<0xB1>(v);
    v = mt_min64_dpp_step<0x4E>(v);
    v = mt_min64_dpp_step<0x141>(v);
    return mt_min64_dpp_step<0x140>(v);
}
__device__ __forceinline__ int mt_rows_max(int v) {   // max over the four rows of a row-uniform value
    int m = __builtin_amdgcn_readlane(v, 0);
    m = max(m, __builtin_amdgcn_readlane(v, 16));
    m = max(m, __builtin_amdgcn_readlane(v, 32));
    return max(m, __builtin_amdgcn_readlane(v, 48));
}
// ST = 1: the frame's keypoints, descriptors and gates staged in LDS (n <= MT_STAGE_MAX); ST = 2: the
// keypoints and gates only (larger frames, e.g. BASELINE config 5's 5,000 keypoints: the box, octave
// and gate tests of every window candidate from LDS, descriptors from memory for the candidates that
// pass them); ST = 0: nothing staged.
template <int ST>
__global__ __launch_bounds__(MT_WNT) void k_sbp_local_wq(FrameDev fr, const orbfe_map_point* mps, int nq, float th,
                                                      int bFar, float thFar, float nnratio, const int* blocked0,
                                                      const int* first, int* assign, int* changed, PassIO io) {
    constexpr int GL = 16;
    extern __shared__ __attribute__((aligned(16))) uint8_t mt_sm[];
    if (pass_gated(io)) return;
    pass_fill(io);
    int2* s_cell = (int2*)mt_sm;                                          // [16 waves][4 rows][16] (start, prefix)
    float4* s_key = (float4*)(mt_sm + (MT_WNT / 64) * 64 * sizeof(int2));  // x, y, octave bits, uR
    uint4* s_desc = (uint4*)(s_key + (ST ? fr.n : 0));             // 2 x uint4 per keypoint (ST == 1)
    int2* s_gate = (int2*)(s_desc + (ST == 1 ? 2 * fr.n : 0));     // {blocked0, first}, read-only in a pass
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, grp = lane >> 4, sl = lane & 15;
    if (ST) {
        for (int i = tid; i < fr.n; i += MT_WNT) {
            const OrbKeyPoint kp = fr.keys[i];
            s_key[i] = make_float4(kp.x, kp.y, __int_as_float(kp.octave), fr.uright ? fr.uright[i] : -1.f);
            if (ST == 1) {
                const uint4* d = (const uint4*)(fr.desc + 8 * i);
                s_desc[2 * i] = d[0];
                s_desc[2 * i + 1] = d[1];
            }
            s_gate[i] = make_int2(blocked0[i], first[i]);
        }
        SYNC();
    }
    int2* my_cells = s_cell + 64 * wave + GL * grp;
    constexpr int WPB = MT_WNT / 64;
    for (int q0 = (blockIdx.x * WPB + wave) * MT_QPW; q0 < nq; q0 += gridDim.x * WPB * MT_QPW) {
        const int q = q0 + grp;
        const bool qv = q < nq;
        int prev = -1, obs = 0, lvl = 0, ncell = 0, cx0 = 0, cy0 = 0, cy1 = -1;
        float R = 0.f, x = 0.f, y = 0.f, xr = 0.f;
        uint32_t qd[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        if (qv) {
            const orbfe_map_point& mp = mps[q];
            prev = assign[q];
            obs = mp.observations;
            if ((mp.flags & ORBFE_MP_IN_VIEW) && !(bFar && mp.depth > thFar) && !(mp.flags & ORBFE_MP_BAD) &&
                mp.scale_level >= 0 && mp.scale_level < fr.nlevels) {
                lvl = mp.scale_level;
                float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;
                if (th != 1.0f) r *= th;
                R = r * fr.scale[lvl];
                x = mp.proj_x;
                y = mp.proj_y;
                xr = mp.proj_xr;
                memcpy(qd, mp.desc, 32);
                cx0 = max(0, (int)floorf((x - fr.minx - R) * fr.invw));
                const int cx1 = min(ORBFE_GRID_COLS - 1, (int)ceilf((x - fr.minx + R) * fr.invw));
                cy0 = max(0, (int)floorf((y - fr.miny - R) * fr.invh));
                cy1 = min(ORBFE_GRID_ROWS - 1, (int)ceilf((y - fr.miny + R) * fr.invh));
                if (cx0 < ORBFE_GRID_COLS && cx1 >= 0 && cy0 < ORBFE_GRID_ROWS && cy1 >= 0 && cx0 <= cx1 && cy0 <= cy1)
                    ncell = cx1 - cx0 + 1;
            }
        }
        const int minLevel = lvl - 1, maxLevel = lvl;
        const bool bCheckLevels = (minLevel > 0) || (maxLevel >= 0);
        const int* pcs = fr.pcstart + lvl * fr.gstride_c;
        const int* pci = fr.pcidx + lvl * fr.gstride_i;
        unsigned long long b1 = ~0ull, b2 = ~0ull;
        int b1idx = -1;
        unsigned nwin = 0, npair = 0;
        int obase = 0;
        const int ncmax = mt_rows_max(ncell);
        // one contiguous CSR run per grid column of the window, 16 columns per round
        for (int cb = 0; cb < ncmax; cb += GL) {
            const int c = cb + sl;
            int st = 0, cnt = 0;
            if (c < ncell) {
                const int ix = cx0 + c;
                st = pcs[ix * ORBFE_GRID_ROWS + cy0];
                cnt = pcs[ix * ORBFE_GRID_ROWS + cy1 + 1] - st;
            }
            const int incl = mt_row_incl_scan(cnt);
            const int tot = __shfl(incl, lane | 15, 64);
            my_cells[sl] = make_int2(st, incl - cnt);
            WAVE_SYNC();
            const int totmax = mt_rows_max(tot);
            for (int j0 = 0; j0 < totmax; j0 += GL) {
                const int j = j0 + sl;
                if (j < tot) {
                    nwin++;
                    int lo = 0, hi = GL;   // last cell with prefix <= j
                    while (hi - lo > 1) {
                        const int mid = (lo + hi) >> 1;
                        if (my_cells[mid].y <= j) lo = mid; else hi = mid;
                    }
                    const int2 ce = my_cells[lo];
                    const int idx = pci[ce.x + (j - ce.y)];
                    float kx, ky, ur;
                    int oct;
                    if (ST) {
                        const float4 k4 = s_key[idx];
                        kx = k4.x; ky = k4.y; oct = __float_as_int(k4.z); ur = k4.w;
                    } else {
                        const OrbKeyPoint kp = fr.keys[idx];
                        kx = kp.x; ky = kp.y; oct = kp.octave; ur = fr.uright ? fr.uright[idx] : -1.f;
                    }
                    bool ok = true;
                    if (bCheckLevels) {
                        if (oct < minLevel) ok = false;
                        if (maxLevel >= 0 && oct > maxLevel) ok = false;
                    }
                    ok = ok && fabsf(kx - x) < R && fabsf(ky - y) < R;
                    if (ST) {
                        const int2 gt = s_gate[idx];
                        ok = ok && !(gt.x || gt.y < q);
                    } else {
                        ok = ok && !(blocked0[idx] || first[idx] < q);
                    }
                    if (ok && ur > 0) ok = !(fabsf(xr - ur) > R);
                    if (ok) {
                        npair++;
                        uint4 d0, d1;
                        if (ST == 1) { d0 = s_desc[2 * idx]; d1 = s_desc[2 * idx + 1]; }
                        else { d0 = ((const uint4*)(fr.desc + 8 * idx))[0]; d1 = ((const uint4*)(fr.desc + 8 * idx))[1]; }
                        const int dist = __popc(qd[0] ^ d0.x) + __popc(qd[1] ^ d0.y) + __popc(qd[2] ^ d0.z) +
                                         __popc(qd[3] ^ d0.w) + __popc(qd[4] ^ d1.x) + __popc(qd[5] ^ d1.y) +
                                         __popc(qd[6] ^ d1.z) + __popc(qd[7] ^ d1.w);
                        if (dist < 256) {
                            const unsigned long long k = ((unsigned long long)dist << 32) |
                                                         ((unsigned long long)(obase + j) << 4) | (unsigned)oct;
                            if (k < b1) { b2 = b1; b1 = k; b1idx = idx; }
                            else if (k < b2) b2 = k;
                        }
                    }
                }
            }
            obase += tot;
            WAVE_SYNC();
        }
        pass_stats(io, nwin, npair);
        const unsigned long long m1 = mt_row_min64(b1);
        const unsigned long long win = (__ballot(b1 == m1 && m1 != ~0ull) >> (GL * grp)) & 0xFFFFull;
        const unsigned long long m2 = mt_row_min64(b1 == m1 ? b2 : b1);
        const int wl = win ? GL * grp + __ffsll((long long)win) - 1 : lane;
        const int bestIdx = __shfl(b1idx, wl, 64);   // every lane takes part
        int result = -1;
        if (m1 != ~0ull) {
            const int bestDist = (int)(m1 >> 32), bestLevel = (int)(m1 & 15);
            const int bestDist2 = m2 != ~0ull ? (int)(m2 >> 32) : 256;
            const int bestLevel2 = m2 != ~0ull ? (int)(m2 & 15) : -1;
            if (bestDist <= MT_TH_HIGH) {
                if (!(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2)) result = bestIdx;
            }
        }
        if (sl == 0 && qv) {
            pass_publish(io, q, result, obs);
            if (result != prev) {
                assign[q] = result;
                mt_flag_changed(changed);
            }
        }
    }
}

// SearchByProjection(Frame&, vector<MapPoint*>, ...) (ORBmatcher.cc:43-213) for a single-camera frame
// of at most MT_BAND_MAXN keypoints, every th: the frame lives in LDS in (octave, 8-row band)
// order (BandGrid), so a query's candidates are two contiguous LDS runs (octaves lvl - 1 and lvl,
// the bands its y window touches, one band of margin each side) that the 16 lanes of its DPP row
// read in order: no grid walk, no per-candidate search. GetFeaturesInArea's candidates are exactly the
// in-grid keypoints of those octaves with |dx| < r and |dy| < r (a keypoint inside the box lies in a
// cell of the reference's window: round() of a value inside [floor(lo), ceil(hi)]), and its
// enumeration order (cell ix, iy, then index, Frame.cc:691-719) is the rank (cell << 13 | index)
// carried in each candidate's key, so the two smallest (dist, rank) keys are the reference's
// best / second best whatever order the lanes visit them in. Four queries per wave, one per row.
#define MT_BAND_MAXN 2048
#define MT_BNT 1024
__global__ __launch_bounds__(MT_BNT) void k_sbp_band(FrameDev fr, BandGrid bg, const orbfe_map_point* mps, int nq,
                                                     float th, int bFar, float thFar, float nnratio,
                                                     const int* blocked0, const int* first, int* assign, int* changed,
                                                     PassIO io, const int* fprev, int qshift) {
    extern __shared__ __attribute__((aligned(16))) uint8_t mt_sm[];
    if (pass_gated(io)) return;
    pass_fill(io);
    const int n = fr.n;
    const int nbk = bg.nlev * bg.NB;
    float4* s_kp = (float4*)mt_sm;                 // {x, y, rank bits, uR} per band position
    uint4* s_desc = (uint4*)(s_kp + n);            // 2 x uint4 per band position
    int* s_gate = (int*)(s_desc + 2 * n);          // -1: blocked initially, else first[] (MT_INF: free)
    int* s_bs = s_gate + n;                        // bucket starts [nbk + 1]
    // per bucket: the query bins (q >> qshift, 128 of them, two words) whose view of some keypoint of
    // the bucket changed since the previous pass (fprev: that pass's first[]; nullptr: no skipping)
    unsigned long long* s_cm = (unsigned long long*)(((uintptr_t)(s_bs + nbk + 1) + 7) & ~(uintptr_t)7);
    int* s_gprev = (int*)(s_cm + 2 * nbk);         // fprev[] per band position
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, grp = lane >> 4, sl = lane & 15;
    for (int p = tid; p < n; p += MT_BNT) {
        const int idx = bg.bidx[p];
        const OrbKeyPoint kp = fr.keys[idx];
        const int px = (int)roundf((kp.x - fr.minx) * fr.invw);   // PosInGrid (Frame.cc:725-735)
        const int py = (int)roundf((kp.y - fr.miny) * fr.invh);
        const bool in_grid = !(px < 0 || px >= ORBFE_GRID_COLS || py < 0 || py >= ORBFE_GRID_ROWS);
        const uint32_t rank = ((uint32_t)(px * ORBFE_GRID_ROWS + py) << 13) | (uint32_t)idx;
        s_kp[p] = make_float4(in_grid ? kp.x : __builtin_nanf(""), kp.y, __uint_as_float(rank),
                              fr.uright ? fr.uright[idx] : -1.f);
        const uint4* d = (const uint4*)(fr.desc + 8 * idx);
        s_desc[2 * p] = d[0];
        s_desc[2 * p + 1] = d[1];
        s_gate[p] = blocked0[idx] ? -1 : first[idx];
        if (fprev) s_gprev[p] = fprev[idx];
    }
    for (int b = tid; b <= nbk; b += MT_BNT) s_bs[b] = bg.bstart[b];
    SYNC();
    // Passes >= 1 skip the queries whose candidates all kept their gate: candidate k is open to query q
    // iff gate_k >= q, so a gate that moved from a to b changes it exactly for q in (min, max]. A
    // query none of whose window buckets holds such a change in its bin computes the previous pass's
    // result again (the same candidates, descriptors and gates), which assign[q] still holds.
    if (fprev) {
        for (int b = tid; b < nbk; b += MT_BNT) {
            unsigned long long m0 = 0ull, m1 = 0ull;
            for (int p = s_bs[b]; p < s_bs[b + 1]; p++) {
                const int gc = s_gate[p];
                if (gc < 0) continue;   // blocked in every pass
                const int gp = s_gprev[p];
                if (gp == gc) continue;
                const int lo = min(gp, gc) + 1, hi = min(max(gp, gc), nq - 1);
                if (lo > hi) continue;
                const int blo = lo >> qshift, bhi = hi >> qshift;   // bins blo .. bhi of 0 .. 127
                auto bits = [](int a, int z) -> unsigned long long {   // bits a .. z of one word, clipped
                    if (z < 0 || a > 63) return 0ull;
                    a = max(a, 0);
                    return (z >= 63 ? ~0ull : ((2ull << z) - 1ull)) & ~((1ull << a) - 1ull);
                };
                m0 |= bits(blo, bhi);
                m1 |= bits(blo - 64, bhi - 64);
            }
            s_cm[2 * b] = m0;
            s_cm[2 * b + 1] = m1;
        }
        SYNC();
    }
    constexpr int WPB = MT_BNT / 64;
    for (int q0 = (blockIdx.x * WPB + wave) * MT_QPW; q0 < nq; q0 += gridDim.x * WPB * MT_QPW) {
        const int q = q0 + grp;
        int prev = -1, obs = 0, lvl = 0, s1 = 0, n1 = 0, s2 = 0, n2 = 0, bk0 = 0, nbd = 0;
        float R = 0.f, x = 0.f, y = 0.f, xr = 0.f;
        uint32_t qd[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
        if (q < nq) {
            const orbfe_map_point& mp = mps[q];
            prev = assign[q];
            obs = mp.observations;
            if ((mp.flags & ORBFE_MP_IN_VIEW) && !(bFar && mp.depth > thFar) && !(mp.flags & ORBFE_MP_BAD) &&
                mp.scale_level >= 0 && mp.scale_level < fr.nlevels) {
                lvl = mp.scale_level;
                float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos (ORBmatcher.cc:215-221)
                if (th != 1.0f) r *= th;
                R = r * fr.scale[lvl];
                x = mp.proj_x;
                y = mp.proj_y;
                xr = mp.proj_xr;
                memcpy(qd, mp.desc, 32);
                // the bands of (y - R, y + R), one band of margin for the rounding of y -+ R
                const int b0 = max(mt_band_of(y - R, bg.NB) - 1, 0), b1 = min(mt_band_of(y + R, bg.NB) + 1, bg.NB - 1);
                if (lvl < bg.nlev) {
                    s2 = s_bs[lvl * bg.NB + b0];
                    n2 = s_bs[lvl * bg.NB + b1 + 1] - s2;
                    if (lvl >= 1) {
                        s1 = s_bs[(lvl - 1) * bg.NB + b0];
                        n1 = s_bs[(lvl - 1) * bg.NB + b1 + 1] - s1;
                    }
                    nbd = b1 - b0 + 1;
                    bk0 = (lvl >= 1 ? lvl - 1 : lvl) * bg.NB + b0;
                }
            }
        }
        bool skip = false;
        if (fprev) {   // the row's lanes test the window's buckets (both octaves) for a change in q's bin
            const int nbt = lvl >= 1 ? 2 * nbd : nbd, bin = q >> qshift;
            bool hit = false;
            for (int i = sl; i < nbt; i += 16) {
                const int bk = i < nbd ? bk0 + i : bk0 + bg.NB + (i - nbd);
                hit = hit || ((s_cm[2 * bk + (bin >> 6)] >> (bin & 63)) & 1ull);
            }
            skip = ((__ballot(hit) >> (16 * grp)) & 0xFFFFull) == 0ull;
        }
        const int tot = skip ? 0 : n1 + n2;
        unsigned long long b1k = ~0ull, b2k = ~0ull;
        unsigned nwin = 0, npair = 0;
        const int totmax = mt_rows_max(tot);
        for (int j0 = 0; j0 < totmax; j0 += 16) {
            const int j = j0 + sl;
            if (j < tot) {
                const bool lo = j < n1;
                const int p = lo ? s1 + j : s2 + (j - n1);
                const int oct = lo ? lvl - 1 : lvl;
                const float4 k4 = s_kp[p];
                bool ok = fabsf(k4.x - x) < R && fabsf(k4.y - y) < R;
                if (ok) {
                    nwin++;
                    ok = s_gate[p] >= q;
                    if (ok && k4.w > 0) ok = !(fabsf(xr - k4.w) > R);
                }
                if (ok) {
                    npair++;
                    const uint4 d0 = s_desc[2 * p], d1 = s_desc[2 * p + 1];
                    const int dist = __popc(qd[0] ^ d0.x) + __popc(qd[1] ^ d0.y) + __popc(qd[2] ^ d0.z) +
                                     __popc(qd[3] ^ d0.w) + __popc(qd[4] ^ d1.x) + __popc(qd[5] ^ d1.y) +
                                     __popc(qd[6] ^ d1.z) + __popc(qd[7] ^ d1.w);
                    const unsigned long long k = ((unsigned long long)dist << 40) |
                                                 ((unsigned long long)__float_as_uint(k4.z) << 4) | (unsigned)oct;
                    if (k < b1k) { b2k = b1k; b1k = k; }
                    else if (k < b2k) b2k = k;
                }
            }
        }
        pass_stats(io, nwin, npair);
        const unsigned long long m1 = mt_row_min64(b1k);
        const unsigned long long m2 = mt_row_min64(b1k == m1 ? b2k : b1k);
        int result = -1;
        if (m1 != ~0ull) {
            const int bestDist = (int)(m1 >> 40), bestLevel = (int)(m1 & 15);
            const int bestDist2 = m2 != ~0ull ? (int)(m2 >> 40) : 256;
            const int bestLevel2 = m2 != ~0ull ? (int)(m2 & 15) : -1;
            if (bestDist <= MT_TH_HIGH) {
                if (!(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2))
                    result = (int)((m1 >> 4) & 0x1FFFu);   // the keypoint index carried in the rank
            }
        }
        if (skip) result = prev;
        if (sl == 0 && q < nq) {
            pass_publish(io, q, result, obs);
            if (result != prev) {
                assign[q] = result;
                mt_flag_changed(changed);
            }
        }
    }
}

// Small single-camera searches (nq <= MT_BLOCK_MAXQ: the per-frame Tracking calls, a few hundred to a
// few thousand queries) in ONE workgroup: the frame in LDS as for k_sbp_band, one thread per query,
// and the whole fixed point (ORBmatcher's ordered "later queries see earlier assignments", see the
// top of this file) iterated inside the block, the first[] states in LDS and a barrier between
// passes. A multi-block pass costs a launch and a round trip through memory per pass and its
// one-thread-per-query grid walk is a chain of dependent global loads; a Tracking call's dependency
// chains need up to ~10 passes (SearchByProjection(CurrentFrame, LastFrame): duplicated corners of
// neighbouring octaves compete for the same keypoints), which here are a few microseconds each.
//   MODE 0: SearchByProjection(F, vpMapPoints, th, bFarPoints, thFar) (ORBmatcher.cc:43-213): best and
//           second best with their levels, ratio test; records orbfe_map_point.
//   MODE 1: SearchByProjection(CurrentFrame, LastFrame, th, bMono) (:1676-1887), MODE 2:
//           SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (:1889-2010): single
//           best (strict <, the first minimum in GetFeaturesInArea order = the smallest (dist, rank)
//           key) within maxDist; records orbfe_proj_point.
// Candidates: the in-grid keypoints of the octave range with |dx| < r and |dy| < r (k_sbp_band's
// argument), read from the (octave, band) runs of the bands (y - r, y + r) touches.
#define MT_BLOCK_MAXQ 2048
#define MT_LDS_MAX (160 * 1024 - 1024)   // dynamic LDS of k_sbp_block (the static part is < 1 KB)
#define MT_BLK_NT 1024
#define MT_BLK_QPT (MT_BLOCK_MAXQ / MT_BLK_NT)
__host__ __device__ __forceinline__ int mt_rot_bin(float a1, float a2);
__host__ __device__ __forceinline__ unsigned mt_three_maxima_keep(const int* hist);
// What k_sbp_block reads besides the frame and the records, and where it reports: the slot state
// (F.mvpMapPoints handles and their Observations(), blocked0 = a held slot that blocks, any held slot
// for the keyframe variant), the record fields the commit needs, and the pinned status words the
// host waits on ({0, assigned, dropped, passes, sequence number, nToMatch}, as k_mt_commit_write).
struct BlkIO {
    const int32_t* mvp_in;     // slots before the search (device)
    const int32_t* obs_in;     // Observations() per slot (nullptr: any held slot blocks)
    int32_t* mvp_out;          // slots after the search (may alias mvp_in)
    int q_stride, qid_off, qangle_off, checkOri;
    const int* ntm;            // k_frustum's nToMatch (nullptr: none)
    int* st_host;              // pinned status words
    int seq;
    unsigned long long* stats;   // [3]: window candidates, Hamming pairs, passes (nullptr: off)
    uint4* qdev;               // device copy of host-memory records for the re-enumerations (nullptr: records in HBM)
};
// Records in mapped host memory are read once over PCIe: the block copies them into HBM scratch
// (before the frame staging, whose barriers publish it), and a list that runs out re-reads its record
// from there instead of paying another PCIe round trip inside a pass.
__device__ __forceinline__ const void* blk_qcopy(const BlkIO& io, const void* recs, int nq) {
    if (!io.qdev) return recs;
    const int nv = nq * io.q_stride / 16;
    for (int i = threadIdx.x; i < nv; i += blockDim.x) io.qdev[i] = ((const uint4*)recs)[i];
    return io.qdev;
}
// k_sbp_block's LDS index: buckets (octave, band of br rows, strip of sw columns), bucket
// c = (octave * NB + band) * NS + strip (the strips of a band are consecutive, so a query's window is one
// contiguous run per (octave, band)); be[c] .. be[c + 1] is bucket c's run of band positions.
struct BlkGeom {
    int NB, NS;
    float inv_br, inv_sw;
    __device__ __forceinline__ int band(float y) const { return min(max((int)floorf(y * inv_br), 0), NB - 1); }
    __device__ __forceinline__ int strip(float x) const { return min(max((int)floorf(x * inv_sw), 0), NS - 1); }
};
// A query of k_sbp_block: its window and descriptor (from its record, pass 0 and fallbacks only)
struct BlkQuery {
    float x, y, R, xr;
    int olo, ohi, obs;
    bool ok;
    uint32_t qd[8];
};
template <int MODE>
__device__ __forceinline__ BlkQuery blk_load(const FrameDev& fr, const void* recs, int q, float th, int a0, int a1,
                                             float thFar) {
    BlkQuery Q;
    Q.x = Q.y = Q.R = Q.xr = 0.f;
    Q.olo = 0;
    Q.ohi = -1;
    if (MODE == 0) {
        const orbfe_map_point& mp = ((const orbfe_map_point*)recs)[q];
        Q.obs = mp.observations;
        Q.ok = (mp.flags & ORBFE_MP_IN_VIEW) && !(a0 && mp.depth > thFar) && !(mp.flags & ORBFE_MP_BAD) &&
               mp.scale_level >= 0 && mp.scale_level < fr.nlevels;
        if (Q.ok) {
            const int lvl = mp.scale_level;
            float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos (ORBmatcher.cc:215-221)
            if (th != 1.0f) r *= th;
            Q.R = r * fr.scale[lvl];
            Q.x = mp.proj_x;
            Q.y = mp.proj_y;
            Q.xr = mp.proj_xr;
            Q.olo = max(lvl - 1, 0);
            Q.ohi = lvl;
            memcpy(Q.qd, mp.desc, 32);
        }
    } else {
        const orbfe_proj_point& pp = ((const orbfe_proj_point*)recs)[q];
        Q.obs = pp.observations;
        Q.ok = pp.valid != 0 && pp.octave >= 0 && pp.octave < fr.nlevels;
        if (Q.ok && MODE == 1) {   // ORBmatcher.cc:1718-1736
            if (pp.invzc < 0) Q.ok = false;
            else if (pp.u < fr.minx || pp.u > fr.maxx) Q.ok = false;
            else if (pp.v < fr.miny || pp.v > fr.maxy) Q.ok = false;
        }
        if (Q.ok) {
            const int oct = pp.octave;
            Q.R = th * fr.scale[oct];
            Q.x = pp.u;
            Q.y = pp.v;
            Q.xr = MODE == 1 ? pp.u - fr.mbf * pp.invzc : 0.f;   // ur of :1752
            // GetFeaturesInArea's level filter (Frame.cc:689,704-711: bCheckLevels)
            int minL, maxL;
            if (MODE == 2) { minL = oct - 1; maxL = oct + 1; }
            else if (a0) { minL = oct; maxL = -1; }
            else if (a1) { minL = 0; maxL = oct; }
            else { minL = oct - 1; maxL = oct + 1; }
            const bool chk = (minL > 0) || (maxL >= 0);
            Q.olo = chk ? max(minL, 0) : 0;
            Q.ohi = (chk && maxL >= 0) ? min(maxL, fr.nlevels - 1) : fr.nlevels - 1;
            memcpy(Q.qd, pp.desc, 32);
        }
    }
    if (Q.ohi >= fr.nlevels) Q.ok = false;
    return Q;
}
// Q's candidates that pass every gate-independent test (box, octave range, stereo), f(key, idx):
// key = dist << 40 | rank << 4 | octave (the reference's enumeration order breaks distance ties)
// cbase: the first bucket of the camera searched (k_sbp_block2: nlev * NB * NS for the right grid);
// nwin: when given, counts every keypoint of the window (GetFeaturesInArea's result, blocked or not).
// MODE 3 = a two-camera frame's last-frame search (k_sbp_block2): MODE 1's gates without the stereo
// test (ORBmatcher.cc:1747-1760 runs for Nleft == -1 only). MODE 4 = a two-camera frame's local-map
// search (k_sbp_block4): no stereo test, and a slot held before the search is NOT skipped here (an
// earlier point's unguarded partner write can replace its holder: the pass gates decide).
template <int MODE, typename Fn>
__device__ __forceinline__ void blk_enum(const BlkQuery& Q, const BlkGeom& gm, const float4* s_kp, const uint4* s_desc,
                                         const int* s_be, const uint8_t* s_blk, Fn&& f, int cbase = 0,
                                         int* nwin = nullptr) {
    if (!Q.ok || Q.olo > Q.ohi) return;
    // the buckets of (x -+ (r + 1), y -+ (r + 1)): a keypoint that passes the box test lies inside (one
    // pixel of margin is far beyond the rounding of the bounds); out-of-grid keypoints are in no bucket
    const int b0 = gm.band(Q.y - Q.R - 1.f), b1 = gm.band(Q.y + Q.R + 1.f);
    const int s0 = gm.strip(Q.x - Q.R - 1.f), s1 = gm.strip(Q.x + Q.R + 1.f);
    for (int o = Q.olo; o <= Q.ohi; o++)
    for (int b = b0; b <= b1; b++) {
        const int c = cbase + (o * gm.NB + b) * gm.NS;
        const int pe = s_be[c + s1 + 1];
        // four positions per step, their box reads issued together (a thread's run is a chain of
        // LDS round trips otherwise)
        for (int p0 = s_be[c + s0]; p0 < pe; p0 += 4) {
            float4 kk[4];
#pragma unroll
            for (int u = 0; u < 4; u++) kk[u] = s_kp[min(p0 + u, pe - 1)];
#pragma unroll
            for (int u = 0; u < 4; u++) {
            const int p = p0 + u;
            const float4 k4 = kk[u];
            if (p >= pe || !(fabsf(k4.x - Q.x) < Q.R && fabsf(k4.y - Q.y) < Q.R)) continue;
            if (nwin) ++*nwin;
            const int idx = (int)(__float_as_uint(k4.z) & 0x1FFFu);
            if (MODE != 4 && s_blk[idx]) continue;
            if (MODE < 2 && k4.w > 0 && fabsf(Q.xr - k4.w) > Q.R) continue;
            const uint4 d0 = s_desc[2 * p], d1 = s_desc[2 * p + 1];
            const int dist = __popc(Q.qd[0] ^ d0.x) + __popc(Q.qd[1] ^ d0.y) + __popc(Q.qd[2] ^ d0.z) +
                             __popc(Q.qd[3] ^ d0.w) + __popc(Q.qd[4] ^ d1.x) + __popc(Q.qd[5] ^ d1.y) +
                             __popc(Q.qd[6] ^ d1.z) + __popc(Q.qd[7] ^ d1.w);
            f(((unsigned long long)dist << 40) | ((unsigned long long)__float_as_uint(k4.z) << 4) | (unsigned)o, idx);
            }
        }
    }
}
// the reference's acceptance from the best / second-best (dist, octave) of a query
template <int MODE>
__device__ __forceinline__ int blk_accept(int bestIdx, int bestDist, int bestLevel, int bestDist2, int bestLevel2,
                                          float nnratio, int maxDist) {
    if (bestIdx < 0) return -1;
    if (MODE == 0)
        return bestDist <= MT_TH_HIGH && !(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) ? bestIdx : -1;
    return bestDist <= maxDist ? bestIdx : -1;
}

#define MT_BLK_LIST 8   // candidates kept per query: the smallest keys, as u32 idx | octave << 13 | dist << 16
// Bucket bounds region: 4 zero words, then one counter per bucket padded to a multiple of 4 NT (each
// thread scans a run of whole int4s); after the placement, word 4 + c = end of bucket c, so the
// enumeration's bounds array ("be", be[c] = start of c, be[c + 1] = end) is region + 3.
__host__ __device__ __forceinline__ int blk_be_words(int nbk, int nt) {
    const int per = ((nbk + nt - 1) / nt + 3) & ~3;
    return per * nt + 4;
}
// k_sbp_block's / k_sbp_multi0's LDS frame: the (octave, band, strip) bucket index (counts, scan,
// placement; the order inside a bucket is irrelevant: every candidate carries its enumeration rank),
// keypoints {x, y, rank bits, uR} and descriptors by bucket position, blocked flags (and angles, the
// first[] state, when given) by keypoint index. s_be: the 16-byte aligned bounds region
// (blk_be_words). Ends with a barrier.
// ncam = 2 (k_sbp_block2): a two-camera frame's right keypoints [nleft, n) in a second bucket set
// after the left one (bucket + nlev * NB * NS); ncam = 1: its single-camera searches read the left
// grid only.
template <int NT>
__device__ __forceinline__ void blk_stage(const FrameDev& fr, const BlkGeom& gm, const int32_t* mvp_in,
                                          const int32_t* obs_in, float4* s_kp, uint4* s_desc, int* s_be,
                                          uint8_t* s_blk, float* s_ang, int* s_first, int* s_ws, int ncam = 1) {
    const int n = fr.n, nlev = fr.nlevels, nbk = ncam * nlev * gm.NB * gm.NS, tid = threadIdx.x;
    const int per = ((nbk + NT - 1) / NT + 3) & ~3;   // buckets per thread in the scan (whole int4s)
    for (int b = tid; b < (per * NT + 4) / 4; b += NT) ((int4*)s_be)[b] = make_int4(0, 0, 0, 0);
    int* a = s_be + 4;   // counters, then starts, then ends
    SYNC();
    auto bucket_of = [&](float x, float y, int oct, int idx) {
        // a two-camera frame's single-camera searches read its left grid only (rows [0, nleft)); a
        // keypoint outside the grid (PosInGrid, Frame.cc:725-735) is in no cell of the reference
        const int px = (int)roundf((x - fr.minx) * fr.invw);
        const int py = (int)roundf((y - fr.miny) * fr.invh);
        const bool in_grid = !(px < 0 || px >= ORBFE_GRID_COLS || py < 0 || py >= ORBFE_GRID_ROWS);
        const int cam = (fr.nleft >= 0 && idx >= fr.nleft) ? 1 : 0;
        return (in_grid && oct >= 0 && oct < nlev && cam < ncam)
                   ? ((cam * nlev + oct) * gm.NB + gm.band(y)) * gm.NS + gm.strip(x) : -1;
    };
    // every keypoint's data is read from memory ONCE, into registers (n <= 2 x NT), before the bucket
    // counts: one round trip for the whole staging (the fields, not the struct: a struct array
    // copy is not promoted to registers)
    constexpr int KPT = (MT_BAND_MAXN + NT - 1) / NT;
    float kx[KPT], ky[KPT], kang[KPT];
    int koct[KPT];
    uint4 rd0[KPT], rd1[KPT];
    float rur[KPT];
    int rblk[KPT], rb[KPT];
#pragma unroll
    for (int u = 0; u < KPT; u++) {
        const int idx = tid + u * NT;
        rb[u] = -1;
        kx[u] = ky[u] = kang[u] = rur[u] = 0.f;
        koct[u] = rblk[u] = 0;
        rd0[u] = rd1[u] = make_uint4(0u, 0u, 0u, 0u);
        if (idx >= n) continue;
        const OrbKeyPoint& kp = fr.keys[idx];
        kx[u] = kp.x;
        ky[u] = kp.y;
        kang[u] = kp.angle;
        koct[u] = kp.octave;
        const uint4* d = (const uint4*)(fr.desc + 8 * idx);
        rd0[u] = d[0];
        rd1[u] = d[1];
        rur[u] = fr.uright ? fr.uright[idx] : -1.f;
        const int hb = mvp_in[idx] >= 0;
        rblk[u] = obs_in ? (hb && obs_in[idx] > 0) : hb;
    }
#pragma unroll
    for (int u = 0; u < KPT; u++) {
        const int idx = tid + u * NT;
        if (idx >= n) continue;
        rb[u] = bucket_of(kx[u], ky[u], koct[u], idx);
        if (rb[u] >= 0) atomicAdd(&a[rb[u]], 1);
    }
    SYNC();
    // counts -> starts (a[c] = start of c); the placement's atomic increments then leave a[c] at the
    // end of bucket c, i.e. the start of c + 1, with a[-1] = 0. One run of whole int4s per thread:
    // one barrier, and 16-byte LDS accesses instead of per-word strided ones.
    {
        int4* a4 = (int4*)a + tid * (per >> 2);
        int sum = 0;
        for (int j = 0; j < (per >> 2); j++) {
            const int4 v = a4[j];
            sum += v.x + v.y + v.z + v.w;
        }
        const int incl = wave_incl_scan_dpp(sum);
        if ((tid & 63) == 63) s_ws[tid >> 6] = incl;
        SYNC();
        int run = incl - sum;
#pragma unroll
        for (int w = 0; w < NT / 64; w++) run += w < (tid >> 6) ? s_ws[w] : 0;
        for (int j = 0; j < (per >> 2); j++) {
            const int4 v = a4[j];
            int4 o;
            o.x = run; run += v.x;
            o.y = run; run += v.y;
            o.z = run; run += v.z;
            o.w = run; run += v.w;
            a4[j] = o;
        }
    }
    SYNC();
#pragma unroll
    for (int u = 0; u < KPT; u++) {
        const int idx = tid + u * NT;
        if (idx >= n) continue;
        s_blk[idx] = (uint8_t)rblk[u];
        if (s_first) s_first[idx] = MT_INF;
        if (s_ang) s_ang[idx] = kang[u];
        if (rb[u] < 0) continue;
        const int p = atomicAdd(&a[rb[u]], 1);
        const int px = (int)roundf((kx[u] - fr.minx) * fr.invw);   // PosInGrid (Frame.cc:725-735)
        const int py = (int)roundf((ky[u] - fr.miny) * fr.invh);
        const uint32_t rank = ((uint32_t)(px * ORBFE_GRID_ROWS + py) << 13) | (uint32_t)idx;
        s_kp[p] = make_float4(kx[u], ky[u], __uint_as_float(rank), rur[u]);
        s_desc[2 * p] = rd0[u];
        s_desc[2 * p + 1] = rd1[u];
    }
    SYNC();
}
// A query's gate-independent candidates: the MT_BLK_LIST smallest keys, sorted, packed as
// idx | octave << 13 | dist << 16 (0xFFFFFFFF: none); returns the candidate count
template <int MODE, int LEN = MT_BLK_LIST>
__device__ __forceinline__ int blk_list(const BlkQuery& Q, const BlkGeom& gm, const float4* kp, const uint4* desc,
                                        const int* be, const uint8_t* blk, uint32_t (&L)[LEN], int cbase = 0,
                                        int* nwin = nullptr) {
    unsigned long long K[LEN];
#pragma unroll
    for (int k = 0; k < LEN; k++) K[k] = ~0ull;
    int c = 0;
    blk_enum<MODE>(Q, gm, kp, desc, be, blk, [&](unsigned long long key, int) {
        c++;
        if (key >= K[LEN - 1]) return;   // not among the LEN smallest so far (keys are unique)
#pragma unroll
        for (int k = 0; k < LEN; k++) {   // sorted insertion (a compare-swap chain)
            const bool lt = key < K[k];
            const unsigned long long t = K[k];
            K[k] = lt ? key : t;
            key = lt ? t : key;
        }
    }, cbase, nwin);
#pragma unroll
    for (int k = 0; k < LEN; k++)
        L[k] = K[k] == ~0ull ? 0xFFFFFFFFu
                             : (uint32_t)((K[k] >> 4) & 0x1FFFu) | (uint32_t)((K[k] & 15) << 13) |
                                   (uint32_t)((K[k] >> 40) << 16);
    return c;
}
template <int MODE>
__global__ __launch_bounds__(MT_BLK_NT) void k_sbp_block(FrameDev fr, BlkGeom gm, const void* recs, int nq, float th,
                                                         int a0, int a1, float thFar, float nnratio, int maxDist,
                                                         int need_obs, BlkIO io) {
    extern __shared__ __attribute__((aligned(16))) uint8_t mt_sm[];
    const int n = fr.n;
    const int nlev = fr.nlevels;
    const int nbk = nlev * gm.NB * gm.NS;
    float4* s_kp = (float4*)mt_sm;                 // {x, y, rank bits, uR} per bucket position
    uint4* s_desc = (uint4*)(s_kp + n);            // 2 x uint4 per bucket position
    int* s_ber = (int*)(s_desc + 2 * n);           // bucket bounds region (blk_be_words)
    const int* s_be = s_ber + 3;                   // be[c] = start of bucket c, be[c + 1] = its end
    int* s_first = s_ber + blk_be_words(nbk, MT_BLK_NT);   // two first[] states by keypoint index (then the commit's slots)
    float* s_ang = (float*)(s_first + 2 * n);      // keypoint angles by index (the rotation check)
    uint8_t* s_blk = (uint8_t*)(s_ang + n);        // blocked initially, by keypoint index
    __shared__ int s_flag, s_ws[MT_BLK_NT / 64], s_hist[MT_HISTO], s_cnt[2];
    __shared__ unsigned s_keep;
    const int tid = threadIdx.x;
    // pass-independent part, once: each query's gate-independent candidates, the MT_BLK_LIST smallest
    // keys sorted (registers) and their count; a pass then only walks the list past the keypoints
    // that earlier queries hold (first[idx] < q). A query whose list runs out while more candidates
    // exist re-enumerates its window with the pass's gates (exact, rare).
    uint32_t L[MT_BLK_QPT][MT_BLK_LIST];
    int cnt[MT_BLK_QPT], obs[MT_BLK_QPT], res[MT_BLK_QPT], qid[MT_BLK_QPT];
    float qang[MT_BLK_QPT];
    unsigned long long npair = 0;
    // every record of the thread read first, before the frame is staged (the two memory round trips
    // overlap: from host memory they are ~7 us each), with the fields the commit needs
    BlkQuery QS[MT_BLK_QPT];
#pragma unroll
    for (int i = 0; i < MT_BLK_QPT; i++) {
        cnt[i] = 0;
        res[i] = -1;
        qid[i] = -1;
        qang[i] = 0.f;
        QS[i].ok = false;
        QS[i].obs = 0;
        const int q = tid + i * MT_BLK_NT;
        if (q >= nq) continue;
        const uint8_t* rec = (const uint8_t*)recs + (size_t)q * io.q_stride;
        qid[i] = *(const int*)(rec + io.qid_off);
        if (io.checkOri) qang[i] = *(const float*)(rec + io.qangle_off);
        QS[i] = blk_load<MODE>(fr, recs, q, th, a0, a1, thFar);
    }
    if (tid < MT_HISTO) s_hist[tid] = 0;
    if (tid < 2) s_cnt[tid] = 0;
    const void* rq = blk_qcopy(io, recs, nq);
    blk_stage<MT_BLK_NT>(fr, gm, io.mvp_in, io.obs_in, s_kp, s_desc, s_ber, s_blk, s_ang, s_first, s_ws);
#pragma unroll
    for (int i = 0; i < MT_BLK_QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        obs[i] = QS[i].obs;
#pragma unroll
        for (int k = 0; k < MT_BLK_LIST; k++) L[i][k] = 0xFFFFFFFFu;
        if (q >= nq) continue;
        const int c = blk_list<MODE>(QS[i], gm, s_kp, s_desc, s_be, s_blk, L[i]);
        npair += (unsigned)c;
        cnt[i] = c;
    }
    int pass = 0;
    for (;; pass++) {
        const int* fcur = s_first + (pass & 1) * n;
        int* fnext = s_first + ((pass + 1) & 1) * n;
        for (int k = tid; k < n; k += MT_BLK_NT) fnext[k] = MT_INF;
        if (tid == 0) s_flag = 0;
        SYNC();
        bool ch = false;
#pragma unroll
        for (int i = 0; i < MT_BLK_QPT; i++) {
            const int q = tid + i * MT_BLK_NT;
            if (q >= nq) continue;   // (not break: the loop must unroll so the per-slot arrays stay in registers)
            // the first (and, MODE 0, second) list entries that no earlier query holds
            // (the eight gate reads issued together, the selection in registers)
            bool free_[MT_BLK_LIST];
#pragma unroll
            for (int k = 0; k < MT_BLK_LIST; k++)
                free_[k] = L[i][k] != 0xFFFFFFFFu && fcur[L[i][k] & 0x1FFFu] >= q;
            uint32_t e1 = 0xFFFFFFFFu, e2 = 0xFFFFFFFFu;
            int found = 0;
#pragma unroll
            for (int k = 0; k < MT_BLK_LIST; k++) {
                if (!free_[k] || found >= (MODE == 0 ? 2 : 1)) continue;
                if (found == 0) e1 = L[i][k];
                else e2 = L[i][k];
                found++;
            }
            int result;
            if (found < (MODE == 0 ? 2 : 1) && cnt[i] > MT_BLK_LIST) {
                // the list ran out: the window again, with this pass's gates
                const BlkQuery Q = blk_load<MODE>(fr, rq, q, th, a0, a1, thFar);
                unsigned long long k1 = ~0ull, k2 = ~0ull;
                blk_enum<MODE>(Q, gm, s_kp, s_desc, s_be, s_blk, [&](unsigned long long key, int idx) {
                    if (fcur[idx] < q) return;
                    const bool lt1 = key < k1, lt2 = key < k2;   // selects, not a store through a chosen pointer
                    k2 = lt1 ? k1 : (lt2 ? key : k2);
                    k1 = lt1 ? key : k1;
                });
                result = blk_accept<MODE>(k1 != ~0ull ? (int)((k1 >> 4) & 0x1FFFu) : -1, (int)(k1 >> 40),
                                          (int)(k1 & 15), k2 != ~0ull ? (int)(k2 >> 40) : 256,
                                          k2 != ~0ull ? (int)(k2 & 15) : -1, nnratio, maxDist);
            } else {
                result = blk_accept<MODE>(e1 != 0xFFFFFFFFu ? (int)(e1 & 0x1FFFu) : -1, (int)(e1 >> 16),
                                          (int)((e1 >> 13) & 7), e2 != 0xFFFFFFFFu ? (int)(e2 >> 16) : 256,
                                          e2 != 0xFFFFFFFFu ? (int)((e2 >> 13) & 7) : -1, nnratio, maxDist);
            }
            if (result >= 0 && (!need_obs || obs[i] > 0)) atomicMin(&fnext[result], q);
            if (result != res[i]) {
                res[i] = result;
                ch = true;
            }
        }
        if (__ballot(ch) && (tid & 63) == 0) s_flag = 1;
        SYNC();
        // after pass t the first t queries are final, so at most nq + 1 passes change anything
        if (s_flag == 0 || pass > nq) break;
    }
    // ---- the commit (k_mt_commit_count / _drop / _write in one block): the last writer of a slot
    // wins, every assignment enters the rotation histogram, ComputeThreeMaxima's dropped bins clear
    // their slots and count once per entry (ORBmatcher.cc:1775-1792,1864-1884) ----
    int* s_res = s_first;   // the pass states are dead
    for (int k = tid; k < n; k += MT_BLK_NT) s_res[k] = -1;
    SYNC();
    int nas = 0;
    int bins[MT_BLK_QPT];
#pragma unroll
    for (int i = 0; i < MT_BLK_QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        bins[i] = -1;
        if (q >= nq || res[i] < 0) continue;
        atomicMax(&s_res[res[i]], q);
        nas++;
        if (io.checkOri) bins[i] = mt_rot_bin(qang[i], s_ang[res[i]]);
    }
    // per-wave counts, one LDS atomic per wave and distinct bin (the assignments of a frame fall in
    // a few bins: same-address atomics from every lane serialise)
    nas = wave_sum_dpp(nas);
    if ((tid & 63) == 0 && nas) atomicAdd(&s_cnt[0], nas);
    if (io.checkOri) {
#pragma unroll
        for (int i = 0; i < MT_BLK_QPT; i++) {
            int b = bins[i];
            for (unsigned long long act = __ballot(b >= 0); act; act = __ballot(b >= 0)) {
                const int lead = __builtin_amdgcn_readlane(b, (int)__builtin_ctzll(act));
                const unsigned long long same = __ballot(b == lead);
                if ((tid & 63) == (int)__builtin_ctzll(same)) atomicAdd(&s_hist[lead], (int)__popcll(same));
                if (b == lead) b = -1;
            }
        }
    }
    SYNC();
    if (tid == 0) s_keep = io.checkOri ? mt_three_maxima_keep(s_hist) : 0xFFFFFFFFu;
    SYNC();
    int ndrop = 0;
#pragma unroll
    for (int i = 0; i < MT_BLK_QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        if (q >= nq || res[i] < 0 || bins[i] < 0 || ((s_keep >> bins[i]) & 1u)) continue;
        s_res[res[i]] = -2;
        io.mvp_out[res[i]] = -1;
        ndrop++;
    }
    ndrop = wave_sum_dpp(ndrop);
    if ((tid & 63) == 0 && ndrop) atomicAdd(&s_cnt[1], ndrop);
    SYNC();
    // the last writer of each slot that no dropped entry cleared stores its record's id
#pragma unroll
    for (int i = 0; i < MT_BLK_QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        if (q < nq && res[i] >= 0 && s_res[res[i]] == q) io.mvp_out[res[i]] = qid[i];
    }
    if (io.stats && npair) {
        atomicAdd(&io.stats[0], npair);
        atomicAdd(&io.stats[1], npair);
    }
    // every wave's slot writes complete (vmcnt 0), the barrier, then ONE system-scope release before the
    // status words (MI355X_MICROARCH.md, correctness boundaries): a release per thread wrote back the
    // L2 sixteen times and cost more than the search
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (tid == 0) {
        __threadfence_system();
        if (io.stats) io.stats[2] = (unsigned long long)(pass + 1);
        volatile int* st = io.st_host;
        st[0] = 0;
        st[1] = s_cnt[0];
        st[2] = s_cnt[1];
        st[3] = pass + 1;
        st[5] = io.ntm ? *io.ntm : 0;
        __threadfence_system();
        st[4] = io.seq;
        __threadfence_system();
    }
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) for a two-camera frame (Nleft != -1,
// ORBmatcher.cc:1695-1858) in ONE workgroup, k_sbp_block's design with two entries per point: entry
// 2 q = the best left keypoint of point q's window (left grid), entry 2 q + 1 = the best right keypoint
// around the caller's right-camera projection right_uv[q] (right grid), searched only when the left
// window holds any keypoint (:1740-1741, blocked ones included). Both cameras' keypoints are staged in
// LDS (two bucket sets); an entry's gate is first[k] < entry (the slot was written by an earlier entry
// of a point with Observations() > 0: such a write is never overwritten, so the earliest one is the
// one that blocks). Each entry keeps its MT_BLK2_LIST smallest gate-independent keys in registers;
// the fixed point, the last-writer commit and the rotation histogram over all entries
// (:1860-1884) run in the block as in k_sbp_block<1>. Up to MT_BLOCK_MAXQ points: two per thread,
// four entries.
#ifndef MT_BLK2_LIST
#define MT_BLK2_LIST 8
#endif
#ifdef ORBFE_BLK2_STAMPS   // diagnostic build (tools/build_variant.sh): phase times of thread 0, printed
#define BLK2_STAMP(k) do { if (threadIdx.x == 0) t_st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BLK2_STAMP(k) do { } while (0)
#endif
__global__ __launch_bounds__(MT_BLK_NT) void k_sbp_block2(FrameDev fr, BlkGeom gm, const orbfe_proj_point* recs,
                                                          const float2* right_uv, int nq, float th, int a0, int a1,
                                                          int maxDist, BlkIO io) {
    extern __shared__ __attribute__((aligned(16))) uint8_t mt_sm[];
    const int n = fr.n;
    const int nbk1 = fr.nlevels * gm.NB * gm.NS;   // buckets of one camera
    float4* s_kp = (float4*)mt_sm;
    uint4* s_desc = (uint4*)(s_kp + n);
    int* s_ber = (int*)(s_desc + 2 * n);
    const int* s_be = s_ber + 3;
    int* s_first = s_ber + blk_be_words(2 * nbk1, MT_BLK_NT);
    float* s_ang = (float*)(s_first + 2 * n);
    uint8_t* s_blk = (uint8_t*)(s_ang + n);
    __shared__ int s_flag, s_ws[MT_BLK_NT / 64], s_hist[MT_HISTO], s_cnt[2];
    __shared__ unsigned s_keep;
    const int tid = threadIdx.x;
#ifdef ORBFE_BLK2_STAMPS
    unsigned long long t_st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    BLK2_STAMP(0);
    constexpr int QPT = MT_BLK_QPT, EPT = 2 * MT_BLK_QPT;   // points / entries per thread (entry j: point j / 2, side j & 1)
    uint32_t L[EPT][MT_BLK2_LIST];
    int cnt[EPT], res[EPT];
    int obs[QPT], qid[QPT];
    float qang[QPT];
    unsigned long long npair = 0;
    BlkQuery QS[QPT];
    float2 uv[QPT];
#pragma unroll
    for (int i = 0; i < QPT; i++) {
        qid[i] = -1;
        qang[i] = 0.f;
        uv[i] = make_float2(0.f, 0.f);
        QS[i].ok = false;
        QS[i].obs = 0;
        const int q = tid + i * MT_BLK_NT;
        if (q >= nq) continue;
        uv[i] = right_uv[q];
    }
    if (tid < MT_HISTO) s_hist[tid] = 0;
    if (tid < 2) s_cnt[tid] = 0;
    BLK2_STAMP(1);
    // the records cross PCIe once, into HBM (their loads in flight during the staging); the points'
    // windows are read from that copy after the staging's barriers
    const orbfe_proj_point* rq = (const orbfe_proj_point*)blk_qcopy(io, recs, nq);
    blk_stage<MT_BLK_NT>(fr, gm, io.mvp_in, io.obs_in, s_kp, s_desc, s_ber, s_blk, s_ang, s_first, s_ws, 2);
    BLK2_STAMP(2);
#pragma unroll
    for (int i = 0; i < QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        if (q >= nq) continue;
        const uint8_t* rec = (const uint8_t*)rq + (size_t)q * io.q_stride;
        qid[i] = *(const int*)(rec + io.qid_off);
        if (io.checkOri) qang[i] = *(const float*)(rec + io.qangle_off);
        QS[i] = blk_load<1>(fr, rq, q, th, a0, a1, 0.f);
    }
#pragma unroll
    for (int i = 0; i < QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        obs[i] = QS[i].obs;
#pragma unroll
        for (int sd = 0; sd < 2; sd++) {
            cnt[2 * i + sd] = 0;
#pragma unroll
            for (int k = 0; k < MT_BLK2_LIST; k++) L[2 * i + sd][k] = 0xFFFFFFFFu;
        }
        if (q >= nq) continue;
        int nwin = 0;
        cnt[2 * i] = blk_list<3, MT_BLK2_LIST>(QS[i], gm, s_kp, s_desc, s_be, s_blk, L[2 * i], 0, &nwin);
        if (nwin > 0) {   // the right camera only after a non-empty left window
            BlkQuery QR = QS[i];
            QR.x = uv[i].x;
            QR.y = uv[i].y;
            cnt[2 * i + 1] = blk_list<3, MT_BLK2_LIST>(QR, gm, s_kp, s_desc, s_be, s_blk, L[2 * i + 1], nbk1);
        }
        npair += (unsigned)(cnt[2 * i] + cnt[2 * i + 1]);
    }
#pragma unroll
    for (int j = 0; j < EPT; j++) res[j] = -1;
    SYNC();
    BLK2_STAMP(3);
    int pass = 0;
    for (;; pass++) {
        const int* fcur = s_first + (pass & 1) * n;
        int* fnext = s_first + ((pass + 1) & 1) * n;
        for (int k = tid; k < n; k += MT_BLK_NT) fnext[k] = MT_INF;
        if (tid == 0) s_flag = 0;
        SYNC();
        bool ch = false;
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            const int i = j >> 1, sd = j & 1;
            const int q = tid + i * MT_BLK_NT;
            if (q >= nq) continue;
            const int e = 2 * q + sd;
            // the first list entry no earlier entry holds (the gate reads issued together)
            bool free_[MT_BLK2_LIST];
#pragma unroll
            for (int k = 0; k < MT_BLK2_LIST; k++)
                free_[k] = L[j][k] != 0xFFFFFFFFu && fcur[L[j][k] & 0x1FFFu] >= e;
            uint32_t e1 = 0xFFFFFFFFu;
#pragma unroll
            for (int k = MT_BLK2_LIST - 1; k >= 0; k--)
                if (free_[k]) e1 = L[j][k];
            int result;
            if (e1 == 0xFFFFFFFFu && cnt[j] > MT_BLK2_LIST) {
                // the list ran out: the window again, with this pass's gates (the smallest key = the
                // first strict minimum in GetFeaturesInArea order)
                BlkQuery Q = blk_load<1>(fr, rq, q, th, a0, a1, 0.f);
                if (sd) {
                    const float2 u = right_uv[q];
                    Q.x = u.x;
                    Q.y = u.y;
                }
                unsigned long long k1 = ~0ull;
                blk_enum<3>(Q, gm, s_kp, s_desc, s_be, s_blk, [&](unsigned long long key, int idx) {
                    if (fcur[idx] < e) return;
                    k1 = key < k1 ? key : k1;
                }, sd ? nbk1 : 0);
                result = blk_accept<1>(k1 != ~0ull ? (int)((k1 >> 4) & 0x1FFFu) : -1, (int)(k1 >> 40), 0, 256, -1,
                                       0.f, maxDist);
            } else {
                result = blk_accept<1>(e1 != 0xFFFFFFFFu ? (int)(e1 & 0x1FFFu) : -1, (int)(e1 >> 16), 0, 256, -1, 0.f,
                                       maxDist);
            }
            if (result >= 0 && obs[i] > 0) atomicMin(&fnext[result], e);
            if (result != res[j]) {
                res[j] = result;
                ch = true;
            }
        }
        if (__ballot(ch) && (tid & 63) == 0) s_flag = 1;
        SYNC();
        if (s_flag == 0 || pass > 2 * nq) break;
    }
    BLK2_STAMP(4);
    // ---- the commit: the last entry writing a slot wins, every assignment enters the rotation
    // histogram, the dropped bins clear their slots and count once per entry ----
    int* s_res = s_first;
    for (int k = tid; k < n; k += MT_BLK_NT) s_res[k] = -1;
    SYNC();
    int nas = 0;
    int bins[EPT];
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int i = j >> 1, q = tid + i * MT_BLK_NT;
        bins[j] = -1;
        if (q >= nq || res[j] < 0) continue;
        atomicMax(&s_res[res[j]], 2 * q + (j & 1));
        nas++;
        if (io.checkOri) bins[j] = mt_rot_bin(qang[i], s_ang[res[j]]);
    }
    nas = wave_sum_dpp(nas);
    if ((tid & 63) == 0 && nas) atomicAdd(&s_cnt[0], nas);
    if (io.checkOri) {
#pragma unroll
        for (int j = 0; j < EPT; j++) {
            int b = bins[j];
            for (unsigned long long act = __ballot(b >= 0); act; act = __ballot(b >= 0)) {
                const int lead = __builtin_amdgcn_readlane(b, (int)__builtin_ctzll(act));
                const unsigned long long same = __ballot(b == lead);
                if ((tid & 63) == (int)__builtin_ctzll(same)) atomicAdd(&s_hist[lead], (int)__popcll(same));
                if (b == lead) b = -1;
            }
        }
    }
    SYNC();
    if (tid == 0) s_keep = io.checkOri ? mt_three_maxima_keep(s_hist) : 0xFFFFFFFFu;
    SYNC();
    int ndrop = 0;
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int q = tid + (j >> 1) * MT_BLK_NT;
        if (q >= nq || res[j] < 0 || bins[j] < 0 || ((s_keep >> bins[j]) & 1u)) continue;
        s_res[res[j]] = -2;
        io.mvp_out[res[j]] = -1;
        ndrop++;
    }
    ndrop = wave_sum_dpp(ndrop);
    if ((tid & 63) == 0 && ndrop) atomicAdd(&s_cnt[1], ndrop);
    SYNC();
#pragma unroll
    for (int j = 0; j < EPT; j++) {
        const int i = j >> 1, q = tid + i * MT_BLK_NT;
        if (q < nq && res[j] >= 0 && s_res[res[j]] == 2 * q + (j & 1)) io.mvp_out[res[j]] = qid[i];
    }
    if (io.stats && npair) {
        atomicAdd(&io.stats[0], npair);
        atomicAdd(&io.stats[1], npair);
    }
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (tid == 0) {
        __threadfence_system();
        if (io.stats) io.stats[2] = (unsigned long long)(pass + 1);
        volatile int* st = io.st_host;
        st[0] = 0;
        st[1] = s_cnt[0];
        st[2] = s_cnt[1];
        st[3] = pass + 1;
        st[5] = 0;
        __threadfence_system();
        st[4] = io.seq;
        __threadfence_system();
    }
#ifdef ORBFE_BLK2_STAMPS
    BLK2_STAMP(5);
    if (tid == 0)   // s_memrealtime ticks at 100 MHz
        printf("blk2 nq %d n %d passes %d  load %.1f stage %.1f lists %.1f passes %.1f commit %.1f us\n", nq, n, pass + 1,
               (t_st[1] - t_st[0]) * 0.01, (t_st[2] - t_st[1]) * 0.01, (t_st[3] - t_st[2]) * 0.01,
               (t_st[4] - t_st[3]) * 0.01, (t_st[5] - t_st[4]) * 0.01);
#endif
}

// SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints) for a two-camera frame (Nleft != -1,
// ORBmatcher.cc:43-213; the per-frame SearchLocalPoints call of a KannalaBrandt8 rig) in ONE
// workgroup. Point q writes up to four slots in the reference's order: entry 4 q = the left best,
// 4 q + 1 = its right partner (mvLeftToRightMatch, written without a check), 4 q + 2 = the right best's
// left partner (mvRightToLeftMatch), 4 q + 3 = the right best; a failed left ratio test skips the right
// search (:124-125). A keypoint is taken for point q when the LAST write to its slot before entry 4 q
// holds a point with Observations() > 0 (no write: the slot's holder before the search); the right
// search sees the point's own partner write as the latest (:158-160). Partner writes are unguarded, so a
// slot's writers are kept per pass: every slot's writer entries (<= MT_B4_WCAP, tagged with their
// point's Observations() > 0) in LDS, rebuilt from the previous pass's results at the start of each
// pass; more writers than that abort the search (status 2) and the caller runs the multi-launch form.
// Each search keeps its MT_BLK_LIST smallest gate-independent keys; the last writer of each slot wins
// (no rotation check in this search), nmatches counts every write (:130-137,196-204).
#define MT_B4_WCAP 6
#define MT_B4_LIST 4   // keys kept per search (registers: two searches per point, two points per thread)
__host__ __device__ constexpr int blk4_bytes_per_kp() { return 16 + 32 + 4 + 2 * MT_B4_WCAP + 2 + 1; }
__device__ __forceinline__ bool b4_taken(const uint16_t* wl, const int* wcnt, const uint8_t* blk0, int k, int e) {
    const int c = min(wcnt[k], MT_B4_WCAP);
    int last = -1;
    for (int j = 0; j < c; j++) {
        const int w = wl[k * MT_B4_WCAP + j];
        if ((w >> 1) < e && w > last) last = w;
    }
    return last < 0 ? blk0[k] != 0 : (last & 1) != 0;
}
// the right-camera search of a point (its record's IN_VIEW_R fields, radius not scaled by th)
__device__ __forceinline__ BlkQuery b4_right(const FrameDev& fr, const orbfe_map_point& mp, int bFar, float thFar) {
    BlkQuery Q;
    Q.x = Q.y = Q.R = Q.xr = 0.f;
    Q.olo = 0;
    Q.ohi = -1;
    Q.obs = mp.observations;
    const int lvl = mp.scale_level_r;
    Q.ok = (mp.flags & ORBFE_MP_IN_VIEW_R) && !(bFar && mp.depth > thFar) && !(mp.flags & ORBFE_MP_BAD) &&
           lvl != -1 && lvl >= 0 && lvl < fr.nlevels;
    if (Q.ok) {
        Q.R = (mp.view_cos_r > 0.998 ? 2.5f : 4.0f) * fr.scale[lvl];   // RadiusByViewingCos, :143-147
        Q.x = mp.proj_xr;
        Q.y = mp.proj_yr;
        Q.olo = max(lvl - 1, 0);
        Q.ohi = lvl;
        memcpy(Q.qd, mp.desc, 32);
    }
    return Q;
}
__global__ __launch_bounds__(MT_BLK_NT) void k_sbp_block4(FrameDev fr, BlkGeom gm, const orbfe_map_point* recs, int nq,
                                                          float th, int bFar, float thFar, float nnratio, BlkIO io) {
    extern __shared__ __attribute__((aligned(16))) uint8_t mt_sm[];
    const int n = fr.n, nl = fr.nleft;
    const int nbk1 = fr.nlevels * gm.NB * gm.NS;
    float4* s_kp = (float4*)mt_sm;
    uint4* s_desc = (uint4*)(s_kp + n);
    int* s_ber = (int*)(s_desc + 2 * n);
    const int* s_be = s_ber + 3;
    int* s_wcnt = s_ber + blk_be_words(2 * nbk1, MT_BLK_NT);                  // writers per slot (this pass)
    uint16_t* s_wl = (uint16_t*)(s_wcnt + n);                                  // their entries << 1 | Observations() > 0
    int16_t* s_link = (int16_t*)(s_wl + (size_t)MT_B4_WCAP * n);              // l2r (left) / r2l (right) partner
    uint8_t* s_blk = (uint8_t*)(s_link + n);                                   // held before the search
    __shared__ int s_flag, s_ovf, s_ws[MT_BLK_NT / 64], s_cnt;
    const int tid = threadIdx.x;
    constexpr int QPT = MT_BLK_QPT;
    uint32_t L[2 * QPT][MT_B4_LIST];   // [2 i]: point i's left list, [2 i + 1]: its right list
    int cnt[2 * QPT], res[QPT][4];
    int obs[QPT];
    bool gl[QPT], gr[QPT];              // the left / right search runs (record flags)
    unsigned long long npair = 0;
    if (tid == 0) { s_cnt = 0; s_ovf = 0; }
    const orbfe_map_point* rq = (const orbfe_map_point*)blk_qcopy(io, recs, nq);
    blk_stage<MT_BLK_NT>(fr, gm, io.mvp_in, io.obs_in, s_kp, s_desc, s_ber, s_blk, nullptr, nullptr, s_ws, 2);
    for (int k = tid; k < n; k += MT_BLK_NT) {
        int p = k < nl ? fr.l2r[k] : fr.r2l[k - nl];
        if (k < nl ? !(p >= 0 && nl + p < n) : !(p >= 0 && p < nl)) p = -1;   // range-guarded links
        s_link[k] = (int16_t)(p < 0 ? -1 : (k < nl ? nl + p : p));
    }
#pragma unroll
    for (int i = 0; i < QPT; i++) {
        const int q = tid + i * MT_BLK_NT;
        obs[i] = 0;
        gl[i] = gr[i] = false;
#pragma unroll
        for (int b = 0; b < 4; b++) res[i][b] = -1;
#pragma unroll
        for (int sd = 0; sd < 2; sd++) {
            cnt[2 * i + sd] = 0;
#pragma unroll
            for (int k = 0; k < MT_B4_LIST; k++) L[2 * i + sd][k] = 0xFFFFFFFFu;
        }
        if (q >= nq) continue;
        const orbfe_map_point& mp = rq[q];
        obs[i] = mp.observations;
        const BlkQuery QL = blk_load<0>(fr, rq, q, th, bFar, 0, thFar);   // mbTrackInView, th-scaled radius
        const BlkQuery QR = b4_right(fr, mp, bFar, thFar);
        gl[i] = QL.ok;
        gr[i] = QR.ok;
        cnt[2 * i] = blk_list<4, MT_B4_LIST>(QL, gm, s_kp, s_desc, s_be, s_blk, L[2 * i]);
        cnt[2 * i + 1] = blk_list<4, MT_B4_LIST>(QR, gm, s_kp, s_desc, s_be, s_blk, L[2 * i + 1], nbk1);
        npair += (unsigned)(cnt[2 * i] + cnt[2 * i + 1]);
    }
    int pass = 0;
    for (;; pass++) {
        // the slots' writers, from the previous pass's results (none in pass 0)
        for (int k = tid; k < n; k += MT_BLK_NT) s_wcnt[k] = 0;
        if (tid == 0) s_flag = 0;
        SYNC();
        bool ovf = false;
#pragma unroll
        for (int i = 0; i < QPT; i++) {
            const int q = tid + i * MT_BLK_NT;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int k = res[i][b];
                if (k < 0) continue;
                const int pos = atomicAdd(&s_wcnt[k], 1);
                if (pos < MT_B4_WCAP) s_wl[k * MT_B4_WCAP + pos] = (uint16_t)(((4 * q + b) << 1) | (obs[i] > 0 ? 1 : 0));
                else ovf = true;
            }
        }
        if (__ballot(ovf) && (tid & 63) == 0) s_ovf = 1;
        SYNC();
        if (s_ovf) break;
        bool ch = false;
#pragma unroll
        for (int i = 0; i < QPT; i++) {
            const int q = tid + i * MT_BLK_NT;
            if (q >= nq) continue;
            const int e0 = 4 * q;
            int r[4] = {-1, -1, -1, -1};
            bool go = true;
#pragma unroll
            for (int sd = 0; sd < 2; sd++) {
                const int j = 2 * i + sd;
                if (!(sd ? (go && gr[i]) : gl[i])) continue;
                const int own = r[1];   // the right search sees this point's own partner write
                auto taken = [&](int k) {
                    return (sd && k == own) ? obs[i] > 0 : b4_taken(s_wl, s_wcnt, s_blk, k, e0);
                };
                bool free_[MT_B4_LIST];
#pragma unroll
                for (int k = 0; k < MT_B4_LIST; k++) free_[k] = L[j][k] != 0xFFFFFFFFu && !taken((int)(L[j][k] & 0x1FFFu));
                uint32_t e1 = 0xFFFFFFFFu, e2 = 0xFFFFFFFFu;
                int found = 0;
#pragma unroll
                for (int k = 0; k < MT_B4_LIST; k++) {
                    if (!free_[k] || found >= 2) continue;
                    if (found == 0) e1 = L[j][k];
                    else e2 = L[j][k];
                    found++;
                }
                int bi = -1, bd = 256, bl = -1, bd2 = 256, bl2 = -1;
                if (found < 2 && cnt[j] > MT_B4_LIST) {
                    // the list ran out: the window again, with this pass's gates
                    const BlkQuery Q = sd ? b4_right(fr, rq[q], bFar, thFar) : blk_load<0>(fr, rq, q, th, bFar, 0, thFar);
                    unsigned long long k1 = ~0ull, k2 = ~0ull;
                    blk_enum<4>(Q, gm, s_kp, s_desc, s_be, s_blk, [&](unsigned long long key, int idx) {
                        if (taken(idx)) return;
                        const bool lt1 = key < k1, lt2 = key < k2;
                        k2 = lt1 ? k1 : (lt2 ? key : k2);
                        k1 = lt1 ? key : k1;
                    }, sd ? nbk1 : 0);
                    if (k1 != ~0ull) { bi = (int)((k1 >> 4) & 0x1FFFu); bd = (int)(k1 >> 40); bl = (int)(k1 & 15); }
                    if (k2 != ~0ull) { bd2 = (int)(k2 >> 40); bl2 = (int)(k2 & 15); }
                } else {
                    if (e1 != 0xFFFFFFFFu) { bi = (int)(e1 & 0x1FFFu); bd = (int)(e1 >> 16); bl = (int)((e1 >> 13) & 7); }
                    if (e2 != 0xFFFFFFFFu) { bd2 = (int)(e2 >> 16); bl2 = (int)((e2 >> 13) & 7); }
                }
                if (bi < 0 || bd > MT_TH_HIGH) continue;
                if (bl == bl2 && bd > nnratio * bd2) {   // :124-125 / :190-191: `continue` to the next point
                    go = false;
                    continue;
                }
                const int p = s_link[bi];
                if (sd == 0) { r[0] = bi; r[1] = p; }
                else { r[2] = p; r[3] = bi; }
            }
#pragma unroll
            for (int b = 0; b < 4; b++) {
                if (r[b] != res[i][b]) ch = true;
                res[i][b] = r[b];
            }
        }
        if (__ballot(ch) && (tid & 63) == 0) s_flag = 1;
        SYNC();
        // after pass t the first t points are final
        if (s_flag == 0 || pass > nq) break;
    }
    const bool aborted = s_ovf != 0;
    // ---- the commit: the last entry writing a slot wins; nmatches counts every write ----
    int* s_res = s_wcnt;
    for (int k = tid; k < n; k += MT_BLK_NT) s_res[k] = -1;
    SYNC();
    int nas = 0;
    if (!aborted) {
#pragma unroll
        for (int i = 0; i < QPT; i++) {
            const int q = tid + i * MT_BLK_NT;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                if (q >= nq || res[i][b] < 0) continue;
                atomicMax(&s_res[res[i][b]], 4 * q + b);
                nas++;
            }
        }
    }
    nas = wave_sum_dpp(nas);
    if ((tid & 63) == 0 && nas) atomicAdd(&s_cnt, nas);
    SYNC();
    if (!aborted)
#pragma unroll
        for (int i = 0; i < QPT; i++) {
            const int q = tid + i * MT_BLK_NT;
#pragma unroll
            for (int b = 0; b < 4; b++)
                if (q < nq && res[i][b] >= 0 && s_res[res[i][b]] == 4 * q + b) io.mvp_out[res[i][b]] = rq[q].id;
        }
    if (io.stats && npair) {
        atomicAdd(&io.stats[0], npair);
        atomicAdd(&io.stats[1], npair);
    }
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (tid == 0) {
        __threadfence_system();
        if (io.stats) io.stats[2] = (unsigned long long)(pass + 1);
        volatile int* st = io.st_host;
        st[0] = aborted ? 2 : 0;
        st[1] = s_cnt;
        st[2] = 0;
        st[3] = pass + 1;
        st[5] = io.ntm ? *io.ntm : 0;
        __threadfence_system();
        st[4] = io.seq;
        __threadfence_system();
    }
}

// ---- Large single-camera local-map searches (nq > MT_BLOCK_MAXQ, frame in LDS): k_sbp_block's design
// over many workgroups. Pass 0 (k_sbp_multi0, one query per thread, every block stages the frame in
// LDS) enumerates each query's window ONCE and keeps its MT_BLK_LIST smallest keys in memory, with
// the queries that have any candidate in an active list; a later pass (k_sbp_multi) walks only the
// active queries' lists past the keypoints earlier queries hold (a list that runs out re-enumerates
// the window over block 0's copy of the LDS frame in memory: exact, rare) and needs no frame at all.
// The first[] states, last writers and change flags carry the pass's generation (a per-call base +
// the pass), so nothing is cleared between passes or calls. The last block of a pass to finish
// commits when the pass changed nothing (slot writes, status words) and otherwise reports "not
// converged" when it ends the host's batch.
struct MultiIO {
    const int32_t* mvp_in;     // slots before the search (device)
    const int32_t* obs_in;     // Observations() per slot
    int32_t* mvp_out;          // slots after the search (device; may alias mvp_in)
    int q_stride, qid_off;
    const int* ntm;            // k_frustum's nToMatch (nullptr: none)
    int* assign;               // [nq] result of the latest pass that ran the query
    uint32_t* lists;           // [nq][MT_BLK_LIST]
    int* lcnt;                 // [nq] candidate count | (Observations() > 0) << 31
    int* active;               // queries with candidates
    int* nactive;
    unsigned long long* first[2];   // generation-tagged first[] states (pass parity)
    unsigned long long* lastw;      // generation-tagged last assigner per slot
    unsigned long long* changed;    // [MT_MAX_PASSES] generation of a pass that changed something
    int* done;                 // [MT_MAX_PASSES] finished blocks (reset by the last one)
    int* cnt;                  // [MT_MAX_PASSES] assigned queries (reset by the last block)
    float4* g_kp;              // block 0's LDS frame, for the re-enumerations
    uint4* g_desc;
    int* g_be;
    uint8_t* g_blk;
    int* st_host;
    int seq;
    unsigned long long gen0;   // generation of pass 0
    unsigned long long* stats;
};
// first[]: gen << 24 | (2^24 - 1 - q), atomicMax keeps the newest generation's smallest query; an
// entry of another generation reads as free (MT_INF). Last writer: gen << 24 | q.
__device__ __forceinline__ unsigned long long mt_ftag(unsigned long long gen, int q) {
    return (gen << 24) | (unsigned long long)(0xFFFFFF - q);
}
__device__ __forceinline__ int mt_fget(unsigned long long v, unsigned long long gen) {
    return (v >> 24) == gen ? 0xFFFFFF - (int)(v & 0xFFFFFFull) : MT_INF;
}
__device__ __forceinline__ void multi_publish(const MultiIO& io, unsigned long long* fnext, unsigned long long gen,
                                              int q, int result, bool hasobs) {
    if (hasobs) {
        const unsigned long long t = mt_ftag(gen + 1, q);
        if (t > __atomic_load_n(&fnext[result], __ATOMIC_RELAXED)) atomicMax(&fnext[result], t);
    }
    atomicMax(&io.lastw[result], (gen << 24) | (unsigned long long)q);
}
// end of pass p: this block's counts and flag, then the last block to finish commits or reports
template <int NT>
__device__ void multi_pass_end(const MultiIO& io, const orbfe_map_point* recs, int n, int p, int final_, int nas,
                               bool ch, unsigned long long npair) {
    __shared__ int s_last, s_nas, s_ch;
    const int tid = threadIdx.x;
    const unsigned long long gen = io.gen0 + (unsigned long long)p;
    // everything the last block reads is an atomic (performed device-wide, no cache write-back
    // needed): counts, the change flag, the last writers; a device-scope release per block wrote
    // back a whole L2 each time and cost more than the pass. The block's counts are summed in LDS
    // first: same-address global atomics serialise at the memory side (one per wave was thousands
    // per pass)
    if (tid == 0) s_nas = s_ch = 0;
    SYNC();
    nas = wave_sum_dpp(nas);
    if ((tid & 63) == 0 && nas) atomicAdd(&s_nas, nas);
    if (__ballot(ch) && (tid & 63) == 0) s_ch = 1;
    if (io.stats && npair) atomicAdd(&io.stats[1], npair);
    // every wave's atomics acknowledged, the barrier, the block's counts, the ticket
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (tid == 0) {
        if (s_nas) atomicAdd(&io.cnt[p], s_nas);
        if (s_ch) atomicMax(&io.changed[p], gen);
        __builtin_amdgcn_s_waitcnt(0);
        s_last = atomicAdd(&io.done[p], 1) == (int)gridDim.x - 1;
    }
    SYNC();
    if (!s_last) return;
    // agent-scope loads (sc1): the atomics' values, not this XCD's cached lines. Converged when this
    // pass changed no result, or when the first[] state it built for the next pass equals the one it
    // read: the next pass would then compute exactly this pass's results (every result is a function
    // of first[] and fixed data), so the pass that would only confirm it is never run
    bool same = true;
    {
        const unsigned long long* fcur = io.first[p & 1];
        const unsigned long long* fnext = io.first[(p + 1) & 1];
        for (int k = tid; k < n && same; k += NT)
            same = mt_fget(__hip_atomic_load(&fnext[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), gen + 1) ==
                   mt_fget(__hip_atomic_load(&fcur[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), gen);
    }
    same = __syncthreads_and(same);
    const bool conv = same || __hip_atomic_load(&io.changed[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != gen;
    // the batch's later passes are gated on this pass's change word: clear it, or a pass that
    // converged by the first[] test (its results did change) would let the next pass run and publish
    // a second status for the same sequence number
    if (conv && tid == 0) __hip_atomic_store(&io.changed[p], 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (conv)
#pragma unroll 4
        for (int k = tid; k < n; k += NT) {
            const unsigned long long v = __hip_atomic_load(&io.lastw[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((v >> 24) == gen)
                io.mvp_out[k] = *(const int*)((const uint8_t*)recs + (size_t)(v & 0xFFFFFFull) * io.q_stride + io.qid_off);
        }
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (tid == 0) {
        if (conv || final_) {
            __threadfence_system();
            if (io.stats) io.stats[2] = (unsigned long long)(p + 1);
            volatile int* st = io.st_host;
            st[0] = conv ? 0 : 1;
            st[1] = __hip_atomic_load(&io.cnt[p], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            st[2] = 0;
            st[3] = p + 1;
            st[5] = io.ntm ? *io.ntm : 0;
            __threadfence_system();
            st[4] = io.seq;
            __threadfence_system();
        }
        __hip_atomic_store(&io.done[p], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&io.cnt[p], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (conv) __hip_atomic_store(io.nactive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}
__global__ __launch_bounds__(MT_BLK_NT) void k_sbp_multi0(FrameDev fr, BlkGeom gm, const orbfe_map_point* recs, int nq,
                                                          float th, int bFar, float thFar, float nnratio, int final_,
                                                          MultiIO io) {
    extern __shared__ __attribute__((aligned(16))) uint8_t mt_sm[];
    const int n = fr.n, nbk = fr.nlevels * gm.NB * gm.NS, tid = threadIdx.x;
    float4* s_kp = (float4*)mt_sm;
    uint4* s_desc = (uint4*)(s_kp + n);
    int* s_ber = (int*)(s_desc + 2 * n);           // bucket bounds region (blk_be_words)
    const int* s_be = s_ber + 3;
    uint8_t* s_blk = (uint8_t*)(s_ber + blk_be_words(nbk, MT_BLK_NT));
    __shared__ int s_ws[MT_BLK_NT / 64];
    // the first round's records are read before the frame is staged: both memory round trips overlap
    BlkQuery Q0;
    Q0.ok = false;
    Q0.obs = 0;
    if (blockIdx.x * MT_BLK_NT + tid < nq) Q0 = blk_load<0>(fr, recs, blockIdx.x * MT_BLK_NT + tid, th, bFar, 0, thFar);
    blk_stage<MT_BLK_NT>(fr, gm, io.mvp_in, io.obs_in, s_kp, s_desc, s_ber, s_blk, nullptr, nullptr, s_ws);
    if (blockIdx.x == 0) {   // the frame as staged, for later passes' re-enumerations
        for (int i = tid; i < n; i += MT_BLK_NT) {
            io.g_kp[i] = s_kp[i];
            io.g_desc[2 * i] = s_desc[2 * i];
            io.g_desc[2 * i + 1] = s_desc[2 * i + 1];
            io.g_blk[i] = s_blk[i];
        }
        for (int b = tid; b <= nbk; b += MT_BLK_NT) io.g_be[b] = s_be[b];
    }
    const unsigned long long gen = io.gen0;
    int nas = 0;
    bool ch = false;
    unsigned long long npair = 0;
    __shared__ int s_acnt, s_abase;
    // block-uniform trip count (the active list is compacted per block: one global atomic per block
    // and round instead of one per wave)
    for (int q0 = blockIdx.x * MT_BLK_NT; q0 < nq; q0 += gridDim.x * MT_BLK_NT) {
        const int q = q0 + tid;
        BlkQuery Q = Q0;
        if (q0 != blockIdx.x * MT_BLK_NT) {
            Q.ok = false;
            Q.obs = 0;
            if (q < nq) Q = blk_load<0>(fr, recs, q, th, bFar, 0, thFar);
        }
        uint32_t L[MT_BLK_LIST];
        const int c = blk_list<0>(Q, gm, s_kp, s_desc, s_be, s_blk, L);
        int result = -1;
        if (c > 0) {
            uint4* lp = (uint4*)(io.lists + (size_t)q * MT_BLK_LIST);
            lp[0] = make_uint4(L[0], L[1], L[2], L[3]);
            lp[1] = make_uint4(L[4], L[5], L[6], L[7]);
            io.lcnt[q] = c | (Q.obs > 0 ? (int)0x80000000 : 0);
            // pass 0: no earlier query holds anything, the list's head decides
            result = blk_accept<0>((int)(L[0] & 0x1FFFu), (int)(L[0] >> 16), (int)((L[0] >> 13) & 7),
                                   L[1] != 0xFFFFFFFFu ? (int)(L[1] >> 16) : 256,
                                   L[1] != 0xFFFFFFFFu ? (int)((L[1] >> 13) & 7) : -1, nnratio, 0);
            npair += (unsigned)c;
        }
        // the active list: wave offsets from an LDS counter, one global reservation per block
        if (tid == 0) s_acnt = 0;
        SYNC();
        const unsigned long long am = __ballot(c > 0);
        int woff = 0;
        if ((tid & 63) == 0 && am) woff = atomicAdd(&s_acnt, (int)__popcll(am));
        woff = __shfl(woff, 0);
        SYNC();
        if (tid == 0) s_abase = s_acnt ? atomicAdd(io.nactive, s_acnt) : 0;
        SYNC();
        if (c > 0) io.active[s_abase + woff + lanes_below(am)] = q;
        if (q < nq) io.assign[q] = result;
        if (result >= 0) {
            nas++;
            ch = true;
            multi_publish(io, io.first[1], gen, q, result, Q.obs > 0);
        }
    }
    multi_pass_end<MT_BLK_NT>(io, recs, n, 0, final_, nas, ch, npair);
}
#define MT_MULTI_NT 256
#define MT_MULTI_TH 4.0f   // k_sbp_multi0 / k_sbp_multi below this th
__global__ __launch_bounds__(MT_MULTI_NT) void k_sbp_multi(FrameDev fr, BlkGeom gm, const orbfe_map_point* recs,
                                                           float th, int bFar, float thFar, float nnratio, int p,
                                                           int final_, MultiIO io) {
    const unsigned long long gen = io.gen0 + (unsigned long long)p;
    if (__atomic_load_n(&io.changed[p - 1], __ATOMIC_RELAXED) != gen - 1) return;   // converged at p - 1
    const unsigned long long* fcur = io.first[p & 1];
    unsigned long long* fnext = io.first[(p + 1) & 1];
    const int na = __hip_atomic_load(io.nactive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int nas = 0;
    bool ch = false;
    for (int i = blockIdx.x * MT_MULTI_NT + threadIdx.x; i < na; i += gridDim.x * MT_MULTI_NT) {
        const int q = io.active[i];
        const int prev = io.assign[q];
        const int lc = io.lcnt[q];
        const int c = lc & 0x7FFFFFFF;
        const uint4* lp = (const uint4*)(io.lists + (size_t)q * MT_BLK_LIST);
        const uint4 l0 = lp[0], l1 = lp[1];
        const uint32_t L[MT_BLK_LIST] = {l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, l1.z, l1.w};
        bool free_[MT_BLK_LIST];
#pragma unroll
        for (int k = 0; k < MT_BLK_LIST; k++)
            free_[k] = L[k] != 0xFFFFFFFFu && mt_fget(fcur[L[k] & 0x1FFFu], gen) >= q;
        uint32_t e1 = 0xFFFFFFFFu, e2 = 0xFFFFFFFFu;
        int found = 0;
#pragma unroll
        for (int k = 0; k < MT_BLK_LIST; k++) {
            if (!free_[k] || found >= 2) continue;
            if (found == 0) e1 = L[k];
            else e2 = L[k];
            found++;
        }
        int result;
        if (found < 2 && c > MT_BLK_LIST) {
            // the list ran out: the window again, over block 0's frame copy, with this pass's gates
            const BlkQuery Q = blk_load<0>(fr, recs, q, th, bFar, 0, thFar);
            unsigned long long k1 = ~0ull, k2 = ~0ull;
            blk_enum<0>(Q, gm, io.g_kp, io.g_desc, io.g_be, io.g_blk, [&](unsigned long long key, int idx) {
                if (mt_fget(fcur[idx], gen) < q) return;
                const bool lt1 = key < k1, lt2 = key < k2;
                k2 = lt1 ? k1 : (lt2 ? key : k2);
                k1 = lt1 ? key : k1;
            });
            result = blk_accept<0>(k1 != ~0ull ? (int)((k1 >> 4) & 0x1FFFu) : -1, (int)(k1 >> 40), (int)(k1 & 15),
                                   k2 != ~0ull ? (int)(k2 >> 40) : 256, k2 != ~0ull ? (int)(k2 & 15) : -1, nnratio, 0);
        } else {
            result = blk_accept<0>(e1 != 0xFFFFFFFFu ? (int)(e1 & 0x1FFFu) : -1, (int)(e1 >> 16), (int)((e1 >> 13) & 7),
                                   e2 != 0xFFFFFFFFu ? (int)(e2 >> 16) : 256,
                                   e2 != 0xFFFFFFFFu ? (int)((e2 >> 13) & 7) : -1, nnratio, 0);
        }
        if (result != prev) {
            io.assign[q] = result;
            ch = true;
        }
        if (result >= 0) {
            nas++;
            multi_publish(io, fnext, gen, q, result, lc < 0);
        }
    }
    multi_pass_end<MT_MULTI_NT>(io, recs, fr.n, p, final_, nas, ch, 0);
}

// ---- SearchByProjection(CurrentFrame, LastFrame, ...) (ORBmatcher.cc:1676-1887) and
//      SearchByProjection(CurrentFrame, pKF, ...) (:1889-2010): single best, then rotation filter ----
__global__ __launch_bounds__(MT_NT) void k_sbp_proj(FrameDev fr, const orbfe_proj_point* pts, int nq, float th,
                                                    int mode /*0 lastframe, 1 kf*/, int bForward, int bBackward,
                                                    int maxDist, const int* blocked0, const int* first, int* assign,
                                                    int* changed, PassIO io) {
    if (pass_gated(io)) return;
    pass_fill(io);
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const orbfe_proj_point& p = pts[q];
    int result = -1;
    bool ok = p.valid != 0 && p.octave >= 0 && p.octave < fr.nlevels;
    if (ok && mode == 0) {
        if (p.invzc < 0) ok = false;
        else if (p.u < fr.minx || p.u > fr.maxx) ok = false;
        else if (p.v < fr.miny || p.v > fr.maxy) ok = false;
    }
    if (ok) {
        const int oct = p.octave;
        const float radius = th * fr.scale[oct];
        int minL, maxL;
        if (mode == 1) { minL = oct - 1; maxL = oct + 1; }
        else if (bForward) { minL = oct; maxL = -1; }
        else if (bBackward) { minL = 0; maxL = oct; }
        else { minL = oct - 1; maxL = oct + 1; }
        int bestDist = 256, bestIdx2 = -1;
        mt_for_area(fr, fr.cstart, fr.cidx, p.u, p.v, radius, minL, maxL, [&](int i2, const OrbKeyPoint&) {
            if (blocked0[i2] || first[i2] < q) return;
            if (mode == 0 && fr.uright && fr.uright[i2] > 0) {
                const float ur = p.u - fr.mbf * p.invzc;
                const float er = fabsf(ur - fr.uright[i2]);
                if (er > radius) return;
            }
            const int dist = mt_hamming(p.desc, fr.desc + 8 * i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        });
        if (bestDist <= maxDist) result = bestIdx2;
    }
    pass_publish(io, q, result, p.observations);
    if (result != assign[q]) {
        assign[q] = result;
        mt_flag_changed(changed);
    }
}

// ---- Two-camera frames (F.Nleft != -1). A query writes up to W slots in the reference's order; the
// entry index 4 q + b (local map) / 2 q + b (last frame) is the write's position in the sequential
// run, and a branch at entry e sees exactly the writes with a smaller entry index. The last-frame
// writes are all guarded by the "already taken" check, so first[k] < e decides as in the
// single-camera kernels. The local map's partner writes are NOT guarded (the reference overwrites
// the partner slot unconditionally), so there the occupant at entry e is the slot's LAST writer
// before e: every pass buckets the writes per slot (k_slot_count / k_slot_fill) and a candidate
// scans its slot's bucket.
// SearchByProjection(F, vpMapPoints, ...) Nleft != -1 (ORBmatcher.cc:62-209): entries
//   b = 0 left best, 1 its right partner nleft + mvLeftToRightMatch[best] (:124-128),
//   b = 2 mvRightToLeftMatch[right best] (:197-201), 3 the right best (nleft + bestIdx, :204).
__device__ __forceinline__ void mt_best2_update(int dist, int oct, int idx, int& bestDist, int& bestLevel,
                                                int& bestDist2, int& bestLevel2, int& bestIdx) {
    if (dist < bestDist) {
        bestDist2 = bestDist; bestDist = dist;
        bestLevel2 = bestLevel; bestLevel = oct;
        bestIdx = idx;
    } else if (dist < bestDist2) {
        bestLevel2 = oct;
        bestDist2 = dist;
    }
}
__global__ void k_slot_count(const int* assign, int nent, int* cnt) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nent && assign[e] >= 0) atomicAdd(&cnt[assign[e]], 1);
}
// exclusive scan of cnt[0, n) into off[0, n] (one 1024-thread block, n <= MT_GRID_MAXN); cursor = off
__global__ __launch_bounds__(1024) void k_slot_scan(const int* cnt, int n, int* off, int* cursor) {
    __shared__ int s_part[1024];
    const int t = threadIdx.x, per = (n + 1023) / 1024, i0 = t * per, i1 = min(i0 + per, n);
    int sum = 0;
    for (int i = i0; i < i1; i++) sum += cnt[i];
    s_part[t] = sum;
    SYNC();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = t >= d ? s_part[t - d] : 0;
        SYNC();
        s_part[t] += v;
        SYNC();
    }
    int run = s_part[t] - sum;
    for (int i = i0; i < i1; i++) { off[i] = run; cursor[i] = run; run += cnt[i]; }
    if (t == 1023) off[n] = s_part[1023];
}
__global__ void k_slot_fill(const int* assign, int nent, int* cursor, int* lst) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e < nent && assign[e] >= 0) lst[atomicAdd(&cursor[assign[e]], 1)] = e;
}
// occupant of slot k before entry e: blocked when it holds a point with Observations() > 0
__device__ __forceinline__ bool mt_taken(const int* off, const int* lst, const orbfe_map_point* mps,
                                         const int* blocked0, int k, int e) {
    int last = -1;
    for (int p = off[k]; p < off[k + 1]; p++) {
        const int w = lst[p];
        if (w < e && w > last) last = w;
    }
    return last < 0 ? blocked0[k] != 0 : mps[last >> 2].observations > 0;
}
__global__ __launch_bounds__(MT_NT) void k_sbp_local2(FrameDev fr, const orbfe_map_point* mps, int nq, float th,
                                                      int bFar, float thFar, float nnratio, const int* blocked0,
                                                      const int* off, const int* lst, int* assign, int* changed) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const orbfe_map_point& mp = mps[q];
    int res[4] = {-1, -1, -1, -1};
    const bool inView = (mp.flags & ORBFE_MP_IN_VIEW) != 0, inViewR = (mp.flags & ORBFE_MP_IN_VIEW_R) != 0;
    bool go = (inView || inViewR) && !(bFar && mp.depth > thFar) && !(mp.flags & ORBFE_MP_BAD);
    const int e0 = 4 * q;
    if (go && inView && mp.scale_level >= 0 && mp.scale_level < fr.nlevels) {
        const int lvl = mp.scale_level;
        float r = mp.view_cos > 0.998 ? 2.5f : 4.0f;
        if (th != 1.0f) r *= th;
        const float R = r * fr.scale[lvl];
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        mt_for_area(fr, fr.pcstart + lvl * fr.gstride_c, fr.pcidx + lvl * fr.gstride_i, mp.proj_x, mp.proj_y, R,
                    lvl - 1, lvl, [&](int idx, const OrbKeyPoint& kp) {
            if (mt_taken(off, lst, mps, blocked0, idx, e0)) return;   // no mvuRight check when Nleft != -1
            mt_best2_update(mt_hamming(mp.desc, fr.desc + 8 * idx), kp.octave, idx, bestDist, bestLevel, bestDist2,
                            bestLevel2, bestIdx);
        });
        if (bestDist <= MT_TH_HIGH) {
            if (bestLevel == bestLevel2 && bestDist > nnratio * bestDist2) {
                go = false;   // the reference's `continue` also skips the right-camera search
            } else {
                res[0] = bestIdx;
                const int p = fr.l2r[bestIdx];
                if (p >= 0 && fr.nleft + p < fr.n) res[1] = fr.nleft + p;   // != -1 (range-guarded)
            }
        }
    }
    if (go && inViewR && mp.scale_level_r != -1 && mp.scale_level_r >= 0 && mp.scale_level_r < fr.nlevels) {
        const int lvl = mp.scale_level_r;
        const float r = mp.view_cos_r > 0.998 ? 2.5f : 4.0f;   // RadiusByViewingCos, not scaled by th (:141)
        const float R = r * fr.scale[lvl];
        // this query's own partner write (entry 4 q + 1, this pass's value) is the slot's latest
        // write when it exists; the other writes seen are those of earlier points (entries < 4 q)
        const int own = res[1], own_obs = mp.observations;
        int bestDist = 256, bestLevel = -1, bestDist2 = 256, bestLevel2 = -1, bestIdx = -1;
        mt_for_area(fr, fr.pcstart + lvl * fr.gstride_c + MT_NCELL, fr.pcidx + lvl * fr.gstride_i, mp.proj_xr,
                    mp.proj_yr, R, lvl - 1, lvl, [&](int idx, const OrbKeyPoint& kp) {
            if (idx == own ? own_obs > 0 : mt_taken(off, lst, mps, blocked0, idx, e0)) return;
            mt_best2_update(mt_hamming(mp.desc, fr.desc + 8 * idx), kp.octave, idx, bestDist, bestLevel, bestDist2,
                            bestLevel2, bestIdx);
        });
        if (bestDist <= MT_TH_HIGH && !(bestLevel == bestLevel2 && bestDist > nnratio * bestDist2)) {
            const int p = fr.r2l[bestIdx - fr.nleft];
            if (p >= 0 && p < fr.nleft) res[2] = p;
            res[3] = bestIdx;
        }
    }
    int ch = 0;
#pragma unroll
    for (int b = 0; b < 4; b++)
        if (res[b] != assign[e0 + b]) { assign[e0 + b] = res[b]; ch = 1; }
    if (ch) mt_flag_changed(changed);
}

// SearchByProjection(CurrentFrame, LastFrame, th, bMono) with CurrentFrame.Nleft != -1
// (ORBmatcher.cc:1695-1858): entry 2 q = the left-grid best, 2 q + 1 = the right-grid best for the
// caller's right-camera projection right_uv[q]; a point whose left window is empty skips both.
__global__ __launch_bounds__(MT_NT) void k_sbp_proj2(FrameDev fr, const orbfe_proj_point* pts, const float2* right_uv,
                                                     int nq, float th, int bForward, int bBackward,
                                                     const int* blocked0, const int* first, int* assign,
                                                     int* changed) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= nq) return;
    const orbfe_proj_point& p = pts[q];
    int res[2] = {-1, -1};
    bool ok = p.valid != 0 && p.octave >= 0 && p.octave < fr.nlevels;
    if (ok && p.invzc < 0) ok = false;
    else if (ok && (p.u < fr.minx || p.u > fr.maxx)) ok = false;
    else if (ok && (p.v < fr.miny || p.v > fr.maxy)) ok = false;
    if (ok) {
        const int oct = p.octave;
        const float radius = th * fr.scale[oct];
        int minL, maxL;
        if (bForward) { minL = oct; maxL = -1; }
        else if (bBackward) { minL = 0; maxL = oct; }
        else { minL = oct - 1; maxL = oct + 1; }
        int bestDist = 256, bestIdx2 = -1, ncand = 0;
        mt_for_area(fr, fr.cstart, fr.cidx, p.u, p.v, radius, minL, maxL, [&](int i2, const OrbKeyPoint&) {
            ncand++;   // vIndices2 non-empty (blocked candidates included)
            if (blocked0[i2] || first[i2] < 2 * q) return;
            const int dist = mt_hamming(p.desc, fr.desc + 8 * i2);
            if (dist < bestDist) { bestDist = dist; bestIdx2 = i2; }
        });
        if (ncand > 0) {
            if (bestDist <= MT_TH_HIGH) res[0] = bestIdx2;
            const float2 uv = right_uv[q];
            int bestDistR = 256, bestIdxR = -1;
            mt_for_area(fr, fr.cstart + MT_NCELL, fr.cidx, uv.x, uv.y, radius, minL, maxL, [&](int i2, const OrbKeyPoint&) {
                if (blocked0[i2] || first[i2] < 2 * q + 1) return;
                const int dist = mt_hamming(p.desc, fr.desc + 8 * i2);
                if (dist < bestDistR) { bestDistR = dist; bestIdxR = i2; }
            });
            if (bestDistR <= MT_TH_HIGH) res[1] = bestIdxR;
        }
    }
    const bool ch = res[0] != assign[2 * q] || res[1] != assign[2 * q + 1];
    if (ch) {
        assign[2 * q] = res[0];
        assign[2 * q + 1] = res[1];
        mt_flag_changed(changed);
    }
}

// ---- Frame::isInFrustum (pinhole, Frame.cc:512-570) + MapPoint::PredictScale (MapPoint.cc:531-546)
// for every local map point (Tracking.cc:3407-3425): one thread per point, float arithmetic in the
// reference's (Eigen's) order, no contraction, glibc logf port. Writes the tracking snapshot the
// SearchByProjection kernels read and counts nToMatch.
struct CamModelDev {
    int type;                 // ORBFE_CAM_*
    float fx, fy, cx, cy, k[4];
};
struct CamDev {
    float R[9], t[3], Ow[3], logsf, cos_limit;
    float minx, maxx, miny, maxy, mbf;
    int nlevels;
    int two;                  // two-camera frame (Nleft != -1): isInFrustumChecks left + right
    CamModelDev cl, cr;       // mpCamera, mpCamera2
    float R2[9], t2[3], Ow2[3];   // right view: Rrl * Rcw, Rrl * tcw + trl, Rwc * tlr + Ow (host-derived)
};
// The 3-term sums of Eigen 3.3's fixed-size expressions (products' coefficients, norm, dot): the
// non-vectorised redux halves the range, sum(a, b, c) = a + (b + c) (Eigen/src/Core/Redux.h,
// redux_novec_unroller; ProductEvaluators.h lazy coeff = (lhs.row(i) .* rhs.col(j)).sum()).
__host__ __device__ __forceinline__ float eig_sum3(float a, float b, float c) { return a + (b + c); }
// Sophus point action in Eigen's order, no contraction; RxSO3 scale = squaredNorm() reduced as one
// SSE packet, (x*x + z*z) + (y*y + w*w) (Eigen's predux<Packet4f>).
__device__ __forceinline__ void be_pose_apply(const orbfe_pose& P, const float p[3], float o[3]) {
    const float vx = P.q[0], vy = P.q[1], vz = P.q[2], w = P.q[3];
    float uv[3] = {vy * p[2] - vz * p[1], vz * p[0] - vx * p[2], vx * p[1] - vy * p[0]};
#pragma unroll
    for (int k = 0; k < 3; k++) uv[k] += uv[k];
    const float c[3] = {vy * uv[2] - vz * uv[1], vz * uv[0] - vx * uv[2], vx * uv[1] - vy * uv[0]};
    if (P.kind == ORBFE_SIM3) {
        const float sc = (vx * vx + vz * vz) + (vy * vy + w * w);
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = (sc * p[k] + (w * uv[k] + c[k])) + P.t[k];
    } else {
#pragma unroll
        for (int k = 0; k < 3; k++) o[k] = ((p[k] + w * uv[k]) + c[k]) + P.t[k];
    }
}

// GeometricCamera::project(Eigen::Vector3f): Pinhole.cpp:43-49, KannalaBrandt8.cpp:67-82 (float
// arithmetic in the source's order; atan2f / cos / sin of float as glibc's atan2f / cosf / sinf).
__device__ __forceinline__ float2 mt_cam_project(const CamModelDev& m, float x, float y, float z) {
    if (m.type == ORBFE_CAM_KANNALA_BRANDT8) {
        const float x2_plus_y2 = x * x + y * y;
        const float theta = glibc_atan2f(sqrtf(x2_plus_y2), z);
        const float psi = glibc_atan2f(y, x);
        const float theta2 = theta * theta;
        const float theta3 = theta * theta2;
        const float theta5 = theta3 * theta2;
        const float theta7 = theta5 * theta2;
        const float theta9 = theta7 * theta2;
        const float r = theta + m.k[0] * theta3 + m.k[1] * theta5 + m.k[2] * theta7 + m.k[3] * theta9;
        return make_float2(m.fx * r * glibc_cosf(psi) + m.cx, m.fy * r * glibc_sinf(psi) + m.cy);
    }
    return make_float2(m.fx * x / z + m.cx, m.fy * y / z + m.cy);
}
// SearchByProjection(CurrentFrame, LastFrame)'s projection (ORBmatcher.cc:1702-1718, 1794-1796) for
// orbfe_search_by_projection_lastframe_pose: one thread per last-frame point, x3Dc = Tcw * x3Dw (Sophus
// SE3f action), invzc = 1.0 / x3Dc(2) in double as the reference's double literal makes it, uv =
// mpCamera->project(x3Dc), and for a two-camera frame the right-camera window centre mpCamera->project(
// Trl * x3Dc). Writes the orbfe_proj_point records the searches read (a point behind the camera keeps
// its negative invzc: the search skips it as the reference's `continue` does).
struct LastProjIn {
    const orbfe_last_point* pts;   // host points (staged by the runner)
    orbfe_pose T, Trl;
    CamModelDev cam;
    int two;
};
__global__ __launch_bounds__(MT_NT) void k_last_proj(LastProjIn g, const orbfe_last_point* pts, int n,
                                                     orbfe_proj_point* out, float2* ruv) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const orbfe_last_point p = pts[i];
    orbfe_proj_point r;
    r.u = r.v = r.invzc = 0.f;
    r.octave = p.octave;
    r.angle = p.angle;
    r.valid = 0;
    r.observations = p.observations;
    r.id = p.id;
    memcpy(r.desc, p.desc, 32);
    float2 uvr = make_float2(0.f, 0.f);
    if (p.valid) {
        float c[3];
        be_pose_apply(g.T, p.pos, c);
        r.invzc = (float)(1.0 / (double)c[2]);
        r.valid = 1;
        if (!(r.invzc < 0)) {
            const float2 uv = mt_cam_project(g.cam, c[0], c[1], c[2]);
            r.u = uv.x;
            r.v = uv.y;
            if (g.two) {
                float cr[3];
                be_pose_apply(g.Trl, c, cr);
                uvr = mt_cam_project(g.cam, cr[0], cr[1], cr[2]);
            }
        }
    }
    out[i] = r;
    if (g.two) ruv[i] = uvr;
}
// The checks shared by isInFrustum's Nleft == -1 branch (Frame.cc:512-570) and isInFrustumChecks
// (Frame.cc:1168-1242) for one view: pose (R, t), camera centre Ow, camera model m. stage = how far
// the point got: 0 behind the camera, 1 outside the image, 2 outside the distance / viewing limits,
// 3 in view (uv, depth, viewCos, level, invz valid from stage 2 / 3 on).
struct FrustumView {
    int stage;
    float u, v, depth, view_cos, invz;
    int level;
};
__device__ __forceinline__ FrustumView mt_frustum_view(const CamDev& c, const float* R, const float* t, const float* Ow,
                                                       const CamModelDev& m, const orbfe_map_point_3d& p) {
    FrustumView o{0, 0.f, 0.f, 0.f, 0.f, 0.f, 0};
    const float P0 = p.pos[0], P1 = p.pos[1], P2 = p.pos[2];
    float Pc[3];
#pragma unroll
    for (int k = 0; k < 3; k++) Pc[k] = eig_sum3(R[3 * k] * P0, R[3 * k + 1] * P1, R[3 * k + 2] * P2) + t[k];
    o.depth = sqrtf(eig_sum3(Pc[0] * Pc[0], Pc[1] * Pc[1], Pc[2] * Pc[2]));
    o.invz = 1.0f / Pc[2];
    if (Pc[2] < 0.0f) return o;
    const float2 uv = mt_cam_project(m, Pc[0], Pc[1], Pc[2]);
    o.u = uv.x;
    o.v = uv.y;
    if (uv.x < c.minx || uv.x > c.maxx || uv.y < c.miny || uv.y > c.maxy) {
        o.stage = 1;
        return o;
    }
    o.stage = 2;
    const float maxDistance = 1.2f * p.max_dist, minDistance = 0.8f * p.min_dist;
    const float PO0 = P0 - Ow[0], PO1 = P1 - Ow[1], PO2 = P2 - Ow[2];
    const float dist = sqrtf(eig_sum3(PO0 * PO0, PO1 * PO1, PO2 * PO2));
    if (dist < minDistance || dist > maxDistance) return o;
    const float viewCos = eig_sum3(PO0 * p.normal[0], PO1 * p.normal[1], PO2 * p.normal[2]) / dist;
    if (viewCos < c.cos_limit) return o;
    // MapPoint::PredictScale (MapPoint.cc:531-546)
    const float ratio = p.max_dist / dist;
    int nScale = (int)ceilf(glibc_logf(ratio) / c.logsf);
    if (nScale < 0) nScale = 0;
    else if (nScale >= c.nlevels) nScale = c.nlevels - 1;
    o.view_cos = viewCos;
    o.level = nScale;
    o.stage = 3;
    return o;
}
__global__ __launch_bounds__(MT_NT) void k_frustum(CamDev c, const orbfe_map_point_3d* pts, int n,
                                                   orbfe_map_point* track, int* n_to_match,
                                                   orbfe_map_point* track_host = nullptr) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const orbfe_map_point_3d p = pts[i];
    orbfe_map_point t;
    // mTrackDepth is only written by a passing left view: otherwise the previous value stays
    t.proj_x = -1.f; t.proj_y = -1.f; t.proj_xr = 0.f; t.view_cos = 0.f; t.depth = p.track_depth;
    t.scale_level = 0;
    t.flags = p.flags & ORBFE_MP_BAD;
    t.observations = p.observations;
    t.id = p.id;
    t.proj_yr = 0.f;
    t.view_cos_r = 0.f;
    t.scale_level_r = -1;
    memcpy(t.desc, p.desc, 32);
    bool in = false;
    if (c.two) {
        // Nleft != -1 (Frame.cc:575-586): both views checked, levels reset to -1, a view's fields
        // written only when it passes (Frame.cc:1225-1239)
        t.scale_level = -1;
        t.proj_xr = -1.f;
        t.proj_yr = -1.f;
        if (!(p.flags & (ORBFE_MP_SKIP | ORBFE_MP_BAD))) {
            const FrustumView L = mt_frustum_view(c, c.R, c.t, c.Ow, c.cl, p);
            if (L.stage == 3) {
                t.flags |= ORBFE_MP_IN_VIEW;
                t.proj_x = L.u;
                t.proj_y = L.v;
                t.scale_level = L.level;
                t.view_cos = L.view_cos;
                t.depth = L.depth;
            }
            const FrustumView Rv = mt_frustum_view(c, c.R2, c.t2, c.Ow2, c.cr, p);
            if (Rv.stage == 3) {
                t.flags |= ORBFE_MP_IN_VIEW_R;
                t.proj_xr = Rv.u;
                t.proj_yr = Rv.v;
                t.scale_level_r = Rv.level;
                t.view_cos_r = Rv.view_cos;
            }
            in = L.stage == 3 || Rv.stage == 3;
        }
    } else if (!(p.flags & (ORBFE_MP_SKIP | ORBFE_MP_BAD))) {
        const FrustumView L = mt_frustum_view(c, c.R, c.t, c.Ow, c.cl, p);
        if (L.stage >= 2) {   // mTrackProjX / Y are written once the projection is in the image
            t.proj_x = L.u;
            t.proj_y = L.v;
        }
        if (L.stage == 3) {
            t.flags |= ORBFE_MP_IN_VIEW;
            t.proj_xr = L.u - c.mbf * L.invz;
            t.depth = L.depth;
            t.scale_level = L.level;
            t.view_cos = L.view_cos;
            in = true;
        }
    }
    track[i] = t;
    // the caller's copy of the records (orbfe_search_local_points_track): vector stores into mapped,
    // coherent host memory, fenced at system scope before the search that follows in the stream
    // publishes its status word, so the host sees them when it sees that word
    if (track_host) {
        track_host[i] = t;
        __threadfence_system();
    }
    const unsigned long long m = __ballot(in);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(n_to_match, __popcll(m));
}

// rotation-histogram bin of an accepted match (ORBmatcher.cc:1775-1792): round(rot * (1/30)).
__host__ __device__ __forceinline__ int mt_rot_bin(float a1, float a2) {
    const float factor = 1.0f / MT_HISTO;
    float rot = a1 - a2;
    if (rot < 0.0) rot += 360.0f;
    int bin = (int)roundf(rot * factor);
    if (bin == MT_HISTO) bin = 0;
    return bin;
}

// ComputeThreeMaxima (ORBmatcher.cc:2012-2053) on 30 bin counts -> keep mask.
__host__ __device__ __forceinline__ unsigned mt_three_maxima_keep(const int* hist) {
    int max1 = 0, max2 = 0, max3 = 0, ind1 = -1, ind2 = -1, ind3 = -1;
    for (int i = 0; i < MT_HISTO; i++) {
        const int s = hist[i];
        if (s > max1) { max3 = max2; max2 = max1; max1 = s; ind3 = ind2; ind2 = ind1; ind1 = i; }
        else if (s > max2) { max3 = max2; max2 = s; ind3 = ind2; ind2 = i; }
        else if (s > max3) { max3 = s; ind3 = i; }
    }
    if (max2 < 0.1f * (float)max1) { ind2 = -1; ind3 = -1; }
    else if (max3 < 0.1f * (float)max1) { ind3 = -1; }
    unsigned keep = 0;
    if (ind1 >= 0) keep |= 1u << ind1;
    if (ind2 >= 0) keep |= 1u << ind2;
    if (ind3 >= 0) keep |= 1u << ind3;
    return keep;
}

// Final write-back for slot-assigning searches: slot k gets the LAST query that chose it; with
// checkOri, every entry of a dropped bin clears its slot and decrements nmatches
// (ORBmatcher.cc:1860-1884). q_angle: the query-side angle per query; frame angle from keys.
// Three grid-wide steps over the queries / slots (result[0] = assigned count, result[1] = dropped
// count, result[2 + k] = last assigner of slot k or -2 when cleared, hist[30] = rotation bins):
// K1 counts, bins and takes the last assigner; K2 (checkOri only) clears the slots of entries in
// dropped bins; K3 writes the slots.
__global__ __launch_bounds__(MT_NT) void k_mt_commit_count(const OrbKeyPoint* keys, const int* assign,
                                                           const float* q_angle, int q_stride_bytes, int nq,
                                                           int checkOri, int* result, int* hist, int W,
                                                           const int* gate = nullptr) {
    if (gate && *gate != 0) return;   // passes not converged yet: the host launches more first
    __shared__ int s_hist[MT_HISTO];
    if (threadIdx.x < MT_HISTO) s_hist[threadIdx.x] = 0;
    SYNC();
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int a = j < nq ? assign[j] : -1;
    if (a >= 0) {
        atomicMax(&result[2 + a], j);
        if (checkOri) {
            const float qa = *(const float*)((const uint8_t*)q_angle + (size_t)(j / W) * q_stride_bytes);
            atomicAdd(&s_hist[mt_rot_bin(qa, keys[a].angle)], 1);
        }
    }
    const unsigned long long m = __ballot(a >= 0);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&result[0], __popcll(m));
    SYNC();
    if (checkOri && threadIdx.x < MT_HISTO && s_hist[threadIdx.x]) atomicAdd(&hist[threadIdx.x], s_hist[threadIdx.x]);
}

__global__ __launch_bounds__(MT_NT) void k_mt_commit_drop(const OrbKeyPoint* keys, const int* assign,
                                                          const float* q_angle, int q_stride_bytes, int nq,
                                                          const int* hist, int* result, int W,
                                                          const int* gate = nullptr) {
    if (gate && *gate != 0) return;
    __shared__ unsigned s_keep;
    if (threadIdx.x == 0) s_keep = mt_three_maxima_keep(hist);
    SYNC();
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    const int a = j < nq ? assign[j] : -1;
    bool drop = false;
    if (a >= 0) {
        const float qa = *(const float*)((const uint8_t*)q_angle + (size_t)(j / W) * q_stride_bytes);
        drop = !((s_keep >> mt_rot_bin(qa, keys[a].angle)) & 1u);
        if (drop) result[2 + a] = -2;   // K1 finished before this kernel: no race with the winner write
    }
    const unsigned long long m = __ballot(drop);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&result[1], __popcll(m));
}

// Status publication (st_host != nullptr): pinned host words {gate value, assigned count, dropped
// count, passes needed, sequence number}; the last block to finish (done counter) stores them after
// every block's slot writes, at system scope, the sequence number last, so a host that sees the
// sequence number sees complete results. changed / npass: the pass change flags of this launch
// batch (passes needed = first pass that changed nothing, + 1).
struct CommitStatus {
    int* st_host;
    int* done;
    const int* changed;
    int npass;
    int seq;
};
__global__ void k_mt_commit_write(int n, const int* qid, int q_stride_bytes, const int* result, int* mvp, int W,
                                  const int* gate = nullptr, int* ch_out = nullptr, CommitStatus cs = CommitStatus{}) {
    // ch_out (result[-1]): the gate's value, so one host read brings the change flag and the counts
    const int g = gate ? *gate : 0;
    if (ch_out && blockIdx.x == 0 && threadIdx.x == 0) *ch_out = g;
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0 && k < n) {
        const int w = result[2 + k];
        if (w == -2) mvp[k] = -1;
        else if (w >= 0) mvp[k] = *(const int*)((const uint8_t*)qid + (size_t)(w / W) * q_stride_bytes);
    }
    if (!cs.st_host) return;
    // this block's slot writes complete (every wave's vmcnt 0, the barrier), then one release by the
    // thread that counts the block done (a release per thread wrote back the L2 once per wave)
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) __threadfence_system();
    if (threadIdx.x == 0 && atomicAdd(cs.done, 1) == (int)gridDim.x - 1) {
        __threadfence_system();
        int need = cs.npass;
        for (int p = 0; p < cs.npass; p++)
            if (cs.changed[p] == 0) { need = p + 1; break; }
        volatile int* st = cs.st_host;
        st[0] = g;
        st[1] = result[0];
        st[2] = result[1];
        st[3] = need;
        __threadfence_system();
        st[4] = cs.seq;
        __threadfence_system();
        *cs.done = 0;   // every block has counted: ready for the next batch's commit
    }
}

// ---- SearchForInitialization (ORBmatcher.cc:648-763) ----
// State seen by query q for candidate i2: vMatchedDistance[i2] = min distance of the queries j < q
// that selected i2 (a new selection must beat the stored distance, so the last selector holds the
// minimum). The state table is rebuilt every pass: (i2 << 16 | j) keys sorted + segmented
// prefix-min of the selecting distances.
#define MT_INIT_MAXQ 8192
// Per candidate i2 the table also keeps its segment (seg_off, seg_cnt; n2 entries, cleared here), so a
// query walks the few selectors of its candidate instead of a binary search over the whole table.
__global__ __launch_bounds__(1024) void k_init_state(const int* assign, const int* adist, int nq, uint32_t* skey,
                                                     int* spmin, int* nsel, int n2, int* seg_off, int* seg_cnt,
                                                     const int* gate) {
    // The selections (i2 << 16 | j) in (i2, j) order as a counting sort by i2: counts, one scan (the
    // segment starts and lengths, written for every i2), atomic placement, then each segment's few
    // selectors put back in j order by one thread (a bitonic network over the selections took ~10 us
    // of barrier stages)
    __shared__ uint32_t s_k[MT_INIT_MAXQ];
    __shared__ int s_c[MT_INIT_MAXQ];
    __shared__ int s_ws[16];
    if (gate && *gate == 0) return;   // the previous pass changed nothing: converged
    const int tid = threadIdx.x, nt = blockDim.x;
    for (int i = tid; i < n2; i += nt) s_c[i] = 0;
    SYNC();
    for (int j = tid; j < nq; j += nt) {
        const int a = assign[j];
        if (a >= 0) atomicAdd(&s_c[a], 1);
    }
    SYNC();
    const int per = (n2 + nt - 1) / nt, c0 = tid * per;
    int sum = 0;
    for (int u = 0; u < per; u++) sum += c0 + u < n2 ? s_c[c0 + u] : 0;
    const int incl = wave_incl_scan_dpp(sum);
    if ((tid & 63) == 63) s_ws[tid >> 6] = incl;
    SYNC();
    int run = incl - sum;
    for (int w = 0; w < (nt >> 6); w++) run += w < (tid >> 6) ? s_ws[w] : 0;
    for (int u = 0; u < per; u++) {
        const int c = c0 + u;
        if (c >= n2) break;
        const int v = s_c[c];
        seg_off[c] = run;
        seg_cnt[c] = v;
        s_c[c] = run;   // placement cursor
        run += v;
    }
    SYNC();
    for (int j = tid; j < nq; j += nt) {
        const int a = assign[j];
        if (a >= 0) s_k[atomicAdd(&s_c[a], 1)] = ((uint32_t)a << 16) | (uint32_t)j;
    }
    SYNC();
    // s_c[i2] is now the end of i2's segment: j order inside it, then the segmented prefix-min of
    // the selecting distances
    for (int c = tid; c < n2; c += nt) {
        const int b = s_c[c], a0 = b - seg_cnt[c];
        if (b <= a0) continue;
        for (int x = a0 + 1; x < b; x++) {
            const uint32_t v = s_k[x];
            int y = x - 1;
            while (y >= a0 && s_k[y] > v) { s_k[y + 1] = s_k[y]; y--; }
            s_k[y + 1] = v;
        }
        int cur = MT_INF;
        for (int t = a0; t < b; t++) {
            cur = min(cur, adist[s_k[t] & 0xFFFFu]);
            spmin[t] = cur;
            skey[t] = s_k[t];
        }
    }
    if (tid == nt - 1) *nsel = run;   // the last thread's running sum: every count
}

// One query per DPP row of 16 lanes (four per wave): lane l walks the window's grid columns
// nMinCellX + l, + l + 16, ... (GetFeaturesInArea, Frame.cc:657-723, one contiguous CSR run per column)
// and keeps its two smallest (dist, CSR position) keys; the CSR position is the reference's
// enumeration order, so the row minimum is its first best and the second minimum its bestDist2.
// A thread per query left most of the machine idle (5,000 queries = 20 blocks) behind a chain of
// dependent loads per candidate.
#define MT_INIT_WNT 256
__global__ __launch_bounds__(MT_INIT_WNT) void k_init_eval(FrameDev f1, FrameDev f2, const float* prev, int windowSize,
                                                           float nnratio, const uint32_t* skey, const int* spmin,
                                                           const int* seg_off, const int* seg_cnt, int* assign,
                                                           int* adist, int* changed, const int* gate) {
    if (gate && *gate == 0) return;   // the previous pass changed nothing: converged
    const int lane = threadIdx.x & 63, grp = lane >> 4, sl = lane & 15;
    const int q = (blockIdx.x * (MT_INIT_WNT / 64) + (threadIdx.x >> 6)) * 4 + grp;
    const bool qv = q < f1.n;
    int level1 = 1;
    float x = 0.f, y = 0.f;
    uint32_t d1[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    if (qv) {
        level1 = f1.keys[q].octave;
        if (level1 <= 0) {
            x = prev[2 * q];
            y = prev[2 * q + 1];
#pragma unroll
            for (int w = 0; w < 8; w++) d1[w] = f1.desc[8 * q + w];
        }
    }
    const float r = (float)windowSize;
    int cx0 = 0, cx1 = -1, cy0 = 0, cy1 = -1;
    if (qv && level1 <= 0) {
        cx0 = max(0, (int)floorf((x - f2.minx - r) * f2.invw));
        cx1 = min(ORBFE_GRID_COLS - 1, (int)ceilf((x - f2.minx + r) * f2.invw));
        cy0 = max(0, (int)floorf((y - f2.miny - r) * f2.invh));
        cy1 = min(ORBFE_GRID_ROWS - 1, (int)ceilf((y - f2.miny + r) * f2.invh));
        if (cx0 >= ORBFE_GRID_COLS || cx1 < 0 || cy0 >= ORBFE_GRID_ROWS || cy1 < 0) cx1 = cx0 - 1;
    }
    const bool bCheckLevels = (level1 > 0) || (level1 >= 0);
    // only level-0 queries search: the octave-0 grid (pcstart) holds exactly the level-0 candidates
    const int* cs = f2.pcstart;
    const int* ci = f2.pcidx;
    unsigned long long b1 = ~0ull, b2 = ~0ull;
    for (int ix = cx0 + sl; ix <= cx1; ix += 16) {
        const int j1 = cs[ix * ORBFE_GRID_ROWS + cy1 + 1];
        for (int j = cs[ix * ORBFE_GRID_ROWS + cy0]; j < j1; j++) {
            const int i2 = ci[j];
            const OrbKeyPoint kp = f2.keys[i2];
            if (bCheckLevels) {
                if (kp.octave < level1) continue;
                if (level1 >= 0 && kp.octave > level1) continue;
            }
            if (!(fabsf(kp.x - x) < r && fabsf(kp.y - y) < r)) continue;
            int dist = 0;
#pragma unroll
            for (int w = 0; w < 8; w++) dist += __popc(d1[w] ^ f2.desc[8 * i2 + w]);
            // vMatchedDistance[i2] as seen by query q: the prefix minimum at the last selector j < q of
            // i2 (its segment lists the selectors in j order; most candidates have none or one)
            int md = MT_INF;
            const int sc = seg_cnt[i2];
            if (sc) {
                const int so = seg_off[i2];
                for (int t = so; t < so + sc && (int)(skey[t] & 0xFFFFu) < q; t++) md = spmin[t];
            }
            if (md <= dist) continue;
            const unsigned long long k = ((unsigned long long)dist << 32) | (unsigned)j;
            if (k < b1) { b2 = b1; b1 = k; }
            else if (k < b2) b2 = k;
        }
    }
    const unsigned long long m1 = mt_row_min64(b1);
    const unsigned long long m2 = mt_row_min64(b1 == m1 ? b2 : b1);
    if (sl != 0 || !qv) return;
    int result = -1, rdist = 0;
    if (m1 != ~0ull) {
        const int bestDist = (int)(m1 >> 32);
        const int bestDist2 = m2 != ~0ull ? (int)(m2 >> 32) : MT_INF;
        if (bestDist <= MT_TH_LOW && bestDist < (float)bestDist2 * nnratio) {
            result = ci[(int)(m1 & 0xFFFFFFFFu)];
            rdist = bestDist;
        }
    }
    if (result != assign[q] || (result >= 0 && rdist != adist[q])) {
        assign[q] = result;
        adist[q] = rdist;
        mt_flag_changed(changed);
    }
}

// The commit runs only once the last pass changed nothing (gate == 0). Its outputs (matches12 and
// the updated prevMatched, the latter pre-filled with the input by the host) go straight into mapped
// pinned memory, then {converged, matches, -, -, sequence number} into the status words the host
// waits on; a gated-off commit publishes "not converged" only (the host enqueues more passes).
__global__ __launch_bounds__(1024) void k_init_commit(FrameDev f1, FrameDev f2, const int* assign, int checkOri,
                                                      float* prev, int* m12, const int* gate, int* st_host, int seq) {
    __shared__ int s_hist[MT_HISTO];
    __shared__ unsigned s_keep;
    __shared__ int s_n;
    __shared__ int s_owner[MT_INIT_MAXQ];
    const bool run = !gate || *gate == 0;
    if (run) {
        if (threadIdx.x < MT_HISTO) s_hist[threadIdx.x] = 0;
        if (threadIdx.x == 0) s_n = 0;
        for (int i = threadIdx.x; i < f2.n && i < MT_INIT_MAXQ; i += blockDim.x) s_owner[i] = -1;
        SYNC();
        for (int j = threadIdx.x; j < f1.n; j += blockDim.x) {
            const int a = assign[j];
            if (a < 0) continue;
            atomicMax(&s_owner[a], j);   // the last selector keeps i2; earlier ones were stolen
            if (checkOri) atomicAdd(&s_hist[mt_rot_bin(f1.keys[j].angle, f2.keys[a].angle)], 1);
        }
        SYNC();
        if (threadIdx.x == 0) s_keep = checkOri ? mt_three_maxima_keep(s_hist) : 0xFFFFFFFFu;
        SYNC();
        int cnt = 0;
        for (int j = threadIdx.x; j < f1.n; j += blockDim.x) {
            const int a = assign[j];
            int out = -1;
            if (a >= 0 && s_owner[a] == j) {
                out = a;
                if (checkOri && !((s_keep >> mt_rot_bin(f1.keys[j].angle, f2.keys[a].angle)) & 1u)) out = -1;
            }
            m12[j] = out;
            if (out >= 0) {
                cnt++;
                prev[2 * j] = f2.keys[out].x;
                prev[2 * j + 1] = f2.keys[out].y;
            }
        }
        atomicAdd(&s_n, cnt);
    }
    // every wave's output stores complete, the barrier, one system-scope release, then the status
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (threadIdx.x == 0) {
        __threadfence_system();
        volatile int* st = st_host;
        st[0] = run ? 0 : 1;
        st[1] = run ? s_n : 0;
        __threadfence_system();
        st[4] = seq;
        __threadfence_system();
    }
}

// ---- SearchByBoW(KF, F) (ORBmatcher.cc:223-425): one thread per node present in both vectors.
// Every frame index belongs to exactly one vocabulary node, so the "already matched" skip is local
// to the node and the node walks are independent (the reference's order inside a node is kept).
// A two-camera F (nleft >= 0) keeps a left and a right best / second-best (:288-313); the right
// match is taken inside the left's bestDist1 <= TH_LOW with its ratio test disabled ("|| true", :359).
__global__ __launch_bounds__(MT_NT) void k_bow_nodes(const int* pairs, int npairs, const int* kf_off,
                                                     const uint32_t* kf_idx, const int* f_off, const uint32_t* f_idx,
                                                     const int32_t* kf_mp, const uint32_t* kf_desc,
                                                     const uint32_t* f_desc, float nnratio, int nleft, int* out_src) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= npairs) return;
    const int a = pairs[2 * t], b = pairs[2 * t + 1];
    for (int ia = kf_off[a]; ia < kf_off[a + 1]; ia++) {
        const unsigned realIdxKF = kf_idx[ia];
        if (kf_mp[realIdxKF] < 0) continue;
        uint32_t dk[8];
#pragma unroll
        for (int w = 0; w < 8; w++) dk[w] = kf_desc[8 * realIdxKF + w];
        int bestDist1 = 256, bestIdxF = -1, bestDist2 = 256;
        int bestDist1R = 256, bestIdxFR = -1, bestDist2R = 256;
        for (int ib = f_off[b]; ib < f_off[b + 1]; ib++) {
            const unsigned realIdxF = f_idx[ib];
            if (out_src[realIdxF] >= 0) continue;
            int dist = 0;
#pragma unroll
            for (int w = 0; w < 8; w++) dist += __popc(dk[w] ^ f_desc[8 * realIdxF + w]);
            if (nleft < 0 || (int)realIdxF < nleft) {
                if (dist < bestDist1) { bestDist2 = bestDist1; bestDist1 = dist; bestIdxF = (int)realIdxF; }
                else if (dist < bestDist2) bestDist2 = dist;
            } else {
                if (dist < bestDist1R) { bestDist2R = bestDist1R; bestDist1R = dist; bestIdxFR = (int)realIdxF; }
                else if (dist < bestDist2R) bestDist2R = dist;
            }
        }
        (void)bestDist2R;
        if (bestDist1 <= MT_TH_LOW) {
            if (static_cast<float>(bestDist1) < nnratio * static_cast<float>(bestDist2)) out_src[bestIdxF] = (int)realIdxKF;
            if (bestDist1R <= MT_TH_LOW) out_src[bestIdxFR] = (int)realIdxKF;
        }
    }
}
__global__ __launch_bounds__(1024) void k_bow_commit(const OrbKeyPoint* kf_keys, const OrbKeyPoint* f_keys, int fn,
                                                     const int32_t* kf_mp, int checkOri, const int* out_src,
                                                     int* out, int* result) {
    __shared__ int s_hist[MT_HISTO];
    __shared__ unsigned s_keep;
    __shared__ int s_n;
    if (threadIdx.x < MT_HISTO) s_hist[threadIdx.x] = 0;
    if (threadIdx.x == 0) s_n = 0;
    SYNC();
    for (int i = threadIdx.x; i < fn; i += blockDim.x) {
        const int s = out_src[i];
        if (s >= 0 && checkOri) atomicAdd(&s_hist[mt_rot_bin(kf_keys[s].angle, f_keys[i].angle)], 1);
    }
    SYNC();
    if (threadIdx.x == 0) s_keep = checkOri ? mt_three_maxima_keep(s_hist) : 0xFFFFFFFFu;
    SYNC();
    int cnt = 0;
    for (int i = threadIdx.x; i < fn; i += blockDim.x) {
        const int s = out_src[i];
        int o = -1;
        if (s >= 0 && (!checkOri || ((s_keep >> mt_rot_bin(kf_keys[s].angle, f_keys[i].angle)) & 1u))) o = kf_mp[s];
        out[i] = o;
        cnt += o >= 0 ? 1 : 0;
    }
    atomicAdd(&s_n, cnt);
    SYNC();
    if (threadIdx.x == 0) result[0] = s_n;
}

// SearchByBoW(KF, F) in ONE workgroup (the Tracking thread's TrackReferenceKeyFrame / Relocalization
// calls, Tracking.cc:2836,3765): both descriptor sets, the node lists and the match state in LDS, the
// node walks of k_bow_nodes (same order, same two-camera rule) reading LDS only, and k_bow_commit's
// rotation histogram in the same block. One launch; the multi-launch pair above serves the sets
// that do not fit.
#define MT_BOW_NT 1024
#define MT_BOW_FR 4   // F features per thread in the commit (fn <= 4096)
// The call's uploads are one contiguous device range (Plan), node pairs first and the F descriptors
// last: the block copies that range into LDS with one flat 16-byte loop (independent loads in flight
// together; a copy loop per array waited one memory latency per array) and addresses every array
// at its byte offset inside the copy. F's keypoints (after the range) are read from memory.
struct BowBlockIn {
    const uint4* region;   // the contiguous uploads (the mapped pinned staging: read over the link once)
    int nvec;              // 16-byte words copied
    int o_pairs, o_kfoff, o_kfidx, o_foff, o_fidx, o_kfmp, o_kfdesc, o_kfkeys, o_fdesc;   // byte offsets
    const OrbKeyPoint* f_keys;
    int npairs, kf_n, fn, nleft, checkOri;
    float nnratio;
    volatile int* st_host;   // status words: [1] = matches, [4] = seq (after the outputs)
    int seq;
};
#ifdef ORBFE_BOW_STAMPS   // diagnostic build (tools/build_variant.sh): phase times of thread 0, printed
#define BOW_STAMP(k) do { if (threadIdx.x == 0) t_st[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define BOW_STAMP(k) do { } while (0)
#endif
__global__ __launch_bounds__(MT_BOW_NT) void k_bow_block(BowBlockIn in, int* out, int* result) {
    extern __shared__ __attribute__((aligned(16))) uint8_t bw_sm[];
    __shared__ int s_hist[MT_HISTO];
    __shared__ unsigned s_keep;
    __shared__ int s_n;
    const int tid = threadIdx.x;
#ifdef ORBFE_BOW_STAMPS
    unsigned long long t_st[5] = {0, 0, 0, 0, 0};
#endif
    BOW_STAMP(0);
    // F's angles for the commit, loaded now (their latency hides under the staging and the walks)
    float fang[MT_BOW_FR];
#pragma unroll
    for (int u = 0; u < MT_BOW_FR; u++) {
        const int i = tid + u * MT_BOW_NT;
        fang[u] = i < in.fn ? in.f_keys[i].angle : 0.f;
    }
    uint4* s_reg = (uint4*)bw_sm;
    int* s_src = (int*)(s_reg + in.nvec);        // F index -> matched KF index (-1)
#pragma unroll 4
    for (int i = tid; i < in.nvec; i += MT_BOW_NT) s_reg[i] = in.region[i];
    for (int i = tid; i < in.fn; i += MT_BOW_NT) s_src[i] = -1;
    if (tid < MT_HISTO) s_hist[tid] = 0;
    if (tid == 0) s_n = 0;
    SYNC();
    BOW_STAMP(1);
    const int* s_pr = (const int*)(bw_sm + in.o_pairs);
    const int* s_kfo = (const int*)(bw_sm + in.o_kfoff);
    const int* s_kfi = (const int*)(bw_sm + in.o_kfidx);
    const int* s_fo = (const int*)(bw_sm + in.o_foff);
    const int* s_fi = (const int*)(bw_sm + in.o_fidx);
    const int* s_mp = (const int*)(bw_sm + in.o_kfmp);
    const uint4* s_kd = (const uint4*)(bw_sm + in.o_kfdesc);
    const OrbKeyPoint* s_kk = (const OrbKeyPoint*)(bw_sm + in.o_kfkeys);
    const uint4* s_fd = (const uint4*)(bw_sm + in.o_fdesc);
    // one quad of lanes per node present in both vectors (ORBmatcher.cc:244-371). The node's KF
    // features run in the reference's order; for each, the quad's lanes score the node's F features
    // (lane l: l, l + 4, ...) and the quad minimum of (dist, position) keys is the reference's first
    // best, the second minimum its bestDist2. An F index belongs to one node only, so the "already
    // matched" state is private to the quad. One thread per node walked the longest node's KF x F
    // pairs alone (16-18 us of the kernel's 26); a row of 16 lanes per node spent more on its
    // reductions than it saved at ~2.5 features per node (28 us).
    const int sl = tid & 3;
    auto quad_min64 = [](unsigned long long v) {
        v = mt_min64_dpp_step<0xB1>(v);
        return mt_min64_dpp_step<0x4E>(v);
    };
    constexpr int FQ = 4;   // F features per lane held in registers (nodes of <= 16 F features)
    for (int t = tid >> 2; t < in.npairs; t += MT_BOW_NT / 4) {
        const int a = s_pr[2 * t], b = s_pr[2 * t + 1];
        const int fb0 = s_fo[b], fb1 = s_fo[b + 1];
        const int ka0 = s_kfo[a], ka1 = s_kfo[a + 1];
        if (fb1 - fb0 <= 4 * FQ) {
            // the node's F features in registers (position p = 4 c + lane: the reference's order), the
            // "already matched" flags as a bit mask: no LDS round trip inside the KF walk
            uint4 fd0[FQ], fd1[FQ];
            int fidx[FQ];
            unsigned taken = 0u, isleft = 0u;
#pragma unroll
            for (int c = 0; c < FQ; c++) {
                const int ib = fb0 + sl + 4 * c;
                fidx[c] = ib < fb1 ? s_fi[ib] : 0;
                if (ib < fb1) {
                    fd0[c] = s_fd[2 * fidx[c]];
                    fd1[c] = s_fd[2 * fidx[c] + 1];
                    if (in.nleft < 0 || fidx[c] < in.nleft) isleft |= 1u << c;
                } else {
                    fd0[c] = fd1[c] = make_uint4(0u, 0u, 0u, 0u);
                    taken |= 1u << c;
                }
            }
            for (int ia = ka0; ia < ka1; ia++) {
                const int realIdxKF = s_kfi[ia];
                if (s_mp[realIdxKF] < 0) continue;
                const uint4 k0 = s_kd[2 * realIdxKF], k1 = s_kd[2 * realIdxKF + 1];
                unsigned long long b1 = ~0ull, b2 = ~0ull, r1 = ~0ull;
#pragma unroll
                for (int c = 0; c < FQ; c++) {
                    if ((taken >> c) & 1u) continue;
                    const int dist = __popc(k0.x ^ fd0[c].x) + __popc(k0.y ^ fd0[c].y) + __popc(k0.z ^ fd0[c].z) +
                                     __popc(k0.w ^ fd0[c].w) + __popc(k1.x ^ fd1[c].x) + __popc(k1.y ^ fd1[c].y) +
                                     __popc(k1.z ^ fd1[c].z) + __popc(k1.w ^ fd1[c].w);
                    const unsigned long long key = ((unsigned long long)dist << 32) | (unsigned)(4 * c + sl);
                    if ((isleft >> c) & 1u) {
                        if (key < b1) { b2 = b1; b1 = key; }
                        else if (key < b2) b2 = key;
                    } else if (key < r1) {
                        r1 = key;
                    }
                }
                const unsigned long long m1 = quad_min64(b1);
                const unsigned long long m2 = quad_min64(b1 == m1 ? b2 : b1);
                const unsigned long long mr = quad_min64(r1);
                const int bestDist1 = m1 != ~0ull ? (int)(m1 >> 32) : 256;
                const int bestDist2 = m2 != ~0ull ? (int)(m2 >> 32) : 256;
                const int bestDist1R = mr != ~0ull ? (int)(mr >> 32) : 256;
                int w1 = -1, wr = -1;   // winning positions
                if (bestDist1 <= MT_TH_LOW) {
                    if (static_cast<float>(bestDist1) < in.nnratio * static_cast<float>(bestDist2)) w1 = (int)(m1 & 0xFFFFFFFFu);
                    if (bestDist1R <= MT_TH_LOW) wr = (int)(mr & 0xFFFFFFFFu);
                }
#pragma unroll
                for (int c = 0; c < FQ; c++) {
                    if (w1 == 4 * c + sl || wr == 4 * c + sl) {
                        taken |= 1u << c;
                        s_src[fidx[c]] = realIdxKF;
                    }
                }
            }
            continue;
        }
        // larger nodes: the F features and their flags read from LDS per KF feature
        for (int ia = ka0; ia < ka1; ia++) {
            const int realIdxKF = s_kfi[ia];
            if (s_mp[realIdxKF] < 0) continue;
            const uint4 k0 = s_kd[2 * realIdxKF], k1 = s_kd[2 * realIdxKF + 1];
            unsigned long long b1 = ~0ull, b2 = ~0ull, r1 = ~0ull;
            for (int ib = fb0 + sl; ib < fb1; ib += 4) {
                const int realIdxF = s_fi[ib];
                if (s_src[realIdxF] >= 0) continue;
                const uint4 f0 = s_fd[2 * realIdxF], f1 = s_fd[2 * realIdxF + 1];
                const int dist = __popc(k0.x ^ f0.x) + __popc(k0.y ^ f0.y) + __popc(k0.z ^ f0.z) + __popc(k0.w ^ f0.w) +
                                 __popc(k1.x ^ f1.x) + __popc(k1.y ^ f1.y) + __popc(k1.z ^ f1.z) + __popc(k1.w ^ f1.w);
                const unsigned long long key = ((unsigned long long)dist << 32) | (unsigned)ib;
                if (in.nleft < 0 || realIdxF < in.nleft) {
                    if (key < b1) { b2 = b1; b1 = key; }
                    else if (key < b2) b2 = key;
                } else if (key < r1) {
                    r1 = key;
                }
            }
            const unsigned long long m1 = quad_min64(b1);
            const unsigned long long m2 = quad_min64(b1 == m1 ? b2 : b1);
            const unsigned long long mr = quad_min64(r1);
            if (sl == 0) {
                const int bestDist1 = m1 != ~0ull ? (int)(m1 >> 32) : 256;
                const int bestDist2 = m2 != ~0ull ? (int)(m2 >> 32) : 256;
                const int bestDist1R = mr != ~0ull ? (int)(mr >> 32) : 256;
                if (bestDist1 <= MT_TH_LOW) {
                    if (static_cast<float>(bestDist1) < in.nnratio * static_cast<float>(bestDist2))
                        s_src[s_fi[(int)(m1 & 0xFFFFFFFFu)]] = realIdxKF;
                    if (bestDist1R <= MT_TH_LOW) s_src[s_fi[(int)(mr & 0xFFFFFFFFu)]] = realIdxKF;
                }
            }
            WAVE_SYNC();   // the quad's next KF feature sees the taken F features
        }
    }
    SYNC();
    BOW_STAMP(2);
    // rotation consistency (ORBmatcher.cc:373-395) and the output (k_bow_commit); F's angles were
    // loaded at the start
    int sidx[MT_BOW_FR], bin[MT_BOW_FR];
#pragma unroll
    for (int u = 0; u < MT_BOW_FR; u++) {
        const int i = tid + u * MT_BOW_NT;
        sidx[u] = i < in.fn ? s_src[i] : -1;
        bin[u] = sidx[u] >= 0 ? mt_rot_bin(s_kk[sidx[u]].angle, fang[u]) : 0;
        if (sidx[u] >= 0 && in.checkOri) atomicAdd(&s_hist[bin[u]], 1);
    }
    SYNC();
    if (tid == 0) s_keep = in.checkOri ? mt_three_maxima_keep(s_hist) : 0xFFFFFFFFu;
    SYNC();
    int cnt = 0;
#pragma unroll
    for (int u = 0; u < MT_BOW_FR; u++) {
        const int i = tid + u * MT_BOW_NT;
        if (i >= in.fn) continue;
        int o = -1;
        if (sidx[u] >= 0 && (!in.checkOri || ((s_keep >> bin[u]) & 1u))) o = s_mp[sidx[u]];
        out[i] = o;
        cnt += o >= 0 ? 1 : 0;
    }
    atomicAdd(&s_n, cnt);
    // every wave's output stores complete (vmcnt 0), the barrier, then one system-scope release before
    // the status words the host waits for (as k_sbp_block)
    __builtin_amdgcn_s_waitcnt(0);
    SYNC();
    if (tid == 0) {
        result[0] = s_n;
        __threadfence_system();
        volatile int* st = in.st_host;
        st[0] = 0;
        st[1] = s_n;
        __threadfence_system();
        st[4] = in.seq;
        __threadfence_system();
    }
#ifdef ORBFE_BOW_STAMPS
    BOW_STAMP(3);
    if (tid == 0)   // s_memrealtime ticks at 100 MHz
        printf("bow npairs %d kf %d f %d nvec %d  stage %.1f walk %.1f commit %.1f us\n", in.npairs, in.kf_n, in.fn,
               in.nvec, (t_st[1] - t_st[0]) * 0.01, (t_st[2] - t_st[1]) * 0.01, (t_st[3] - t_st[2]) * 0.01);
#endif
}

// ---- ComputeStereoFishEyeMatches' knnMatch(k=2) + ratio (Frame.cc:1144-1151) ----
__global__ __launch_bounds__(MT_NT) void k_knn2(const uint32_t* L, int nl, const uint32_t* R, int nr, float ratio,
                                                int* out_train, int* out_dist) {
    __shared__ uint32_t s_r[MT_NT * 8];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t d[8];
#pragma unroll
    for (int w = 0; w < 8; w++) d[w] = i < nl ? L[8 * i + w] : 0u;
    int d0 = MT_INF, d1 = MT_INF, t0 = -1;
    for (int base = 0; base < nr; base += MT_NT) {
        SYNC();
        for (int k = threadIdx.x; k < MT_NT * 8; k += blockDim.x) s_r[k] = (base * 8 + k < nr * 8) ? R[base * 8 + k] : 0u;
        SYNC();
        const int lim = min(MT_NT, nr - base);
        for (int jj = 0; jj < lim; jj++) {
            int dist = 0;
#pragma unroll
            for (int w = 0; w < 8; w++) dist += __popc(d[w] ^ s_r[8 * jj + w]);
            if (dist < d0) { d1 = d0; d0 = dist; t0 = base + jj; }
            else if (dist < d1) d1 = dist;
        }
    }
    if (i < nl) {
        const bool ok = nr >= 2 && (float)d0 < (float)d1 * (double)ratio;
        out_train[i] = ok ? t0 : -1;
        out_dist[i] = ok ? d0 : -1;
    }
}

// Batched form of the same descriptor stage over the extractor's device outputs: frame f's queries
// are rows [monoL, nL) of left image (lbase + f lstep), its train set rows [monoR, nR) of right
// image (rbase + f rstep) (ComputeStereoFishEyeMatches' stereoDescLeft / stereoDescRight,
// Frame.cc:1129-1133). One 256-thread block per (frame, 64 query slots): the frame's train rows
// are staged in LDS once per block, each wave scans a quarter of them for the same 64 queries
// (LDS broadcast reads), and the four partial top-2 lists are merged in train order so ties keep
// the earlier train row (cv::BFMatcher's strict-less insertion). Outputs in the frame's full keypoint
// numbering: l2r[f][i] = right keypoint index (trainIdx + monoRight) when Lowe's test passes, else -1;
// dist[f][i] its Hamming distance or -1; ngood[f] += passed queries (zeroed by the launcher).
// W waves per block split the train rows: 4 for batches (the grid fills the machine), 16 for a few
// frames (the one-frame fisheye Frame: 16 blocks would otherwise leave each lane a 250-row chain)
#define KNN_Q 64
template <int W>
__global__ __launch_bounds__(64 * W) void k_knn2_batch(StereoSide SL, StereoSide SR, int cap, float ratio,
                                                       int* __restrict__ l2r, int* __restrict__ dist, int* ngood) {
    extern __shared__ __attribute__((aligned(16))) uint32_t s_train[];   // [cap][8]
    __shared__ int s_part[W][KNN_Q][3];
    const int f = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int li = SL.base + f * SL.step, ri = SR.base + f * SR.step;
    const int nL = SL.counts[2 * li], monoL = SL.counts[2 * li + 1];
    const int nR = SR.counts[2 * ri], monoR = SR.counts[2 * ri + 1];
    const int q = blockIdx.x * KNN_Q + lane;
    int* o_t = l2r + (size_t)f * cap;
    int* o_d = dist + (size_t)f * cap;
    const int q0 = max(blockIdx.x * KNN_Q, monoL), q1 = min(blockIdx.x * KNN_Q + KNN_Q, nL);
    if (q0 >= q1) {   // no query in this slot range: only the -1 fill
        if (wave == 0 && q < cap) { o_t[q] = -1; o_d[q] = -1; }
        return;
    }
    const int nt = max(nR - monoR, 0);
    const uint32_t* rdesc = (const uint32_t*)(SR.desc + ((size_t)ri * cap + monoR) * 32);
    for (int k = threadIdx.x; k < nt * 8; k += 64 * W) s_train[k] = rdesc[k];
    const bool valid = q >= monoL && q < nL;
    uint32_t d[8];
    const uint32_t* ld = (const uint32_t*)(SL.desc + ((size_t)li * cap + (valid ? q : q0)) * 32);
#pragma unroll
    for (int w = 0; w < 8; w++) d[w] = ld[w];
    SYNC();
    const int j0 = (int)((long)nt * wave / W), j1 = (int)((long)nt * (wave + 1) / W);
    int d0 = MT_INF, d1 = MT_INF, t0 = -1;
    for (int j = j0; j < j1; j++) {
        const uint4 a = *(const uint4*)&s_train[8 * j];
        const uint4 b = *(const uint4*)&s_train[8 * j + 4];
        int dd = __popc(d[0] ^ a.x) + __popc(d[1] ^ a.y) + __popc(d[2] ^ a.z) + __popc(d[3] ^ a.w) +
                 __popc(d[4] ^ b.x) + __popc(d[5] ^ b.y) + __popc(d[6] ^ b.z) + __popc(d[7] ^ b.w);
        if (dd < d0) { d1 = d0; d0 = dd; t0 = j; }
        else if (dd < d1) d1 = dd;
    }
    s_part[wave][lane][0] = d0;
    s_part[wave][lane][1] = d1;
    s_part[wave][lane][2] = t0;
    SYNC();
    if (wave == 0) {
        // merge the later ranges into the running top-2: a later row wins only when strictly closer
        for (int w = 1; w < W; w++) {
            const int b0 = s_part[w][lane][0], b1 = s_part[w][lane][1], bt = s_part[w][lane][2];
            if (b0 < d0) { d1 = min(d0, b1); d0 = b0; t0 = bt; }
            else d1 = min(d1, b0);
        }
        if (q < cap) {
            // (*it).size() >= 2 && d0 < d1 * 0.7 (DMatch distances are float; the product in double, as k_knn2)
            const bool ok = valid && nt >= 2 && (float)d0 < (float)d1 * (double)ratio;
            o_t[q] = ok ? t0 + monoR : -1;
            o_d[q] = ok ? d0 : -1;
            const unsigned long long m = __ballot(ok);
            if (lane == 0 && m) atomicAdd(ngood + f, (int)__popcll(m));
        }
    }
}

// =============================================================================================
// Host side (compiled in the engine TU after HIPCHK is defined).
// Every call is synchronous from the caller's point of view (the reference methods return
// nmatches), stateless and re-entrant: each calling thread owns a device arena, a pinned staging
// buffer and a non-blocking stream (Tracking, LocalMapping and LoopClosing call the matcher
// concurrently in the reference). All host inputs are packed into the pinned buffer and uploaded
// with ONE copy; results come back with one copy per output array.
// =============================================================================================
namespace {

// The zero-copy status words: a commit kernel stores the slots and st[0..3,5], fences at system
// scope, then stores the sequence word st[4]. The host spin reads st[4] with ACQUIRE semantics, so
// neither the compiler nor the CPU may move the later reads of the slots (memcpy from the mapped
// block) or of st[0..5] above the read that saw the new sequence number.
inline int host_seq_acquire(volatile int* st) { return __atomic_load_n((int*)&st[4], __ATOMIC_ACQUIRE); }

struct MatchScratch {
    int device = -1;
    // the last fused local-map search's isInFrustum records (device arena) and their count, for
    // orbfe_search_local_points_track's read-back
    const orbfe_map_point* last_track = nullptr;
    int last_track_n = 0;
    orbfe_map_point* th = nullptr;       // mapped pinned track records (orbfe_search_local_points_track)
    orbfe_map_point* th_dev = nullptr;
    size_t th_cap = 0;
    hipStream_t stream = nullptr;
    uint8_t* d = nullptr;
    size_t dcap = 0;
    uint8_t* h = nullptr;   // pinned
    size_t hcap = 0;
    uint8_t* hd = nullptr;  // h as the device addresses it (mapped): the zero-copy inputs of k_sbp_block
    int32_t* ho = nullptr;  // pinned, mapped: k_sbp_block's slot results
    int32_t* ho_dev = nullptr;
    size_t ocap = 0;
    int* hs = nullptr;      // pinned status words read back at the end of a call
    int* hs_dev = nullptr;  // hs as the device addresses it (kernels store the status there)
    int seq = 0;            // sequence number of the last published status
    int pass_hint[3] = {4, 4, 4};   // passes the previous single-camera search of each mode needed
    // A device-resident search returns as soon as its status words are published, before its last
    // commit block has retired (and reset its completion counter): `tail` is recorded on its stream
    // after the last launch, and the next call of this thread orders its own stream after it when
    // that is a different stream (ms_after_tail), so the shared scratch is never reused early.
    hipEvent_t tail = nullptr;
    hipStream_t tail_stream = nullptr;
    // sbp_multi_run's persistent state (MultiBuf), the generation of the next call's pass 0 (tags of
    // 0 never match) and whether an unfinished call may have left its counters set
    uint8_t* mbuf = nullptr;
    unsigned long long gen = MT_MAX_PASSES;
    bool mdirty = false;
    // Deliberately never freed: thread_local destructors of the main thread can run after the HIP
    // runtime has been torn down at exit; the arena is reused for the thread's lifetime.
};
thread_local MatchScratch t_ms;

// Optional per-thread device timing of matcher calls (orbfe_matcher_set_timing): events bracket
// the kernels of a call on the thread's stream (after the input upload, before the result copy).
thread_local bool t_timing = false;
// orbfe_matcher_set_stats: window candidates / Hamming pairs / passes of the last counted search
thread_local bool t_stats = false;
thread_local long long t_last_stats[3] = {-1, -1, -1};
thread_local float t_last_ms = -1.f;
thread_local hipEvent_t t_ev[2] = {nullptr, nullptr};
struct MsTimer {
    bool on = false, ended = false;
    hipStream_t s;
    explicit MsTimer(hipStream_t stream = t_ms.stream) : s(stream) {
        t_last_ms = -1.f;
        if (!t_timing) return;
        if (!t_ev[0] && (hipEventCreate(&t_ev[0]) != hipSuccess || hipEventCreate(&t_ev[1]) != hipSuccess)) return;
        on = hipEventRecord(t_ev[0], s) == hipSuccess;
    }
    void end() {
        if (on) ended = hipEventRecord(t_ev[1], s) == hipSuccess;
    }
    ~MsTimer() {
        float ms = 0.f;
        if (ended && hipEventSynchronize(t_ev[1]) == hipSuccess && hipEventElapsedTime(&ms, t_ev[0], t_ev[1]) == hipSuccess)
            t_last_ms = ms;
    }
};

struct Plan {
    struct Up { const void* src; size_t bytes; size_t off; };
    std::vector<Up> ups;
    size_t up_end = 0, end = 0;
    static size_t a256(size_t b) { return (b + 255) & ~(size_t)255; }
    size_t upload(const void* src, size_t bytes) {   // all uploads must be planned before scratch
        const size_t o = end;
        ups.push_back(Up{src, bytes, o});
        end += a256(bytes);
        up_end = end;
        return o;
    }
    size_t scratch(size_t bytes) { const size_t o = end; end += a256(bytes); return o; }
};

// order stream s after the previous device-resident search of this thread (see MatchScratch::tail)
hipError_t ms_after_tail(hipStream_t s) {
    if (t_ms.tail_stream && t_ms.tail_stream != s) return hipStreamWaitEvent(s, t_ms.tail, 0);
    return hipSuccess;
}

int ms_prepare(const Plan& p, bool zero_copy = false) {
    MatchScratch& m = t_ms;
    int dev = 0;
    HIPCHK(hipGetDevice(&dev));
    if (m.device != dev) {   // new thread or device switch: fresh resources on this device
        m = MatchScratch();
        m.device = dev;
        HIPCHK(hipStreamCreateWithFlags(&m.stream, hipStreamNonBlocking));
        HIPCHK(hipHostMalloc((void**)&m.hs, 128, hipHostMallocMapped | hipHostMallocCoherent));
        // the status words are compared against sequence numbers: start from zeros, not from
        // whatever the allocation held
        memset(m.hs, 0, 128);
        HIPCHK(hipHostGetDevicePointer((void**)&m.hs_dev, m.hs, 0));
        HIPCHK(hipEventCreateWithFlags(&m.tail, hipEventDisableTiming));
    }
    HIPCHK(ms_after_tail(m.stream));
    if (p.end > m.dcap) {
        if (m.d) HIPCHK(hipFree(m.d));
        m.d = nullptr;
        const size_t cap = std::max<size_t>(p.end + p.end / 2, 1 << 20);
        HIPCHK(hipMalloc(&m.d, cap));
        m.dcap = cap;
    }
    if (p.up_end > m.hcap) {
        if (m.h) HIPCHK(hipHostFree(m.h));
        m.h = nullptr;
        const size_t cap = std::max<size_t>(p.up_end + p.up_end / 2, 1 << 20);
        // mapped and fine-grained as well: the one-workgroup searches read their inputs from here
        // directly, uncached, so a later call never sees an earlier call's lines
        HIPCHK(hipHostMalloc((void**)&m.h, cap, hipHostMallocMapped | hipHostMallocCoherent));
        m.hcap = cap;
        HIPCHK(hipHostGetDevicePointer((void**)&m.hd, m.h, 0));
    }
    for (const auto& u : p.ups)
        if (u.bytes) memcpy(m.h + u.off, u.src, u.bytes);
    if (p.up_end && !zero_copy) HIPCHK(hipMemcpyAsync(m.d, m.h, p.up_end, hipMemcpyHostToDevice, m.stream));
    return ORBFE_OK;
}

template <typename T> T* ms_ptr(size_t off) { return reinterpret_cast<T*>(t_ms.d + off); }
// an uploaded input: the device arena copy, or (zero copy) the mapped pinned staging itself
template <typename T> T* up_ptr(size_t off, bool zc) { return reinterpret_cast<T*>((zc ? t_ms.hd : t_ms.d) + off); }

// Upload a frame and plan its grid; returns the device view after ms_prepare (fill_frame).
struct FramePlan {
    const orbfe_frame* F;
    size_t keys, desc, uright, scale, cstart, cidx, l2r = 0, r2l = 0;
    bool has_uright;
    bool two = false;   // Nleft != -1: left + right grids, l2r / r2l uploaded
    void plan(Plan& p, const orbfe_frame* f, bool want_grid, bool want_uright) {
        F = f;
        two = f->two_cams != 0;
        keys = p.upload(f->keys, (size_t)f->n * sizeof(orbfe_keypoint));
        desc = p.upload(f->desc, (size_t)f->n * 32);
        has_uright = !two && want_uright && f->uright != nullptr;
        uright = has_uright ? p.upload(f->uright, (size_t)f->n * 4) : 0;
        scale = p.upload(f->scale_factors, (size_t)f->nlevels * 4);
        if (two) {
            l2r = p.upload(f->l2r, (size_t)f->nleft * 4);
            r2l = p.upload(f->r2l, (size_t)(f->n - f->nleft) * 4);
        }
        (void)want_grid;
    }
    int ngrids = 1;
    int gfirst = 0;   // grids below gfirst are not built (a search that reads only level grids)
    // k_sbp_band's (octave, band) index, built by the grid launch when planned (plan_band)
    bool band = false;
    int band_nb = 0;
    size_t bstart = 0, bidx = 0;
    void plan_band(Plan& p) {
        band = true;
        band_nb = std::min(std::max((int)std::floor(F->max_y * (1.0f / MT_BAND_ROWS)) + 2, 1), 4096);
        bstart = p.scratch((size_t)(F->nlevels * band_nb + 1) * 4);
        bidx = p.scratch((size_t)std::max(F->n, 1) * 4);
    }
    int cells() const { return (two ? 2 : 1) * MT_NCELL; }
    void plan_grid(Plan& p, int grids) {   // grids = 1 (full) + level-restricted grids
        ngrids = grids;
        cstart = p.scratch((size_t)grids * (cells() + 1) * 4);
        cidx = p.scratch((size_t)grids * std::max(F->n, 1) * 4);
    }
    // device-resident frame: F's arrays are already device pointers (no upload)
    bool dev = false;
    void plan_dev(const orbfe_frame* f, bool want_uright) {
        F = f;
        dev = true;
        two = f->two_cams != 0;
        has_uright = !two && want_uright && f->uright != nullptr;
    }
    bool zc = false;   // uploads read in place from the mapped pinned staging (no DMA)
    FrameDev view() const {
        FrameDev v;
        v.n = F->n;
        v.keys = dev ? (const OrbKeyPoint*)F->keys : up_ptr<const OrbKeyPoint>(keys, zc);
        v.desc = dev ? (const uint32_t*)F->desc : up_ptr<const uint32_t>(desc, zc);
        v.uright = has_uright ? (dev ? F->uright : up_ptr<const float>(uright, zc)) : nullptr;
        v.minx = F->min_x; v.maxx = F->max_x; v.miny = F->min_y; v.maxy = F->max_y;
        // mfGridElementWidthInv / HeightInv (Frame.cc:163-164)
        v.invw = static_cast<float>(ORBFE_GRID_COLS) / (F->max_x - F->min_x);
        v.invh = static_cast<float>(ORBFE_GRID_ROWS) / (F->max_y - F->min_y);
        v.mbf = F->mbf;
        v.nlevels = F->nlevels;
        v.scale = dev ? F->scale_factors : up_ptr<const float>(scale, zc);
        v.cstart = ms_ptr<const int>(cstart);
        v.cidx = ms_ptr<const int>(cidx);
        v.gstride_c = cells() + 1;
        v.gstride_i = std::max(F->n, 1);
        v.pcstart = v.cstart + v.gstride_c;
        v.pcidx = v.cidx + v.gstride_i;
        v.nleft = two ? F->nleft : -1;
        v.l2r = two ? (dev ? F->l2r : up_ptr<const int>(l2r, zc)) : nullptr;
        v.r2l = two ? (dev ? F->r2l : up_ptr<const int>(r2l, zc)) : nullptr;
        return v;
    }
    // the grids on the thread's matcher stream, or on stream s; with `init`, the same launch also
    // runs the search initialisation in extra blocks
    void launch_grid(const FrameDev& v) const { launch_grid_on(v, t_ms.stream, nullptr); }
    void launch_grid_on(const FrameDev& v, hipStream_t s, const SbpInit* init) const {
        SbpInit none;
        memset(&none, 0, sizeof(none));
        const SbpInit& ia = init ? *init : none;
        const int nib = (sbp_init_extent(ia) + 1023) / 1024;
        BandGrid bg{nullptr, nullptr, 0, 0};
        if (band) bg = BandGrid{ms_ptr<int>(bstart), ms_ptr<int>(bidx), band_nb, F->nlevels};
        hipLaunchKernelGGL(k_mt_grid, dim3(ngrids - gfirst + (band ? 1 : 0) + nib), dim3(1024), 0, s, v.keys, v.n,
                           v.nleft, v.minx, v.miny, v.invw, v.invh, (int*)v.cstart, (int*)v.cidx, v.gstride_c,
                           v.gstride_i, ngrids, ia, bg, gfirst);
    }
};

// device views (orbfe_frame_device_view) are taken by sbp_run's one-workgroup path only
bool frame_ok(const orbfe_frame* f) {
    return f && !f->device && f->n >= 0 && f->n <= MT_GRID_MAXN && (f->n == 0 || (f->keys && f->desc)) && f->scale_factors &&
           f->nlevels > 0 &&
           (!f->two_cams || (f->nleft >= 0 && f->nleft <= f->n && (f->nleft == 0 || f->l2r) &&
                             (f->nleft == f->n || f->r2l)));
}
// single-camera frames only: the back-end matchers and SearchForInitialization restate the
// reference's Nleft == -1 branches
bool frame1_ok(const orbfe_frame* f) { return frame_ok(f) && !f->two_cams; }
// host check of a two-camera frame's stereo links (they index slots)
bool links_ok(const orbfe_frame* f) {
    if (!f->two_cams) return true;
    const int nr = f->n - f->nleft;
    for (int i = 0; i < f->nleft; i++)
        if (f->l2r[i] < -1 || f->l2r[i] >= nr) return false;
    for (int i = 0; i < nr; i++)
        if (f->r2l[i] < -1 || f->r2l[i] >= f->nleft) return false;
    return true;
}

inline void fill(int* p, int n, int v, hipStream_t s = t_ms.stream) {
    if (n > 0) hipLaunchKernelGGL(k_mt_fill, dim3((n + 255) / 256), dim3(256), 0, s, p, n, v);
}

// Shared driver of the three slot-assigning SearchByProjection variants.
// mode: 0 local map, 1 last frame, 2 keyframe.
// Local-map projection feeding sbp_run (mode 0): the query records are produced on the device by
// k_frustum from map point geometry instead of being uploaded.
struct FrustumIn {
    const orbfe_camera* cam;
    const orbfe_map_point_3d* pts;
    int32_t* n_to_match;
    const orbfe_stereo_rig* rig;   // camera models / right view (NULL: pinhole from cam, one camera)
    orbfe_map_point* track_dev = nullptr;   // mapped host copy of the isInFrustum records (device view)
};

// isInFrustum's per-frame constants (Frame.cc:512-586, 1168-1242): pose, bounds, camera models and,
// for a two-camera frame, the right view's pose in the reference's Eigen order. false = bad input.
bool make_camdev(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig, CamDev& cd) {
    if (!F || !cam || (F->two_cams && !rig)) return false;
    memset(&cd, 0, sizeof(cd));
    memcpy(cd.R, cam->Rcw, sizeof(cd.R));
    memcpy(cd.t, cam->tcw, sizeof(cd.t));
    memcpy(cd.Ow, cam->Ow, sizeof(cd.Ow));
    cd.logsf = cam->log_scale_factor;
    cd.cos_limit = cam->view_cos_limit;
    cd.minx = F->min_x; cd.maxx = F->max_x; cd.miny = F->min_y; cd.maxy = F->max_y;
    cd.mbf = F->mbf;
    cd.nlevels = F->nlevels;
    auto model = [](const orbfe_camera_model& m, CamModelDev& o) {
        if (m.type != ORBFE_CAM_PINHOLE && m.type != ORBFE_CAM_KANNALA_BRANDT8) return false;
        o.type = m.type;
        o.fx = m.params[0]; o.fy = m.params[1]; o.cx = m.params[2]; o.cy = m.params[3];
        for (int k = 0; k < 4; k++) o.k[k] = m.type == ORBFE_CAM_KANNALA_BRANDT8 ? m.params[4 + k] : 0.f;
        return true;
    };
    if (rig) {
        if (!model(rig->left, cd.cl)) return false;
    } else {
        cd.cl.type = ORBFE_CAM_PINHOLE;
        cd.cl.fx = cam->fx; cd.cl.fy = cam->fy; cd.cl.cx = cam->cx; cd.cl.cy = cam->cy;
    }
    cd.two = F->two_cams ? 1 : 0;
    if (cd.two) {
        if (!model(rig->right, cd.cr)) return false;
        const float* A = rig->Rrl;
        for (int i = 0; i < 3; i++) {
            for (int j = 0; j < 3; j++)   // mR = Rrl * mRcw
                cd.R2[3 * i + j] = eig_sum3(A[3 * i] * cam->Rcw[j], A[3 * i + 1] * cam->Rcw[3 + j], A[3 * i + 2] * cam->Rcw[6 + j]);
            cd.t2[i] = eig_sum3(A[3 * i] * cam->tcw[0], A[3 * i + 1] * cam->tcw[1], A[3 * i + 2] * cam->tcw[2]) + rig->trl[i];
            cd.Ow2[i] = eig_sum3(rig->Rwc[3 * i] * rig->tlr[0], rig->Rwc[3 * i + 1] * rig->tlr[1],
                                 rig->Rwc[3 * i + 2] * rig->tlr[2]) + cam->Ow[i];
        }
    }
    return true;
}

// Device-resident call (the *_device entry points): F's arrays, mvp, mvp_obs and the query
// records are device pointers produced on `caller`; the matcher's stream waits for it, results
// are written in place and the call returns after they are complete.
struct DevIn {
    hipStream_t caller;
};

// k_sbp_block's bucket geometry for a frame: bands of 16 rows, then as many column strips (<= 32, >= 24
// columns wide) as 8192 buckets and the LDS allow; false: the frame does not fit the block form
// (ncam = 2: both cameras' bucket sets, k_sbp_block2 / k_sbp_block4; bpk: LDS bytes per keypoint)
size_t blk_lds(int n, int nlev, const BlkGeom& gm, int ncam = 1, int bpk = 61) {
    return (size_t)n * bpk + (size_t)blk_be_words(ncam * nlev * gm.NB * gm.NS, MT_BLK_NT) * 4 + 16;
}
bool blk_geom(const orbfe_frame* F, BlkGeom& gm, int ncam = 1, int bpk = 61) {
    constexpr int BR = 16;
    if (!(F->max_y > 0.f && F->max_y < 65536.f && F->max_x > 0.f && F->max_x < 65536.f)) return false;
    gm.NB = (int)std::floor(F->max_y / BR) + 2;
    gm.inv_br = 1.0f / BR;
    const int lev_bands = ncam * F->nlevels * gm.NB;
    const long budget = std::min<long>(8192, ((long)MT_LDS_MAX - (long)bpk * F->n - 4) / 4);
    gm.NS = (int)std::min<long>(std::min<long>(32, budget / std::max(lev_bands, 1)), (long)std::ceil(F->max_x / 24.f));
    if (gm.NS < 1) return false;
    while (gm.NS > 1 && blk_lds(F->n, F->nlevels, gm, ncam, bpk) > MT_LDS_MAX) gm.NS--;   // the scan's padding
    gm.inv_sw = (float)gm.NS / (F->max_x + 1.f);
    return blk_lds(F->n, F->nlevels, gm, ncam, bpk) <= MT_LDS_MAX;
}

// sbp_run's one-launch form (k_sbp_block, k_sbp_block4): arguments already validated by sbp_run.
// kBlockAborted: k_sbp_block4 gave up (more writers of one slot than it tracks) before writing
// anything; the caller runs the multi-launch form.
constexpr int kBlockAborted = -1000;
int sbp_block_run(int mode, const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs, const void* queries, int nq,
                  size_t qstride, size_t qid_off, size_t qangle_off, float th, int a0, int a1, float thFar,
                  float nnratio, int maxDist, int checkOri, const BlkGeom& gm, const FrustumIn* fin, const DevIn* dev,
                  const LastProjIn* lp = nullptr) {
    const int n = F->n;
    Plan p;
    FramePlan fp;
    if (dev || F->device) fp.plan_dev(F, mode != 2);   // a device frame: read in place
    else fp.plan(p, F, true, mode != 2);
    const size_t o_q = dev ? 0 : fin ? p.upload(fin->pts, (size_t)nq * sizeof(orbfe_map_point_3d))
                                     : lp ? p.upload(lp->pts, (size_t)nq * sizeof(orbfe_last_point))
                                          : p.upload(queries, (size_t)nq * qstride);
    const size_t o_rec = lp ? p.scratch((size_t)nq * sizeof(orbfe_proj_point)) : 0;   // device-projected records
    const size_t o_mvp = dev ? 0 : p.upload(mvp, (size_t)n * 4);
    const size_t o_obs = (dev || mode == 2) ? 0 : p.upload(mvp_obs, (size_t)n * 4);
    const size_t o_track = fin ? p.scratch((size_t)nq * sizeof(orbfe_map_point)) : 0;
    const size_t o_ntm = fin ? p.scratch(16) : 0;
    const size_t o_stats = t_stats ? p.scratch(24) : 0;
#ifndef ORBFE_BLK_DMA
#define ORBFE_BLK_DMA 0
#endif
    // host-API calls: zero copy both ways. The kernel reads its inputs straight from the mapped pinned
    // staging and writes the slots into mapped pinned memory; the host waits for the status words
    // only (no DMA, no stream synchronisation: the call is one launch). (ORBFE_BLK_DMA: inputs by one
    // DMA instead, an A/B build.)
    const bool zc = !dev, zin = zc && !ORBFE_BLK_DMA;
    const size_t o_qdev = (!dev && !fin && !lp && zin) ? p.scratch((size_t)nq * qstride) : 0;
    int rc = ms_prepare(p, zin);
    if (rc) return rc;
    MatchScratch& m = t_ms;
    if (zc && m.ocap < (size_t)n) {
        if (m.ho) HIPCHK(hipHostFree(m.ho));
        m.ho = nullptr;
        m.ocap = 0;
        const size_t cap = std::max<size_t>((size_t)n, 2048);
        HIPCHK(hipHostMalloc((void**)&m.ho, cap * 4, hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&m.ho_dev, m.ho, 0));
        m.ocap = cap;
    }
    fp.zc = zin;
    hipStream_t s = dev ? dev->caller : t_ms.stream;
    if (dev) HIPCHK(ms_after_tail(s));
    unsigned long long* stats = t_stats ? ms_ptr<unsigned long long>(o_stats) : nullptr;
    t_last_stats[0] = t_last_stats[1] = t_last_stats[2] = -1;
    if (stats) HIPCHK(hipMemsetAsync(stats, 0, 24, s));
    MsTimer timer(s);
    const FrameDev fr = fp.view();
    const uint8_t* q = dev ? (const uint8_t*)(fin ? (const void*)fin->pts : queries) : up_ptr<const uint8_t>(o_q, zin);
    int* ntm = fin ? ms_ptr<int>(o_ntm) : nullptr;
    if (fin) {   // Tracking::SearchLocalPoints' isInFrustum, then the search (nothing in view: no match)
        CamDev cd;
        if (!make_camdev(F, fin->cam, fin->rig, cd)) return ORBFE_E_ARG;
        HIPCHK(hipMemsetAsync(ntm, 0, 4, s));
        hipLaunchKernelGGL(k_frustum, dim3((nq + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, cd,
                           (const orbfe_map_point_3d*)q, nq, ms_ptr<orbfe_map_point>(o_track), ntm, fin->track_dev);
        t_ms.last_track = ms_ptr<const orbfe_map_point>(o_track);
        t_ms.last_track_n = nq;
        q = ms_ptr<const uint8_t>(o_track);
        qstride = sizeof(orbfe_map_point);
        qid_off = offsetof(orbfe_map_point, id);
    }
    if (lp) {   // SearchByProjection(CurrentFrame, LastFrame)'s projection on the device
        hipLaunchKernelGGL(k_last_proj, dim3((nq + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, *lp,
                           up_ptr<const orbfe_last_point>(o_q, zin), nq, ms_ptr<orbfe_proj_point>(o_rec), (float2*)nullptr);
        q = ms_ptr<const uint8_t>(o_rec);
    }
    const int32_t* mvp_in = dev ? mvp : up_ptr<const int32_t>(o_mvp, zin);
    int32_t* mvp_out = dev ? mvp : m.ho_dev;
    const int32_t* obs_d = mode == 2 ? nullptr : dev ? mvp_obs : up_ptr<const int32_t>(o_obs, zin);
    const int seq = ++t_ms.seq;
    if (zc) memcpy(m.ho, mvp, (size_t)n * 4);   // the slots the search leaves alone keep their value
    const BlkIO io{mvp_in, obs_d, mvp_out, (int)qstride, (int)qid_off, (int)qangle_off, checkOri, ntm, t_ms.hs_dev, seq,
                   stats, (!dev && !fin && !lp && zin) ? ms_ptr<uint4>(o_qdev) : nullptr};
    const bool two4 = F->two_cams && mode == 0;
    const size_t lds = two4 ? blk_lds(n, F->nlevels, gm, 2, blk4_bytes_per_kp()) : blk_lds(n, F->nlevels, gm);
    if (two4)
        hipLaunchKernelGGL(k_sbp_block4, dim3(1), dim3(MT_BLK_NT), lds, s, fr, gm, (const orbfe_map_point*)q, nq, th, a0,
                           thFar, nnratio, io);
    else if (mode == 0)
        hipLaunchKernelGGL(k_sbp_block<0>, dim3(1), dim3(MT_BLK_NT), lds, s, fr, gm, (const void*)q, nq, th, a0, a1,
                           thFar, nnratio, maxDist, 1, io);
    else if (mode == 1)
        hipLaunchKernelGGL(k_sbp_block<1>, dim3(1), dim3(MT_BLK_NT), lds, s, fr, gm, (const void*)q, nq, th, a0, a1,
                           thFar, nnratio, maxDist, 1, io);
    else
        hipLaunchKernelGGL(k_sbp_block<2>, dim3(1), dim3(MT_BLK_NT), lds, s, fr, gm, (const void*)q, nq, th, a0, a1,
                           thFar, nnratio, maxDist, 0, io);
    HIPCHK(hipGetLastError());
    if (dev) {
        HIPCHK(hipEventRecord(t_ms.tail, s));
        t_ms.tail_stream = s;
    }
    timer.end();
    volatile int* st = t_ms.hs;
    for (unsigned spin = 1; host_seq_acquire(st) != seq; spin++) {
        if ((spin & 1023) == 0) {   // bounded: a stream that finished without publishing is an error
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess && host_seq_acquire(st) != seq) return ORBFE_E_DEVICE;
            if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
        }
        __builtin_ia32_pause();
    }
    if (st[0] == 2) return kBlockAborted;   // k_sbp_block4: a slot with too many writers, nothing written
    if (zc) memcpy(mvp, m.ho, (size_t)n * 4);   // complete: the status words come after the slot writes
    if (fin && fin->n_to_match) *fin->n_to_match = st[5];
    if (stats) {   // counting mode only: one more copy and synchronisation
        unsigned long long hst[3];
        HIPCHK(hipMemcpyAsync(hst, stats, 24, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        t_last_stats[0] = (long long)hst[0];
        t_last_stats[1] = (long long)hst[1];
        t_last_stats[2] = (long long)hst[2];
    }
    return st[1] - st[2];
}

// sbp_run's one-launch form for a two-camera frame's last-frame search (k_sbp_block2): host buffers
// read in place from the mapped pinned staging, slots written to mapped pinned memory, the status
// words awaited (as sbp_block_run); arguments already validated by sbp_run.
int sbp_block2_run(const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs, const orbfe_proj_point* pts,
                   const float* right_uv, int nq, float th, int a0, int a1, int maxDist, int checkOri,
                   const BlkGeom& gm, const LastProjIn* lp = nullptr) {
    const int n = F->n;
    Plan p;
    FramePlan fp;
    fp.plan(p, F, true, false);
    const size_t o_q = lp ? p.upload(lp->pts, (size_t)nq * sizeof(orbfe_last_point))
                          : p.upload(pts, (size_t)nq * sizeof(orbfe_proj_point));
    const size_t o_ruv = lp ? p.scratch((size_t)nq * 8) : p.upload(right_uv, (size_t)nq * 8);
    const size_t o_rec = lp ? p.scratch((size_t)nq * sizeof(orbfe_proj_point)) : 0;
    const size_t o_mvp = p.upload(mvp, (size_t)n * 4);
    const size_t o_obs = p.upload(mvp_obs, (size_t)n * 4);
    const size_t o_stats = t_stats ? p.scratch(24) : 0;
    const size_t o_qdev = lp ? 0 : p.scratch((size_t)nq * sizeof(orbfe_proj_point));
    int rc = ms_prepare(p, true);
    if (rc) return rc;
    MatchScratch& m = t_ms;
    if (m.ocap < (size_t)n) {
        if (m.ho) HIPCHK(hipHostFree(m.ho));
        m.ho = nullptr;
        m.ocap = 0;
        const size_t cap = std::max<size_t>((size_t)n, 2048);
        HIPCHK(hipHostMalloc((void**)&m.ho, cap * 4, hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&m.ho_dev, m.ho, 0));
        m.ocap = cap;
    }
    fp.zc = true;
    hipStream_t s = t_ms.stream;
    unsigned long long* stats = t_stats ? ms_ptr<unsigned long long>(o_stats) : nullptr;
    t_last_stats[0] = t_last_stats[1] = t_last_stats[2] = -1;
    if (stats) HIPCHK(hipMemsetAsync(stats, 0, 24, s));
    MsTimer timer(s);
    const FrameDev fr = fp.view();
    const int seq = ++t_ms.seq;
    memcpy(m.ho, mvp, (size_t)n * 4);   // the slots the search leaves alone keep their value
    const BlkIO io{up_ptr<const int32_t>(o_mvp, true), up_ptr<const int32_t>(o_obs, true), m.ho_dev,
                   (int)sizeof(orbfe_proj_point), (int)offsetof(orbfe_proj_point, id),
                   (int)offsetof(orbfe_proj_point, angle), checkOri, nullptr, t_ms.hs_dev, seq, stats,
                   lp ? nullptr : ms_ptr<uint4>(o_qdev)};
    const orbfe_proj_point* recs = up_ptr<const orbfe_proj_point>(o_q, true);
    const float2* ruv = up_ptr<const float2>(o_ruv, true);
    if (lp) {   // the projection into both cameras on the device; records and right centres in HBM
        recs = ms_ptr<const orbfe_proj_point>(o_rec);
        ruv = ms_ptr<const float2>(o_ruv);
        hipLaunchKernelGGL(k_last_proj, dim3((nq + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, *lp,
                           up_ptr<const orbfe_last_point>(o_q, true), nq, ms_ptr<orbfe_proj_point>(o_rec),
                           ms_ptr<float2>(o_ruv));
    }
    hipLaunchKernelGGL(k_sbp_block2, dim3(1), dim3(MT_BLK_NT), blk_lds(n, F->nlevels, gm, 2), s, fr, gm, recs, ruv, nq,
                       th, a0, a1, maxDist, io);
    HIPCHK(hipGetLastError());
    timer.end();
    volatile int* st = t_ms.hs;
    for (unsigned spin = 1; host_seq_acquire(st) != seq; spin++) {
        if ((spin & 1023) == 0) {   // bounded: a stream that finished without publishing is an error
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess && host_seq_acquire(st) != seq) return ORBFE_E_DEVICE;
            if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
        }
        __builtin_ia32_pause();
    }
    memcpy(mvp, m.ho, (size_t)n * 4);
    if (stats) {
        unsigned long long hst[3];
        HIPCHK(hipMemcpyAsync(hst, stats, 24, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        t_last_stats[0] = (long long)hst[0];
        t_last_stats[1] = (long long)hst[1];
        t_last_stats[2] = (long long)hst[2];
    }
    return st[1] - st[2];
}

// the multi-block local-map search's persistent state (MatchScratch::mbuf): generation-tagged arrays
// and self-resetting counters, zeroed once at allocation
struct MultiBuf {
    static constexpr size_t kFirst = (size_t)MT_BAND_MAXN * 8;
    static constexpr size_t off_first0 = 0, off_first1 = kFirst, off_lastw = 2 * kFirst;
    static constexpr size_t off_changed = 3 * kFirst;
    static constexpr size_t off_done = off_changed + (size_t)MT_MAX_PASSES * 8;
    static constexpr size_t off_cnt = off_done + (size_t)MT_MAX_PASSES * 4;
    static constexpr size_t off_nactive = off_cnt + (size_t)MT_MAX_PASSES * 4;
    static constexpr size_t counters = off_done, counters_bytes = off_nactive + 256 - off_done;
    static constexpr size_t bytes = off_nactive + 256;
};
size_t multi_lds(int n, int nlev, const BlkGeom& gm) {
    return (size_t)n * 49 + (size_t)blk_be_words(nlev * gm.NB * gm.NS, MT_BLK_NT) * 4 + 16;
}

// sbp_run's multi-block form for single-camera local-map searches of more than MT_BLOCK_MAXQ points
// (k_sbp_multi0 / k_sbp_multi): arguments already validated by sbp_run.
int sbp_multi_run(const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs, const void* queries, int nq,
                  size_t qstride, size_t qid_off, float th, int a0, float thFar, float nnratio, const BlkGeom& gm,
                  const FrustumIn* fin, const DevIn* dev) {
    const int n = F->n;
    const int nbk = F->nlevels * gm.NB * gm.NS;
    Plan p;
    FramePlan fp;
    if (dev) fp.plan_dev(F, true);
    else fp.plan(p, F, true, true);
    const size_t o_q = dev ? 0 : fin ? p.upload(fin->pts, (size_t)nq * sizeof(orbfe_map_point_3d))
                                     : p.upload(queries, (size_t)nq * qstride);
    const size_t o_mvp = dev ? 0 : p.upload(mvp, (size_t)n * 4);
    const size_t o_obs = dev ? 0 : p.upload(mvp_obs, (size_t)n * 4);
    const size_t o_track = fin ? p.scratch((size_t)nq * sizeof(orbfe_map_point)) : 0;
    const size_t o_ntm = fin ? p.scratch(16) : 0;
    const size_t o_assign = p.scratch((size_t)nq * 4);
    const size_t o_lists = p.scratch((size_t)nq * MT_BLK_LIST * 4);
    const size_t o_lcnt = p.scratch((size_t)nq * 4);
    const size_t o_active = p.scratch((size_t)nq * 4);
    const size_t o_gkp = p.scratch((size_t)n * 16);
    const size_t o_gdesc = p.scratch((size_t)n * 32);
    const size_t o_gbe = p.scratch((size_t)(nbk + 1) * 4);
    const size_t o_gblk = p.scratch((size_t)n);
    const size_t o_stats = t_stats ? p.scratch(24) : 0;
    int rc = ms_prepare(p);
    if (rc) return rc;
    MatchScratch& m = t_ms;
    hipStream_t s = dev ? dev->caller : m.stream;
    if (dev) HIPCHK(ms_after_tail(s));
    if (!m.mbuf) {   // zeroed on the search's stream (a non-blocking stream does not wait for the null stream)
        HIPCHK(hipMalloc(&m.mbuf, MultiBuf::bytes));
        HIPCHK(hipMemsetAsync(m.mbuf, 0, MultiBuf::bytes, s));
        m.mdirty = false;
    }
    if (m.mdirty) {   // an earlier call ended early: its counters may not have been reset
        HIPCHK(hipMemsetAsync(m.mbuf + MultiBuf::counters, 0, MultiBuf::counters_bytes, s));
        m.mdirty = false;
    }
    unsigned long long* stats = t_stats ? ms_ptr<unsigned long long>(o_stats) : nullptr;
    t_last_stats[0] = t_last_stats[1] = t_last_stats[2] = -1;
    if (stats) HIPCHK(hipMemsetAsync(stats, 0, 24, s));
    MsTimer timer(s);
    const FrameDev fr = fp.view();
    const uint8_t* q = dev ? (const uint8_t*)(fin ? (const void*)fin->pts : queries) : ms_ptr<const uint8_t>(o_q);
    int* ntm = fin ? ms_ptr<int>(o_ntm) : nullptr;
    if (fin) {   // Tracking::SearchLocalPoints' isInFrustum, then the search
        CamDev cd;
        if (!make_camdev(F, fin->cam, fin->rig, cd)) return ORBFE_E_ARG;
        HIPCHK(hipMemsetAsync(ntm, 0, 4, s));
        hipLaunchKernelGGL(k_frustum, dim3((nq + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, cd,
                           (const orbfe_map_point_3d*)q, nq, ms_ptr<orbfe_map_point>(o_track), ntm, fin->track_dev);
        t_ms.last_track = ms_ptr<const orbfe_map_point>(o_track);
        t_ms.last_track_n = nq;
        q = ms_ptr<const uint8_t>(o_track);
        qstride = sizeof(orbfe_map_point);
        qid_off = offsetof(orbfe_map_point, id);
    }
    uint8_t* mb = m.mbuf;
    MultiIO io;
    io.mvp_in = dev ? mvp : ms_ptr<const int32_t>(o_mvp);
    io.obs_in = dev ? mvp_obs : ms_ptr<const int32_t>(o_obs);
    io.mvp_out = dev ? mvp : ms_ptr<int32_t>(o_mvp);
    io.q_stride = (int)qstride;
    io.qid_off = (int)qid_off;
    io.ntm = ntm;
    io.assign = ms_ptr<int>(o_assign);
    io.lists = ms_ptr<uint32_t>(o_lists);
    io.lcnt = ms_ptr<int>(o_lcnt);
    io.active = ms_ptr<int>(o_active);
    io.nactive = (int*)(mb + MultiBuf::off_nactive);
    io.first[0] = (unsigned long long*)(mb + MultiBuf::off_first0);
    io.first[1] = (unsigned long long*)(mb + MultiBuf::off_first1);
    io.lastw = (unsigned long long*)(mb + MultiBuf::off_lastw);
    io.changed = (unsigned long long*)(mb + MultiBuf::off_changed);
    io.done = (int*)(mb + MultiBuf::off_done);
    io.cnt = (int*)(mb + MultiBuf::off_cnt);
    io.g_kp = ms_ptr<float4>(o_gkp);
    io.g_desc = ms_ptr<uint4>(o_gdesc);
    io.g_be = ms_ptr<int>(o_gbe);
    io.g_blk = ms_ptr<uint8_t>(o_gblk);
    io.st_host = m.hs_dev;
    io.stats = stats;
    io.gen0 = m.gen;
    m.gen += MT_MAX_PASSES;
    const orbfe_map_point* recs = (const orbfe_map_point*)q;
    const int nb0 = std::min((nq + MT_BLK_NT - 1) / MT_BLK_NT, 1024);
    // later passes walk the active queries (a fraction of nq): each thread's chain of dependent
    // loads (list -> gates) is the pass's latency, so more blocks (32: 10.8 us per pass, 128: 8.1)
    const int nb1 = std::min((nq + MT_MULTI_NT - 1) / MT_MULTI_NT, 256);
    const size_t lds = multi_lds(n, F->nlevels, gm);
    // passes per round trip: as many as the previous search needed, plus one (a gated pass is one
    // short dispatch; another round trip costs far more)
    int batch = std::min(std::max(m.pass_hint[0] + 1, 2), 8);
    int pass = 0;
    volatile int* st = m.hs;
    while (true) {
        io.seq = ++m.seq;
        for (int c = 0; c < batch; c++, pass++) {
            if (pass >= MT_MAX_PASSES) {
                m.mdirty = true;
                return ORBFE_E_CAPACITY;
            }
            const int final_ = c == batch - 1;
            if (pass == 0)
                hipLaunchKernelGGL(k_sbp_multi0, dim3(nb0), dim3(MT_BLK_NT), lds, s, fr, gm, recs, nq, th, a0, thFar,
                                   nnratio, final_, io);
            else
                hipLaunchKernelGGL(k_sbp_multi, dim3(nb1), dim3(MT_MULTI_NT), 0, s, fr, gm, recs, th, a0, thFar,
                                   nnratio, pass, final_, io);
        }
        HIPCHK(hipGetLastError());
        if (dev) {
            HIPCHK(hipEventRecord(m.tail, s));
            m.tail_stream = s;
        }
        timer.end();
        for (unsigned spin = 1; host_seq_acquire(st) != io.seq; spin++) {
            if ((spin & 1023) == 0) {   // bounded: a stream that finished without publishing is an error
                const hipError_t e = hipStreamQuery(s);
                if (e == hipSuccess && host_seq_acquire(st) != io.seq) {
                    m.mdirty = true;
                    return ORBFE_E_DEVICE;
                }
                if (e != hipSuccess && e != hipErrorNotReady) {
                    m.mdirty = true;
                    HIPCHK(e);
                }
            }
            __builtin_ia32_pause();
        }
        if (st[0] == 0) break;
        batch = 6;
    }
    m.pass_hint[0] = st[3];
    if (!dev) {
        HIPCHK(hipMemcpyAsync(mvp, io.mvp_out, (size_t)n * 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    }
    if (fin && fin->n_to_match) *fin->n_to_match = st[5];
    if (stats) {   // counting mode only: one more copy and synchronisation
        unsigned long long hst[3];
        HIPCHK(hipMemcpyAsync(hst, stats, 24, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        t_last_stats[0] = (long long)hst[1];
        t_last_stats[1] = (long long)hst[1];
        t_last_stats[2] = (long long)hst[2];
    }
    return st[1];
}

// k_last_proj for the multi-launch forms: records and right-camera centres back to the host
int last_proj_host(const LastProjIn& lp, int nq, std::vector<orbfe_proj_point>& rec, std::vector<float>& ruv) {
    Plan p;
    const size_t o_in = p.upload(lp.pts, (size_t)nq * sizeof(orbfe_last_point));
    const size_t o_rec = p.scratch((size_t)nq * sizeof(orbfe_proj_point));
    const size_t o_ruv = p.scratch((size_t)nq * 8);
    int rc = ms_prepare(p);
    if (rc) return rc;
    hipStream_t s = t_ms.stream;
    hipLaunchKernelGGL(k_last_proj, dim3((nq + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, lp,
                       ms_ptr<const orbfe_last_point>(o_in), nq, ms_ptr<orbfe_proj_point>(o_rec), ms_ptr<float2>(o_ruv));
    HIPCHK(hipGetLastError());
    rec.resize(nq);
    ruv.assign((size_t)nq * 2, 0.f);
    HIPCHK(hipMemcpyAsync(rec.data(), ms_ptr<orbfe_proj_point>(o_rec), (size_t)nq * sizeof(orbfe_proj_point),
                          hipMemcpyDeviceToHost, s));
    if (lp.two) HIPCHK(hipMemcpyAsync(ruv.data(), ms_ptr<float2>(o_ruv), (size_t)nq * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return 0;
}

int sbp_run(int mode, const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs, const void* queries, int nq,
            size_t qstride, size_t qobs_off, size_t qid_off, size_t qangle_off, size_t qlevel_off, float th, int a0, int a1, float thFar,
            float nnratio, int maxDist, int checkOri, const FrustumIn* fin = nullptr, const DevIn* dev = nullptr,
            const float* right_uv = nullptr, const LastProjIn* lp = nullptr) {
    // a device view of the current frame (orbfe_frame_device_view): the frame's arrays are read in HBM
    // by k_sbp_block; any other path would read them on the host, so other shapes are refused
    const bool fdev = F && F->device != 0;
    orbfe_frame Fchk;
    if (fdev) {
        Fchk = *F;
        Fchk.device = 0;
        BlkGeom g0;
        if (F->two_cams || F->n > MT_BAND_MAXN || nq > MT_BLOCK_MAXQ || !blk_geom(F, g0)) return ORBFE_E_ARG;
    }
    if (!frame_ok(fdev ? &Fchk : F) || !mvp || nq < 0 || (nq > 0 && !queries && !fin && !lp)) return ORBFE_E_ARG;
    if (fin && (!fin->cam || (nq > 0 && !fin->pts) || mode != 0)) return ORBFE_E_ARG;
    if (mode != 2 && !mvp_obs) return ORBFE_E_ARG;
    const bool two = F->two_cams != 0;
    // two-camera frames: a device projection needs the rig (camera models, right view); the
    // last-frame search needs the right projections
    if (two && ((fin && !fin->rig) || (mode == 1 && nq > 0 && !right_uv && !lp))) return ORBFE_E_ARG;
    if (two && !dev && !links_ok(F)) return ORBFE_E_ARG;
    // slot writes per query, in the reference's order (entry index = W q + b)
    const int W = !two ? 1 : mode == 0 ? 4 : mode == 1 ? 2 : 1;
    if (fin && fin->n_to_match) *fin->n_to_match = 0;
    if (F->n == 0 || nq == 0) return 0;
    if (nq > (1 << 24)) return ORBFE_E_CAPACITY;
    const int n = F->n;
    // level indices address mvScaleFactors: reject out-of-range ones instead of reading past it
    // (frustum-produced levels are clamped to [0, nlevels) by PredictScale; device-resident
    // records are not visible to the host: the kernels skip out-of-range levels instead)
    for (int j = 0; !fin && !dev && !lp && j < nq; j++) {
        const uint8_t* rec = (const uint8_t*)queries + (size_t)j * qstride;
        const bool used = mode == 0 ? (((const orbfe_map_point*)rec)->flags & ORBFE_MP_IN_VIEW) != 0
                                    : ((const orbfe_proj_point*)rec)->valid != 0;
        const int lvl = *(const int32_t*)(rec + qlevel_off);
        if (used && (lvl < 0 || lvl >= F->nlevels)) return ORBFE_E_ARG;
        if (two && mode == 0) {
            const orbfe_map_point* m = (const orbfe_map_point*)rec;
            if ((m->flags & ORBFE_MP_IN_VIEW_R) && m->scale_level_r != -1 &&
                (m->scale_level_r < 0 || m->scale_level_r >= F->nlevels))
                return ORBFE_E_ARG;
        }
    }
    // single-camera searches of a frame that fits in LDS run on its (octave, band) index: a small
    // search (the per-frame Tracking calls) entirely in one workgroup, one launch (k_sbp_block), a
    // large local-map search as one multi-block pass per fixed-point step (k_sbp_band)
    const int band_nb = std::min(std::max((int)std::floor(F->max_y * (1.0f / MT_BAND_ROWS)) + 2, 1), 4096);
    // 16-bit bucket keys, and k_sbp_band's LDS (frame, bucket starts, change bins) within 160 KB
    const bool band_ok = (size_t)F->nlevels * band_nb < 65535 &&
                         (size_t)n * 56 + (size_t)F->nlevels * band_nb * 20 + 32 <= 160 * 1024;
    BlkGeom gm;
    if (W == 1 && n <= MT_BAND_MAXN && blk_geom(F, gm)) {
        if (nq <= MT_BLOCK_MAXQ)
            return sbp_block_run(mode, F, mvp, mvp_obs, queries, nq, qstride, qid_off, qangle_off, th, a0, a1, thFar,
                                 nnratio, maxDist, checkOri, gm, fin, dev, lp);
        // narrow windows only: a wide window is a long serial walk for one thread, where k_sbp_band's
        // sixteen lanes per query win (config 5: th 1 / 3 here, th 5 / 15 there; r05_kernel_ab.txt)
        if (mode == 0 && th < MT_MULTI_TH)
            return sbp_multi_run(F, mvp, mvp_obs, queries, nq, qstride, qid_off, th, a0, thFar, nnratio, gm, fin, dev);
    }
    // a two-camera frame's local-map search (SearchLocalPoints of a KannalaBrandt8 rig) in one
    // workgroup: four slot writes per point, the slots' writers tracked per pass (k_sbp_block4)
    if (two && mode == 0 && n <= MT_BAND_MAXN && nq <= MT_BLOCK_MAXQ && blk_geom(F, gm, 2, blk4_bytes_per_kp())) {
        const int r = sbp_block_run(0, F, mvp, mvp_obs, queries, nq, qstride, qid_off, qangle_off, th, a0, a1, thFar,
                                    nnratio, maxDist, 0, gm, fin, dev);
        if (r != kBlockAborted) return r;
    }
    // a two-camera frame's last-frame search (the per-frame Tracking call of a KannalaBrandt8 rig) in
    // one workgroup as well: both cameras' keypoints in LDS, two entries per point
    if (two && mode == 1 && !dev && n <= MT_BAND_MAXN && nq <= MT_BLOCK_MAXQ && blk_geom(F, gm, 2))
        return sbp_block2_run(F, mvp, mvp_obs, (const orbfe_proj_point*)queries, right_uv, nq, th, a0, a1, maxDist,
                              checkOri, gm, lp);
    // the multi-launch forms read host records: a device-projected search projects first and brings the
    // records back (searches beyond the one-workgroup limits only)
    std::vector<orbfe_proj_point> lp_rec;
    std::vector<float> lp_ruv;
    if (lp) {
        const int rc = last_proj_host(*lp, nq, lp_rec, lp_ruv);
        if (rc) return rc;
        queries = lp_rec.data();
        right_uv = lp_ruv.data();
    }
    std::vector<int32_t> blocked0(dev ? 0 : n);
    for (int k = 0; !dev && k < n; k++) blocked0[k] = mode == 2 ? (mvp[k] >= 0) : (mvp[k] >= 0 && mvp_obs[k] > 0);
    Plan p;
    FramePlan fp;
    if (dev) fp.plan_dev(F, mode != 2);
    else fp.plan(p, F, true, mode != 2);
    const size_t o_q = dev ? 0 : fin ? p.upload(fin->pts, (size_t)nq * sizeof(orbfe_map_point_3d))
                                     : p.upload(queries, (size_t)nq * qstride);
    const size_t o_b0 = dev ? 0 : p.upload(blocked0.data(), (size_t)n * 4);
    const size_t o_mvp = dev ? 0 : p.upload(mvp, (size_t)n * 4);
    const size_t o_b0d = dev ? p.scratch((size_t)n * 4) : 0;
    fp.plan_grid(p, mode == 0 ? F->nlevels + 1 : 1);
    // single-camera searches of a frame that fits in LDS run on its (octave, band) index: a small
    // search (the per-frame Tracking calls) entirely in one workgroup (k_sbp_block), a large local-map
    // search as one multi-block pass per fixed-point step (k_sbp_band)
    bool use_band = mode == 0 && W == 1 && n <= MT_BAND_MAXN && band_ok;
    if (use_band) {
        fp.plan_band(p);
        fp.ngrids = 0;   // the cell grids are not read
    }
    const size_t o_track = fin ? p.scratch((size_t)nq * sizeof(orbfe_map_point)) : 0;
    const size_t o_ntm = fin ? p.scratch(16) : 0;
    const size_t o_ruv = (two && mode == 1 && !dev) ? p.upload(right_uv, (size_t)nq * 8) : 0;
    const size_t o_first = p.scratch((size_t)n * 4);
    const size_t o_first1 = p.scratch((size_t)n * 4);   // rotating pass states (W == 1)
    const size_t o_first2 = p.scratch((size_t)n * 4);
    const size_t o_first3 = p.scratch((size_t)n * 4);
    const size_t o_assign = p.scratch((size_t)nq * W * 4);
    const bool buckets = two && mode == 0;
    const size_t o_soff = buckets ? p.scratch((size_t)(n + 1) * 4) : 0;
    const size_t o_scur = buckets ? p.scratch((size_t)n * 4) : 0;
    const size_t o_slst = buckets ? p.scratch((size_t)nq * W * 4) : 0;
    const size_t o_changed = p.scratch(MT_MAX_PASSES * 4);
    const size_t o_result = p.scratch((size_t)(n + 3) * 4);   // [change flag copy | counts | slots]
    const size_t o_hist = p.scratch((MT_HISTO + 1) * 4);   // rotation bins + commit completion counter
    const size_t o_stats = t_stats ? p.scratch(24) : 0;
    int rc = ms_prepare(p);
    if (rc) return rc;
    // a device-resident search runs on the caller's stream, after the producer of its inputs; it
    // returns once its status is published and records MatchScratch::tail, after which the next
    // call of the thread orders itself (host-API calls also end with a stream synchronisation)
    hipStream_t s = dev ? dev->caller : t_ms.stream;
    if (dev) HIPCHK(ms_after_tail(s));
    unsigned long long* stats = t_stats ? ms_ptr<unsigned long long>(o_stats) : nullptr;
    t_last_stats[0] = t_last_stats[1] = t_last_stats[2] = -1;
    if (stats) HIPCHK(hipMemsetAsync(stats, 0, 24, s));
    MsTimer timer(s);
    const FrameDev fr = fp.view();
    const int* b0 = dev ? ms_ptr<const int>(o_b0d) : ms_ptr<const int>(o_b0);
    int32_t* mvp_d = dev ? mvp : ms_ptr<int32_t>(o_mvp);
    int* first = ms_ptr<int>(o_first);
    int* assign = ms_ptr<int>(o_assign);
    int* changed = ms_ptr<int>(o_changed);
    int* resb = ms_ptr<int>(o_result);
    int* hist = ms_ptr<int>(o_hist);
    {   // the grids and the search initialisation in one launch
        const SbpInit ia{mvp, mvp_obs, mode == 2 ? 1 : 0, dev ? ms_ptr<int>(o_b0d) : nullptr, first,
                         ms_ptr<int>(o_first1), assign, nq * W, changed, hist, resb, n};
        fp.launch_grid_on(fr, s, &ia);
    }
    const float2* ruv = (two && mode == 1) ? (dev ? (const float2*)right_uv : ms_ptr<const float2>(o_ruv)) : nullptr;
    const uint8_t* q = dev ? (const uint8_t*)(fin ? (const void*)fin->pts : queries) : ms_ptr<const uint8_t>(o_q);
    if (fin) {   // Tracking::SearchLocalPoints: project, count nToMatch, match only if > 0
        CamDev cd;
        if (!make_camdev(F, fin->cam, fin->rig, cd)) return ORBFE_E_ARG;
        int* ntm = ms_ptr<int>(o_ntm);
        HIPCHK(hipMemsetAsync(ntm, 0, 4, s));
        hipLaunchKernelGGL(k_frustum, dim3((nq + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, cd,
                           (const orbfe_map_point_3d*)q, nq, ms_ptr<orbfe_map_point>(o_track), ntm, fin->track_dev);
        t_ms.last_track = ms_ptr<const orbfe_map_point>(o_track);
        t_ms.last_track_n = nq;
        int h_ntm = 0;
        HIPCHK(hipMemcpyAsync(t_ms.hs, ntm, 4, hipMemcpyDeviceToHost, s));   // pinned
        HIPCHK(hipStreamSynchronize(s));
        h_ntm = t_ms.hs[0];
        if (fin->n_to_match) *fin->n_to_match = h_ntm;
        if (h_ntm <= 0) return 0;
        q = ms_ptr<const uint8_t>(o_track);
    }
    const dim3 gq((nq + MT_NT - 1) / MT_NT);
    const bool staged = n <= MT_STAGE_MAX;
    int* result = resb + 1;
    const dim3 ge((nq * W + MT_NT - 1) / MT_NT);
    // the commit runs once (a gated commit that does not run leaves result / hist as the
    // initialisation set them); st_host: where the last kernel stores the status the host reads
    auto commit = [&](const int* gate, const CommitStatus& cs) {
        hipLaunchKernelGGL(k_mt_commit_count, ge, dim3(MT_NT), 0, s, fr.keys, assign, (const float*)(q + qangle_off),
                           (int)qstride, nq * W, checkOri, result, hist, W, gate);
        if (checkOri)
            hipLaunchKernelGGL(k_mt_commit_drop, ge, dim3(MT_NT), 0, s, fr.keys, assign,
                               (const float*)(q + qangle_off), (int)qstride, nq * W, hist, result, W, gate);
        hipLaunchKernelGGL(k_mt_commit_write, dim3((n + 255) / 256), dim3(256), 0, s, n, (const int*)(q + qid_off),
                           (int)qstride, result, mvp_d, W, gate, resb, cs);
        return ORBFE_OK;
    };
    int pass = 0;
    if (W == 1) {
        // single camera: one gated kernel per pass (PassIO), a batch of passes and the gated commit
        // per host round trip; most searches converge within the first batch (2-4 passes)
        // fb[0], fb[1] = MT_INF (init); four states so that pass p still sees its predecessor's
        // (k_sbp_band's skip of unchanged queries) while it clears the state of pass p + 2
        int* fb[4] = {first, ms_ptr<int>(o_first1), ms_ptr<int>(o_first2), ms_ptr<int>(o_first3)};
        // passes per round trip: as many as the previous search of this mode needed, plus one (a
        // gated pass costs a dispatch; an extra round trip costs far more)
        int batch = std::min(std::max(t_ms.pass_hint[mode] + 1, 2), 8);
        while (true) {
            const int pass0 = pass;
            for (int c = 0; c < batch; c++, pass++) {
                if (pass >= MT_MAX_PASSES) return ORBFE_E_CAPACITY;
                PassIO io{pass ? changed + pass - 1 : nullptr, fb[(pass + 1) % 4], fb[(pass + 2) % 4], n,
                          mode == 2 ? 0 : 1, stats};
                const int* fcur = fb[pass % 4];
                // pass 1 sees nearly every gate move (free -> first claimer): skipping from pass 2 on
                const int* fprev = pass >= 2 ? fb[(pass + 3) % 4] : nullptr;
                if (use_band) {
                    const int qpb = (MT_BNT / 64) * MT_QPW;
                    const int nb = std::min((nq + qpb - 1) / qpb, 512);
                    const BandGrid bg{ms_ptr<int>(fp.bstart), ms_ptr<int>(fp.bidx), fp.band_nb, F->nlevels};
                    const size_t nbk = (size_t)F->nlevels * fp.band_nb;
                    const size_t lds = ((size_t)n * 56 + (nbk + 1) * 4 + 8 + nbk * 16 + 15) & ~(size_t)15;
                    int qshift = 0;
                    while ((((nq - 1) >> qshift) >> 7) > 0) qshift++;   // 128 query bins
                    hipLaunchKernelGGL(k_sbp_band, dim3(nb), dim3(MT_BNT), lds, s, fr, bg, (const orbfe_map_point*)q, nq,
                                       th, a0, thFar, nnratio, b0, fcur, assign, changed + pass, io, fprev, qshift);
                } else if (mode == 0 && th >= MT_WAVE_TH) {
                    const int qpb = (MT_WNT / 64) * MT_QPW;   // queries per block and round
                    const int nb = std::min((nq + qpb - 1) / qpb, 512);
                    const size_t cellb = (MT_WNT / 64) * 64 * sizeof(int2);
                    const int st = staged ? 1 : (cellb + (size_t)n * 24 <= 150 * 1024 ? 2 : 0);
                    const size_t lds = cellb + (st == 1 ? (size_t)n * 56 : st == 2 ? (size_t)n * 24 : 0);
                    if (st == 1)
                        hipLaunchKernelGGL(k_sbp_local_wq<1>, dim3(nb), dim3(MT_WNT), lds, s, fr,
                                           (const orbfe_map_point*)q, nq, th, a0, thFar, nnratio, b0, fcur, assign,
                                           changed + pass, io);
                    else if (st == 2)
                        hipLaunchKernelGGL(k_sbp_local_wq<2>, dim3(nb), dim3(MT_WNT), lds, s, fr,
                                           (const orbfe_map_point*)q, nq, th, a0, thFar, nnratio, b0, fcur, assign,
                                           changed + pass, io);
                    else
                        hipLaunchKernelGGL(k_sbp_local_wq<0>, dim3(nb), dim3(MT_WNT), lds, s, fr,
                                           (const orbfe_map_point*)q, nq, th, a0, thFar, nnratio, b0, fcur, assign,
                                           changed + pass, io);
                } else if (mode == 0) {
                    hipLaunchKernelGGL(k_sbp_local, gq, dim3(MT_NT), 0, s, fr, (const orbfe_map_point*)q, nq, th, a0,
                                       thFar, nnratio, b0, fcur, assign, changed + pass, io);
                } else {
                    hipLaunchKernelGGL(k_sbp_proj, gq, dim3(MT_NT), 0, s, fr, (const orbfe_proj_point*)q, nq, th,
                                       mode == 1 ? 0 : 1, a0, a1, maxDist, b0, fcur, assign, changed + pass, io);
                }
            }
            // the commit (gated: runs only if the last pass changed nothing) ends with its last
            // block storing {change flag, assigned, dropped, passes needed, sequence number} straight
            // into the pinned host words: no copy operation, and a device-resident call waits for
            // the sequence number instead of the stream
            volatile int* st = t_ms.hs;
            const int seq = ++t_ms.seq;
            commit(changed + pass - 1, CommitStatus{t_ms.hs_dev, hist + MT_HISTO, changed + pass0, batch, seq});
            HIPCHK(hipGetLastError());
            if (dev) {
                HIPCHK(hipEventRecord(t_ms.tail, s));
                t_ms.tail_stream = s;
            }
            timer.end();
            if (!dev) {
                HIPCHK(hipMemcpyAsync(mvp, mvp_d, (size_t)n * 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
            for (unsigned spin = 1; host_seq_acquire(st) != seq; spin++) {
                if ((spin & 1023) == 0) {   // bounded: a stream that finished without publishing is an error
                    const hipError_t e = hipStreamQuery(s);
                    if (e == hipSuccess && host_seq_acquire(st) != seq) return ORBFE_E_DEVICE;
                    if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
                }
                __builtin_ia32_pause();
            }
            if (st[0] == 0) {
                t_ms.pass_hint[mode] = pass0 + st[3];
                if (stats) {   // counting mode only: one more copy and synchronisation
                    unsigned long long hst[3];
                    HIPCHK(hipMemcpyAsync(hst, stats, 24, hipMemcpyDeviceToHost, s));
                    HIPCHK(hipStreamSynchronize(s));
                    t_last_stats[0] = (long long)hst[0];
                    t_last_stats[1] = (long long)hst[1];
                    t_last_stats[2] = pass0 + st[3];
                }
                return st[1] - st[2];
            }
            batch = 6;
        }
    }
    const int chunk = 2;   // passes launched between host checks (two-camera frames)
    while (true) {
        for (int c = 0; c < chunk; c++, pass++) {
            if (pass >= MT_MAX_PASSES) return ORBFE_E_CAPACITY;
            const dim3 gw((nq * W + MT_NT - 1) / MT_NT);
            if (two && mode == 0) {   // per-slot write buckets (unguarded partner writes)
                int* cntb = first;   // n counters, then the scan's offsets / cursors / lists
                int* off = ms_ptr<int>(o_soff);
                int* cur = ms_ptr<int>(o_scur);
                int* lst = ms_ptr<int>(o_slst);
                HIPCHK(hipMemsetAsync(cntb, 0, (size_t)n * 4, s));
                hipLaunchKernelGGL(k_slot_count, gw, dim3(MT_NT), 0, s, assign, nq * W, cntb);
                hipLaunchKernelGGL(k_slot_scan, dim3(1), dim3(1024), 0, s, cntb, n, off, cur);
                hipLaunchKernelGGL(k_slot_fill, gw, dim3(MT_NT), 0, s, assign, nq * W, cur, lst);
                hipLaunchKernelGGL(k_sbp_local2, gq, dim3(MT_NT), 0, s, fr, (const orbfe_map_point*)q, nq, th, a0, thFar,
                                   nnratio, b0, (const int*)off, (const int*)lst, assign, changed + pass);
                continue;
            }
            fill(first, n, MT_INF, s);
            hipLaunchKernelGGL(k_mt_first_strided, gw, dim3(MT_NT), 0, s, assign, q + qobs_off, (int)qstride, nq * W,
                               mode == 2 ? 0 : 1, first, W);
            hipLaunchKernelGGL(k_sbp_proj2, gq, dim3(MT_NT), 0, s, fr, (const orbfe_proj_point*)q, ruv, nq, th, a0,
                               a1, b0, first, assign, changed + pass);
        }
        int* ch = t_ms.hs;   // pinned: a pageable 4-byte read back costs more than the passes
        HIPCHK(hipMemcpyAsync(ch, changed + pass - 1, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        if (*ch == 0) break;
    }
    commit(nullptr, CommitStatus{});
    HIPCHK(hipGetLastError());
    timer.end();
    int* cnt = t_ms.hs;
    if (!dev) HIPCHK(hipMemcpyAsync(mvp, mvp_d, (size_t)n * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cnt, result, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return cnt[0] - cnt[1];
}

}  // namespace

extern "C" {

int orbfe_search_by_projection_local(const orbfe_frame* F, int32_t* mvp, const int32_t* mvp_obs,
                                     const orbfe_map_point* mps, int32_t n_mps, float th, int32_t bFarPoints,
                                     float thFarPoints, float nnratio) {
    return sbp_run(0, F, mvp, mvp_obs, mps, n_mps, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                   offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0, thFarPoints, nnratio, 0, 0);
}

int orbfe_search_by_projection_lastframe_stereo(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs,
                                                const orbfe_proj_point* pts, const float* right_uv, int32_t n_pts,
                                                float th, int32_t bForward, int32_t bBackward, int32_t checkOri) {
    return sbp_run(1, cur, mvp, mvp_obs, pts, n_pts, sizeof(orbfe_proj_point), offsetof(orbfe_proj_point, observations),
                   offsetof(orbfe_proj_point, id), offsetof(orbfe_proj_point, angle), offsetof(orbfe_proj_point, octave),
                   th, bForward, bBackward, 0.f, 0.f, MT_TH_HIGH, checkOri, nullptr, nullptr, right_uv);
}

int orbfe_search_by_projection_lastframe_pose(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs,
                                              const orbfe_last_point* pts, int32_t n_pts, const orbfe_pose* Tcw,
                                              const orbfe_pose* Trl, const orbfe_camera_model* cam, float th,
                                              int32_t bForward, int32_t bBackward, int32_t checkOri) {
    if (!cur || !Tcw || !cam || n_pts < 0 || (n_pts > 0 && !pts)) return ORBFE_E_ARG;
    const bool two = cur->two_cams != 0;
    if (two && !Trl) return ORBFE_E_ARG;
    if (cam->type != ORBFE_CAM_PINHOLE && cam->type != ORBFE_CAM_KANNALA_BRANDT8) return ORBFE_E_ARG;
    // nLastOctave addresses mvScaleFactors (as the host-projected entry points check)
    for (int j = 0; j < n_pts; j++)
        if (pts[j].valid && (pts[j].octave < 0 || pts[j].octave >= cur->nlevels)) return ORBFE_E_ARG;
    LastProjIn lp;
    memset(&lp, 0, sizeof(lp));
    lp.pts = pts;
    lp.T = *Tcw;
    lp.T.kind = ORBFE_SE3;
    if (two) {
        lp.Trl = *Trl;
        lp.Trl.kind = ORBFE_SE3;
    }
    lp.two = two ? 1 : 0;
    lp.cam.type = cam->type;
    lp.cam.fx = cam->params[0]; lp.cam.fy = cam->params[1]; lp.cam.cx = cam->params[2]; lp.cam.cy = cam->params[3];
    for (int k = 0; k < 4; k++) lp.cam.k[k] = cam->type == ORBFE_CAM_KANNALA_BRANDT8 ? cam->params[4 + k] : 0.f;
    return sbp_run(1, cur, mvp, mvp_obs, nullptr, n_pts, sizeof(orbfe_proj_point),
                   offsetof(orbfe_proj_point, observations), offsetof(orbfe_proj_point, id),
                   offsetof(orbfe_proj_point, angle), offsetof(orbfe_proj_point, octave), th, bForward, bBackward, 0.f, 0.f,
                   MT_TH_HIGH, checkOri, nullptr, nullptr, nullptr, &lp);
}

int orbfe_search_by_projection_lastframe(const orbfe_frame* cur, int32_t* mvp, const int32_t* mvp_obs,
                                         const orbfe_proj_point* pts, int32_t n_pts, float th, int32_t bForward,
                                         int32_t bBackward, int32_t checkOri) {
    return sbp_run(1, cur, mvp, mvp_obs, pts, n_pts, sizeof(orbfe_proj_point),
                   offsetof(orbfe_proj_point, observations), offsetof(orbfe_proj_point, id),
                   offsetof(orbfe_proj_point, angle), offsetof(orbfe_proj_point, octave), th, bForward, bBackward, 0.f, 0.f, MT_TH_HIGH, checkOri);
}

int orbfe_search_by_projection_kf(const orbfe_frame* cur, int32_t* mvp, const orbfe_proj_point* pts, int32_t n_pts,
                                  float th, int32_t ORBdist, int32_t checkOri) {
    return sbp_run(2, cur, mvp, nullptr, pts, n_pts, sizeof(orbfe_proj_point),
                   offsetof(orbfe_proj_point, observations), offsetof(orbfe_proj_point, id),
                   offsetof(orbfe_proj_point, angle), offsetof(orbfe_proj_point, octave), th, 0, 0, 0.f, 0.f, ORBdist, checkOri);
}

static int sfi_core(const orbfe_frame* F1, const orbfe_frame* F2, float* prev_matched, int32_t* matches12,
                    int32_t windowSize, float nnratio, int32_t checkOri);

int orbfe_search_for_initialization(const orbfe_frame* F1, const orbfe_frame* F2, float* prev_matched,
                                    int32_t* matches12, int32_t windowSize, float nnratio, int32_t checkOri) {
    if (!frame1_ok(F1) || !frame1_ok(F2) || !prev_matched || !matches12) return ORBFE_E_ARG;
    // Only F1's level-0 features search (ORBmatcher.cc:661-663: level1 > 0 continues), and their
    // windows read F2's level-0 features only (GetFeaturesInArea(.., level1, level1)). The call runs
    // on those two subsets (order-preserving, so "earlier query" and the enumeration order are
    // unchanged) and scatters the results back: a fifth of the monocular initialiser's 5 x nFeatures
    // to pack, upload and grid. A negative octave (no level filter in the reference) keeps the
    // whole frames.
    bool neg = false;
    for (int i = 0; i < F1->n && !neg; i++) neg = F1->keys[i].octave < 0;
    if (neg || F1->n == 0 || F2->n == 0)
        return sfi_core(F1, F2, prev_matched, matches12, windowSize, nnratio, checkOri);
    std::vector<int32_t> i1, i2;
    for (int i = 0; i < F1->n; i++)
        if (F1->keys[i].octave == 0) i1.push_back(i);
    for (int i = 0; i < F2->n; i++)
        if (F2->keys[i].octave == 0) i2.push_back(i);
    const int m1 = (int)i1.size(), m2 = (int)i2.size();
    std::vector<orbfe_keypoint> k1(std::max(m1, 1)), k2(std::max(m2, 1));
    std::vector<uint8_t> d1((size_t)std::max(m1, 1) * 32), d2((size_t)std::max(m2, 1) * 32);
    std::vector<float> pv((size_t)std::max(m1, 1) * 2);
    for (int j = 0; j < m1; j++) {
        k1[j] = F1->keys[i1[j]];
        memcpy(&d1[(size_t)j * 32], F1->desc + (size_t)i1[j] * 32, 32);
        pv[2 * j] = prev_matched[2 * i1[j]];
        pv[2 * j + 1] = prev_matched[2 * i1[j] + 1];
    }
    for (int j = 0; j < m2; j++) {
        k2[j] = F2->keys[i2[j]];
        memcpy(&d2[(size_t)j * 32], F2->desc + (size_t)i2[j] * 32, 32);
    }
    orbfe_frame c1 = *F1, c2 = *F2;
    c1.n = m1; c1.keys = k1.data(); c1.desc = d1.data(); c1.uright = nullptr;
    c2.n = m2; c2.keys = k2.data(); c2.desc = d2.data(); c2.uright = nullptr;
    std::vector<int32_t> mc((size_t)std::max(m1, 1));
    const int r = sfi_core(&c1, &c2, pv.data(), mc.data(), windowSize, nnratio, checkOri);
    if (r < 0) return r;
    for (int i = 0; i < F1->n; i++) matches12[i] = -1;
    for (int j = 0; j < m1; j++) {
        matches12[i1[j]] = mc[j] >= 0 ? i2[mc[j]] : -1;
        prev_matched[2 * i1[j]] = pv[2 * j];
        prev_matched[2 * i1[j] + 1] = pv[2 * j + 1];
    }
    return r;
}

static int sfi_core(const orbfe_frame* F1, const orbfe_frame* F2, float* prev_matched, int32_t* matches12,
                    int32_t windowSize, float nnratio, int32_t checkOri) {
    const int n1 = F1->n;
    if (n1 == 0) return 0;
    if (F2->n == 0) {
        for (int i = 0; i < n1; i++) matches12[i] = -1;
        return 0;
    }
    Plan p;
    FramePlan f1p, f2p;
    f1p.plan(p, F1, false, false);
    f2p.plan(p, F2, true, false);
    const size_t o_prev = p.upload(prev_matched, (size_t)n1 * 8);
    f1p.cstart = f1p.cidx = 0;
    f2p.plan_grid(p, 2);
    f2p.gfirst = 1;   // k_init_eval reads the octave-0 grid only
    const size_t o_assign = p.scratch((size_t)n1 * 4);
    const size_t o_adist = p.scratch((size_t)n1 * 4);
    const size_t o_skey = p.scratch((size_t)n1 * 4);
    const size_t o_spmin = p.scratch((size_t)n1 * 4);
    const size_t o_nsel = p.scratch(4);
    const size_t o_segoff = p.scratch((size_t)F2->n * 4);
    const size_t o_segcnt = p.scratch((size_t)F2->n * 4);
    const size_t o_changed = p.scratch(MT_MAX_PASSES * 4);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    const FrameDev v1 = f1p.view(), v2 = f2p.view();
    f2p.launch_grid(v2);
    int* assign = ms_ptr<int>(o_assign);
    int* adist = ms_ptr<int>(o_adist);
    int* changed = ms_ptr<int>(o_changed);
    HIPCHK(hipMemsetAsync(changed, 0, MT_MAX_PASSES * 4, s));
    fill(assign, n1, -1);
    fill(adist, n1, 0);
    const dim3 gq((n1 + MT_INIT_WNT / 16 - 1) / (MT_INIT_WNT / 16));   // four queries per wave
    // outputs in mapped pinned memory: matches12, then prevMatched (the input, updated by the commit)
    MatchScratch& m = t_ms;
    if (m.ocap < (size_t)n1 * 3) {
        if (m.ho) HIPCHK(hipHostFree(m.ho));
        m.ho = nullptr;
        m.ocap = 0;
        const size_t cap = std::max<size_t>((size_t)n1 * 3, 2048);
        HIPCHK(hipHostMalloc((void**)&m.ho, cap * 4, hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&m.ho_dev, m.ho, 0));
        m.ocap = cap;
    }
    memcpy(m.ho + n1, prev_matched, (size_t)n1 * 8);
    // gated passes (a pass after an unchanged one returns at once) and a gated commit per round trip:
    // the host waits for the commit's status words, and enqueues more passes only when the last one
    // still changed something
    int pass = 0, batch = 3;
    while (true) {
        for (int c = 0; c < batch; c++, pass++) {
            if (pass >= MT_MAX_PASSES) return ORBFE_E_CAPACITY;
            const int* gate = pass ? changed + pass - 1 : nullptr;
            hipLaunchKernelGGL(k_init_state, dim3(1), dim3(1024), 0, s, assign, adist, n1, ms_ptr<uint32_t>(o_skey),
                               ms_ptr<int>(o_spmin), ms_ptr<int>(o_nsel), F2->n, ms_ptr<int>(o_segoff),
                               ms_ptr<int>(o_segcnt), gate);
            hipLaunchKernelGGL(k_init_eval, gq, dim3(MT_INIT_WNT), 0, s, v1, v2, ms_ptr<const float>(o_prev), windowSize,
                               nnratio, ms_ptr<const uint32_t>(o_skey), ms_ptr<const int>(o_spmin),
                               ms_ptr<const int>(o_segoff), ms_ptr<const int>(o_segcnt), assign, adist, changed + pass,
                               gate);
        }
        const int seq = ++t_ms.seq;
        hipLaunchKernelGGL(k_init_commit, dim3(1), dim3(1024), 0, s, v1, v2, assign, checkOri,
                           (float*)(m.ho_dev + n1), m.ho_dev, changed + pass - 1, t_ms.hs_dev, seq);
        HIPCHK(hipGetLastError());
        timer.end();
        volatile int* st = t_ms.hs;
        for (unsigned spin = 1; host_seq_acquire(st) != seq; spin++) {
            if ((spin & 1023) == 0) {   // bounded: a stream that finished without publishing is an error
                const hipError_t e = hipStreamQuery(s);
                if (e == hipSuccess && host_seq_acquire(st) != seq) return ORBFE_E_DEVICE;
                if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
            }
            __builtin_ia32_pause();
        }
        if (st[0] == 0) {   // converged and committed: the outputs precede the status words
            memcpy(matches12, m.ho, (size_t)n1 * 4);
            memcpy(prev_matched, m.ho + n1, (size_t)n1 * 8);
            return st[1];
        }
        batch = 4;
    }
}

int orbfe_search_by_bow(const orbfe_keypoint* kf_keys, const uint8_t* kf_desc, const int32_t* kf_mp, int32_t kf_n,
                        const orbfe_feature_vector* kf_fv, const orbfe_frame* F, const orbfe_feature_vector* f_fv,
                        int32_t* out, float nnratio, int32_t checkOri) {
    if (!F || F->n < 0 || kf_n < 0 || !kf_fv || !f_fv || !out || (kf_n > 0 && (!kf_keys || !kf_desc || !kf_mp)))
        return ORBFE_E_ARG;
    if (F->two_cams && (F->nleft < 0 || F->nleft > F->n)) return ORBFE_E_ARG;
    const int fn = F->n;
    for (int i = 0; i < fn; i++) out[i] = -1;
    if (fn == 0 || kf_n == 0 || kf_fv->n_nodes <= 0 || f_fv->n_nodes <= 0) return 0;
    // ordered merge-join of the two node lists (the reference's lower_bound walk, ORBmatcher.cc:244-371)
    std::vector<int32_t> pairs;
    int a = 0, b = 0;
    while (a < kf_fv->n_nodes && b < f_fv->n_nodes) {
        if (kf_fv->node_ids[a] == f_fv->node_ids[b]) { pairs.push_back(a); pairs.push_back(b); a++; b++; }
        else if (kf_fv->node_ids[a] < f_fv->node_ids[b]) a++;
        else b++;
    }
    if (pairs.empty()) return 0;
    for (const orbfe_feature_vector* fv : {kf_fv, f_fv}) {
        if (!fv->node_ids || !fv->offsets || fv->offsets[0] != 0) return ORBFE_E_ARG;
        for (int i = 0; i < fv->n_nodes; i++)
            if (fv->offsets[i + 1] < fv->offsets[i] || (i > 0 && fv->node_ids[i] <= fv->node_ids[i - 1]))
                return ORBFE_E_ARG;
    }
    // each frame index must belong to one node only (DBoW2 transform); the per-node threads rely on it
    std::vector<uint8_t> seen(fn, 0);
    const int nfi = f_fv->offsets[f_fv->n_nodes];
    for (int i = 0; i < nfi; i++) {
        const uint32_t x = f_fv->indices[i];
        if (x >= (uint32_t)fn || seen[x]) return ORBFE_E_ARG;
        seen[x] = 1;
    }
    const int nki = kf_fv->offsets[kf_fv->n_nodes];
    for (int i = 0; i < nki; i++)
        if (kf_fv->indices[i] >= (uint32_t)kf_n) return ORBFE_E_ARG;
    const int npairs = (int)pairs.size() / 2;
    Plan p;
    const size_t o_pairs = p.upload(pairs.data(), pairs.size() * 4);
    const size_t o_kfoff = p.upload(kf_fv->offsets, (size_t)(kf_fv->n_nodes + 1) * 4);
    const size_t o_kfidx = p.upload(kf_fv->indices, (size_t)nki * 4);
    const size_t o_foff = p.upload(f_fv->offsets, (size_t)(f_fv->n_nodes + 1) * 4);
    const size_t o_fidx = p.upload(f_fv->indices, (size_t)nfi * 4);
    const size_t o_kfmp = p.upload(kf_mp, (size_t)kf_n * 4);
    const size_t o_kfdesc = p.upload(kf_desc, (size_t)kf_n * 32);
    const size_t o_kfkeys = p.upload(kf_keys, (size_t)kf_n * sizeof(orbfe_keypoint));
    const size_t o_fdesc = p.upload(F->desc, (size_t)fn * 32);
    const size_t o_fkeys = p.upload(F->keys, (size_t)fn * sizeof(orbfe_keypoint));
    const size_t o_src = p.scratch((size_t)fn * 4);
    const size_t o_out = p.scratch((size_t)fn * 4);
    const size_t o_result = p.scratch(16);
    // the uploads from the node pairs to the F descriptors, in Plan order (k_bow_block copies them whole)
    const size_t reg_bytes = o_fdesc + (size_t)fn * 32 - o_pairs;
    const size_t blds = ((reg_bytes + 15) & ~(size_t)15) + (size_t)fn * 4 + 16;
    const bool block = o_pairs < o_kfoff && o_kfoff < o_kfidx && o_kfidx < o_foff && o_foff < o_fidx &&
                       o_fidx < o_kfmp && o_kfmp < o_kfdesc && o_kfdesc < o_kfkeys && o_kfkeys < o_fdesc &&
                       blds <= 150 * 1024 && fn <= MT_BOW_FR * MT_BOW_NT;
    // one workgroup: zero copy both ways (inputs read in place from the mapped pinned staging, the
    // output written to mapped pinned memory, the status words awaited: no DMA, no stream sync)
    int rc = ms_prepare(p, block);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    if (block) {
        MatchScratch& m = t_ms;
        if (m.ocap < (size_t)fn) {
            if (m.ho) HIPCHK(hipHostFree(m.ho));
            m.ho = nullptr;
            m.ocap = 0;
            const size_t cap = std::max<size_t>((size_t)fn, 2048);
            HIPCHK(hipHostMalloc((void**)&m.ho, cap * 4, hipHostMallocMapped | hipHostMallocCoherent));
            HIPCHK(hipHostGetDevicePointer((void**)&m.ho_dev, m.ho, 0));
            m.ocap = cap;
        }
        auto rel = [&](size_t o) { return (int)(o - o_pairs); };
        const int seq = ++t_ms.seq;
        BowBlockIn in{up_ptr<const uint4>(o_pairs, true), (int)((reg_bytes + 15) / 16), rel(o_pairs), rel(o_kfoff),
                      rel(o_kfidx), rel(o_foff), rel(o_fidx), rel(o_kfmp), rel(o_kfdesc), rel(o_kfkeys), rel(o_fdesc),
                      up_ptr<const OrbKeyPoint>(o_fkeys, true), npairs, kf_n, fn, F->two_cams ? F->nleft : -1,
                      checkOri, nnratio, t_ms.hs_dev, seq};
        hipLaunchKernelGGL(k_bow_block, dim3(1), dim3(MT_BOW_NT), blds, s, in, m.ho_dev, ms_ptr<int>(o_result));
        HIPCHK(hipGetLastError());
        timer.end();
        volatile int* st = t_ms.hs;
        for (unsigned spin = 1; host_seq_acquire(st) != seq; spin++) {
            if ((spin & 1023) == 0) {   // bounded: a stream that finished without publishing is an error
                const hipError_t e = hipStreamQuery(s);
                if (e == hipSuccess && host_seq_acquire(st) != seq) return ORBFE_E_DEVICE;
                if (e != hipSuccess && e != hipErrorNotReady) HIPCHK(e);
            }
            __builtin_ia32_pause();
        }
        memcpy(out, m.ho, (size_t)fn * 4);   // complete: the status words come after the output stores
        return st[1];
    }
    fill(ms_ptr<int>(o_src), fn, -1);
    hipLaunchKernelGGL(k_bow_nodes, dim3((npairs + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, ms_ptr<const int>(o_pairs),
                       npairs, ms_ptr<const int>(o_kfoff), ms_ptr<const uint32_t>(o_kfidx), ms_ptr<const int>(o_foff),
                       ms_ptr<const uint32_t>(o_fidx), ms_ptr<const int32_t>(o_kfmp), ms_ptr<const uint32_t>(o_kfdesc),
                       ms_ptr<const uint32_t>(o_fdesc), nnratio, F->two_cams ? F->nleft : -1, ms_ptr<int>(o_src));
    hipLaunchKernelGGL(k_bow_commit, dim3(1), dim3(1024), 0, s, ms_ptr<const OrbKeyPoint>(o_kfkeys),
                       ms_ptr<const OrbKeyPoint>(o_fkeys), fn, ms_ptr<const int32_t>(o_kfmp), checkOri,
                       ms_ptr<const int>(o_src), ms_ptr<int>(o_out), ms_ptr<int>(o_result));
    HIPCHK(hipGetLastError());
    timer.end();
    int nm = 0;
    HIPCHK(hipMemcpyAsync(out, ms_ptr<int>(o_out), (size_t)fn * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ms_ptr<int>(o_result), 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    nm = t_ms.hs[0];
    return nm;
}

int orbfe_stereo_knn_ratio(const uint8_t* left_desc, int32_t nl, const uint8_t* right_desc, int32_t nr, float ratio,
                           int32_t* out_train, int32_t* out_dist) {
    if (nl < 0 || nr < 0 || (nl > 0 && (!left_desc || !out_train || !out_dist)) || (nr > 0 && !right_desc))
        return ORBFE_E_ARG;
    if (nl == 0) return 0;
    Plan p;
    const size_t o_l = p.upload(left_desc, (size_t)nl * 32);
    const size_t o_r = p.upload(right_desc, (size_t)nr * 32);
    const size_t o_t = p.scratch((size_t)nl * 4);
    const size_t o_d = p.scratch((size_t)nl * 4);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    hipLaunchKernelGGL(k_knn2, dim3((nl + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, ms_ptr<const uint32_t>(o_l), nl,
                       ms_ptr<const uint32_t>(o_r), nr, ratio, ms_ptr<int>(o_t), ms_ptr<int>(o_d));
    HIPCHK(hipGetLastError());
    timer.end();
    HIPCHK(hipMemcpyAsync(out_train, ms_ptr<int>(o_t), (size_t)nl * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(out_dist, ms_ptr<int>(o_d), (size_t)nl * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int good = 0;
    for (int i = 0; i < nl; i++) good += out_train[i] >= 0;
    return good;
}

static void knn2_batch_launch(const StereoSide& SL, const StereoSide& SR, int cap, int nframes, float ratio,
                              int32_t* d_l2r, int32_t* d_dist, int32_t* d_ngood, hipStream_t s) {
    const size_t lds = (size_t)cap * 32;
    const dim3 grid((cap + KNN_Q - 1) / KNN_Q, nframes);
    if (nframes < 16)   // a few frames: the whole CU on each block's 64 queries
        hipLaunchKernelGGL(k_knn2_batch<16>, grid, dim3(1024), lds, s, SL, SR, cap, ratio, (int*)d_l2r, (int*)d_dist,
                           (int*)d_ngood);
    else
        hipLaunchKernelGGL(k_knn2_batch<4>, grid, dim3(256), lds, s, SL, SR, cap, ratio, (int*)d_l2r, (int*)d_dist,
                           (int*)d_ngood);
}

int orbfe_stereo_knn_slabs(const int32_t* d_counts_l, const uint8_t* d_desc_l, int lbase, int lstep,
                           const int32_t* d_counts_r, const uint8_t* d_desc_r, int rbase, int rstep, int cap,
                           int nframes, float ratio, int32_t* d_l2r, int32_t* d_dist, int32_t* d_ngood, void* stream) {
    if (!d_counts_l || !d_desc_l || !d_counts_r || !d_desc_r || nframes <= 0 || cap <= 0 || !d_l2r || !d_dist ||
        !d_ngood || lbase < 0 || rbase < 0 || lstep < 0 || rstep < 0)
        return ORBFE_E_ARG;
    const size_t lds = (size_t)cap * 32;
    if (lds > 128 * 1024) return ORBFE_E_ARG;
    StereoSide SL{nullptr, 0, nullptr, 0, nullptr, d_desc_l, d_counts_l, lbase, lstep};
    StereoSide SR{nullptr, 0, nullptr, 0, nullptr, d_desc_r, d_counts_r, rbase, rstep};
    hipStream_t s = (hipStream_t)stream;
    HIPCHK(hipMemsetAsync(d_ngood, 0, (size_t)nframes * 4, s));
    knn2_batch_launch(SL, SR, cap, nframes, ratio, d_l2r, d_dist, d_ngood, s);
    HIPCHK(hipGetLastError());
    return ORBFE_OK;
}

int orbfe_stereo_knn_batch(orbfe_extractor* left, int lbase, int lstep, orbfe_extractor* right, int rbase, int rstep,
                           int nframes, float ratio, int32_t* d_l2r, int32_t* d_dist, int32_t* d_ngood, void* stream) {
    if (!left || !right || nframes <= 0 || !d_l2r || !d_dist || !d_ngood) return ORBFE_E_ARG;
    std::lock_guard<std::mutex> lk(left->mu_stereo);
    if (!left->cap_b || !right->cap_b || left->g.kp_cap != right->g.kp_cap) return ORBFE_E_ARG;
    if (lbase < 0 || rbase < 0 || lbase + (nframes - 1) * lstep >= left->last_nimg ||
        rbase + (nframes - 1) * rstep >= right->last_nimg)
        return ORBFE_E_ARG;
    const int cap = left->g.kp_cap;
    const size_t lds = (size_t)cap * 32;
    if (lds > 128 * 1024) return ORBFE_E_ARG;
    StereoSide SL{left->d_ptrs, left->last_pitch, left->d_pyr, left->g.pyr_bytes, left->last_kps, left->last_desc,
                  left->last_counts, lbase, lstep};
    StereoSide SR{right->d_ptrs, right->last_pitch, right->d_pyr, right->g.pyr_bytes, right->last_kps,
                  right->last_desc, right->last_counts, rbase, rstep};
    hipStream_t s = pick_stream(left, stream);
    HIPCHK(hipMemsetAsync(d_ngood, 0, (size_t)nframes * 4, s));
    knn2_batch_launch(SL, SR, cap, nframes, ratio, d_l2r, d_dist, d_ngood, s);
    HIPCHK(hipGetLastError());
    return ORBFE_OK;
}

// A frame without keypoints matches nothing, but Tracking::SearchLocalPoints still runs isInFrustum
// over every point (Tracking.cc:3407-3425), so nToMatch is the projection's count.
static int empty_frame_n_to_match(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                  const orbfe_map_point_3d* pts, int32_t n, int32_t* n_to_match) {
    std::vector<orbfe_map_point> track((size_t)n);
    const int k = orbfe_is_in_frustum_rig(F, cam, rig, pts, n, track.data());
    if (k < 0) return k;
    if (n_to_match) *n_to_match = k;
    return 0;
}

int orbfe_search_local_points(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts,
                              int32_t n, int32_t* mvp, const int32_t* mvp_obs, float th, int32_t bFarPoints,
                              float thFarPoints, float nnratio, int32_t* n_to_match) {
    if (F && F->n == 0 && n > 0 && pts && cam && !F->two_cams)
        return empty_frame_n_to_match(F, cam, nullptr, pts, n, n_to_match);
    const FrustumIn fin{cam, pts, n_to_match, nullptr};
    return sbp_run(0, F, mvp, mvp_obs, nullptr, n, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                   offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0,
                   thFarPoints, nnratio, 0, 0, &fin);
}

int orbfe_search_by_projection_local_device(const orbfe_frame* F, int32_t* d_mvp, const int32_t* d_mvp_obs,
                                            const orbfe_map_point* d_mps, int32_t n_mps, float th,
                                            int32_t bFarPoints, float thFarPoints, float nnratio, void* stream) {
    const DevIn dv{(hipStream_t)stream};
    return sbp_run(0, F, d_mvp, d_mvp_obs, d_mps, n_mps, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                   offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0,
                   thFarPoints, nnratio, 0, 0, nullptr, &dv);
}

int orbfe_search_local_points_device(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* d_pts,
                                     int32_t n, int32_t* d_mvp, const int32_t* d_mvp_obs, float th,
                                     int32_t bFarPoints, float thFarPoints, float nnratio, int32_t* n_to_match,
                                     void* stream) {
    const FrustumIn fin{cam, d_pts, n_to_match, nullptr};
    const DevIn dv{(hipStream_t)stream};
    return sbp_run(0, F, d_mvp, d_mvp_obs, nullptr, n, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                   offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0,
                   thFarPoints, nnratio, 0, 0, &fin, &dv);
}

int orbfe_search_local_points_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                  const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* mvp_obs,
                                  float th, int32_t bFarPoints, float thFarPoints, float nnratio, int32_t* n_to_match) {
    if (!rig) return ORBFE_E_ARG;
    if (F && F->n == 0 && n > 0 && pts && cam) return empty_frame_n_to_match(F, cam, rig, pts, n, n_to_match);
    const FrustumIn fin{cam, pts, n_to_match, rig};
    return sbp_run(0, F, mvp, mvp_obs, nullptr, n, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                   offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0,
                   thFarPoints, nnratio, 0, 0, &fin);
}

int orbfe_search_local_points_rig_device(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                         const orbfe_map_point_3d* d_pts, int32_t n, int32_t* d_mvp,
                                         const int32_t* d_mvp_obs, float th, int32_t bFarPoints, float thFarPoints,
                                         float nnratio, int32_t* n_to_match, void* stream) {
    if (!rig) return ORBFE_E_ARG;
    const FrustumIn fin{cam, d_pts, n_to_match, rig};
    const DevIn dv{(hipStream_t)stream};
    return sbp_run(0, F, d_mvp, d_mvp_obs, nullptr, n, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                   offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0,
                   thFarPoints, nnratio, 0, 0, &fin, &dv);
}

int orbfe_search_local_points_track(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                                    const orbfe_map_point_3d* pts, int32_t n, int32_t* mvp, const int32_t* mvp_obs,
                                    float th, int32_t bFarPoints, float thFarPoints, float nnratio,
                                    int32_t* n_to_match, orbfe_map_point* track) {
    if (n < 0 || (n > 0 && !track)) return ORBFE_E_ARG;
    if (n == 0 || !F || F->n == 0 || !pts || !cam) {
        // no projection inside the search (a frame without keypoints, nothing to project): the
        // reference still runs isInFrustum over every point, so the records come from it alone
        int r = rig ? orbfe_search_local_points_rig(F, cam, rig, pts, n, mvp, mvp_obs, th, bFarPoints, thFarPoints,
                                                    nnratio, n_to_match)
                    : orbfe_search_local_points(F, cam, pts, n, mvp, mvp_obs, th, bFarPoints, thFarPoints, nnratio,
                                                n_to_match);
        if (r < 0 || n == 0) return r;
        const int k = rig ? orbfe_is_in_frustum_rig(F, cam, rig, pts, n, track) : orbfe_is_in_frustum(F, cam, pts, n, track);
        return k < 0 ? k : r;
    }
    // the records come back zero-copy: k_frustum stores them into mapped pinned memory as well, and
    // the host copies them out once the search's status word has arrived
    {   // this thread's scratch on the current device first (a first call or a device switch resets it)
        Plan p0;
        const int rc0 = ms_prepare(p0);
        if (rc0) return rc0;
    }
    MatchScratch& m = t_ms;
    if (m.th_cap < (size_t)n) {
        if (m.th) HIPCHK(hipHostFree(m.th));
        m.th = nullptr;
        m.th_cap = 0;
        const size_t cap = std::max<size_t>((size_t)n, 4096);
        HIPCHK(hipHostMalloc((void**)&m.th, cap * sizeof(orbfe_map_point), hipHostMallocMapped | hipHostMallocCoherent));
        HIPCHK(hipHostGetDevicePointer((void**)&m.th_dev, m.th, 0));
        m.th_cap = cap;
    }
    if (rig == nullptr && F->two_cams) return ORBFE_E_ARG;   // the pinhole API has no right camera
    FrustumIn fin{cam, pts, n_to_match, rig};
    fin.track_dev = m.th_dev;
    const orbfe_map_point* th_host = m.th;
    const int r = sbp_run(0, F, mvp, mvp_obs, nullptr, n, sizeof(orbfe_map_point), offsetof(orbfe_map_point, observations),
                          offsetof(orbfe_map_point, id), 0, offsetof(orbfe_map_point, scale_level), th, bFarPoints, 0,
                          thFarPoints, nnratio, 0, 0, &fin);
    if (r < 0) return r;
    std::atomic_thread_fence(std::memory_order_acquire);
    memcpy(track, th_host, (size_t)n * sizeof(orbfe_map_point));
    return r;
}

int orbfe_is_in_frustum(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_map_point_3d* pts, int32_t n,
                        orbfe_map_point* track) {
    if (F && F->two_cams) return ORBFE_E_ARG;   // the pinhole API has no right camera
    return orbfe_is_in_frustum_rig(F, cam, nullptr, pts, n, track);
}

int orbfe_is_in_frustum_rig(const orbfe_frame* F, const orbfe_camera* cam, const orbfe_stereo_rig* rig,
                            const orbfe_map_point_3d* pts, int32_t n, orbfe_map_point* track) {
    if (!F || !cam || n < 0 || (n > 0 && (!pts || !track)) || F->nlevels <= 0) return ORBFE_E_ARG;
    if (n == 0) return 0;
    Plan p;
    const size_t o_pts = p.upload(pts, (size_t)n * sizeof(orbfe_map_point_3d));
    const size_t o_track = p.scratch((size_t)n * sizeof(orbfe_map_point));
    const size_t o_ntm = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    CamDev cd;
    if (!make_camdev(F, cam, rig, cd)) return ORBFE_E_ARG;
    int* ntm = ms_ptr<int>(o_ntm);
    HIPCHK(hipMemsetAsync(ntm, 0, 4, s));
    hipLaunchKernelGGL(k_frustum, dim3((n + MT_NT - 1) / MT_NT), dim3(MT_NT), 0, s, cd,
                       ms_ptr<const orbfe_map_point_3d>(o_pts), n, ms_ptr<orbfe_map_point>(o_track), ntm);
    HIPCHK(hipGetLastError());
    timer.end();
    int h_ntm = 0;
    HIPCHK(hipMemcpyAsync(track, ms_ptr<orbfe_map_point>(o_track), (size_t)n * sizeof(orbfe_map_point),
                          hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(t_ms.hs, ntm, 4, hipMemcpyDeviceToHost, s));   // pinned
    HIPCHK(hipStreamSynchronize(s));
    h_ntm = t_ms.hs[0];
    return h_ntm;
}

int orbfe_matcher_set_timing(int enable) {
    t_timing = enable != 0;
    return ORBFE_OK;
}

int orbfe_matcher_set_stats(int enable) {
    t_stats = enable != 0;
    return ORBFE_OK;
}

int orbfe_matcher_last_stats(long long* out) {
    if (!out) return ORBFE_E_ARG;
    for (int i = 0; i < 3; i++) out[i] = t_last_stats[i];
    return t_last_stats[2] >= 0 ? ORBFE_OK : ORBFE_E_ARG;
}

float orbfe_matcher_last_ms(void) { return t_last_ms; }

}  // extern "C"
