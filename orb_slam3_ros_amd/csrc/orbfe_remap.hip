// cv::remap(src, dst, map1, map2, INTER_LINEAR) for 8UC1 images and CV_32FC1 map pairs, the stereo
// rectification of System::TrackStereo (System.cc:233-240, maps from initUndistortRectifyMap(...,
// CV_32F, ...), Settings.cc:506-509), restated from OpenCV 4.2 imgwarp.cpp:
//  * map -> fixed point: X = cvRound(mapx * 32), sx = X >> 5, fx = X & 31 (same for y);
//  * BilinearTab_i[fy][fx] = ((32 - fy)(32 - fx), (32 - fy) fx, fy (32 - fx), fy fx) * 32 — exact
//    integers summing to 32768 — except cell (0, 0), whose 32768 saturates to 32767 and whose
//    deficit initInterTab2D adds to the (1, 1) weight: (32767, 0, 0, 1);
//  * D = (w0 S00 + w1 S01 + w2 S10 + w3 S11 + 2^14) >> 15 (FixedPtCast, INTER_REMAP_COEF_BITS = 15);
//  * BORDER_CONSTANT (value 0): a sample outside the source reads 0; a pixel whose 2x2 footprint
//    is entirely outside is 0.
#pragma once

// The map-only part of one output pixel (identical for every image of a batch: one map pair
// serves one camera): source offset of the 2x2 footprint, the BilinearTab_i weights packed as
// u16 pairs, which footprint samples lie inside the source (bits 0-3: S00, S01, S10, S11) and
// whether the whole footprint is outside (the pixel is 0).
struct RemapPx {
    int off;
    uint32_t w01, w23;
    uint32_t inside;   // bits 0-3 as above, bit 4 = at least one sample inside
};
__device__ __forceinline__ RemapPx remap_setup(int sw, int sh, int sstride, float mx, float my) {
    const float fxs = mx * 32.f, fys = my * 32.f;
    // saturate_cast<int>(float): round half to even, saturating
    const int X = fxs >= 2147483520.f ? INT_MAX : (fxs <= -2147483648.f ? INT_MIN : __float2int_rn(fxs));
    const int Y = fys >= 2147483520.f ? INT_MAX : (fys <= -2147483648.f ? INT_MIN : __float2int_rn(fys));
    const int sx = min(max(X >> 5, -32768), 32767), sy = min(max(Y >> 5, -32768), 32767);
    const int ax = X & 31, ay = Y & 31;
    uint32_t w0, w1, w2, w3;
    if (ax == 0 && ay == 0) {
        w0 = 32767; w1 = 0; w2 = 0; w3 = 1;
    } else {
        w0 = (uint32_t)((32 - ay) * (32 - ax) * 32);
        w1 = (uint32_t)((32 - ay) * ax * 32);
        w2 = (uint32_t)(ay * (32 - ax) * 32);
        w3 = (uint32_t)(ay * ax * 32);
    }
    RemapPx r;
    r.w01 = w0 | (w1 << 16);
    r.w23 = w2 | (w3 << 16);
    if (sx >= sw || sx + 1 < 0 || sy >= sh || sy + 1 < 0) {
        r.off = 0;
        r.inside = 0;
        return r;
    }
    r.off = sy * sstride + sx;   // sx, sy in [-1, sw - 1] x [-1, sh - 1] here
    r.inside = 16u | (sx >= 0 && sy >= 0 ? 1u : 0u) | (sx + 1 < sw && sy >= 0 ? 2u : 0u) |
               (sx >= 0 && sy + 1 < sh ? 4u : 0u) | (sx + 1 < sw && sy + 1 < sh ? 8u : 0u);
    return r;
}
// D = (w0 S00 + w1 S01 + w2 S10 + w3 S11 + 2^14) >> 15 (FixedPtCast, INTER_REMAP_COEF_BITS = 15);
// BORDER_CONSTANT: a sample outside the source reads 0
__device__ __forceinline__ uint32_t remap_apply(gptr_u8 src, int sstride, const RemapPx& r) {
    if (!(r.inside & 16u)) return 0u;
    gptr_u8 p = src + r.off;
    int v0, v1, v2, v3;
    if ((r.inside & 15u) == 15u) {
        v0 = p[0]; v1 = p[1]; v2 = p[sstride]; v3 = p[sstride + 1];
    } else {
        v0 = (r.inside & 1u) ? p[0] : 0;
        v1 = (r.inside & 2u) ? p[1] : 0;
        v2 = (r.inside & 4u) ? p[sstride] : 0;
        v3 = (r.inside & 8u) ? p[sstride + 1] : 0;
    }
    const int v = (v0 * (int)(r.w01 & 0xFFFFu) + v1 * (int)(r.w01 >> 16) + v2 * (int)(r.w23 & 0xFFFFu) +
                   v3 * (int)(r.w23 >> 16) + (1 << 14)) >> 15;
    return (uint32_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// One thread per 4 adjacent output pixels, for RM_IPB images of the batch: the map is read and
// converted once per pixel and image group (the maps are larger than the images: 8 B per pixel).
// Fast path (every sample of the 4 footprints inside the source, one source row pair, and the 4
// footprints inside one 8-byte window from (off_0 & ~3)): 4 aligned dword loads per image, the
// (S00, S01) and (S10, S11) pairs of a pixel by one v_perm each, and the weighted sum by two
// v_dot2_u32_u16 against the BilinearTab_i weights, which RemapPx already packs as u16 pairs.
// Otherwise the 16 guarded byte loads of remap_apply. Measured (512 images, 752x480): 516 ->
// 443 us; image-group-major block order and issuing a group's loads before its stores were slower.
#define RM_IPB 8

typedef unsigned short orbfe_ushort2_rm __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_remap(const uint8_t* const* __restrict__ srcs, int sw, int sh, int sstride,
                                               const float* __restrict__ mapx, const float* __restrict__ mapy,
                                               int dw, int dh, uint8_t* const* __restrict__ dsts, int dstride, int n,
                                               int src_al) {
    // XCD-aware order: the blocks one XCD runs are consecutive tiles of one image group, so the
    // source rows two adjacent tiles share are fetched into that XCD's L2 once
    const int lb = xcd_logical(block_linear(), gridDim.x * gridDim.y);
    const int grp = lb / gridDim.x, tile = lb - grp * gridDim.x;
    const int ng = (dw + 3) >> 2;
    const int t = tile * blockDim.x + threadIdx.x;
    if (t >= ng * dh) return;
    const int y = t / ng, x0 = 4 * (t - y * ng);
    const float* mxr = mapx + (size_t)y * dw;
    const float* myr = mapy + (size_t)y * dw;
    const bool full = x0 + 4 <= dw;
    float mx[4], my[4];
    if (full && ((dw & 3) == 0)) {
        const float4 a = *(const float4*)(mxr + x0), c = *(const float4*)(myr + x0);
        mx[0] = a.x; mx[1] = a.y; mx[2] = a.z; mx[3] = a.w;
        my[0] = c.x; my[1] = c.y; my[2] = c.z; my[3] = c.w;
    } else {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            mx[q] = x0 + q < dw ? mxr[x0 + q] : 0.f;
            my[q] = x0 + q < dw ? myr[x0 + q] : 0.f;
        }
    }
    RemapPx r[4];
#pragma unroll
    for (int q = 0; q < 4; q++) r[q] = remap_setup(sw, sh, sstride, mx[q], my[q]);
    // the fast path's window: base = off_0 & ~3 (4-byte aligned when the sources' rows are), every
    // pixel's pair at d = off - base in [0, 6], and the window's columns inside the row
    const int base = r[0].off & ~3;
    bool fast = src_al && full;
    uint32_t sel[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int d = r[q].off - base;
        fast = fast && (r[q].inside & 15u) == 15u && d >= 0 && d <= 6;
        sel[q] = 0x0c000c00u | (uint32_t)(d & 7) | ((uint32_t)((d + 1) & 7) << 16);
    }
    // (inside the image width, not the pitch: the last row of a pitched buffer may end at sw)
    fast = fast && (base - (r[0].off - (r[0].off % sstride))) + 8 <= sw;
    const int i0 = grp * RM_IPB, i1 = min(i0 + RM_IPB, n);
    // the fast path's two 8-byte windows of image img, as one dwordx2 load each (4-byte aligned:
    // the hardware's unaligned global access). Every lane loads (the others from offset 0, never
    // used), so the loads are unconditional and the next image's pair is in flight while this
    // image is computed and stored.
    const int woff = fast ? base : 0, woff2 = fast ? base + sstride : 0;
    auto ldw = [&](int img, uint2& wa, uint2& wb) {
        gptr_u8 src = as_global(srcs[img]);
        __builtin_memcpy(&wa, (const void*)(src + woff), 8);
        __builtin_memcpy(&wb, (const void*)(src + woff2), 8);
    };
    uint2 na = {0u, 0u}, nb = {0u, 0u};
    if (src_al) ldw(i0, na, nb);   // src_al (wave-uniform) also guarantees >= 16 bytes per source
    for (int img = i0; img < i1; img++) {
        const uint2 wa = na, wb = nb;
        if (src_al && img + 1 < i1) ldw(img + 1, na, nb);
        ORBFE_GLOBAL uint8_t* dst = (ORBFE_GLOBAL uint8_t*)dsts[img] + (size_t)y * dstride;   // global stores, not flat
        uint32_t packed = 0;
        if (fast) {
            const uint32_t a0 = wa.x, a1 = wa.y, b0 = wb.x, b1 = wb.y;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const uint32_t t0 = __builtin_amdgcn_perm(a1, a0, sel[q]), t1 = __builtin_amdgcn_perm(b1, b0, sel[q]);
                uint32_t acc = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2_rm, t0),
                                                      __builtin_bit_cast(orbfe_ushort2_rm, r[q].w01), 1u << 14, false);
                acc = __builtin_amdgcn_udot2(__builtin_bit_cast(orbfe_ushort2_rm, t1),
                                             __builtin_bit_cast(orbfe_ushort2_rm, r[q].w23), acc, false);
                packed |= (acc >> 15) << (8 * q);   // <= 255: the weights sum to 32768
            }
        } else {
            gptr_u8 src = as_global(srcs[img]);
#pragma unroll
            for (int q = 0; q < 4; q++) packed |= remap_apply(src, sstride, r[q]) << (8 * q);
        }
        if (full && ((((uintptr_t)(dst + x0)) & 3) == 0)) {
            *(ORBFE_GLOBAL uint32_t*)(dst + x0) = packed;
        } else {
            for (int q = 0; q < 4 && x0 + q < dw; q++) dst[x0 + q] = (uint8_t)(packed >> (8 * q));
        }
    }
}

// cv::undistortPoints(pts, pts, K, D, noArray(), K) for CV_32FC2 points (Frame::UndistortKeyPoints,
// Frame.cc:747-780), restated from OpenCV 4.2 cvUndistortPointsInternal: double arithmetic, the
// default criteria (COUNT, 5 iterations), identity tilt and rectification, P = K. One thread per
// point; the expression order follows the OpenCV source (no contraction).
struct UndistArgs {
    double fx, fy, cx, cy, ifx, ify;
    double k[12];
};
__global__ __launch_bounds__(256) void k_undistort(const float* __restrict__ in, int n, UndistArgs a, float* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* k = a.k;
    double x = in[2 * i], y = in[2 * i + 1];
    const double u = x, v = y;
    x = (x - a.cx) * a.ifx;
    y = (y - a.cy) * a.ify;
    // invMatTilt = identity: vecUntilt = (1*x + 0*y + 0*1, 0*x + 1*y + 0*1, 0*x + 0*y + 1*1)
    const double ux = (1.0 * x + 0.0 * y) + 0.0 * 1.0, uy = (0.0 * x + 1.0 * y) + 0.0 * 1.0;
    const double uz = (0.0 * x + 0.0 * y) + 1.0 * 1.0;
    const double invProj = uz != 0.0 ? 1. / uz : 1;
    double x0 = x = invProj * ux;
    double y0 = y = invProj * uy;
    for (int j = 0; j < 5; j++) {
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        if (icdist < 0) {
            x = (u - a.cx) * a.ifx;
            y = (v - a.cy) * a.ify;
            break;
        }
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x) + k[8] * r2 + k[9] * r2 * r2;
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y + k[10] * r2 + k[11] * r2 * r2;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I = K
    const double xx = a.fx * x + 0.0 * y + a.cx;
    const double yy = 0.0 * x + a.fy * y + a.cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    out[2 * i] = (float)(xx * ww);
    out[2 * i + 1] = (float)(yy * ww);
}

extern "C" {

int orbfe_undistort_points(const float* pts, int n, const float* K4, const float* dist, int ndist, float* out) {
    if (n < 0 || (n > 0 && (!pts || !out)) || !K4 || (ndist > 0 && !dist) || ndist < 0 || ndist > 12) return ORBFE_E_ARG;
    if (n == 0) return 0;
    UndistArgs a;
    memset(&a, 0, sizeof(a));
    a.fx = (double)K4[0]; a.fy = (double)K4[1]; a.cx = (double)K4[2]; a.cy = (double)K4[3];
    a.ifx = 1. / a.fx;
    a.ify = 1. / a.fy;
    for (int i = 0; i < ndist; i++) a.k[i] = (double)dist[i];
    Plan p;
    const size_t o_in = p.upload(pts, (size_t)n * 8);
    const size_t o_out = p.scratch((size_t)n * 8);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, s, ms_ptr<const float>(o_in), n, a,
                       ms_ptr<float>(o_out));
    HIPCHK(hipGetLastError());
    timer.end();
    HIPCHK(hipMemcpyAsync(out, ms_ptr<float>(o_out), (size_t)n * 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return n;
}

int orbfe_remap_linear_batch(const uint8_t* const* d_src, int sw, int sh, int sstride, const float* d_mapx,
                             const float* d_mapy, int dw, int dh, uint8_t* const* d_dst, int dstride, int n,
                             void* stream) {
    if (n <= 0 || sw < 0 || sh < 0 || dw <= 0 || dh <= 0 || !d_src || !d_dst || !d_mapx || !d_mapy ||
        sstride < sw || dstride < dw)
        return n == 0 ? ORBFE_OK : ORBFE_E_ARG;
    if ((size_t)sw * sh == 0) return ORBFE_E_EMPTY;
    // the pointer tables live in a small per-thread ring of device tables keyed by the caller's
    // pointers (a rectification loop passes the same buffers every frame, a double-buffered one
    // alternates two sets): a hit launches without any upload; a miss takes the least recently
    // used slot, waits only for the last launch that read it (its event), refills its pinned
    // staging and uploads it asynchronously on s ahead of the launch
    struct RemapSlot {
        std::vector<const void*> key;
        void** dev = nullptr;
        void** pinned = nullptr;
        size_t cap = 0;
        hipEvent_t done = nullptr;
        uint64_t used = 0;
    };
    static thread_local RemapSlot ring[4];
    static thread_local uint64_t tick = 0;
    hipStream_t s = (hipStream_t)stream;
    RemapSlot* slot = nullptr;
    for (RemapSlot& r : ring)
        if (r.dev && r.key.size() == (size_t)2 * n && std::equal(d_src, d_src + n, r.key.begin()) &&
            std::equal(d_dst, d_dst + n, r.key.begin() + n))
            slot = &r;
    if (!slot) {
        slot = &ring[0];
        for (RemapSlot& r : ring)
            if (r.used < slot->used) slot = &r;
        if (slot->done) HIPCHK(hipEventSynchronize(slot->done));
        else HIPCHK(hipEventCreateWithFlags(&slot->done, hipEventDisableTiming));
        slot->key.clear();
        if (slot->cap < (size_t)2 * n) {
            if (slot->dev) HIPCHK(hipFree(slot->dev));
            if (slot->pinned) HIPCHK(hipHostFree(slot->pinned));
            slot->dev = slot->pinned = nullptr;
            slot->cap = 0;
            HIPCHK(hipMalloc((void**)&slot->dev, (size_t)2 * n * sizeof(void*)));
            HIPCHK(hipHostMalloc((void**)&slot->pinned, (size_t)2 * n * sizeof(void*), hipHostMallocDefault));
            slot->cap = (size_t)2 * n;
        }
        slot->key.assign(d_src, d_src + n);
        slot->key.insert(slot->key.end(), d_dst, d_dst + n);
        memcpy(slot->pinned, slot->key.data(), (size_t)2 * n * sizeof(void*));
        HIPCHK(hipMemcpyAsync(slot->dev, slot->pinned, (size_t)2 * n * sizeof(void*), hipMemcpyHostToDevice, s));
    } else {
        // a hit may come on another stream than the miss that uploaded the table (or than the
        // slot's earlier readers): order this launch after the slot's last use, whose event
        // follows the upload and, through this same wait on every hit, every earlier reader
        HIPCHK(hipStreamWaitEvent(s, slot->done, 0));
    }
    slot->used = ++tick;
    const uint8_t* const* dsrc = (const uint8_t* const*)slot->dev;
    uint8_t* const* ddst = (uint8_t* const*)(slot->dev + n);
    const int ng = (dw + 3) >> 2;
    // the fast path's dword loads need 4-byte aligned source rows
    bool al = (sstride & 3) == 0 && (size_t)sstride * (size_t)(sh - 1) + (size_t)sw >= 16;
    for (int i = 0; al && i < n; i++) al = (((uintptr_t)d_src[i]) & 3) == 0;
    const dim3 grid((ng * dh + 255) / 256, (n + RM_IPB - 1) / RM_IPB);
    hipLaunchKernelGGL(k_remap, grid, dim3(256), 0, s, dsrc, sw, sh,
                       sstride, d_mapx, d_mapy, dw, dh, ddst, dstride, n, al ? 1 : 0);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(slot->done, s));
    return ORBFE_OK;
}

int orbfe_remap_linear(const uint8_t* src, int sw, int sh, int sstride, const float* mapx, const float* mapy, int dw,
                       int dh, uint8_t* dst, int dstride) {
    if (!src || !mapx || !mapy || !dst || sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || sstride < sw || dstride < dw)
        return ORBFE_E_ARG;
    Plan p;
    const size_t o_mx = p.upload(mapx, (size_t)dw * dh * 4), o_my = p.upload(mapy, (size_t)dw * dh * 4);
    const size_t o_src = p.upload(src, (size_t)sstride * (sh - 1) + sw);
    const size_t o_dst = p.scratch((size_t)dw * dh);
    const size_t o_ptr = p.scratch(16);
    int rc = ms_prepare(p);
    if (rc) return rc;
    MsTimer timer;
    hipStream_t s = t_ms.stream;
    const uint8_t* ptrs[2] = {ms_ptr<const uint8_t>(o_src), ms_ptr<uint8_t>(o_dst)};
    HIPCHK(hipMemcpyAsync(ms_ptr<uint8_t>(o_ptr), ptrs, 16, hipMemcpyHostToDevice, s));
    const int nt = (((dw + 3) >> 2) * dh + 255) / 256;
    hipLaunchKernelGGL(k_remap, dim3(nt, 1), dim3(256), 0, s,
                       (const uint8_t* const*)ms_ptr<uint8_t>(o_ptr), sw, sh, sstride, ms_ptr<const float>(o_mx),
                       ms_ptr<const float>(o_my), dw, dh, (uint8_t* const*)(ms_ptr<uint8_t>(o_ptr) + 8), dw, 1,
                       (((uintptr_t)ms_ptr<uint8_t>(o_src) & 3) == 0 && (sstride & 3) == 0 &&
                        (size_t)sstride * (size_t)(sh - 1) + (size_t)sw >= 16) ? 1 : 0);
    HIPCHK(hipGetLastError());
    timer.end();
    HIPCHK(hipMemcpy2DAsync(dst, dstride, ms_ptr<uint8_t>(o_dst), dw, dw, dh, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return ORBFE_OK;
}

}  // extern "C"
