// Bit-exact restatement of glibc's single-precision logf (sysdeps/ieee754/flt-32/e_logf.c,
// e_logf_data.c; glibc >= 2.28, the implementation Ubuntu 20.04 / 22.04 ship) for positive normal
// and subnormal inputs. MapPoint::PredictScale computes ceil(log(ratio) / mfLogScaleFactor) on a
// float ratio (MapPoint.cc:531-546), which resolves to logf through OpenCV's <math.h>.
// glibc dispatches logf through an ifunc: every AVX2/FMA host runs the FMA variant (the products
// below fused), older hosts the SSE2 variant; ORBFE_LOGF_FMA picks the modelled one (default 1).
// The 16-entry (invc, logc) table, Ln2 and the polynomial were read from the host libm (the FMA
// variant's RIP-relative constants); tests/native/check_logf.cpp compares this port with the host
// logf for every float in [2^-10, 2^10).
// Host + device (HIP) code; must be compiled with -ffp-contract=off.
#pragma once
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifndef ORBFE_HD
#if defined(__HIPCC__)
#define ORBFE_HD __host__ __device__ inline
#else
#define ORBFE_HD inline
#endif
#endif

#ifndef ORBFE_LOGF_FMA
#define ORBFE_LOGF_FMA 1
#endif

namespace orbfe {

ORBFE_HD double logf_tab(int i, int which) {
    const double t[16][2] = {
        {0x1.661ec79f8f3bep+0, -0x1.57bf7808caadep-2}, {0x1.571ed4aaf883dp+0, -0x1.2bef0a7c06ddbp-2},
        {0x1.49539f0f010b0p+0, -0x1.01eae7f513a67p-2}, {0x1.3c995b0b80385p+0, -0x1.b31d8a68224e9p-3},
        {0x1.30d190c8864a5p+0, -0x1.6574f0ac07758p-3}, {0x1.25e227b0b8ea0p+0, -0x1.1aa2bc79c8100p-3},
        {0x1.1bb4a4a1a343fp+0, -0x1.a4e76ce8c0e5ep-4}, {0x1.12358f08ae5bap+0, -0x1.1973c5a611cccp-4},
        {0x1.0953f419900a7p+0, -0x1.252f438e10c1ep-5}, {0x1.0000000000000p+0, 0x0.0p+0},
        {0x1.e608cfd9a47acp-1, 0x1.aa5aa5df25984p-5}, {0x1.ca4b31f026aa0p-1, 0x1.c5e53aa362eb4p-4},
        {0x1.b2036576afce6p-1, 0x1.526e57720db08p-3}, {0x1.9c2d163a1aa2dp-1, 0x1.bc2860d224770p-3},
        {0x1.886e6037841edp-1, 0x1.1058bc8a07ee1p-2}, {0x1.767dcf5534862p-1, 0x1.4043057b6ee09p-2}};
    return t[i][which];
}

ORBFE_HD float glibc_logf(float x) {
    const double Ln2 = 0x1.62e42fefa39efp-1;
    const double A0 = -0x1.00ea348b88334p-2, A1 = 0x1.5575b0be00b6ap-2, A2 = -0x1.ffffef20a4123p-2;
    uint32_t ix;
    memcpy(&ix, &x, 4);
    if (ix == 0x3f800000u) return 0.0f;
    if (ix - 0x00800000u >= 0x7f800000u - 0x00800000u) {
        // zero, negative, inf, nan, subnormal
        if (ix * 2 == 0) return -INFINITY;
        if (ix == 0x7f800000u) return x;
        if ((ix & 0x80000000u) || ix * 2 >= 0xff000000u) return (x - x) / (x - x);
        // subnormal: normalise
        float xs = x * 0x1p23f;
        memcpy(&ix, &xs, 4);
        ix -= 23u << 23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const int k = (int32_t)tmp >> 23;
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const double invc = logf_tab(i, 0), logc = logf_tab(i, 1);
    float zf;
    memcpy(&zf, &iz, 4);
    const double z = (double)zf;
#if ORBFE_LOGF_FMA
    const double r = fma(z, invc, -1.0);
    const double y0 = fma((double)k, Ln2, logc);
    const double r2 = r * r;
    double y = fma(A1, r, A2);
    y = fma(A0, r2, y);
    y = fma(y, r2, y0 + r);
#else
    const double r = z * invc - 1.0;
    const double y0 = logc + (double)k * Ln2;
    const double r2 = r * r;
    double y = A1 * r + A2;
    y = A0 * r2 + y;
    y = y * r2 + (y0 + r);
#endif
    return (float)y;
}

}  // namespace orbfe
