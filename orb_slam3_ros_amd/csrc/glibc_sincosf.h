// Bit-exact restatement of glibc's single-precision cosf/sinf (sysdeps/ieee754/flt-32/s_sinf.c,
// s_cosf.c, sincosf.h; glibc >= 2.28, the implementation Ubuntu 20.04/22.04 ship) for the argument
// range the ORB descriptor uses: angle * pi/180 with angle in [0, 360] (ORBextractor.cc:111-112,
// where `cos(float)` resolves to cosf). Two code paths exist in glibc on x86-64: the FMA ifunc
// variant (selected on every AVX2/FMA host) and the SSE2 variant; ORBFE_SINCOSF_FMA picks which
// one is modelled (default 1). The polynomial table was read from the host libm
// (__sincosf_table); tests/test_sincosf.py checks this port against the host libm for EVERY float
// in [0, 2*pi + 1e-3], so a host whose libm disagrees is detected rather than assumed.
// Host + device (HIP) code; must be compiled with -ffp-contract=off.
#pragma once
#include <stdint.h>
#include <string.h>

#ifndef ORBFE_HD
#if defined(__HIPCC__)
#define ORBFE_HD __host__ __device__ inline
#else
#define ORBFE_HD inline
#endif
#endif

#ifndef ORBFE_SINCOSF_FMA
#define ORBFE_SINCOSF_FMA 1
#endif

namespace orbfe {

struct SinCosTable {
    double hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4;
};

ORBFE_HD double sc_coef(int neg, int i) {
    // {hpi_inv, hpi, c0, c1, s1, c2, s2, c3, s3, c4}; entry 1 negates the cosine polynomial.
    const double t0[10] = {0x1.45f306dc9c883p+23, 0x1.921fb54442d18p+0, 0x1.0p+0, -0x1.ffffffd0c621cp-2,
                           -0x1.555545995a603p-3, 0x1.55553e1068f19p-5, 0x1.1107605230bc4p-7,
                           -0x1.6c087e89a359dp-10, -0x1.994eb3774cf24p-13, 0x1.99343027bf8c3p-16};
    const double v = t0[i];
    const bool is_cos = (i == 2 || i == 3 || i == 5 || i == 7 || i == 9);
    return (neg && is_cos) ? -v : v;
}

ORBFE_HD double sc_madd(double a, double b, double c) {  // a*b + c as the glibc build evaluates it
#if ORBFE_SINCOSF_FMA
    return __builtin_fma(a, b, c);
#else
    return a * b + c;
#endif
}

ORBFE_HD uint32_t sc_abstop12(float x) {
    uint32_t u;
    memcpy(&u, &x, 4);
    return (u >> 20) & 0x7ff;
}

// sinf_poly(x, x2, p, n)
ORBFE_HD float sc_poly(double x, double x2, int neg, int n) {
    if ((n & 1) == 0) {
        double x3 = x * x2;
        double s1 = sc_madd(x2, sc_coef(neg, 8), sc_coef(neg, 6));   // s2 + x2*s3
        double x7 = x3 * x2;
        double s = sc_madd(x3, sc_coef(neg, 4), x);                    // x + x3*s1
        return (float)sc_madd(x7, s1, s);                              // s + x7*s1
    } else {
        double x4 = x2 * x2;
        double c2 = sc_madd(x2, sc_coef(neg, 9), sc_coef(neg, 7));   // c3 + x2*c4
        double c1 = sc_madd(x2, sc_coef(neg, 3), sc_coef(neg, 2));   // c0 + x2*c1
        double x6 = x4 * x2;
        double c = sc_madd(x4, sc_coef(neg, 5), c1);                   // c1 + x4*c2
        return (float)sc_madd(x6, c2, c);                              // c + x6*c2
    }
}

// reduce_fast (non-TOINT_INTRINSICS form used on x86-64)
ORBFE_HD double sc_reduce(double x, int* np) {
    double r = x * sc_coef(0, 0);
    int n = ((int32_t)r + 0x800000) >> 24;
    *np = n;
#if ORBFE_SINCOSF_FMA
    return __builtin_fma(-(double)n, sc_coef(0, 1), x);
#else
    return x - n * sc_coef(0, 1);
#endif
}

// Valid for |y| < 120 (the ORB range is [0, 2*pi]); larger inputs are never produced here.
ORBFE_HD float glibc_cosf(float y) {
    double x = y;
    const float pio4 = 0x1.921FB6p-1f;
    if (sc_abstop12(y) < sc_abstop12(pio4)) {
        double x2 = x * x;
        if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) return 1.0f;
        return sc_poly(x, x2, 0, 1);
    }
    int n;
    x = sc_reduce(x, &n);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sc_poly(x * s, x * x, (n & 2) ? 1 : 0, n ^ 1);
}

ORBFE_HD float glibc_sinf(float y) {
    double x = y;
    const float pio4 = 0x1.921FB6p-1f;
    if (sc_abstop12(y) < sc_abstop12(pio4)) {
        double s = x * x;
        if (sc_abstop12(y) < sc_abstop12(0x1p-12f)) return y;
        return sc_poly(x, s, 0, 0);
    }
    int n;
    x = sc_reduce(x, &n);
    const double s = ((n & 3) == 1 || (n & 3) == 2) ? -1.0 : 1.0;
    return sc_poly(x * s, x * x, (n & 2) ? 1 : 0, n);
}

}  // namespace orbfe
