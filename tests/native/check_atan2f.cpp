// CPU check of the glibc atan2f port (orb_slam3_ros_amd/csrc/glibc_atan2f.h) against the host libm:
// random bit patterns (every exponent, NaN / Inf / subnormals included), camera-ray-like values
// (1e-3 grid in [-1000, 1000]) and the special-value grid. usage: check_atan2f [pairs]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "../../orb_slam3_ros_amd/csrc/glibc_atan2f.h"

int main(int argc, char** argv) {
    const long pairs = argc > 1 ? atol(argv[1]) : 20000000;
    std::mt19937_64 rng(1);
    long bad = 0, n = 0;
    auto chk = [&](float y, float x) {
        const float a = atan2f(y, x), b = orbfe::glibc_atan2f(y, x);
        n++;
        if (memcmp(&a, &b, 4) && !(a != a && b != b)) {
            if (bad < 10) printf("y %a x %a host %a port %a\n", y, x, a, b);
            bad++;
        }
    };
    for (long i = 0; i < pairs; i++) {
        const uint32_t u = (uint32_t)rng(), v = (uint32_t)rng();
        float y, x;
        memcpy(&y, &u, 4);
        memcpy(&x, &v, 4);
        chk(y, x);
        chk((float)((int32_t)(rng() % 2000001) - 1000000) * 1e-3f, (float)((int32_t)(rng() % 2000001) - 1000000) * 1e-3f);
    }
    const float sp[] = {0.f, -0.f, 1.f, -1.f, INFINITY, -INFINITY, NAN, 1e-30f, -1e-30f, 1e30f, 3.f, 0.5f, 1e-45f};
    for (float a : sp)
        for (float b : sp) chk(a, b);
    printf("checked %ld mismatches %ld\n", n, bad);
    return bad != 0;
}
