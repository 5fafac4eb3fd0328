// Exhaustive check: orbfe::glibc_cosf/sinf (the port the HIP descriptor kernel uses) against the
// host libm cosf/sinf for every float in [lo, hi]. Prints mismatches count; exit 1 on any mismatch.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <thread>
#include <vector>
#include <atomic>
#include "../../orb_slam3_ros_amd/csrc/glibc_sincosf.h"
int main(int argc, char** argv) {
    float lo = argc > 1 ? strtof(argv[1], 0) : 0.f, hi = argc > 2 ? strtof(argv[2], 0) : 6.2842f;
    int nth = argc > 3 ? atoi(argv[3]) : 8;
    uint32_t ulo, uhi; memcpy(&ulo, &lo, 4); memcpy(&uhi, &hi, 4);
    std::atomic<long> bad{0}, tot{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++) th.emplace_back([&, t]() {
        long b = 0, n = 0;
        for (uint64_t u = ulo + t; u <= uhi; u += nth) {
            float x; uint32_t uu = (uint32_t)u; memcpy(&x, &uu, 4);
            volatile float xv = x;
            float c0 = cosf(xv), s0 = sinf(xv);
            float c1 = orbfe::glibc_cosf(x), s1 = orbfe::glibc_sinf(x);
            if (memcmp(&c0, &c1, 4) || memcmp(&s0, &s1, 4)) {
                if (b < 3) fprintf(stderr, "mismatch x=%a cos %a/%a sin %a/%a\n", x, c0, c1, s0, s1);
                b++;
            }
            n++;
        }
        bad += b; tot += n;
    });
    for (auto& t : th) t.join();
    printf("checked %ld floats, mismatches %ld\n", tot.load(), bad.load());
    return bad.load() ? 1 : 0;
}
