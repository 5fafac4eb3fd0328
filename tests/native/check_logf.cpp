// Exhaustive check: orbfe::glibc_logf (the port the HIP frustum / PredictScale kernel uses) against
// the host libm logf for every float in [lo, hi] plus subnormals and special values. Prints the
// mismatch count; exit 1 on any mismatch.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <thread>
#include <vector>
#include "../../orb_slam3_ros_amd/csrc/glibc_logf.h"
static bool same(float a, float b) { return memcmp(&a, &b, 4) == 0 || (isnan(a) && isnan(b)); }
int main(int argc, char** argv) {
    float lo = argc > 1 ? strtof(argv[1], 0) : 0x1p-10f, hi = argc > 2 ? strtof(argv[2], 0) : 0x1p10f;
    int nth = argc > 3 ? atoi(argv[3]) : 8;
    uint32_t ulo, uhi;
    memcpy(&ulo, &lo, 4);
    memcpy(&uhi, &hi, 4);
    std::atomic<long> bad{0}, tot{0};
    std::vector<std::thread> th;
    for (int t = 0; t < nth; t++)
        th.emplace_back([&, t]() {
            long b = 0, n = 0;
            for (uint64_t u = ulo + t; u <= uhi; u += nth) {
                float x;
                uint32_t uu = (uint32_t)u;
                memcpy(&x, &uu, 4);
                volatile float xv = x;
                const float a = logf(xv), c = orbfe::glibc_logf(x);
                if (!same(a, c)) {
                    if (b < 3) fprintf(stderr, "mismatch x=%a libm %a port %a\n", x, a, c);
                    b++;
                }
                n++;
            }
            bad += b;
            tot += n;
        });
    for (auto& x : th) x.join();
    const float specials[] = {0.f, -0.f, 1.f, 0x1p-149f, 0x1p-130f, 0x1.fffffep-127f, 0x1p-126f, 3.0e38f, INFINITY, -1.f};
    for (float x : specials) {
        volatile float xv = x;
        if (!same(logf(xv), orbfe::glibc_logf(x))) {
            fprintf(stderr, "special mismatch x=%a\n", x);
            bad++;
        }
        tot++;
    }
    printf("checked %ld floats, mismatches %ld\n", tot.load(), bad.load());
    return bad ? 1 : 0;
}
