// Checks orbfe::stl_sort / st_heap_sort (the replica the octree kernel uses) against the host
// libstdc++ std::sort / std::partial_sort element-for-element on tie-heavy inputs.
#include <algorithm>
#include <cstdio>
#include <random>
#include <vector>
#include "../../orb_slam3_ros_amd/csrc/stl_sort.h"
struct E { int size, x, id; };
static bool cmp(const E& a, const E& b) {   // compareNodes shape: (size, UL.x), ties possible
    if (a.size < b.size) return true;
    if (a.size > b.size) return false;
    return a.x < b.x;
}
int main() {
    std::mt19937 rng(12345);
    long bad = 0, cases = 0;
    for (int it = 0; it < 20000; it++) {
        int n = it < 3000 ? it % 300 : (int)(rng() % 3000);
        int range_s = 1 + rng() % 8, range_x = 1 + rng() % 16;
        std::vector<E> a(n);
        for (int i = 0; i < n; i++) a[i] = E{(int)(rng() % range_s) + 2, (int)(rng() % range_x) * 7, i};
        if (it % 7 == 0) std::sort(a.begin(), a.end(), [](const E& p, const E& q) { return p.size > q.size; });
        std::vector<E> b = a, c = a, d = a;
        std::sort(a.begin(), a.end(), cmp);
        orbfe::stl_sort(b.data(), n, cmp);
        std::partial_sort(c.begin(), c.end(), c.end(), cmp);
        orbfe::st_heap_sort(d.data(), n, cmp);
        for (int i = 0; i < n; i++) {
            if (a[i].id != b[i].id) { bad++; if (bad < 5) printf("sort mismatch n=%d i=%d\n", n, i); break; }
        }
        for (int i = 0; i < n; i++) {
            if (c[i].id != d[i].id) { bad++; if (bad < 5) printf("heap mismatch n=%d i=%d\n", n, i); break; }
        }
        cases++;
    }
    printf("cases %ld mismatches %ld\n", cases, bad);
    return bad ? 1 : 0;
}
