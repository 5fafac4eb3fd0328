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
// Host emulation of the device block sort: stop-based partitions + stable sort of each leaf
// (heap-sorted leaves when the depth budget is exhausted).
static void par_emul(std::vector<E>& a) {
    const int n = (int)a.size();
    if (n <= 1) return;
    struct Seg { int lo, hi, depth; };
    std::vector<Seg> st{{0, n, 2 * orbfe::st_lg(n)}};
    std::vector<Seg> leaves;
    std::vector<int> ls(n), rs(n);
    while (!st.empty()) {
        Seg s = st.back(); st.pop_back();
        if (s.hi - s.lo <= 16) { leaves.push_back({s.lo, s.hi, 1}); continue; }
        if (s.depth == 0) { leaves.push_back({s.lo, s.hi, 0}); continue; }
        E* f = a.data() + s.lo;
        orbfe::st_move_median_to_first(f, f + 1, f + (s.hi - s.lo) / 2, a.data() + s.hi - 1, cmp);
        int cut = orbfe::partition_by_stops(a.data(), s.lo, s.hi, cmp, ls.data(), rs.data());
        st.push_back({cut, s.hi, s.depth - 1});
        st.push_back({s.lo, cut, s.depth - 1});
    }
    for (auto& lf : leaves) {
        if (lf.depth == 0) orbfe::st_heap_sort(a.data() + lf.lo, lf.hi - lf.lo, cmp);
        else std::stable_sort(a.begin() + lf.lo, a.begin() + lf.hi, cmp);
    }
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
        std::vector<E> b = a, c = a, d = a, e = a;
        std::sort(a.begin(), a.end(), cmp);
        orbfe::stl_sort(b.data(), n, cmp);
        par_emul(e);
        for (int i = 0; i < n; i++) {
            if (a[i].id != e[i].id) { bad++; if (bad < 5) printf("par-emul mismatch n=%d i=%d\n", n, i); break; }
        }
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
    // partition_by_stops == st_unguarded_partition (same array, same cut)
    long pbad = 0;
    for (int it = 0; it < 20000; it++) {
        int n = 17 + (int)(rng() % 400);   // introsort only partitions segments of > 16 elements
        int rs = 1 + rng() % 6, rx = 1 + rng() % 5;
        std::vector<E> a(n);
        for (int i = 0; i < n; i++) a[i] = E{(int)(rng() % rs), (int)(rng() % rx), i};
        // the unguarded partition needs the median-of-three sentinel arrangement
        E* f = a.data();
        orbfe::st_move_median_to_first(f, f + 1, f + n / 2, f + n - 1, cmp);
        std::vector<E> b = a;
        E* cut1 = orbfe::st_unguarded_partition(a.data() + 1, a.data() + n, a.data(), cmp);
        std::vector<int> ls(n), rs2(n);
        int cut2 = orbfe::partition_by_stops(b.data(), 0, n, cmp, ls.data(), rs2.data());
        bool ok = (int)(cut1 - a.data()) == cut2;
        for (int i = 0; ok && i < n; i++) ok = a[i].id == b[i].id;
        if (!ok) { pbad++; if (pbad < 5) printf("partition mismatch n=%d\n", n); }
    }
    bad += pbad;
    printf("cases %ld mismatches %ld (partition mismatches %ld)\n", cases, bad, pbad);
    return bad ? 1 : 0;
}
