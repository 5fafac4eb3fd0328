// Replica of libstdc++'s std::sort (bits/stl_algo.h / stl_heap.h, GCC 7-13: introsort with
// _S_threshold = 16, median-of-three pivot moved to *first, unguarded partition, heapsort fallback
// at depth 2*lg(n), final insertion sort). DistributeOctTree sorts (size, node) pairs with a
// comparator that has ties (ORBextractor.cc:538-553,700), so the ORDER OF TIED ELEMENTS — which
// decides which octree nodes get split before the feature budget is reached and the final
// keypoint order — is whatever this exact algorithm produces. Reproducing it element-for-element
// is therefore part of bit-exact parity. tests/test_stl_sort.py checks this replica against the
// host's std::sort on tie-heavy inputs. Host + device (HIP) code, no recursion depth issues
// (the right-hand recursion of __introsort_loop is kept on an explicit stack).
#pragma once

#ifndef ORBFE_HD
#if defined(__HIPCC__)
#define ORBFE_HD __host__ __device__ inline
#else
#define ORBFE_HD inline
#endif
#endif

namespace orbfe {

template <typename T>
ORBFE_HD void st_swap(T* a, T* b) { T t = *a; *a = *b; *b = t; }

template <typename T, typename Cmp>
ORBFE_HD void st_push_heap(T* first, int hole, int top, T value, Cmp comp) {
    int parent = (hole - 1) / 2;
    while (hole > top && comp(first[parent], value)) {
        first[hole] = first[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    first[hole] = value;
}

template <typename T, typename Cmp>
ORBFE_HD void st_adjust_heap(T* first, int hole, int len, T value, Cmp comp) {
    const int top = hole;
    int second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (comp(first[second], first[second - 1])) second--;
        first[hole] = first[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        first[hole] = first[second - 1];
        hole = second - 1;
    }
    st_push_heap(first, hole, top, value, comp);
}

template <typename T, typename Cmp>
ORBFE_HD void st_heap_sort(T* first, int len, Cmp comp) {   // __partial_sort(first, last, last)
    if (len >= 2) {                                          // __make_heap
        int parent = (len - 2) / 2;
        while (true) {
            T v = first[parent];
            st_adjust_heap(first, parent, len, v, comp);
            if (parent == 0) break;
            parent--;
        }
    }
    // __heap_select with middle == last has no extra elements; then __sort_heap
    while (len > 1) {
        --len;
        T v = first[len];
        first[len] = first[0];
        st_adjust_heap(first, 0, len, v, comp);
    }
}

template <typename T, typename Cmp>
ORBFE_HD void st_move_median_to_first(T* result, T* a, T* b, T* c, Cmp comp) {
    if (comp(*a, *b)) {
        if (comp(*b, *c)) st_swap(result, b);
        else if (comp(*a, *c)) st_swap(result, c);
        else st_swap(result, a);
    } else if (comp(*a, *c)) st_swap(result, a);
    else if (comp(*b, *c)) st_swap(result, c);
    else st_swap(result, b);
}

template <typename T, typename Cmp>
ORBFE_HD T* st_unguarded_partition(T* first, T* last, T* pivot, Cmp comp) {
    while (true) {
        while (comp(*first, *pivot)) ++first;
        --last;
        while (comp(*pivot, *last)) --last;
        if (!(first < last)) return first;
        st_swap(first, last);
        ++first;
    }
}

template <typename T, typename Cmp>
ORBFE_HD void st_unguarded_linear_insert(T* last, Cmp comp) {
    T val = *last;
    T* next = last - 1;
    while (comp(val, *next)) {
        *last = *next;
        last = next;
        --next;
    }
    *last = val;
}

template <typename T, typename Cmp>
ORBFE_HD void st_insertion_sort(T* first, T* last, Cmp comp) {
    if (first == last) return;
    for (T* i = first + 1; i != last; ++i) {
        if (comp(*i, *first)) {
            T val = *i;
            for (T* p = i; p != first; --p) *p = *(p - 1);   // move_backward
            *first = val;
        } else {
            st_unguarded_linear_insert(i, comp);
        }
    }
}

ORBFE_HD int st_lg(int n) { int r = 0; while (n >>= 1) r++; return r; }

struct StSeg { int lo, hi, depth; };
#define ORBFE_SORT_STACK 64

// `stack` must hold ORBFE_SORT_STACK entries (the device passes an LDS buffer).
template <typename T, typename Cmp>
ORBFE_HD void stl_sort_with_stack(T* first, int n, Cmp comp, StSeg* stack) {
    if (n <= 1) return;
    const int kThreshold = 16;
    // __introsort_loop(first, last, 2*lg(n)): iterate on the left part, "recurse" on the right part.
    typedef StSeg Seg;
    int sp = 0;
    stack[sp++] = Seg{0, n, 2 * st_lg(n)};
    while (sp > 0) {
        Seg s = stack[--sp];
        int lo = s.lo, hi = s.hi, depth = s.depth;
        while (hi - lo > kThreshold) {
            if (depth == 0) { st_heap_sort(first + lo, hi - lo, comp); break; }
            --depth;
            T* f = first + lo;
            T* l = first + hi;
            T* mid = f + (hi - lo) / 2;
            st_move_median_to_first(f, f + 1, mid, l - 1, comp);
            T* cut = st_unguarded_partition(f + 1, l, f, comp);
            const int c = (int)(cut - first);
            // libstdc++ recurses on [cut, last) first, then loops on [first, cut). The two ranges are
            // disjoint, so the processing order does not change the result; push right, loop left.
            stack[sp++] = Seg{c, hi, depth};
            hi = c;
        }
    }
    // __final_insertion_sort
    if (n > kThreshold) {
        st_insertion_sort(first, first + kThreshold, comp);
        for (T* i = first + kThreshold; i != first + n; ++i) st_unguarded_linear_insert(i, comp);
    } else {
        st_insertion_sort(first, first + n, comp);
    }
}

template <typename T, typename Cmp>
ORBFE_HD void stl_sort(T* first, int n, Cmp comp) {
    StSeg stack[ORBFE_SORT_STACK];
    stl_sort_with_stack(first, n, comp, stack);
}

// ------------------------------------------------------------------------------------------------
// Data-parallel formulation of the SAME libstdc++ introsort (used by the octree kernel's block
// sort). The result is element-for-element identical to stl_sort because:
//  * __unguarded_partition(first, last, pivot) pairs the k-th "left stop" (scanning right, first
//    element with !(x < P)) with the k-th "right stop" (scanning left, first element with
//    !(P < x)) of the ORIGINAL segment for k = 1..s, s = #k with Lstop_k < Rstop_k; it returns
//    cut = Lstop_{s+1} if that exists and lies left of Rstop_s, else Rstop_s (s >= 1), or Lstop_1.
//  * after the introsort loop every leaf segment (<= 16 elements) holds only elements that are
//    not-greater than everything to its right, so __final_insertion_sort never moves an element
//    across a leaf boundary and acts as a STABLE sort inside each leaf; any stable sort gives the
//    same order. Leaves whose depth budget ran out are heap-sorted by the serial replica.
// partition_by_stops is the sequential statement of the first point (checked against
// st_unguarded_partition in tests/native/check_stl_sort.cpp); the device version computes the
// stops with block scans.
template <typename T, typename Cmp>
ORBFE_HD int partition_by_stops(T* a, int lo, int hi, Cmp comp, int* lstop, int* rstop) {
    const T P = a[lo];
    int nl = 0, nr = 0;
    for (int i = lo + 1; i < hi; i++)
        if (!comp(a[i], P)) lstop[nl++] = i;
    for (int j = hi - 1; j > lo; j--)
        if (!comp(P, a[j])) rstop[nr++] = j;
    int s = 0;
    while (s < nl && s < nr && lstop[s] < rstop[s]) s++;
    int cut;
    if (s == 0) cut = lstop[0];
    else cut = (s < nl && lstop[s] < rstop[s - 1]) ? lstop[s] : rstop[s - 1];
    for (int k = 0; k < s; k++) st_swap(&a[lstop[k]], &a[rstop[k]]);
    return cut;
}

}  // namespace orbfe
