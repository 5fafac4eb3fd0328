"""GPU: the block-parallel libstdc++ std::sort replica used by DistributeOctTree (k_octree) against
the host's std::sort, element for element, on tie-heavy (size, UL.x) keys."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_block_sort_matches_std_sort(gpu, oracle_lib, orbfe_lib):
    L = oracle_lib.lib()
    rng = np.random.default_rng(7)
    for it in range(300):
        n = int(rng.integers(0, 1200)) if it > 40 else it
        size = rng.integers(2, 2 + int(rng.integers(1, 9)), n).astype(np.uint64)
        x0 = (rng.integers(0, int(rng.integers(1, 12)), n) * 7).astype(np.uint64)
        vals = (size << np.uint64(44)) | (x0 << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        if it % 5 == 0:
            vals = np.sort(vals)[::-1].copy()
        a = np.ascontiguousarray(vals.copy())
        b = np.ascontiguousarray(vals.copy())
        L.oro_std_sort_u64_hi(a.ctypes.data, n)
        assert orbfe_lib.orbfe_debug_block_sort(b.ctypes.data, n) == n
        assert np.array_equal(a, b), f"iteration {it} n={n}"


def _introsort_adversary(n):
    """McIlroy's adversary against libstdc++'s introsort (median of three, unguarded partition):
    keys fixed lazily so every partition is as lopsided as possible, which exhausts the 2*lg(n)
    depth budget and sends segments of every size to the heapsort fallback. Returns the keys."""
    gas = n
    val = [gas] * n
    state = {"solid": 0, "cand": 0}

    def less(x, y):
        if val[x] == gas and val[y] == gas:
            z = x if x == state["cand"] else y
            val[z] = state["solid"]
            state["solid"] += 1
        if val[x] == gas:
            state["cand"] = x
        elif val[y] == gas:
            state["cand"] = y
        return val[x] < val[y]

    a = list(range(n))

    def sift(lo, hole, length, v):   # __adjust_heap + __push_heap
        top = hole
        child = hole
        while child < (length - 1) // 2:
            child = 2 * (child + 1)
            if less(a[lo + child], a[lo + child - 1]):
                child -= 1
            a[lo + hole] = a[lo + child]
            hole = child
        if (length & 1) == 0 and child == (length - 2) // 2:
            child = 2 * (child + 1)
            a[lo + hole] = a[lo + child - 1]
            hole = child - 1
        parent = (hole - 1) // 2
        while hole > top and less(a[lo + parent], v):
            a[lo + hole] = a[lo + parent]
            hole = parent
            parent = (hole - 1) // 2
        a[lo + hole] = v

    def heapsort(lo, hi):
        length = hi - lo
        for p in range((length - 2) // 2, -1, -1):
            sift(lo, p, length, a[lo + p])
        for last in range(hi - 1, lo, -1):
            v = a[last]
            a[last] = a[lo]
            sift(lo, 0, last - lo, v)

    def loop(lo, hi, depth):
        while hi - lo > 16:
            if depth == 0:
                heapsort(lo, hi)
                return
            depth -= 1
            m = lo + (hi - lo) // 2
            ia, ib, ic = lo + 1, m, hi - 1
            if less(a[ia], a[ib]):
                p = ib if less(a[ib], a[ic]) else (ic if less(a[ia], a[ic]) else ia)
            else:
                p = ia if less(a[ia], a[ic]) else (ic if less(a[ib], a[ic]) else ib)
            a[lo], a[p] = a[p], a[lo]
            f, l = lo + 1, hi
            while True:
                while less(a[f], a[lo]):
                    f += 1
                l -= 1
                while less(a[lo], a[l]):
                    l -= 1
                if not f < l:
                    break
                a[f], a[l] = a[l], a[f]
                f += 1
            loop(f, hi, depth)
            hi = f

    loop(0, n, 2 * (n.bit_length() - 1))
    for i in range(n):
        if val[i] == gas:
            val[i] = state["solid"]
            state["solid"] += 1
    return np.array(val, dtype=np.uint64)


def test_block_sort_depth_exhausted(gpu, oracle_lib, orbfe_lib):
    """Adversarial inputs: the heapsort fallback (__partial_sort) on large and small leaves."""
    L = oracle_lib.lib()
    for n in (40, 70, 150, 400, 1000):
        keys = _introsort_adversary(n)
        vals = (keys << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        a = np.ascontiguousarray(vals.copy())
        b = np.ascontiguousarray(vals.copy())
        L.oro_std_sort_u64_hi(a.ctypes.data, n)
        assert orbfe_lib.orbfe_debug_block_sort(b.ctypes.data, n) == n
        assert np.array_equal(a, b), f"n={n}"
