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
