"""ORBVocabulary — host mirror of DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>
(Thirdparty/DBoW2/DBoW2/TemplatedVocabulary.h, typedef'd as ORB_SLAM3::ORBVocabulary) over the
C-ABI: loadFromBinFile and transform(features, BowVector, FeatureVector, levelsup), the call of
Frame::ComputeBoW. The tree lives in HBM; transform runs in liborbfe.so's HIP kernels.
Also writes the binary format (saveToBinFile layout) for synthetic vocabularies.
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from . import _lib
from .matcher import FeatureVector

TF_IDF, TF, IDF, BINARY = 0, 1, 2, 3
L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = 0, 1, 2, 3, 4, 5


def save_bin(k, L, scoring, weighting, parents, is_leaf, desc, weights) -> bytes:
    """TemplatedVocabulary::saveToBinFile layout: int k, L, scoring, weighting; then per node
    1..n-1: int parent, uchar isLeaf, uchar desc[32], double weight."""
    out = [struct.pack("<4i", k, L, scoring, weighting)]
    for i in range(1, len(parents)):
        out.append(struct.pack("<iB", int(parents[i]), int(is_leaf[i])) + bytes(desc[i]) +
                   struct.pack("<d", float(weights[i])))
    return b"".join(out)


class ORBVocabulary:
    def __init__(self, handle, lib):
        self._h = handle
        self._lib = lib
        k, L, nn, nw = (ctypes.c_int32() for _ in range(4))
        _lib.check(lib.orbfe_vocabulary_info(handle, ctypes.byref(k), ctypes.byref(L), ctypes.byref(nn),
                                             ctypes.byref(nw)), "vocabulary_info")
        self.k, self.L, self.n_nodes, self.n_words = k.value, L.value, nn.value, nw.value

    @classmethod
    def from_bin(cls, data: bytes):
        """loadFromBinFile from the file's bytes."""
        lib = _lib.load()
        h = ctypes.c_void_p()
        buf = np.frombuffer(data, np.uint8)
        _lib.check(lib.orbfe_vocabulary_load_bin(buf.ctypes.data, len(buf), ctypes.byref(h)), "vocabulary_load_bin")
        return cls(h, lib)

    @classmethod
    def from_arrays(cls, k, L, scoring, weighting, parents, is_leaf, desc, weights):
        lib = _lib.load()
        h = ctypes.c_void_p()
        par = np.ascontiguousarray(parents, np.int32)
        leaf = np.ascontiguousarray(is_leaf, np.uint8)
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        w = np.ascontiguousarray(weights, np.float64)
        _lib.check(lib.orbfe_vocabulary_create(k, L, scoring, weighting, len(par), par.ctypes.data, leaf.ctypes.data,
                                               d.ctypes.data, w.ctypes.data, ctypes.byref(h)), "vocabulary_create")
        return cls(h, lib)

    def transform(self, desc, levelsup: int = 4):
        """-> (BowVector as (word ids, weights), FeatureVector)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = len(d)
        bid = np.zeros(max(n, 1), np.uint32)
        bw = np.zeros(max(n, 1), np.float64)
        fid = np.zeros(max(n, 1), np.uint32)
        foff = np.zeros(n + 1, np.int32)
        fidx = np.zeros(max(n, 1), np.uint32)
        nb, nf = ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self._lib.orbfe_vocabulary_transform(self._h, d.ctypes.data, n, int(levelsup), bid.ctypes.data,
                                                        bw.ctypes.data, ctypes.byref(nb), fid.ctypes.data,
                                                        foff.ctypes.data, fidx.ctypes.data, ctypes.byref(nf)),
                   "vocabulary_transform")
        nb, nf = nb.value, nf.value
        fv = FeatureVector({int(fid[i]): fidx[foff[i]:foff[i + 1]].tolist() for i in range(nf)})
        return (bid[:nb].copy(), bw[:nb].copy()), fv

    def close(self):
        if self._h:
            self._lib.orbfe_vocabulary_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def synth_vocabulary(rng, k: int = 10, L: int = 4, stop_frac: float = 0.02):
    """A full k-ary tree of depth L in DBoW2's node order (breadth-first, children consecutive) with
    random descriptors; leaf weights are idf-like positive values, a few 0 (stopped words)."""
    parents = [0]
    is_leaf = [0]
    level_nodes = [0]
    for lv in range(1, L + 1):
        nxt = []
        for p in level_nodes:
            for _ in range(k):
                parents.append(p)
                is_leaf.append(1 if lv == L else 0)
                nxt.append(len(parents) - 1)
        level_nodes = nxt
    n = len(parents)
    desc = rng.integers(0, 256, (n, 32), dtype=np.uint8)
    w = rng.uniform(0.1, 6.0, n)
    w[rng.random(n) < stop_frac] = 0.0
    w[0] = 0.0
    return np.array(parents, np.int32), np.array(is_leaf, np.uint8), desc, w
