"""CPU: the DBoW2 transform oracle (oracle/orb_oracle_bow.cpp) against an independent Python
restatement on a small synthetic vocabulary, and the binary-format loader round trip."""
import numpy as np
import pytest

from orb_slam3_ros_amd.vocabulary import (BINARY, DOT_PRODUCT, IDF, L1_NORM, L2_NORM, TF, TF_IDF, save_bin,
                                          synth_vocabulary)


def py_transform(k, L, scoring, weighting, parents, is_leaf, desc, weights, feats, levelsup):
    children = {i: [] for i in range(len(parents))}
    word = {}
    for i in range(1, len(parents)):
        children[int(parents[i])].append(i)
        if is_leaf[i]:
            word[i] = len(word)
    ham = lambda a, b: int(np.unpackbits(a ^ b).sum())
    bv, fv = {}, {}
    tf = weighting in (TF_IDF, TF)
    for i, f in enumerate(feats):
        nid_level = L - levelsup
        nid = 0
        fin, lev = 0, 0
        while children[fin]:
            lev += 1
            ch = children[fin]
            best, bd = ch[0], ham(f, desc[ch[0]])
            for c in ch[1:]:
                d = ham(f, desc[c])
                if d < bd:
                    best, bd = c, d
            fin = best
            if lev == nid_level:
                nid = fin
        wid, w = word.get(fin, 0), float(weights[fin])
        if w > 0:
            if tf:
                bv[wid] = bv.get(wid, 0.0) + w
            elif wid not in bv:
                bv[wid] = w
            fv.setdefault(nid, []).append(i)
    must = scoring != DOT_PRODUCT
    ids = sorted(bv)
    vals = [bv[i] for i in ids]
    if tf and vals and not must:
        vals = [v / float(len(vals)) for v in vals]
    if must:
        if scoring == L2_NORM:
            norm = 0.0
            for v in vals:
                norm += v * v
            norm = np.sqrt(norm)
        else:
            norm = 0.0
            for v in vals:
                norm += abs(v)
        if norm > 0:
            vals = [v / norm for v in vals]
    return ids, vals, {k2: fv[k2] for k2 in sorted(fv)}


@pytest.mark.parametrize("scoring,weighting", [(L1_NORM, TF_IDF), (DOT_PRODUCT, TF), (L2_NORM, IDF), (L1_NORM, BINARY)])
@pytest.mark.parametrize("levelsup", [0, 1, 2, 4])
def test_oracle_transform_vs_python(oracle_lib, scoring, weighting, levelsup):
    rng = np.random.default_rng(levelsup * 10 + weighting)
    k, L = 4, 3
    par, leaf, desc, w = synth_vocabulary(rng, k, L, stop_frac=0.1)
    feats = rng.integers(0, 256, (120, 32), dtype=np.uint8)
    feats[:40] = desc[rng.integers(1, len(desc), 40)]
    ov = oracle_lib.OracleVocabulary.from_arrays(k, L, scoring, weighting, par, leaf, desc, w)
    (bid, bw), (fid, foff, fidx) = ov.transform(feats, levelsup)
    ids, vals, fv = py_transform(k, L, scoring, weighting, par, leaf, desc, w, feats, levelsup)
    assert bid.tolist() == ids
    assert bw.tobytes() == np.array(vals, np.float64).tobytes()
    assert fid.tolist() == list(fv)
    assert [fidx[foff[i]:foff[i + 1]].tolist() for i in range(len(fid))] == list(fv.values())


def test_oracle_loader_roundtrip(oracle_lib):
    rng = np.random.default_rng(3)
    par, leaf, desc, w = synth_vocabulary(rng, 5, 3)
    blob = save_bin(5, 3, L1_NORM, TF_IDF, par, leaf, desc, w)
    assert len(blob) == 16 + 45 * (len(par) - 1)
    a = oracle_lib.OracleVocabulary.from_bin(blob)
    b = oracle_lib.OracleVocabulary.from_arrays(5, 3, L1_NORM, TF_IDF, par, leaf, desc, w)
    feats = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    ra, rb = a.transform(feats), b.transform(feats)
    for x, y in zip(ra[0] + ra[1], rb[0] + rb[1]):
        assert np.array_equal(x, y)
    # the reference's header sanity checks (TemplatedVocabulary.h:1499-1503)
    bad = bytearray(blob)
    bad[0:4] = (25).to_bytes(4, "little")
    assert oracle_lib.OracleVocabulary.from_bin(bytes(bad)) is None
