#!/usr/bin/env python3
"""Regenerate tests/golden/matcher_golden.npz: ORBmatcher cases with per-query expected outputs.

The reference ships no matcher fixtures and cannot run here (no OpenCV / Eigen / Sophus), so the
expected outputs come from the CPU oracle (oracle/orb_oracle_match.cpp), itself cross-checked on
small cases by the independent Python restatement in tests/test_oracle_matcher.py. The inputs are
regenerated from seeds by orb_slam3_ros_amd.synth_match (a SHA-256 of the packed inputs guards
against generator drift). Parity w.r.t. the real reference: unpinned.
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "matcher_golden.npz")


def digest(*arrays):
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return np.frombuffer(h.digest(), np.uint8)


def cases():
    """Yields (name, kind, inputs dict, runner) for both the generator and the tests."""
    from orb_slam3_ros_amd import synth_match as sm
    out = []
    rng = np.random.default_rng(101)
    F = sm.synth_frame(rng, 500, w=400, h=300)
    mps = sm.synth_local_map(rng, F, 3000, copy_frac=0.5)
    mvp, obs = sm.initial_slots(rng, F.N, 0.2)
    for th in (1, 3):
        out.append((f"local_th{th}", "local", dict(F=F, mps=mps, mvp=mvp, obs=obs, th=th, ratio=0.8)))
    rng = np.random.default_rng(102)
    F = sm.synth_frame(rng, 600, w=400, h=300)
    pts = sm.synth_proj_points(rng, F, 500)
    mvp, obs = sm.initial_slots(rng, F.N, 0.2)
    out.append(("lastframe", "lastframe", dict(F=F, pts=pts, mvp=mvp, obs=obs, th=7, fw=0, bw=0)))
    out.append(("lastframe_fw", "lastframe", dict(F=F, pts=pts, mvp=mvp, obs=obs, th=15, fw=1, bw=0)))
    out.append(("keyframe", "kf", dict(F=F, pts=pts, mvp=mvp, th=10, orbdist=64)))
    rng = np.random.default_rng(103)
    F1 = sm.synth_frame(rng, 800, w=400, h=300, stereo=False)
    F2, src = sm.perturbed_frame(rng, F1, shift=(3.0, -2.0), flip_p=0.05, drop=0.2)
    prev = np.stack([F1.keys["x"], F1.keys["y"]], 1).astype(np.float32)
    out.append(("init", "init", dict(F1=F1, F2=F2, prev=prev, window=50)))
    kf_mp = np.where(rng.random(F1.N) < 0.2, -1, np.arange(F1.N) + 7).astype(np.int32)
    fk, ff = sm.synth_bow(rng, 60, F1, F2, src)
    out.append(("bow", "bow", dict(KF=F1, F=F2, kf_mp=kf_mp, fk=fk, ff=ff)))
    L = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    R = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    L[:100] = sm.flip_bits(rng, R[rng.integers(0, 300, 100)], 0.05)
    out.append(("knn", "knn", dict(L=L, R=R)))
    return out


def input_digest(kind, d):
    if kind == "local":
        return digest(d["F"].keys, d["F"].desc, d["F"].uright, d["mps"], d["mvp"], d["obs"])
    if kind in ("lastframe", "kf"):
        return digest(d["F"].keys, d["F"].desc, d["F"].uright, d["pts"], d["mvp"])
    if kind == "init":
        return digest(d["F1"].keys, d["F1"].desc, d["F2"].keys, d["F2"].desc, d["prev"])
    if kind == "bow":
        return digest(d["KF"].keys, d["KF"].desc, d["F"].keys, d["F"].desc, d["kf_mp"], d["fk"].indices,
                      d["ff"].indices, d["fk"].node_ids, d["ff"].node_ids)
    return digest(d["L"], d["R"])


def run(m, kind, d):
    """m: an object with the OracleMatcher-style API (oracle) -> (n, outputs...)."""
    if kind == "local":
        mvp = d["mvp"].copy()
        n = m(d["ratio"], True).sbp_local(d["F"], mvp, d["obs"], d["mps"], d["th"])
        return n, mvp
    if kind == "lastframe":
        mvp = d["mvp"].copy()
        n = m(0.9, True).sbp_lastframe(d["F"], mvp, d["obs"], d["pts"], d["th"], d["fw"], d["bw"])
        return n, mvp
    if kind == "kf":
        mvp = d["mvp"].copy()
        n = m(0.9, True).sbp_kf(d["F"], mvp, d["pts"], d["th"], d["orbdist"])
        return n, mvp
    if kind == "init":
        prev = d["prev"].copy()
        m12 = np.zeros(d["F1"].N, np.int32)
        n = m(0.9, True).search_for_init(d["F1"], d["F2"], prev, m12, d["window"])
        return n, m12, prev
    if kind == "bow":
        n, out = m(0.75, True).search_by_bow(d["KF"].keys, d["KF"].desc, d["kf_mp"], d["fk"], d["F"], d["ff"])
        return n, out
    return oracle.stereo_knn_ratio(d["L"], d["R"])


def main():
    oracle.build()
    g = {}
    for name, kind, d in cases():
        res = run(oracle.OracleMatcher, kind, d)
        g[name + "_in"] = input_digest(kind, d)
        g[name + "_n"] = np.array([res[0]], np.int32)
        for i, a in enumerate(res[1:]):
            g[f"{name}_out{i}"] = a
    np.savez_compressed(OUT, **g)
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
