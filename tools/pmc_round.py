#!/usr/bin/env python3
"""Summarise tools/gpu_profile_round.sh output into the three per-round JSON files bench.py reads
from profiles/:

  <prefix>_pmc_traffic.json  HBM bytes per step and kernel: read = 2 x FETCH_SIZE(KB) x 1024 (gfx950
                             reports half the bytes of wide streaming reads, calibrated in
                             profiles/r01_fetch_calibration.txt), write = WRITE_SIZE(KB) x 1024
  <prefix>_pmc_cache.json    L2 hit rate TCC_HIT / (TCC_HIT + TCC_MISS); LDS bank-conflict share
                             SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  <prefix>_pmc_valu.json     VALU / SALU / LDS instructions per step, the kernel's isolated time per
                             step (kernel trace of the same build and command) and the VALU issue
                             fraction = VALU instructions / (time x 1024 SIMDs x 2.4 GHz / 2 cycles per
                             wave64 instruction) (MI355X_MICROARCH.md §Wave scheduling); wave states
                             as fractions of SQ_WAVE_CYCLES (active / parked in s_waitcnt or barrier /
                             issue-stalled)

A "step" is one bench step (one launch sequence over the batch): counts are divided by the number of
k_octree launches (one per step); k_remap (the rectification leg) is per launch.

usage: pmc_round.py <dir> <prefix> [--outdir profiles] [--images 1024 --width 752 --height 480]
"""
import argparse
import collections
import csv
import glob
import json
import os

VALU_PEAK = 1024 * 2.4e9 / 2


def kname(full):
    """'void orbfe::k_describe<4>(...)' -> 'k_describe' (template instances of a kernel pooled)."""
    k = full.split("(")[0].replace("orbfe::", "")
    if k.startswith("void "):
        k = k[5:]
    return k.split("<")[0].strip()


def counters(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kname(r["Kernel_Name"])
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            n[k].add(r["Dispatch_Id"])
    return acc, {k: len(v) for k, v in n.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("prefix")
    ap.add_argument("--outdir", default="profiles")
    ap.add_argument("--images", type=int, default=1024)
    ap.add_argument("--width", type=int, default=752)
    ap.add_argument("--height", type=int, default=480)
    a = ap.parse_args()
    tr = glob.glob(os.path.join(a.dir, "trace", "**", "*kernel_trace.csv"), recursive=True)[0]
    dur = collections.defaultdict(float)
    launches = collections.Counter()
    for r in csv.DictReader(open(tr)):
        k = kname(r["Kernel_Name"])
        dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        launches[k] += 1
    steps = launches["k_octree"] or 1
    per = lambda k: 1 if k == "k_remap" else steps   # noqa: E731
    c = {}
    for i in range(1, 7):
        acc, _ = counters(os.path.join(a.dir, f"p{i}"))
        for k, v in acc.items():
            c.setdefault(k, {}).update(v)
    kerns = sorted(k for k in c if k.startswith("k_"))
    hdr = {"images_per_step": a.images, "width": a.width, "height": a.height, "steps_profiled": steps,
           "build": "isolated-timing build (-DFAST_NO_OVERLAP), tools/gpu_profile_round.sh"}
    traffic = {}
    for k in kerns:
        v = c[k]
        runs = launches[k] // per(k) if k == "k_remap" else steps
        traffic[k] = {"launches_per_step": launches[k] // steps if k != "k_remap" else 1,
                      "fetch_kb_raw_per_step": round(v.get("FETCH_SIZE", 0.0) / runs, 1),
                      "read_bytes_per_step": int(2 * 1024 * v.get("FETCH_SIZE", 0.0) / runs),
                      "write_bytes_per_step": int(1024 * v.get("WRITE_SIZE", 0.0) / runs)}
    pf = [traffic[k] for k in traffic if k.startswith("k_resize") or k == "k_fast"]
    t = dict(hdr, source="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes)",
             correction="read = 2 x FETCH_SIZE(KB) x 1024 (gfx950 streaming-read factor); write = WRITE_SIZE x 1024",
             kernels=traffic,
             pyramid_fast_traffic_bytes_per_step=sum(x["read_bytes_per_step"] + x["write_bytes_per_step"] for x in pf))
    cache = {}
    for k in kerns:
        v = c[k]
        hit, miss = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
        conf, act = v.get("SQ_LDS_BANK_CONFLICT", 0.0), v.get("SQ_LDS_IDX_ACTIVE", 0.0)
        cache[k] = {"l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
                    "lds_conflict_share": round(conf / act, 4) if act else None,
                    "lds_bank_conflict_cycles": conf, "lds_active_cycles": act}
    ca = dict(hdr, source="rocprofv3 --pmc 'TCC_HIT_sum TCC_MISS_sum' and 'SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE'",
              kernels=cache)
    valu = {}
    for k in kerns:
        v = c[k]
        runs = launches[k] if k == "k_remap" else steps
        t_step = dur[k] / runs if runs else 0.0
        wc = v.get("SQ_WAVE_CYCLES", 0.0)
        valu[k] = {"valu_per_step": v.get("SQ_INSTS_VALU", 0.0) / runs,
                   "salu_per_step": v.get("SQ_INSTS_SALU", 0.0) / runs,
                   "lds_per_step": v.get("SQ_INSTS_LDS", 0.0) / runs,
                   "kernel_us_per_step": round(t_step * 1e6, 2),
                   "valu_issue_frac": round(v.get("SQ_INSTS_VALU", 0.0) / runs / t_step / VALU_PEAK, 4) if t_step else None,
                   "wave_state": {s: round(v.get(n, 0.0) / wc, 4) if wc else None for s, n in
                                  (("active", "SQ_ACTIVE_INST_ANY"), ("wait_any", "SQ_WAIT_ANY"),
                                   ("wait_inst", "SQ_WAIT_INST_ANY"))}}
    va = dict(hdr, source="rocprofv3 --pmc SQ_INSTS_* / SQ_WAVE_CYCLES / SQ_WAIT_* (separate passes) + kernel trace",
              valu_issue_peak_wave_instr_per_s=VALU_PEAK, kernels=valu)
    os.makedirs(a.outdir, exist_ok=True)
    for name, obj in (("traffic", t), ("cache", ca), ("valu", va)):
        p = os.path.join(a.outdir, f"{a.prefix}_pmc_{name}.json")
        json.dump(obj, open(p, "w"), indent=1)
        print("wrote", p)
    for k in kerns:
        print(f"{k:14s} {valu[k]['kernel_us_per_step']:9.1f} us/step  VALU issue {valu[k]['valu_issue_frac']}  "
              f"traffic {(traffic[k]['read_bytes_per_step'] + traffic[k]['write_bytes_per_step']) / 1e6:9.1f} MB  "
              f"L2 hit {cache[k]['l2_hit_rate']}  LDS conflicts {cache[k]['lds_conflict_share']}  states {valu[k]['wave_state']}")


if __name__ == "__main__":
    main()
