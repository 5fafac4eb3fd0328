#!/usr/bin/env python3
"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/gpu_round.sh) into a per-launch
HBM-traffic table committed under profiles/.

Units and corrections follow /opt/skills/guides/MI355X_MICROARCH.md §HBM: the counters are in KB
(1024 B); on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced streaming reads, so the
corrected read bytes are 2x the counter. WRITE_SIZE is taken as reported. One "step" of bench.py =
one launch sequence (resize x7, fast, octree, describe, stereo, stereo_cut), so per-step numbers
divide the per-kernel sums by the number of steps profiled.

usage: pmc_summary.py <pmc_dir> <out.json> --images N --width W --height H
"""
import argparse
import collections
import csv
import json
import os


def load(path, counter):
    per = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("orbfe::", "")
        per[short].append(float(r["Counter_Value"]))
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--images", type=int, required=True)
    ap.add_argument("--width", type=int, default=752)
    ap.add_argument("--height", type=int, default=480)
    a = ap.parse_args()
    fetch = load(os.path.join(a.pmc_dir, "p1", "run_counter_collection.csv"), "FETCH_SIZE")
    write = load(os.path.join(a.pmc_dir, "p2", "run_counter_collection.csv"), "WRITE_SIZE")
    steps = len(fetch.get("k_fast", [])) or 1
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        if not k.startswith("k_"):
            continue
        f = fetch.get(k, [])
        w = write.get(k, [])
        kernels[k] = {
            "launches_per_step": len(f) // steps if f else len(w) // steps,
            "fetch_kb_raw_per_step": round(sum(f) / steps, 1),
            "read_bytes_per_step": int(2 * 1024 * sum(f) / steps),
            "write_bytes_per_step": int(1024 * sum(w) / steps),
        }
    pf = [kernels[k] for k in ("k_resize", "k_fast") if k in kernels]
    out = {
        "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (separate passes), tools/gpu_round.sh",
        "correction": "read = 2 x FETCH_SIZE(KB) x 1024 (gfx950 streaming-read factor); write = WRITE_SIZE x 1024",
        "images_per_step": a.images, "width": a.width, "height": a.height, "steps_profiled": steps,
        "kernels": kernels,
        "pyramid_fast_traffic_bytes_per_step": sum(k["read_bytes_per_step"] + k["write_bytes_per_step"] for k in pf),
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
