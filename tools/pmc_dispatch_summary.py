#!/usr/bin/env python3
"""Per-dispatch view of tools/gpu_pmc_dispatch.sh: for the last bench step's launch sequence, each
dispatch's kernel, duration (kernel trace) and counters (all passes merged by dispatch order)."""
import collections
import csv
import glob
import os
import sys


def main(d):
    merged = collections.OrderedDict()
    for p in sorted(glob.glob(os.path.join(d, "p*"))):
        for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
            per = collections.OrderedDict()
            for r in csv.DictReader(open(f)):
                key = int(r["Dispatch_Id"])
                e = per.setdefault(key, {"name": r["Kernel_Name"].split("(")[0].replace("orbfe::", ""),
                                         "grid": r.get("Grid_Size", "")})
                e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            dur = {}
            for t in glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True):
                for r in csv.DictReader(open(t)):
                    dur[int(r["Dispatch_Id"])] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
            items = [(k, v) for k, v in per.items() if v["name"].startswith("k_")]
            # the last launch sequence: from the last k_resize run of 7 onward
            idx = [i for i, (k, v) in enumerate(items) if v["name"] == "k_resize"]
            start = idx[-7] if len(idx) >= 7 else 0
            for j, (k, v) in enumerate(items[start:]):
                m = merged.setdefault(j, {"name": v["name"], "grid": v["grid"], "us": []})
                m["us"].append(dur.get(k, 0.0))
                for c, x in v.items():
                    if c not in ("name", "grid"):
                        m[c] = x
    for j, m in merged.items():
        us = sum(m["us"]) / max(1, len(m["us"]))
        cs = {c: (f"{x / 1e6:.2f}M" if x > 1e4 else f"{x:.3g}") for c, x in m.items() if c not in ("name", "grid", "us")}
        print(f"{j:2d} {m['name']:14s} grid={m['grid']:>10s} {us:8.1f} us {cs}")


if __name__ == "__main__":
    main(sys.argv[1])
