#!/usr/bin/env python3
"""Per-ablation-mode counter totals of k_fast / k_describe (tools/gpu_ablate_pmc.sh output):
VALU / LDS / SALU / VMEM instructions per launch and their increments per phase."""
import collections
import csv
import glob
import os
import sys


def main(d):
    rows = {}
    for m in sorted(glob.glob(os.path.join(d, "m*"))):
        if not os.path.isdir(m):
            continue
        f = glob.glob(os.path.join(m, "**", "*counter_collection.csv"), recursive=True)
        if not f:
            continue
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        n = collections.Counter()
        seen = set()
        for r in csv.DictReader(open(f[0])):
            k = r["Kernel_Name"].split("(")[0].replace("orbfe::", "")
            if not k.startswith("k_"):
                continue
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            key = (k, r["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                n[k] += 1
        rows[os.path.basename(m)] = {k: {c: v / n[k] for c, v in acc[k].items()} for k in acc}
    for k in sorted({k for r in rows.values() for k in r}):
        print(k)
        prev = None
        for mode in sorted(rows):
            r = rows[mode].get(k, {})
            line = {c: f"{v / 1e6:.1f}M" for c, v in sorted(r.items())}
            print(" ", mode, line)


if __name__ == "__main__":
    main(sys.argv[1])
