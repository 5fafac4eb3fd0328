#!/usr/bin/env python3
"""Per-kernel (and per-level for k_pyrfast, by dispatch order) mean durations from a rocprofv3
--kernel-trace csv directory."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
seq = []
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("orbfe::", "")
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    per[k].append(dur)
    seq.append((k, dur))
for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
    print(f"{k:28s} n={len(v):4d} mean={sum(v)/len(v):9.2f} us total={sum(v):10.1f} us")
# k_pyrfast per level: consecutive runs of 8 dispatches
pf = [d for k, d in seq if k == "k_pyrfast"]
if pf:
    n = len(pf) // 8
    lv = [sum(pf[8 * i + l] for i in range(n)) / n for l in range(8)]
    print("k_pyrfast per level (us):", " ".join(f"{v:.1f}" for v in lv), " sum", round(sum(lv), 1))
