#!/usr/bin/env python3
"""Timeline (start / duration, microseconds from the first kernel) of the last batch's kernels in a
rocprofv3 --kernel-trace csv directory: shows the overlap of the split path's two streams."""
import csv
import glob
import os
import sys

d = sys.argv[1]
last = sys.argv[2] if len(sys.argv) > 2 else "k_describe"
f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("orbfe::", ""), int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
        r["Grid_Size_X"], r["Queue_Id"]) for r in rows]
ends = [i for i, s in enumerate(seq) if s[0] == last]
i1 = ends[-1]
i0 = ends[-2] + 1 if len(ends) > 1 else 0
t0 = seq[i0][1]
for k, a, b, gx, q in seq[i0:i1 + 1]:
    print(f"{k:14s} q{q:>3s} start {(a - t0) / 1e3:8.1f} end {(b - t0) / 1e3:8.1f} dur {(b - a) / 1e3:7.1f} grid {gx}")
