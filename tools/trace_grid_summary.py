#!/usr/bin/env python3
"""Per-(kernel, grid) mean durations from a rocprofv3 --kernel-trace csv directory, plus the span of
the pyramid+FAST pass per step (first k_resize / k_fast / k_pyrfast start -> k_octree start)."""
import collections
import csv
import glob
import os
import sys

f = glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
per = collections.defaultdict(list)
spans, st = [], None
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("orbfe::", "")
    if "at::native" in k or "rocclr" in k:
        continue
    t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    per[(k, int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]))].append((t1 - t0) / 1e3)
    if k in ("k_fast", "k_resize", "k_pyrfast") and st is None:
        st = t0
    if k == "k_octree" and st is not None:
        spans.append((t0 - st) / 1e3)
        st = None
for (k, gx, gy), d in sorted(per.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    print(f"{k:16s} grid {gx:7d} x {gy:4d} n={len(d):3d} mean={sum(d) / len(d):8.1f} us")
if spans:
    s = sorted(spans)
    print(f"pyramid+FAST span per step: median {s[len(s) // 2]:.1f} us, min {s[0]:.1f} (n={len(s)})")
