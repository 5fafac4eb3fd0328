"""Per-call kernel timeline of the matcher from a rocprofv3 kernel-trace CSV: a call starts at its
k_mt_grid launch; prints the median span (first start -> last end), busy time (sum of kernel
durations) and the median gap before each kernel position."""
import csv
import sys
from collections import defaultdict

import numpy as np

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
calls, cur = [], None
for r in rows:
    name = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
    if "k_mt_grid" in name:
        cur = []
        calls.append(cur)
    if cur is not None:
        cur.append((name, int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
by_len = defaultdict(list)
for c in calls:
    by_len[len(c)].append(c)
for n, cs in sorted(by_len.items()):
    span = np.median([c[-1][2] - c[0][1] for c in cs]) / 1e3
    busy = np.median([sum(e - s for _, s, e in c) for c in cs]) / 1e3
    print(f"{len(cs)} calls of {n} kernels: span {span:.1f} us, busy {busy:.1f} us")
    for i in range(n):
        gap = np.median([c[i][1] - c[i - 1][2] for c in cs]) / 1e3 if i else 0.0
        dur = np.median([c[i][2] - c[i][1] for c in cs]) / 1e3
        print(f"   {i:2d} {cs[0][i][0][:40]:40s} gap {gap:6.1f} dur {dur:6.1f}")
    if len(cs) > 1:
        between = np.median([cs[k + 1][0][1] - cs[k][-1][2] for k in range(len(cs) - 1)]) / 1e3
        print(f"   median idle between consecutive calls: {between:.1f} us")
