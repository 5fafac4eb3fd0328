#!/usr/bin/env python3
"""Per-kernel PMC counter means per dispatch from rocprofv3 --pmc csv directories p1..pN."""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(set)
for p in sorted(glob.glob(os.path.join(d, "p*"))) or [d]:
    for f in glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("orbfe::", "")
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
for k in sorted(acc):
    print(k)
    for c, v in sorted(acc[k].items()):
        n = len(cnt[(k, c)]) or 1
        print(f"   {c:24s} per-dispatch {v / n / 1e6:10.3f} M")
