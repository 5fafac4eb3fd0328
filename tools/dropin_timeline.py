#!/usr/bin/env python3
"""Summarise a kernel (+ memory copy) trace of capi_frontend --latency: mean duration per kernel
and the GPU timeline of one late frame (start offsets from the frame's first GPU op, durations,
idle gaps), so the batch-1 critical path and its launch gaps can be read off.
usage: dropin_timeline.py <rocprofv3 output dir> [--frame-after KERNEL]
(--frame-after: a frame starts at the first host-to-device copy after KERNEL, e.g. k_sbp_block<0> for
capi_frontend --tracking; default: after >= 100 us of GPU idleness)"""
import collections
import csv
import glob
import os
import sys


def kname(full):
    k = full.split("(")[0].replace("orbfe::", "")
    if k.startswith("void "):
        k = k[5:]
    return k.strip()


def main():
    d = sys.argv[1]
    after = sys.argv[3] if len(sys.argv) > 3 and sys.argv[2] == "--frame-after" else None
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"]),
                        r.get("Queue_Id", "")))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy_" + r.get("Direction", "?"),
                        r.get("Queue_Id", "")))
    ops.sort()
    per = collections.defaultdict(list)
    for s, e, k, _ in ops:
        per[k].append((e - s) / 1e3)
    for k, v in sorted(per.items(), key=lambda x: -sum(x[1])):
        print(f"{k:16s} n={len(v):5d} mean={sum(v) / len(v):8.1f} us")
    # frames: a frame starts at an H2D copy that follows >= 100 us of GPU idleness
    h2d = [i for i, o in enumerate(ops) if o[2].startswith("copy_") and "HOST_TO_DEVICE" in o[2].upper()]
    if after:
        starts = [i for i in h2d if i > 0 and ops[i - 1][2] == after]
    else:
        starts = [i for i in h2d if i == 0 or ops[i][0] - max(x[1] for x in ops[max(0, i - 40):i]) > 100e3]
    if len(starts) < 3:
        print("frames not found")
        return
    a, b = starts[-3], starts[-2]
    t0 = ops[a][0]
    end = t0
    print(f"--- one frame ({b - a} GPU ops), offsets from its first op ---")
    for s, e, k, q in ops[a:b]:
        gap = (s - end) / 1e3
        print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  gap {gap:6.1f}  {k} q{q}")
        end = max(end, e)
    print(f"frame GPU span {(end - t0) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
