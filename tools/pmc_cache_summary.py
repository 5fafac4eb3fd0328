#!/usr/bin/env python3
"""Summarise rocprofv3 cache / LDS counter passes (tools/gpu_pmc_cache.sh) per kernel into a JSON
committed under profiles/: L2 hit rate = TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
(/opt/skills/guides/MI355X_MICROARCH.md §L2) and the LDS bank-conflict share =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over all LDS-array cycles, §LDS).

usage: pmc_cache_summary.py <pmc_dir> <out.json> --images N --width W --height H
"""
import argparse
import collections
import csv
import json
import os


def load(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        short = r["Kernel_Name"].split("(")[0].replace("orbfe::", "")
        per[short][r["Counter_Name"]] += float(r["Counter_Value"])
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("out")
    ap.add_argument("--images", type=int, required=True)
    ap.add_argument("--width", type=int, default=752)
    ap.add_argument("--height", type=int, default=480)
    a = ap.parse_args()
    c = collections.defaultdict(dict)
    for sub in ("c1", "c2"):
        p = os.path.join(a.pmc_dir, sub, "run_counter_collection.csv")
        for k, v in load(p).items():
            c[k].update(v)
    kernels = {}
    for k, v in sorted(c.items()):
        if not k.startswith("k_"):
            continue
        hit, miss = v.get("TCC_HIT_sum", 0.0), v.get("TCC_MISS_sum", 0.0)
        conf, act = v.get("SQ_LDS_BANK_CONFLICT", 0.0), v.get("SQ_LDS_IDX_ACTIVE", 0.0)
        kernels[k] = {
            "l2_hit_rate": round(hit / (hit + miss), 4) if hit + miss else None,
            "tcc_hit": hit, "tcc_miss": miss,
            "lds_bank_conflict_cycles": conf, "lds_active_cycles": act,
            "lds_conflict_share": round(conf / act, 4) if act else None,
        }
    out = {
        "source": "rocprofv3 --pmc 'TCC_HIT_sum TCC_MISS_sum' and 'SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE' "
                  "--kernel-trace (separate passes), tools/gpu_pmc_cache.sh",
        "images_per_step": a.images, "width": a.width, "height": a.height,
        "kernels": kernels,
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
