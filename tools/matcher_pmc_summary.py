"""Summarise tools/gpu_matcher_pmc.sh: per th, the pass kernel's counters per call and its VALU issue
fraction = SQ_INSTS_VALU / (kernel time x the wave64 issue peak, 1024 SIMD-32s x 2.4 GHz / 2 cycles).
usage: python tools/matcher_pmc_summary.py gpurun_out PREFIX -> gpurun_out/PREFIX_pmc_matcher.json"""
import collections
import csv
import glob
import json
import os
import sys

VALU_PEAK = 1024 * 2.4e9 / 2
root, prefix = sys.argv[1], sys.argv[2]
per_th = {}
for th in (1, 3, 5, 15):
    cnt = collections.defaultdict(float)
    dur, ndisp, names = 0.0, 0, set()
    for i in (1, 2):
        for f in glob.glob(os.path.join(root, f"mp_th{th}_{i}", "**", "*counter_collection.csv"), recursive=True):
            seen = set()
            for r in csv.DictReader(open(f)):
                cnt[r["Counter_Name"]] += float(r["Counter_Value"])
                k = r["Kernel_Name"].split("(")[0].split("<")[0]
                names.add(k[5:] if k.startswith("void ") else k)
        if i == 1:
            for f in glob.glob(os.path.join(root, f"mp_th{th}_{i}", "**", "*kernel_trace.csv"), recursive=True):
                for r in csv.DictReader(open(f)):
                    if any(k in r["Kernel_Name"] for k in ("k_sbp_local", "k_sbp_band", "k_sbp_multi")):
                        dur += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
                        ndisp += 1
    if not dur:
        continue
    calls = 20
    wc = cnt.get("SQ_WAVE_CYCLES", 0.0)
    per_th[f"th{th}"] = {
        "kernel": "/".join(sorted(names)),
        "dispatches_per_call": ndisp / calls,
        "kernel_us_per_call": round(dur / calls * 1e6, 2),
        "valu_per_call": cnt["SQ_INSTS_VALU"] / calls,
        "salu_per_call": cnt["SQ_INSTS_SALU"] / calls,
        "lds_per_call": cnt["SQ_INSTS_LDS"] / calls,
        "vmem_per_call": cnt["SQ_INSTS_VMEM"] / calls,
        "waves_per_call": cnt["SQ_WAVES"] / calls,
        "valu_issue_frac": round(cnt["SQ_INSTS_VALU"] / (dur * VALU_PEAK), 4),
        "wave_state": {k: round(cnt[c] / wc, 4) for k, c in (("active", "SQ_ACTIVE_INST_ANY"), ("wait_any", "SQ_WAIT_ANY"),
                                                           ("wait_inst", "SQ_WAIT_INST_ANY"))} if wc else None,
    }
out = {"workload": "config 5: SearchByProjection(local map), 100k map points vs 1000 keypoints, 20 host calls per th",
       "source": "rocprofv3 --pmc (2 passes per th) + kernel trace, tools/gpu_matcher_pmc.sh",
       "valu_issue_peak_wave_instr_per_s": VALU_PEAK, "per_th": per_th}
path = os.path.join(root, f"{prefix}_pmc_matcher.json")
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(out, indent=1))
