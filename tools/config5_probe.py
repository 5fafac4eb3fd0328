"""Config-5 SearchByProjection timings alone (bench.matcher_config5): per th the host-call, device and
resident times and the fixed-point passes. python tools/config5_probe.py [calls]"""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402

r = bench.matcher_config5(int(sys.argv[1]) if len(sys.argv) > 1 else 20)
for th, v in r["per_th"].items():
    print(th, json.dumps({k: v.get(k) for k in ("ms_per_call", "device_ms_per_call", "resident_ms_per_call", "passes",
                                                "pairs", "nmatches", "kernel")}))
