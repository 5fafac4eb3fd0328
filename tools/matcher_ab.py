#!/usr/bin/env python3
"""Config-5 matcher A/B: bench.py's matcher_config5 leg (device ms per call per th) against the
library named by ORBFE_LIB, one JSON line. usage: ORBFE_LIB=... python tools/matcher_ab.py [CALLS]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = bench.matcher_config5(int(sys.argv[1]) if len(sys.argv) > 1 else 30)
print(json.dumps({th: {k: v.get(k) for k in ("kernel", "device_ms_per_call", "resident_ms_per_call", "nmatches")}
                  for th, v in out["per_th"].items()}))
