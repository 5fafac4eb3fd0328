"""bench.py's config-5 matcher leg alone (device vs device-resident call time per th)."""
import json
import sys
sys.path.insert(0, ".")
import bench

print(json.dumps(bench.matcher_config5(int(sys.argv[1]) if len(sys.argv) > 1 else 10), indent=1))
