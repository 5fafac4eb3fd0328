"""Print chosen keys of the last JSON line of a bench output: python tools/show_bench.py FILE KEY..."""
import json
import sys

d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k in sys.argv[2:]:
    print(k, json.dumps(d.get(k))[:2000])
