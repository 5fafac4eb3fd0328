#!/usr/bin/env python3
"""Per-basic-block instruction census of one kernel in a device assembly file (hipcc
--cuda-device-only -S): instructions, VALU, SALU (no waitcnt / branches), LDS, global, last branch.

usage: isa_census.py <file.s> <kernel-mangled-substring>
"""
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r'^(_Z\w*' + re.escape(sys.argv[2]) + r'\w*):', s, re.M)
i = m.start()
e = s.find('.Lfunc_end', i)
blocks, cur = [], None
for line in s[i:e].split('\n'):
    if re.match(r'^\.?L\w+:|^_Z\w+:', line):
        cur = [line.split()[0], []]
        blocks.append(cur)
    elif cur and line.startswith('\t') and not line.startswith('\t.') and not line.startswith('\t;'):
        cur[1].append(line.strip())
tot = 0
for name, ins in blocks:
    v = sum(1 for x in ins if x.startswith('v_'))
    sa = sum(1 for x in ins if x.startswith('s_') and not x.startswith(('s_waitcnt', 's_cbranch', 's_branch')))
    ld = sum(1 for x in ins if x.startswith('ds_'))
    gl = sum(1 for x in ins if x.startswith(('global_', 'buffer_')))
    tot += len(ins)
    br = [x for x in ins if 'branch' in x]
    print(f"{name[:14]:14s} n={len(ins):4d} v={v:3d} s={sa:3d} ds={ld:3d} g={gl:2d} {br[-1][:40] if br else ''}")
print("total", tot)
