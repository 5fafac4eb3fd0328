#!/usr/bin/env python3
"""Print the instructions of the basic blocks of one kernel in a device assembly file
(hipcc --cuda-device-only -S) whose instruction count of a given opcode prefix is at least N.

usage: isa_block.py <file.s> <kernel-substring> <opcode-prefix> <min-count> [grep-substring]
"""
import re
import sys


def main(path, kern, prefix, mincount, pat=None):
    s = open(path).read()
    m = re.search(r'^(_Z\w*' + re.escape(kern) + r'\w*):', s, re.M)
    if not m:
        sys.exit("kernel not found")
    i = m.start()
    e = s.find('.Lfunc_end', i)
    blocks, cur = [], None
    for line in s[i:e].split('\n'):
        if re.match(r'^\.?L\w+:|^_Z\w+:', line):
            cur = [line.split()[0], []]
            blocks.append(cur)
        elif cur and line.startswith('\t') and not line.startswith('\t.') and not line.startswith('\t;'):
            cur[1].append(line.strip())
    for name, ins in blocks:
        if sum(1 for x in ins if x.startswith(prefix)) >= mincount:
            print(name, len(ins))
            for x in ins:
                if pat is None or pat in x:
                    print("   ", x[:90])


if __name__ == '__main__':
    a = sys.argv
    main(a[1], a[2], a[3], int(a[4]), a[5] if len(a) > 5 else None)
