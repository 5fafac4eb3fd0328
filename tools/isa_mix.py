#!/usr/bin/env python3
"""Instruction mix per kernel of a device assembly file (hipcc --cuda-device-only -S)."""
import re
import sys

OPS = ['v_mul_lo_u32', 'v_mul_hi_u32', 'v_mul_u32_u24', 'v_mad_u32_u24', 'v_mad_u64_u32', 'v_mul_i32_i24',
       'v_mad_i32_i24', 'v_cvt_f32', 'v_rcp', 'v_perm_b32', 'v_pk_', 'ds_read', 'ds_write', 'v_cndmask',
       'scratch_', 'buffer_', 'global_load', 's_waitcnt']


def main(path, filt):
    s = open(path).read()
    labels = [(m.start(), m.group(1)) for m in re.finditer(r'^(_Z\w+):', s, re.M)]
    for i, (pos, name) in enumerate(labels):
        end = labels[i + 1][0] if i + 1 < len(labels) else len(s)
        body = s[pos:end]
        if filt and not any(f in name for f in filt):
            continue
        ninstr = sum(1 for l in body.splitlines() if l.startswith('\t') and not l.startswith('\t.') and
                     not l.startswith('\t;'))
        cnt = {op: len(re.findall(r'\b' + op, body)) for op in OPS}
        print(name[:48], ninstr, {k: v for k, v in cnt.items() if v})


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])
