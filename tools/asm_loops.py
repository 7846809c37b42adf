#!/usr/bin/env python
"""Instruction mix of the loops of a kernel in a hipcc -S listing.
    python tools/asm_loops.py file.s name_substring"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read().splitlines()
want = sys.argv[2]
i = 0
while i < len(s):
    m = re.match(r'^(_Z\w+):', s[i])
    if m and want in m.group(1):
        name = m.group(1)
        j = i
        while not s[j].strip().startswith('.Lfunc_end'):
            j += 1
        body = s[i:j]
        labels = {l.split(':')[0]: k for k, l in enumerate(body) if re.match(r'^\.LBB\w+:', l)}
        print(name, len(body), 'lines')
        for k, l in enumerate(body):
            mm = re.search(r's_(?:c)?branch\w*\s+(\.LBB\w+)', l)
            if mm and mm.group(1) in labels and labels[mm.group(1)] < k:
                seg = body[labels[mm.group(1)]:k + 1]
                c = Counter()
                for x in seg:
                    x = x.strip()
                    if not x or x[0] in ';.':
                        continue
                    op = x.split()[0]
                    key = ('mfma' if op.startswith('v_mfma') else 'exp' if op.startswith('v_exp') else
                           op if op.startswith(('v_cvt', 'v_max', 'v_add', 'v_fma', 'v_mul', 'v_pk', 'v_mov',
                                                'v_cndmask', 'v_perm', 'v_accvgpr', 'v_sub', 'v_perm'))
                           else 'valu_other' if op.startswith('v_') else 'ds' if op.startswith('ds_') else
                           's_waitcnt' if op == 's_waitcnt' else 'salu' if op.startswith('s_') else
                           'vmem' if op.startswith(('global_', 'buffer_')) else op)
                    c[key] += 1
                print('  loop', mm.group(1), 'lines', len(seg))
                for kk, v in sorted(c.items(), key=lambda kv: -kv[1]):
                    print(f'    {kk:24s} {v}')
        i = j
    i += 1
