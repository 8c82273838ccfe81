#!/usr/bin/env python3
"""Instruction mix between consecutive s_barrier of one kernel in a device .s file:
python tools/asm_steps.py <file.s> <mangled-name-substring>"""
import re
import sys
from collections import Counter

s = open(sys.argv[1]).read()
names = [m.group(1) for m in re.finditer(r'^(_Z\w+):', s, re.M) if sys.argv[2] in m.group(1)]
for name in names[:1]:
    i = s.find(name + ':')
    j = s.find('.Lfunc_end', i)
    lines = s[i:j].split('\n')
    bar = [n for n, l in enumerate(lines) if 's_barrier' in l]
    meta = s[s.find('amdhsa.kernels'):]
    e = [x for x in meta.split('\n  - ') if name in x][0]
    g = lambda k: (re.search(r'\.' + k + r':\s+(\d+)', e) or [None, None])[1]
    print(name[:80], 'vgpr', g('vgpr_count'), 'agpr', g('agpr_count'), 'spill', g('vgpr_spill_count'))
    for a, b in zip(bar, bar[1:]):
        body = [l.split()[0] for l in lines[a + 1:b] if l.strip() and not l.strip().startswith(';') and not l.startswith('.')]
        c = Counter(body)
        print(a, b, 'mfma', c['v_mfma_f32_32x32x16_f16'], 'valu',
              sum(v for k, v in c.items() if k.startswith('v_') and 'mfma' not in k),
              'salu', sum(v for k, v in c.items() if k.startswith('s_')), 'ds', sum(v for k, v in c.items() if k.startswith('ds_')),
              'buf', c['buffer_load_dwordx4'])
        print('    ', [(k, v) for k, v in c.most_common(24) if k.startswith('v_') and 'mfma' not in k])
