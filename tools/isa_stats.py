#!/usr/bin/env python3
"""VALU / scratch / VGPR statistics per kernel of a device assembly file (hipcc -S
--cuda-device-only).  Usage: tools/isa_stats.py file.s [substring]"""
import collections
import re
import sys

L = open(sys.argv[1]).read().split('\n')
sub = sys.argv[2] if len(sys.argv) > 2 else ''
for i, l in enumerate(L):
    m = re.match(r'^(_Z\S+):\s', l)
    if not m or sub not in m.group(1):
        continue
    name = m.group(1)
    en = next(j for j in range(i, len(L)) if L[j].strip().startswith('.Lfunc_end'))
    c = collections.Counter(re.match(r'\s+(v_\w+)', x).group(1) for x in L[i:en] if re.match(r'\s+v_', x))
    scr = sum('scratch_' in x for x in L[i:en])
    ds = sum(bool(re.match(r'\s+ds_', x)) for x in L[i:en])
    vm = sum(bool(re.match(r'\s+(buffer|global)_', x)) for x in L[i:en])
    vg = next(x for x in L[en:] if 'next_free_vgpr' in x).split()[-1]
    print(f"{name[:70]:70s} valu {sum(c.values()):6d} ds {ds:5d} vmem {vm:4d} scratch {scr:3d} vgpr {vg}")
