#!/bin/bash
# ISA statistics of the 4-wave tile kernel (k_pq_lin) only: compiles ezrs_ps.hip with
# -DEZRS_PQ_ONLY (the 8-wave kernels are not instantiated), prints VALU / spill counts per
# instantiation.  Usage: tools/pq_isa.sh [extra hipcc flags]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -w -I$R/include -DEZRS_PQ_ONLY "$@" \
    --cuda-device-only -S -o /tmp/pq_only.s $R/ezpwd-reed-solomon_amd/csrc/ezrs_ps.hip
python3 - <<'PY'
import re, collections
L = open('/tmp/pq_only.s').read().split('\n')
names = [l.split(':')[0] for l in L if l.startswith('_ZN4ezrs2ps2pq8k_pq_lin') and ':' in l]
for name in names:
    st = L.index(next(l for l in L if l.startswith(name + ':')))
    en = next(i for i in range(st, len(L)) if L[i].strip().startswith('.Lfunc_end'))
    c = collections.Counter(re.match(r'\s+(v_\w+)', l).group(1) for l in L[st:en] if re.match(r'\s+v_', l))
    scr = sum('scratch_' in l for l in L[st:en])
    vg = next(l for l in L[en:] if 'next_free_vgpr' in l).split()[-1]
    print(name[38:70], 'valu', sum(c.values()), 'b3', c['v_bitop3_b32'], 'xor', c['v_xor_b32_e32'],
          'mov', c['v_mov_b32_e32'] + 2 * c['v_mov_b64_e32'], 'scratch', scr, 'vgpr', vg)
PY
