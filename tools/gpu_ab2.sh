#!/bin/bash
# A/B timing of variant libraries on the GPU box: the C2 bench line (value, per-call averages) of
# the default library and of each variant (tools/build_variant.sh), 200 timed steps each, twice in
# alternating order.  Optional quick parity spot-check per variant (PARITY=1).
# Usage: tools/gpu_ab2.sh <tag> [variant names...]
set -u
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    if [ "${PARITY:-0}" = 1 ] && [ $rep = 1 ] && [ $v != default ]; then
      timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread \
          -k "c2_past or RS_255_223 or (bulk and 223 and not CCSDS)" > $OUT/pytest_$v.log 2>&1
      rc=$?; echo "variant $v parity rc=$rc: $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
    fi
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extras > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -3 $OUT/bench_${v}_$rep.err; exit $rc; }
    python3 -c "
import json; d=json.loads(open('$OUT/bench_${v}_$rep.json').read().splitlines()[-1])
print('$rep $v', d['value'], d['roofline']['avg_ms'])"
  done
done
unset EZRS_LIB_VARIANT
exit 0
