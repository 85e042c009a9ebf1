#!/bin/bash
# One GPU session: the full GPU suite + smoke on the default library, a parity spot-check of each
# variant library (tools/build_variant.sh), the C2 bench line of the default and each variant, and
# the stamp micro-benchmarks named in STAMPS.  Every GPU step has its own time limit; the first
# failure ends the script.  Usage: tools/gpu_session.sh <tag> "<variants>" "<stamp binaries>"
set -u
TAG=$1; VARS=${2:-}; STAMPS=${3:-}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 3 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
rc=$?; tail -n 1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
for v in $VARS; do
  EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py \
      -m gpu -x -q --timeout 240 --timeout-method thread -k "c2_past or RS_255_223 or (bulk and 223 and not CCSDS)" > $OUT/pytest_$v.log 2>&1
  rc=$?; echo "variant $v parity rc=$rc: $(tail -n 1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for v in default $VARS; do
  if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $OUT/bench_$v.json 2> $OUT/bench_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -3 $OUT/bench_$v.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$v.json').read().splitlines()[-1])
print('$v', d['value'], d['roofline']['avg_ms'], d['roofline']['frac'])"
done
unset EZRS_LIB_VARIANT
for b in $STAMPS; do
  timeout -k 10 60 tools/micro/$b > $OUT/$b.txt 2>&1 || { echo "stamps $b failed"; exit 1; }
  case $b in pq_*) timeout -k 10 60 tools/micro/$b 1 >> $OUT/$b.txt 2>&1 || exit 1;; esac
done
exit 0
