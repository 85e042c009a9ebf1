#!/bin/bash
# A/B timing on the GPU box: selected GPU tests on the default library, then the C2 bench line of
# the default library and of each variant library (tools/build_variant.sh), plus a kernel trace of
# the default.  Usage: tools/gpu_ab.sh <tag> "<pytest -k expr>" [variant names...]
set -u
TAG=$1; K=$2; shift 2
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -n 5 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for v in default "$@"; do
  if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$v.json 2> $OUT/bench_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; tail -3 $OUT/bench_$v.err; exit $rc; }
  python3 -c "
import json; d=json.loads(open('$OUT/bench_$v.json').read().splitlines()[-1])
print('$v', d['value'], d.get('avg_ms'), d['roofline']['frac'])"
done
unset EZRS_LIB_VARIANT
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/kt.log 2>&1 || { echo "kt failed"; exit 1; }
python3 - <<EOF
import csv, glob
for f in glob.glob("$OUT/kt/**/run_kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:80], r['Calls'], r['AverageNs'])
EOF
exit 0
