#!/bin/bash
# Round-end check, part A: every GPU test, smoke, the default bench line (the driver's command) and
# a 200-step line.  Usage: tools/gpu_final_a.sh <tag>
set -u
TAG=${1:-final}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -n 2 $OUT/$name.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
cd $GRAFT_REPO_ROOT
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 500 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_k200 500 python bench.py --steps 200 --warmup 20 --no-cpu-baseline
exit 0
