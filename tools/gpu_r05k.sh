#!/bin/bash
# r05k: GPU suite, smoke, the driver's bench line (K = 20) and a K = 200 line on the final kernels.
set -u
TAG=${1:-r05k}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -n 2 $OUT/$name.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
cd $GRAFT_REPO_ROOT
[ "${SKIP_SUITE:-0}" = 1 ] || run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 500 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_k200 500 python bench.py --steps 200 --warmup 20 --no-extras --e2e
exit 0
