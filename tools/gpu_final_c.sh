#!/bin/bash
# Round-end workload lines: shard sweep, C1, C3, C4, C5 (1 M and 8 M) and the default line.
# Usage: tools/gpu_final_c.sh <tag>
set -u
TAG=${1:-final}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -n 1 $OUT/$name.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
cd $GRAFT_REPO_ROOT
run bench_shards 400 python bench.py --workload shards --steps 20 --warmup 3 --no-cpu-baseline
run bench_c1 300 python bench.py --workload c1 --steps 200 --warmup 20 --no-cpu-baseline
run bench_c3 400 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c4 400 python bench.py --workload c4 --steps 5 --warmup 1 --no-cpu-baseline
run bench_c5 300 python bench.py --workload c5 --steps 200 --warmup 20 --no-cpu-baseline
run bench_c5_8m 300 python bench.py --workload c5 --ncw 8388608 --steps 50 --warmup 5 --no-cpu-baseline
run bench_driver 500 python bench.py --gpus 1 --steps 20 --warmup 5
exit 0
