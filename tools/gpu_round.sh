#!/bin/bash
# One round-check on the GPU box: all GPU tests, smoke, the bench lines of every config, kernel-trace
# summaries (C2, C3, C4, C5) and the FETCH_SIZE / WRITE_SIZE PMC passes (one counter group per run).
set -u
TAG=${1:-round}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
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
run bench_c2 400 python bench.py --steps 20 --warmup 3 --e2e
run bench_c1 300 python bench.py --workload c1 --steps 20 --warmup 3 --no-cpu-baseline
run bench_shards 400 python bench.py --workload shards --steps 10 --warmup 2 --no-cpu-baseline
run bench_c3 400 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
run bench_c4 400 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline
run bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline"
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- $B --steps 5 --warmup 1
run prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- $B --workload c4 --steps 2 --warmup 1
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- $B --workload c5 --steps 5 --warmup 1
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- $B --workload c3 --steps 5 --warmup 1
for w in c2 c3 c4 c5; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    run pmc_${w}_$grp 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$w/$grp -o run -- $B --workload $w --steps 2 --warmup 1
  done
done
exit 0
