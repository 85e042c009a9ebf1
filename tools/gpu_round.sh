#!/bin/bash
# One round-check on the GPU box: all GPU tests, smoke, C2 + C5 benches, kernel-trace summaries,
# and the FETCH_SIZE / WRITE_SIZE PMC passes (one counter group per rocprofv3 run) for both.
set -u
TAG=${1:-round}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -n 3 $OUT/$name.log
  [ $rc -eq 0 ] || exit $rc
}
run pytest 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench_c2 400 python bench.py --steps 20 --warmup 3 --e2e
run bench_c1 300 python bench.py --workload c1 --steps 20 --warmup 3
run bench_shards 400 python bench.py --workload shards --steps 10 --warmup 2 --no-cpu-baseline
run bench_c3 400 python bench.py --workload c3 --steps 10 --warmup 2
run bench_c4 400 python bench.py --workload c4 --steps 3 --warmup 1
run bench_c5 400 python bench.py --workload c5 --steps 20 --warmup 3
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- python bench.py --workload c5 --steps 5 --warmup 1
i=0
for w in c2 c5; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    run pmc_${w}_$grp 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc/p$i -o run -- python bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline
  done
done
python tools/pmc_summary.py $OUT/pmc $OUT/pmc_summary.json --all > $OUT/pmc_summary.txt
exit 0
