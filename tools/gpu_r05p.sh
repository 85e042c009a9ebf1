#!/bin/bash
# r05p: the final round-5 tree -- GPU suite, smoke, the driver's bench line, a K = 200 line, kernel
# traces (C2, C3, C5 at 1M and 8M) and FETCH / WRITE passes (C3, C5 at 8M), one counter per run.
set -u
TAG=${1:-r05x}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -n 1 $OUT/$name.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
}
cd $GRAFT_REPO_ROOT
[ "${SKIP_SUITE:-0}" = 1 ] || run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
run smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
run bench_driver 500 python bench.py --gpus 1 --steps 20 --warmup 5
run bench_k200 300 python bench.py --steps 200 --warmup 20 --no-extras --e2e
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras"
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- $B --steps 20 --warmup 5
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- $B --workload c3 --steps 5 --warmup 1
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- $B --workload c5 --steps 5 --warmup 1
run prof_c5_8m 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_8m -o run -- $B --workload c5 --ncw 8388608 --steps 3 --warmup 1
for grp in FETCH_SIZE WRITE_SIZE; do
  run pmc_c3_$grp 180 timeout -s KILL 170 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c3/$grp -o run -- $B --workload c3 --steps 2 --warmup 1
  run pmc_c5_8m_$grp 180 timeout -s KILL 170 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c5_8m/$grp -o run -- $B --workload c5 --ncw 8388608 --steps 2 --warmup 1
done
exit 0
