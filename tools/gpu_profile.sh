#!/bin/bash
# Round profile on the GPU box (no tests): the default bench line (extras + CPU baseline), the
# other workloads' lines (C5 also at 8 M codewords on one GPU), rocprofv3 kernel-trace summaries
# and the PMC passes that profiles/traffic.json and the VALU counts come from (one counter group
# per run, as MI355X_MICROARCH.md prescribes).  Usage: tools/gpu_profile.sh <tag>
set -u
TAG=${1:-prof}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name"
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 $OUT/$name.log | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
}
cd $GRAFT_REPO_ROOT
run bench_c2 300 python bench.py --steps 20 --warmup 3 --e2e
run bench_c3 200 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
run bench_c5 200 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c5_8m 300 python bench.py --workload c5 --ncw 8388608 --steps 10 --warmup 2 --no-cpu-baseline
run bench_shards 300 python bench.py --workload shards --steps 10 --warmup 2 --no-cpu-baseline
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras"
run prof_c2 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- $B --steps 5 --warmup 1
run prof_c3 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- $B --workload c3 --steps 3 --warmup 1
run prof_c5 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- $B --workload c5 --steps 3 --warmup 1
for w in c2 c3 c5; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    run pmc_${w}_$grp 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$w/$grp -o run -- $B --workload $w --steps 2 --warmup 1
  done
done
run pmc_c2_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    --output-format csv -d $OUT/pmc_c2_sq -o run -- $B --steps 2 --warmup 1
exit 0
