#!/bin/bash
# Round-end check, part B: kernel-trace summaries and FETCH_SIZE / WRITE_SIZE passes (one counter
# group per run) of C2, C3, C4, C5 (1 M) and C5 at 8 M.  Usage: tools/gpu_final_b.sh <tag>
set -u
TAG=${1:-final}; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
run() {
  local name=$1 to=$2; shift 2
  echo "== $name" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  [ $rc -eq 0 ] || { tail -n 3 $OUT/$name.log; exit $rc; }
}
cd /tmp
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-extras"
run prof_c2 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c2 -o run -- $B --steps 20 --warmup 3
run prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- $B --workload c3 --steps 5 --warmup 1
run prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4 -o run -- $B --workload c4 --steps 2 --warmup 1
run prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5 -o run -- $B --workload c5 --steps 20 --warmup 3
run prof_c5_8m 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c5_8m -o run -- $B --workload c5 --ncw 8388608 --steps 5 --warmup 1
for w in c2 c3 c4 c5; do
  for grp in FETCH_SIZE WRITE_SIZE; do
    run pmc_${w}_$grp 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$w/$grp -o run -- $B --workload $w --steps 2 --warmup 1
  done
done
for grp in FETCH_SIZE WRITE_SIZE; do
  run pmc_c5_8m_$grp 180 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_c5_8m/$grp -o run -- $B --workload c5 --ncw 8388608 --steps 2 --warmup 1
done
exit 0
