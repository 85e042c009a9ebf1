#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout/fault status stops the script.
# Usage: tools/gpu_check.sh <tag> [pytest-args...]
set -u
TAG=${1:-r01}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
fatal() { case $1 in 0|1|2|5) return 1;; *) return 0;; esac; }
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" | tee -a $OUT/steps.log
  timeout -k 10 $to "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a $OUT/steps.log
  tail -n 5 $OUT/$name.log
  if fatal $rc; then echo "FATAL rc=$rc in $name; stopping" | tee -a $OUT/steps.log; exit $rc; fi
  return 0
}
nproc > $OUT/host.txt; lscpu | grep -E "Model name|Socket|Thread|Core" >> $OUT/host.txt
step pytest_gpu 600 python -m pytest tests -m gpu -x -q "$@"
step smoke 240 python -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python bench.py --steps 10 --warmup 2
step rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline
find $OUT/prof -name "*stats*" | head
exit 0
