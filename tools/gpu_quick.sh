#!/bin/bash
# Quick GPU iteration: selected tests + the C2 bench (+ optional extra bench args).
# Usage: tools/gpu_quick.sh <tag> "<pytest -k expr>" [bench args...]
set -u
TAG=$1; K=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -n 3 $OUT/bench.err
exit $rc
