#!/bin/bash
# Wide-symbol (GF(2^16)) iteration: parity tests, the C4 bench, a kernel trace of it.
set -u
TAG=${1:-wide}; OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_wide_gpu.py tests/test_gpu_parity.py -k "wide" -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 25 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench_c4.json; tail -n 3 $OUT/bench_c4.err
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/kt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/$OUT/kt.log 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
