#!/bin/bash
# r05o: error-path parity tests on the default library, then C3 decode A/B against the previous
# error kernel (eprev).
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05o; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
    -k "c3 or erasure or bulk or karn or full_length or shard or positions or generic or decode" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_c3_ab.sh r05o ${VARIANTS:-eprev} || exit 1
exit 0
