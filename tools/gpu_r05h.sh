set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05h; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_early.so
timeout -k 10 500 python -u -m pytest tests/test_pq2_gpu.py tests/test_gpu_parity.py tests/test_shards_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "full_length or c2_c3 or c2_past or (bulk and 223 and not CCSDS) or (shapes and RS and 223 and not CCSDS) or shards" > $OUT/pytest_early.log 2>&1
rc=$?; tail -n 5 $OUT/pytest_early.log; [ $rc -eq 0 ] || exit $rc
unset EZRS_LIB_VARIANT
bash tools/gpu_ab2.sh r05h pq1 early pq2
