set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r05e; mkdir -p $OUT
cd $GRAFT_REPO_ROOT
export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_pq2.so
timeout -k 10 400 python -u -m pytest tests/test_pq2_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "full_length or c2_c3 or c2_past" > $OUT/pytest_pq2.log 2>&1
rc=$?; tail -n 5 $OUT/pytest_pq2.log; [ $rc -eq 0 ] || exit $rc
unset EZRS_LIB_VARIANT
bash tools/gpu_ab2.sh r05e pq1 pq2
