set -u
cd $GRAFT_REPO_ROOT
export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_pqmore.so
[ "${SKIP_PARITY:-0}" = 1 ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_shards_gpu.py tests/test_launch_split_gpu.py tests/test_ref_harness_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pqmore_pytest.log 2>&1
rc=$?; echo "variant parity rc=$rc: $(tail -n 1 gpurun_out/pqmore_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for K in 228 247; do
  for v in default pqmore; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    timeout -k 10 200 python bench.py --k $K --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/pqmore_${K}_$v.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/pqmore_${K}_$v.json').read().splitlines()[-1]); print('$K $v', d['value'], d['roofline']['avg_ms'])"
  done
done
