set -u
OUT=gpurun_out/r03j; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_shards_gpu.py -x -q --timeout 300 --timeout-method thread -k "bulk or shapes or golden or shards or host or c2" > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in round persist; do
  EZRS_PARITY_KERNEL=$v timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c2_$v.json 2>/dev/null || exit 1
  echo $v; grep -o "avg_ms.*}}" $OUT/c2_$v.json
done
timeout -k 10 200 python tools/e2e_probe.py 2>&1 | grep -v amdgpu.ids
