set -u
OUT=gpurun_out/r03o; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_bch_gpu.py -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o "\"value\": [0-9.]*\|avg_ms.*}}" || exit 1
for v in prio1 prio2; do
  EZRS_LIB_VARIANT=tools/variants/libezrs_$v.so timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o "avg_ms.*}}" || exit 1
done
timeout -k 10 120 python bench.py --steps 20 --warmup 3 --no-cpu-baseline 2>/dev/null | grep -o "avg_ms.*}}"
