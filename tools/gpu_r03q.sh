set -u
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python tools/c3_decode_time.py || exit 1
for w in c3 c2 shards; do
timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$w.json 2>$OUT/bench_$w.err || exit 1
grep -o "\"value\": [0-9.]*\|avg_ms.*}}" $OUT/bench_$w.json | head -4
done
