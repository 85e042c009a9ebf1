set -u
OUT=gpurun_out/r03y; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bulk or golden or c3 or shards or karn or host or errors or eras" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python tools/c3_decode_time.py || exit 1
timeout -k 10 120 python tools/c3_decode_time.py || exit 1
