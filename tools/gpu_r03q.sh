set -u
OUT=gpurun_out/r03zc; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bulk or golden or c3 or karn or errors or eras or erasure_split" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 120 python tools/c3_decode_time.py || exit 1
