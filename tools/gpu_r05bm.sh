#!/bin/bash
# r05bm: full GPU suite on the default library (two lanes per parity row, log-domain BCH BM), C5
# timing A/B against the previous BM (bmold), 1M and 8M, twice; then the driver's bench line.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05bm; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in default bmold; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    for n in 1048576 8388608; do
      echo -n "$rep $v $n: " >> $OUT/c5_ab.txt
      timeout -k 10 120 python3 tools/c5_decode_time.py $n 30 >> $OUT/c5_ab.txt 2>> $OUT/c5.err || { echo "c5 $v $n failed"; tail -3 $OUT/c5.err; exit 1; }
      tail -n 1 $OUT/c5_ab.txt
    done
  done
done
unset EZRS_LIB_VARIANT
timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_driver.json 2> $OUT/bench_driver.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -3 $OUT/bench_driver.err; exit $rc; }
python3 -c "
import json; d=json.loads(open('$OUT/bench_driver.json').read().splitlines()[-1])
print(d['value'], d['roofline']['avg_ms'], d['c5'], d['shards'])"
exit 0
