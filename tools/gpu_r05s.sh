#!/bin/bash
# r05s: shard parity tests, then shard-point timings (1 KiB, 16 KiB, 1 MiB) and their kernel traces.
set -u
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r05s; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "shard or split or full_length" > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -n 2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for S in 1024 16384 1048576; do
  timeout -k 10 120 python3 tools/shard_time.py $S 100 > $OUT/shard_$S.txt 2>&1 || { echo "shard $S failed"; tail -3 $OUT/shard_$S.txt; exit 1; }
  tail -1 $OUT/shard_$S.txt | cut -c1-400
done
exit 0
