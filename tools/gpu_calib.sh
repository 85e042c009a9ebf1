#!/bin/bash
# FETCH_SIZE calibration on known byte counts (tools/micro/ps_stream2: linear 1-KiB LDS-DMA tiles
# "T" and the 128-B row-chunk gather "G128_2_1" of the pair kernel), then FETCH/WRITE of the C2
# bench at 4M codewords (1.07 GB, past the 256 MiB Infinity Cache).  One counter group per run.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-calib}; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for pat in T G128_2_1; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_$pat -o run -- $GRAFT_REPO_ROOT/tools/micro/ps_stream2 $pat > $OUT/cal_$pat.log 2>&1 || { echo "cal $pat failed"; tail -5 $OUT/cal_$pat.log; exit 1; }
  grep -E "TB/s" $OUT/cal_$pat.log
done
B="python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline --ncw 4194304"
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $grp --output-format csv -d $OUT/c2_4m_$grp -o run -- $B > $OUT/c2_4m_$grp.log 2>&1 || { echo "c2 4m $grp failed"; tail -5 $OUT/c2_4m_$grp.log; exit 1; }
done
timeout -k 10 200 $B > $OUT/bench_c2_4m.json 2>$OUT/bench_c2_4m.err || exit 1
cat $OUT/bench_c2_4m.json
exit 0
