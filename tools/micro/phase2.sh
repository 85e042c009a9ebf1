set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/phase2; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/micro -o run -- python3 $GRAFT_REPO_ROOT/tools/wide_phase.py 65536 > $OUT/micro.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench.log 2>&1 || exit 1
