set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_bch_gpu.py tests/test_bch_dropin.py > gpurun_out/r06f_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06f_pytest.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --workload c5 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/r06f_c5.json 2> gpurun_out/r06f_c5.err && cat gpurun_out/r06f_c5.json
timeout -k 10 200 python bench.py --workload c5 --ncw 8388608 --steps 50 --warmup 5 --no-cpu-baseline > gpurun_out/r06f_c5_8m.json 2> gpurun_out/r06f_c5_8m.err && cat gpurun_out/r06f_c5_8m.json
bash tools/gpu_kt.sh r06f_kt --workload c5 --ncw 8388608
