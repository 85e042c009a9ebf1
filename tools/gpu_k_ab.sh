#!/bin/bash
# A/B of one RS(255,K) codec's bench line (bench.py --k K) for the default library and a variant,
# after the variant's parity tests for that codec.  Usage: tools/gpu_k_ab.sh <K> <variant>
set -u
K=$1; V=$2
cd $GRAFT_REPO_ROOT
export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$V.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/k_ab_pytest.log 2>&1
rc=$?; echo "variant parity rc=$rc: $(tail -n 1 gpurun_out/k_ab_pytest.log)"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in default $V; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    timeout -k 10 200 python bench.py --k $K --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/k_ab_$v.json 2>/dev/null || exit 1
    python3 -c "
import json; d=json.loads(open('gpurun_out/k_ab_$v.json').read().splitlines()[-1]); print('$rep $v', d['value'], d['roofline']['avg_ms'])"
  done
done
