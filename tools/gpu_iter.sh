#!/bin/bash
# One iteration on the GPU box: parity tests, bench, rocprof kernel trace, ablations.
set -u
TAG=${1:-iter}
bash tools/gpu_check.sh $TAG --timeout 120 || exit $?
bash tools/gpu_ablate.sh || exit $?
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/$TAG/prof/run_kernel_stats.csv')):
    print(r['Name'][:70], r['Calls'], r['AverageNs'], r['Percentage'])
"
