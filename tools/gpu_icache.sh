#!/bin/bash
# Instruction-fetch / issue counters of the C2 kernels: lists the gfx950 counters once, then one
# rocprofv3 --pmc pass per group (counters the box does not have are dropped from the group), then
# a per-kernel summary.  Usage: tools/gpu_icache.sh <tag> [extra bench args]
set -u
TAG=${1:-icache}; shift || true
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters.txt; }
GROUPS_=(
  "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH"
  "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"
  "SQ_IFETCH_LEVEL SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS"
)
i=0
for grp in "${GROUPS_[@]}"; do
  i=$((i+1))
  sel=""
  for c in $grp; do have $c && sel="$sel $c"; done
  echo "== pass $i:$sel"
  [ -z "$sel" ] && continue
  timeout -s KILL 120 rocprofv3 --pmc $sel --output-format csv -d $OUT/p$i -o run -- \
      python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --spinup 0 --no-cpu-baseline --no-extras "$@" \
      > $OUT/p$i.log 2>&1
  rc=$?
  echo "== pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done
python3 - $OUT <<'EOF'
import csv, glob, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:80]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in acc.items():
    if "pq_lin" not in k and "parity" not in k:
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:12.4g}")
EOF
exit 0
