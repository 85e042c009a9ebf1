#!/bin/bash
# PMC passes (one rocprofv3 --pmc run per group; counters the box lacks are dropped) over a short
# bench run, then a per-kernel summary of the kernels matching KFILT.
# Usage: KFILT=regex tools/gpu_pmc_groups.sh <tag> "<group1>" "<group2>" ... -- [bench args]
set -u
TAG=$1; shift
GROUPS_=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do GROUPS_+=("$1"); shift; done
[ $# -gt 0 ] && shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
have() { grep -qw "$1" $OUT/counters.txt || [ "$1" = FETCH_SIZE ] || [ "$1" = WRITE_SIZE ]; }
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
python3 - $OUT "${KFILT:-.}" <<'PY'
import csv, glob, re, sys, collections
out, kf = sys.argv[1], re.compile(sys.argv[2])
acc = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.defaultdict(set)
for f in glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:80]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[k].add((f, r.get("Dispatch_Id", "")))
for k, d in acc.items():
    if not kf.search(k):
        continue
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:28s} {v:12.4g}")
PY
exit 0
