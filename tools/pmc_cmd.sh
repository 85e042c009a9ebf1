#!/bin/bash
# PMC passes over an arbitrary command.  Usage: tools/pmc_cmd.sh <tag> "<grp1>" "<grp2>" ... -- cmd args
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
sets=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do sets+=("$1"); shift; done
shift
i=0
for grp in "${sets[@]}"; do
  i=$((i+1))
  echo "== pass $i: $grp"
  timeout -k 10 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1
  rc=$?; echo "== pass $i rc=$rc"; tail -2 $OUT/p$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
