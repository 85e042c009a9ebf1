#!/bin/bash
# A/B of C5 encode / decode call times (tools/c5_decode_time.py) for the default library and
# variants (tools/build_variant.sh), twice in alternating order.
# Usage: tools/gpu_c5_ab.sh <ncw> [variant names...]
set -u
NCW=$1; shift
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for v in default "$@"; do
    if [ $v = default ]; then unset EZRS_LIB_VARIANT; else export EZRS_LIB_VARIANT=$GRAFT_REPO_ROOT/tools/variants/libezrs_$v.so; fi
    timeout -k 10 120 python tools/c5_decode_time.py $NCW 20 || exit $?
  done
done
exit 0
