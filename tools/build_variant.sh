#!/bin/bash
# Variant build of libezrs_hip.so for A/B timing: one source (ezrs_ps.hip by default) recompiled with extra flags, linked
# with the other objects of the regular build.  Usage: tools/build_variant.sh <name> <flags...>
# SRC="<file stems>" picks the sources (default ezrs_ps).
# -> tools/variants/libezrs_<name>.so (load it with EZRS_LIB_VARIANT=<path>).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
O=$R/ezpwd-reed-solomon_amd/lib/obj
SRC=${SRC:-ezrs_ps}
mkdir -p $R/tools/variants
objs=""
keep=$(ls $O/*.o)
for s in $SRC; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -I$R/include "$@" \
      -c $R/ezpwd-reed-solomon_amd/csrc/$s.hip -o /tmp/${s}_$NAME.o &
  objs="$objs /tmp/${s}_$NAME.o"
  keep=$(echo "$keep" | grep -v "/$s.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/variants/libezrs_$NAME.so $keep $objs
echo $R/tools/variants/libezrs_$NAME.so
