#!/bin/bash
# Variant build of libezrs_hip.so for A/B timing: one source (ezrs_ps.hip by default) recompiled with extra flags, linked
# with the other objects of the regular build.  Usage: tools/build_variant.sh <name> <flags...>
# SRC=<file stem> picks the source (default ezrs_ps).
# -> tools/variants/libezrs_<name>.so (load it with EZRS_LIB_VARIANT=<path>).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
O=$R/ezpwd-reed-solomon_amd/lib/obj
SRC=${SRC:-ezrs_ps}
mkdir -p $R/tools/variants
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -I$R/include "$@" \
    -c $R/ezpwd-reed-solomon_amd/csrc/$SRC.hip -o /tmp/${SRC}_$NAME.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/tools/variants/libezrs_$NAME.so \
    $(ls $O/*.o | grep -v $SRC.o) /tmp/${SRC}_$NAME.o
echo $R/tools/variants/libezrs_$NAME.so
