#!/bin/bash
# A/B or ablation library: one translation unit recompiled with extra flags, linked with the in-tree objects of the
# rest (make first). The result is abv/<name>/libdmip.so, loaded with DMIP_LIB=abv/<name>/libdmip.so.
#   usage: bash scripts/build_variant.sh <name> <tu-basename, e.g. dmip_train> <extra hipcc flags...>
set -eu
NAME=$1; TU=$2; shift 2
C=diffusion-modelling-for-inverse-problems_amd/csrc
mkdir -p abv/$NAME
SLP=""
case $TU in dmip_kernels|dmip_x3*|dmip_dps_x3) SLP="-fno-slp-vectorize" ;; esac
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-parameter $SLP "$@" \
  -c $C/$TU.hip -o abv/$NAME/$TU.o
OBJS=$(ls $C/*.o | grep -v "/$TU.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS abv/$NAME/$TU.o -o abv/$NAME/libdmip.so
echo "built abv/$NAME/libdmip.so"
