#!/bin/bash
# A same-box A/B variant of the x3k engine: dmip_x3k.hip compiled with extra defines, linked with the in-tree
# objects into abv/<name>/libdmip.so.   bash scripts/build_x3k_variant.sh <name> "-DDMIP_X3K_PF=2 ..."
set -e
NAME=$1; DEFS=$2
PKG=diffusion-modelling-for-inverse-problems_amd
C=$PKG/csrc
mkdir -p abv/$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -Wno-unused-parameter $DEFS \
  -c $C/dmip_x3k.hip -o abv/$NAME/dmip_x3k.o
OBJS=$(ls $C/*.o | grep -v "/dmip_x3k.o$")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS abv/$NAME/dmip_x3k.o -o abv/$NAME/libdmip.so
rm abv/$NAME/dmip_x3k.o
echo "abv/$NAME/libdmip.so"
