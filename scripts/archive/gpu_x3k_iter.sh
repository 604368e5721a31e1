#!/bin/bash
# x3k iteration: tests, timing of NT 3/2, stamps (NT 3)
set -u
TAG=${1:-x3ki}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
VARIANTS="nt3:DMIP_X3K_NT=3 nt2:DMIP_X3K_NT=2 nt1:DMIP_X3K_NT=1" bash scripts/gpu_x3k_quick.sh "$TAG" || exit $?
DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=2 timeout -k 10 200 python scripts/x3k_stamps.py > "$OUT/stamps_nt3.json" 2>&1 || exit 3
DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=2 DMIP_X3K_NT=1 timeout -k 10 200 python scripts/x3k_stamps.py > "$OUT/stamps_nt1.json" 2>&1 || exit 3
tail -1 "$OUT/stamps_nt3.json"; tail -1 "$OUT/stamps_nt1.json"
