#!/bin/bash
# per-phase cycle stamps of the k-major fp32x3 sampler (diagnostic build path) for NT = 3 and 2
set -u
OUT=gpurun_out/${1:-x3kst}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for nt in 3 2 1; do
  DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=2 DMIP_X3K_NT=$nt timeout -k 10 200 python scripts/x3k_stamps.py > "$OUT/stamps_nt$nt.json" 2>&1 || { tail -5 "$OUT/stamps_nt$nt.json"; exit 3; }
  echo "nt=$nt $(tail -1 $OUT/stamps_nt$nt.json)"
done
