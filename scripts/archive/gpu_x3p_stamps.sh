#!/bin/bash
set -u
OUT=gpurun_out/${1:-x3ps}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
DMIP_LIB=abv/diag/libdmip_diag.so timeout -k 10 200 python scripts/x3p_stamps.py > "$OUT/stamps.json" 2>&1 || { tail -5 "$OUT/stamps.json"; exit 3; }
tail -1 "$OUT/stamps.json"
timeout -k 10 60 ./scripts/ubench/mfma_chain > "$OUT/mfma_chain.txt" 2>&1 || exit 3
cat "$OUT/mfma_chain.txt"
