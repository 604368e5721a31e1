#!/bin/bash
# one iteration on the paired-tile engine: its tests, same-box timing vs the k-major engine, stamps, ubench
set -u
TAG=${1:-x3pi}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
SKIP_X3=1 bash scripts/gpu_x3p.sh "$TAG" || exit $?
DMIP_LIB=abv/diag/libdmip_diag.so timeout -k 10 200 python scripts/x3p_stamps.py > "$OUT/stamps.json" 2>&1 || { tail -5 "$OUT/stamps.json"; exit 3; }
tail -1 "$OUT/stamps.json"
if [ -x scripts/ubench/mfma_chain ]; then timeout -k 10 60 ./scripts/ubench/mfma_chain > "$OUT/mfma_chain.txt" 2>&1 || exit 3; cat "$OUT/mfma_chain.txt"; fi
