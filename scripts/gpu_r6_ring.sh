#!/bin/bash
# Round-6 ring-cost split at width 512: the diagnostic library's DMIP_X3_DIAG 8 (no ring barrier), 16 (no LDS-DMA
# pieces) and 24 (neither) beside 0 and 1 (no ring at all), CDE row (the ablations are CDE-only). Every step has its own limit.
#   usage: bash scripts/gpu_r6_ring.sh [tag]
set -u
TAG=${1:-r6_ring}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for d in ${DIAGS:-0 1 8 16 24}; do
  echo "=== diag $d ($(date +%T))" | tee -a "$OUT/steps.log"
  DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=$d timeout -k 10 300 python -u scripts/bench_x3_rows.py \
    --rows cde512 --reps 2 > "$OUT/diag_$d.log" 2>&1
  rc=$?
  echo "=== diag $d rc=$rc" | tee -a "$OUT/steps.log"
  tail -3 "$OUT/diag_$d.log"
  [ $rc -eq 0 ] || exit $rc
done
echo done | tee -a "$OUT/steps.log"
