#!/bin/bash
# one iteration on the paired-tile engine: its tests, same-box timing vs the k-major engine, stamps, ubench
set -u
TAG=${1:-x3pi}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
SKIP_X3=1 bash scripts/gpu_x3p.sh "$TAG" || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_x3k.py -m gpu -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "fp16_range or handover or tiles_per_wave" > "$OUT/pytest_range.log" 2>&1
rc=$?; echo "pytest range rc=$rc"; grep -E "FAILED|Error|passed|failed|\[x3\]" "$OUT/pytest_range.log" | tail -20
case $rc in 0|1) ;; *) exit $rc ;; esac
DMIP_LIB=abv/diag/libdmip_diag.so timeout -k 10 200 python scripts/x3p_stamps.py > "$OUT/stamps.json" 2>&1 || { tail -5 "$OUT/stamps.json"; exit 3; }
tail -1 "$OUT/stamps.json"
if [ -x scripts/ubench/mfma_chain ]; then timeout -k 10 60 ./scripts/ubench/mfma_chain > "$OUT/mfma_chain.txt" 2>&1 || exit 3; cat "$OUT/mfma_chain.txt"; fi
