#!/bin/bash
# round 5: DPS tests + chain-wise drift of the two DPS engines with the step count
set -u
OUT=gpurun_out/${1:-r5g}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_surrogate.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -rf -s -k dps > "$OUT/pytest_sur.log" 2>&1
rc=$?; echo "pytest sur rc=$rc"; grep -E "FAILED|passed|failed|\[dps\]" "$OUT/pytest_sur.log" | tail -14
case $rc in 0|1) ;; *) exit 3 ;; esac
timeout -k 10 400 python -u scripts/dps_x3_drift.py > "$OUT/drift.json" 2> "$OUT/drift.err" || { tail -5 "$OUT/drift.err"; exit 3; }
cut -c1-400 "$OUT/drift.json"
