#!/bin/bash
# k-major engine iteration: its GPU tests, then a same-box A/B of the headline against a baseline build
# (alternating processes), optionally followed by one more command.
#   usage: bash scripts/gpu_r4_x3k.sh <tag> <baseline.so>
set -u
TAG=${1:-r4x3k}
BASE=${2:-abv/x3k_r3/libdmip.so}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3k.py -m gpu -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -8
case $rc in 0) ;; *) exit 3 ;; esac
bash scripts/gpu_ab_libs.sh "$TAG/ab" "$BASE" || exit 3
