#!/bin/bash
# round 5: DPS tests (both engines) + the config-5 A/B
set -u
OUT=gpurun_out/${1:-r5f}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_surrogate.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -rf -s > "$OUT/pytest_sur.log" 2>&1
rc=$?; echo "pytest sur rc=$rc"; grep -E "FAILED|passed|failed|\[dps\]" "$OUT/pytest_sur.log" | tail -14
case $rc in 0|1) ;; *) exit 3 ;; esac
bash scripts/gpu_r5d.sh "${1:-r5f}/c5"
