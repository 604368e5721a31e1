#!/bin/bash
# x3 engine: chain index recomputed after the step loop -- its tests (snapshots, shards, balanced schedule) + rows
set -u
OUT=gpurun_out/${1:-r5p}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_x3k.py tests/test_gpu_parity.py tests/test_gpu_drivers.py -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider -rf > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -6
case $rc in 0|1) ;; *) exit 3 ;; esac
timeout -k 10 300 python -u scripts/bench_x3_rows.py > "$OUT/rows.json" 2>/dev/null || exit 3
cat "$OUT/rows.json"
