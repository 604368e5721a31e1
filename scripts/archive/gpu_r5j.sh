#!/bin/bash
# the x3 engine's resident-weights mode at width 64: its tests, then config 1's latency breakdown
set -u
OUT=gpurun_out/${1:-r5j}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_gpu_drivers.py -m gpu -v --timeout 300 \
  --timeout-method thread -p no:cacheprovider -rf > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -8
case $rc in 0|1) ;; *) exit 3 ;; esac
timeout -k 10 200 python -u scripts/config1_breakdown.py > "$OUT/c1.json" 2> "$OUT/c1.err" || { tail -5 "$OUT/c1.err"; exit 3; }
cat "$OUT/c1.json"
DMIP_LIB=abv/r5_base/libdmip.so DMIP_LIB_AB=1 timeout -k 10 200 python -u scripts/config1_breakdown.py > "$OUT/c1_base.json" 2> "$OUT/c1_base.err" || { tail -5 "$OUT/c1_base.err"; exit 3; }
cat "$OUT/c1_base.json"
