#!/bin/bash
# the one-tile fp32x3 engine's per-chunk LDS drain removed: its tests, then a same-box A/B of its bench rows against the
# drain build (abv/drain)
set -u
OUT=gpurun_out/${1:-r5m}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_gpu_drivers.py -m gpu -q --timeout 300 \
  --timeout-method thread -p no:cacheprovider -rf > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -6
case $rc in 0|1) ;; *) exit 3 ;; esac
for r in 1 2; do
  timeout -k 10 300 python -u scripts/bench_x3_rows.py > "$OUT/new_$r.json" 2>/dev/null || exit 3
  echo "new   $(cat $OUT/new_$r.json)"
  DMIP_LIB=abv/drain/libdmip.so DMIP_LIB_AB=1 timeout -k 10 300 python -u scripts/bench_x3_rows.py > "$OUT/drain_$r.json" 2>/dev/null || exit 3
  echo "drain  $(cat $OUT/drain_$r.json)"
done
