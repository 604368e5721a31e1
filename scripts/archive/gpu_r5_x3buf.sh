#!/bin/bash
# x3 one-tile engine with buffer LDS-DMA: the x3 GPU tests, then the bench rows alternating with DMIP_LIB=$1
set -u
OUT=gpurun_out/${2:-r5x3buf}
BASE=$1
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_x3.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 3; }
tail -1 "$OUT/pytest.log"
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export DMIP_LIB=$BASE DMIP_LIB_AB=1; else unset DMIP_LIB DMIP_LIB_AB; fi
    timeout -k 10 300 python -u scripts/bench_x3_rows.py --reps 3 > "$OUT/rows_${lib}_$r.json" 2> "$OUT/rows_${lib}_$r.err" || { tail -5 "$OUT/rows_${lib}_$r.err"; exit 3; }
    echo "$lib $r $(tail -1 $OUT/rows_${lib}_$r.json)"
  done
done
