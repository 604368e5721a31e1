#!/bin/bash
# same-box A/B of the x3 rows: in-tree vs abv/prev
set -u
OUT=gpurun_out/${1:-r5q}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  timeout -k 10 300 python -u scripts/bench_x3_rows.py > "$OUT/new_$r.json" 2>/dev/null || exit 3
  echo "new  $(cat $OUT/new_$r.json)"
  DMIP_LIB=abv/prev/libdmip.so DMIP_LIB_AB=1 timeout -k 10 300 python -u scripts/bench_x3_rows.py > "$OUT/prev_$r.json" 2>/dev/null || exit 3
  echo "prev $(cat $OUT/prev_$r.json)"
done
