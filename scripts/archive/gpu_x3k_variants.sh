#!/bin/bash
# same-box A/B of x3k engine variants (abv/<name>/libdmip.so, scripts/build_x3k_variant.sh) against the in-tree
# library, alternating processes: bash scripts/gpu_x3k_variants.sh <tag> <name>...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  timeout -k 10 200 python -u scripts/sweep.py --chains 100000 --rounds 2 > "$OUT/base_$r.json" 2>/dev/null || exit 3
  echo "base $(grep -o '"ms_median": [0-9.]*' $OUT/base_$r.json | head -1)"
  for v in "$@"; do
    DMIP_LIB=abv/$v/libdmip.so DMIP_LIB_AB=1 timeout -k 10 200 python -u scripts/sweep.py --chains 100000 --rounds 2 \
      > "$OUT/${v}_$r.json" 2>/dev/null || exit 3
    echo "$v $(grep -o '"ms_median": [0-9.]*' $OUT/${v}_$r.json | head -1)"
  done
done
