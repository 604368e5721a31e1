#!/bin/bash
# config-5 reverse half: timing ablations (wrong results, timing only) against the product library, same box
#   usage: bash scripts/gpu_c5_ablate.sh <tag> <ablation.so>...
set -u
OUT=gpurun_out/${1:-c5ab}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/prod_$r.json" 2>/dev/null || exit 3
  echo "prod $(tail -1 $OUT/prod_$r.json | cut -c1-120)"
  for L in "$@"; do
    n=$(basename $(dirname $L))
    DMIP_LIB=$L timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/${n}_$r.json" 2>/dev/null || exit 3
    echo "$n $(tail -1 $OUT/${n}_$r.json | cut -c1-120)"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/bench_config5.py --steps 20 > "$OUT/prof.log" 2>&1 || exit 3
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-8 "$OUT/kernel_stats.csv" | head -12
