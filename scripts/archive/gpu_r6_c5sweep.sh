#!/bin/bash
# Config 5 reverse half: fixed vs per-tile cost (batch sweep under rocprof) and the turn-barrier ablation.
set -u
OUT=gpurun_out/${1:-r6_c5sweep}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 16384 32768 65536 131072; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$b" -o run --output-format csv -- \
    python scripts/bench_config5.py --steps 20 --batch $b > "$OUT/b_$b.log" 2>&1 || exit 3
  echo "batch $b: $(tail -1 $OUT/b_$b.log | cut -c1-120)"
  find "$OUT/prof_$b" -name "*kernel_stats*" -exec grep -h "loss_grad_kernel" {} \; | cut -d, -f1-4
done
for r in 1 2; do
  timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/prod_$r.log" 2>&1 || exit 3
  DMIP_LIB=abv/c5nb/libdmip.so timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/nb_$r.log" 2>&1 || exit 3
  echo "prod $(tail -1 $OUT/prod_$r.log | cut -c1-100)"; echo "nobarrier $(tail -1 $OUT/nb_$r.log | cut -c1-100)"
done
