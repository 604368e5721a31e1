#!/bin/bash
# Config 5 reverse-half ablations (timing only; wrong gradients): rocprof kernel times of the product library and of
# variant libraries (DMIP_LIB), batch 65,536.
#   usage: bash scripts/gpu_r6_c5abl.sh <tag> <variant.so>...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for L in prod "$@"; do
    n=prod; [ $L != prod ] && n=$(basename $(dirname $L))
    if [ $L = prod ]; then E=""; else E="DMIP_LIB=$L"; fi
    env $E timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${n}_$r" -o run --output-format csv -- \
      python scripts/bench_config5.py --steps 20 > "$OUT/${n}_$r.log" 2>&1 || exit 3
    echo "$n: $(tail -1 $OUT/${n}_$r.log | cut -c1-90)"
    find "$OUT/prof_${n}_$r" -name "*kernel_stats*" -exec grep -h "loss_grad_kernel" {} \; | cut -d, -f1-4
  done
done
