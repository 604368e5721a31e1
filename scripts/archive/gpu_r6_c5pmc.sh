#!/bin/bash
# Config 5 evidence: PMC of both halves (scripts/pmc_train_split.sh) and the batch sweep under rocprof.
set -u
TAG=${1:-r6_c5pmc}
bash scripts/pmc_train_split.sh $TAG > gpurun_out/${TAG}_pmc.log 2>&1 || exit 3
OUT=gpurun_out/$TAG/sweep
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 16384 32768 65536 131072; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$b" -o run --output-format csv -- \
    python scripts/bench_config5.py --steps 20 --batch $b > "$OUT/b_$b.log" 2>&1 || exit 3
  echo "batch $b: $(tail -1 $OUT/b_$b.log | cut -c1-100)"
  find "$OUT/prof_$b" -name "*kernel_stats*" -exec grep -h "loss_grad_kernel" {} \; | cut -d, -f1-4
done
