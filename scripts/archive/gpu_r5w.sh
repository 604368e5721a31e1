#!/bin/bash
# the reference evaluation pipeline with the fp32x3 MH ground truth; kernel trace of the surrogate bench (both MH kernels)
set -u
OUT=gpurun_out/${1:-r5w}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/bench_evaluate_pipeline.py --gt-precision fp32x3 > "$OUT/evaluate_x3gt.json" 2> "$OUT/evaluate_x3gt.err" || { tail -5 "$OUT/evaluate_x3gt.err"; exit 3; }
cut -c1-900 "$OUT/evaluate_x3gt.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o mh --output-format csv -- python -u scripts/bench_surrogate.py --no-cpu --reps 2 > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 3; }
find "$OUT/prof" -name "*kernel_stats.csv"
