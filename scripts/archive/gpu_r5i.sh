#!/bin/bash
set -u
OUT=gpurun_out/${1:-r5i}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 200 python -u scripts/config1_breakdown.py > "$OUT/c1.json" 2> "$OUT/c1.err" || { tail -5 "$OUT/c1.err"; exit 3; }
cat "$OUT/c1.json"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python scripts/config1_breakdown.py > "$OUT/prof.log" 2>&1 || exit 3
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -12 | cut -c1-160
