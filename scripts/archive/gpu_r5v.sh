#!/bin/bash
# fp32x3 Metropolis-Hastings: the MH GPU tests, then the surrogate bench (exact f32 beside fp32x3) and a kernel trace
set -u
OUT=gpurun_out/${1:-r5v}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py -k "mh or gt" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 3; }
tail -3 "$OUT/pytest.log"
timeout -k 10 300 python -u scripts/bench_surrogate.py --no-cpu > "$OUT/bench_surrogate.json" 2> "$OUT/bench_surrogate.err" || { tail -5 "$OUT/bench_surrogate.err"; exit 3; }
cut -c1-900 "$OUT/bench_surrogate.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o mh -- python -u scripts/bench_surrogate.py --no-cpu --reps 2 > "$OUT/prof.log" 2>&1 || { tail -5 "$OUT/prof.log"; exit 3; }
find "$OUT/prof" -name "*kernel_stats.csv" | head -2
