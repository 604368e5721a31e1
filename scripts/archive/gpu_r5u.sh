#!/bin/bash
# round-5 end-to-end checks at the reference's sizes: the scatterometry evaluation pipeline (MCMC ground truth +
# evaluate over 100 ys) and the linear fixture's evaluation
set -u
OUT=gpurun_out/${1:-r5u}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u scripts/bench_evaluate_pipeline.py > "$OUT/evaluate.json" 2> "$OUT/evaluate.err" || { tail -5 "$OUT/evaluate.err"; exit 3; }
tail -1 "$OUT/evaluate.json" | cut -c1-600
timeout -k 10 300 python -u scripts/bench_linear_e2e.py --fixture > "$OUT/linear_fixture.json" 2> "$OUT/linear_fixture.err" || { tail -5 "$OUT/linear_fixture.err"; exit 3; }
tail -1 "$OUT/linear_fixture.json" | cut -c1-600
