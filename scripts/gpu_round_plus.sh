#!/bin/bash
# gpu_round.sh (tests, smoke, bench, rocprof, PMC traffic), then the config-3 CDiffE quality run on the
# committed trained checkpoint and the k-major engine's phase stamps. Each step time-limited.
set -u
TAG=${1:-roundplus}
bash scripts/gpu_round.sh "$TAG" || exit $?
OUT=gpurun_out/$TAG
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/bench_posterior_e2e.py --no-cde --no-posterior \
  --load-cdiffe tests/golden/ckpt_cdiffe_scat.npz --snr-sweep 0.01,0.05,0.1 > "$OUT/e2e_cdiffe.json" 2> "$OUT/e2e_cdiffe.err" \
  || { echo "e2e failed"; tail -5 "$OUT/e2e_cdiffe.err"; exit 3; }
tail -c 600 "$OUT/e2e_cdiffe.json"
bash scripts/gpu_x3k_stamps.sh "$TAG/stamps"
