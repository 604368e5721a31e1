#!/bin/bash
# round 3: CDiffE trained 4x longer, predictor-only vs predictor-corrector over a corrector snr sweep
set -u
OUT=gpurun_out/r3d
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u scripts/bench_posterior_e2e.py --no-posterior --no-cde --epochs 12000 \
  --snr-sweep 0.005,0.01,0.02,0.05,0.1 --save-cdiffe "$OUT/ckpt_cdiffe_scat.npz" > "$OUT/e2e_cdiffe.json" 2> "$OUT/e2e_cdiffe.err"
rc=$?; echo "e2e rc=$rc"; tail -c 2500 "$OUT/e2e_cdiffe.json"; tail -3 "$OUT/e2e_cdiffe.err"
exit $rc
