#!/bin/bash
# round 3: tightened parity bounds (with -s reports) + CDiffE trained end to end and scored vs MCMC
set -u
OUT=gpurun_out/r3c
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train_f32.py -m gpu -v -s --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_s.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest_s.log" | tail -5
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 900 python -u scripts/bench_posterior_e2e.py --no-posterior --no-cde --epochs 3000 \
  --save-cdiffe "$OUT/ckpt_cdiffe_scat.npz" > "$OUT/e2e_cdiffe.json" 2> "$OUT/e2e_cdiffe.err"
rc=$?; echo "e2e rc=$rc"; tail -c 1500 "$OUT/e2e_cdiffe.json"; tail -3 "$OUT/e2e_cdiffe.err"
exit $rc
