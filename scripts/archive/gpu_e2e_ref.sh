#!/bin/bash
# Verdict r3 item 3: the reference's own training configuration run to completion on the device and scored.
#   ref      config_scatterometry.yml (CDE [512]^3, PINNLoss, lr 1e-4, batch 1000, 20,000 epochs x 8 batches), then
#            the reference-size evaluation of that checkpoint (100 ys x 10 repeats x 30k samples vs fused MH)
#   fixture  the CPU fixture's recipe on the device (the control: its KL2 of 6.6 vs MH)
set -u
PART=${1:-ref}
OUT=gpurun_out/e2e
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$PART" = ref ]; then
  timeout -k 10 900 python -u scripts/bench_posterior_e2e.py --recipe reference --save-cde "$OUT/ckpt_ref512.npz" \
    > "$OUT/ref.json" 2> "$OUT/ref.err" || { tail -5 "$OUT/ref.err"; exit 3; }
  tail -1 "$OUT/ref.json"
  timeout -k 10 250 python -u scripts/bench_evaluate_pipeline.py --ckpt "$OUT/ckpt_ref512.npz" --width 512 \
    > "$OUT/eval_ref.json" 2> "$OUT/eval_ref.err" || { tail -5 "$OUT/eval_ref.err"; exit 3; }
  tail -1 "$OUT/eval_ref.json"
else
  timeout -k 10 900 python -u scripts/bench_posterior_e2e.py --recipe fixture --save-cde "$OUT/ckpt_fix256.npz" \
    > "$OUT/fix.json" 2> "$OUT/fix.err" || { tail -5 "$OUT/fix.err"; exit 3; }
  tail -1 "$OUT/fix.json"
fi
