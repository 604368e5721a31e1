#!/bin/bash
# Config 5 (the PINNLoss bf16 training step): the record reverse half (default) vs the recomputing one
# (DMIP_TRAIN_REC=0) -- the training GPU tests, then alternating timings on one box, then rocprof stats.
#   usage: bash scripts/gpu_r6_c5.sh [tag]
set -u
TAG=${1:-r6_c5}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -2 "$OUT/$name.log"
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc ;; esac
}
step pytest_train 600 python -u -m pytest -v --timeout 240 --timeout-method thread -p no:cacheprovider -rf -s \
  tests/test_gpu_train_split.py tests/test_gpu_train_step.py \
  tests/test_gpu_parity.py -k "loss_grad or config5 or train"
for r in 1 2 3; do
  DMIP_TRAIN_REC=1 step "rec_$r" 120 python -u scripts/bench_config5.py --steps 50
  DMIP_TRAIN_REC=0 step "recompute_$r" 120 python -u scripts/bench_config5.py --steps 50
done
step rocprof 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/bench_config5.py --steps 20
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
grep -h ms_loss "$OUT"/rec_*.log "$OUT"/recompute_*.log | cut -c1-140
echo done | tee -a "$OUT/steps.log"
