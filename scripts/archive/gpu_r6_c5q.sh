#!/bin/bash
# Config 5 quick loop: the training parity tests, then record vs recomputing reverse timings (alternating), rocprof.
#   usage: bash scripts/gpu_r6_c5q.sh [tag]
set -u
TAG=${1:-r6_c5q}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc: $(tail -1 $OUT/$name.log | cut -c1-150)"
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name: stopping"; exit $rc ;; esac
}
step pytest_train 600 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf \
  tests/test_gpu_train_split.py tests/test_gpu_train_step.py tests/test_gpu_parity.py -k "loss_grad or config5 or train"
for r in 1 2; do
  DMIP_TRAIN_REC=1 step "rec_$r" 120 python -u scripts/bench_config5.py --steps 50
  DMIP_TRAIN_REC=0 step "recompute_$r" 120 python -u scripts/bench_config5.py --steps 50
done
step rocprof 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/bench_config5.py --steps 20
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -5
