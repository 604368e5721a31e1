#!/bin/bash
# config-5 training kernel: forward / reverse split vs the fused kernel -- GPU training tests on the split
# (default), then a same-box timing of both (DMIP_TRAIN_SPLIT=0 | 1).
set -u
TAG=${1:-trsplit}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train_step.py tests/test_gpu_drivers.py -m gpu \
  -k "loss_grad or config5 or train or linear" -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed|config5|ragged|G5" "$OUT/pytest.log" | tail -40
case $rc in 0|1) ;; *) exit $rc ;; esac
for s in 1 0 1 0; do
  DMIP_TRAIN_SPLIT=$s timeout -k 10 200 python scripts/bench_config5.py > "$OUT/config5_split$s.json" 2>&1 || { echo "config5 $s failed"; tail -5 "$OUT/config5_split$s.json"; exit 3; }
  echo "split=$s $(tail -1 $OUT/config5_split$s.json)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python scripts/bench_config5.py > "$OUT/prof.log" 2>&1 || exit 3
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -12
