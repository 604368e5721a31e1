#!/bin/bash
# config-5 training kernels: their GPU tests, then a same-box A/B of bench_config5 against a baseline build
#   usage: bash scripts/gpu_r4_c5.sh <tag> <baseline.so>
set -u
TAG=${1:-r4c5}
BASE=${2:-abv/x3k_r3/libdmip.so}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_train_split.py tests/test_gpu_train_step.py \
  -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "loss_grad or split or step or config5" \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -8
case $rc in 0) ;; *) exit 3 ;; esac
for r in 1 2; do
  timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/new_$r.json" 2>/dev/null || exit 3
  DMIP_LIB=$BASE timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/base_$r.json" 2>/dev/null || exit 3
  echo "new  $(tail -1 $OUT/new_$r.json)"; echo "base $(tail -1 $OUT/base_$r.json)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/bench_config5.py --steps 20 > "$OUT/prof.log" 2>&1 || exit 3
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
grep -E "loss_grad" "$OUT/kernel_stats.csv" | cut -c1-200
