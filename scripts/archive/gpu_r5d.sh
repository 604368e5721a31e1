#!/bin/bash
# config-5 fused step: training tests, then a same-box A/B of bench_config5 against the round-5 base library and
# its rocprof kernel stats
set -u
OUT=gpurun_out/${1:-r5d}
BASE=${2:-abv/r5_base/libdmip.so}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_train_step.py tests/test_gpu_train_split.py tests/test_gpu_parity.py \
  tests/test_gpu_train_f32.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rf > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -12
case $rc in 0|1) ;; *) exit 3 ;; esac
for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/c5_new_$r.json" 2>/dev/null || exit 3
  DMIP_LIB=$BASE DMIP_LIB_AB=1 timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/c5_base_$r.json" 2>/dev/null || exit 3
  echo "new  $(tail -1 $OUT/c5_new_$r.json | cut -c1-110)"; echo "base $(tail -1 $OUT/c5_base_$r.json | cut -c1-110)"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python scripts/bench_config5.py --steps 20 > "$OUT/prof.log" 2>&1 || exit 3
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/kernel_stats.csv" | head -12 | cut -c1-150
