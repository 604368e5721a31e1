#!/bin/bash
# Config 5: training parity tests, then the in-tree library against A/B variant libraries (DMIP_LIB), alternating.
#   usage: bash scripts/gpu_r6_c5ab.sh <tag> <variant.so>...
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf \
  tests/test_gpu_train_split.py tests/test_gpu_train_step.py tests/test_gpu_parity.py -k "loss_grad or config5 or train" \
  > "$OUT/pytest_train.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_train.log)"; case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2 3; do
  timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/prod_$r.log" 2>&1 || exit 3
  echo "prod $(tail -1 $OUT/prod_$r.log | cut -c1-110)"
  for L in "$@"; do
    n=$(basename $(dirname $L))
    DMIP_LIB=$L timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/${n}_$r.log" 2>&1 || exit 3
    echo "$n $(tail -1 $OUT/${n}_$r.log | cut -c1-110)"
  done
done
