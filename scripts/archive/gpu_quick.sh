#!/bin/bash
# Short GPU iteration: parity tests then one bench line (no profiler).
#   usage: bash scripts/gpu_quick.sh [tag] [pytest -k expr]
set -u
TAG=${1:-quick}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$K" ]; then KARGS=(-k "$K"); else KARGS=(); fi
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider -rf "${KARGS[@]}" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 "$OUT/bench.log"
exit $rc
