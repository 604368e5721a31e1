#!/bin/bash
# Round validation on one GPU: full GPU tests -> smoke -> bench line -> rocprofv3 kernel stats of the same
# command -> FETCH_SIZE / WRITE_SIZE passes (per-kernel HBM traffic, profiles/pmc_traffic.json).
# Every GPU step has its own time limit; a timeout / abort / segfault ends the script.
#   usage: bash scripts/gpu_round.sh <tag>
set -u
TAG=${1:-round}
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
  tail -3 "$OUT/$name.log"
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc ;; esac
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --steps 10 --warmup 3
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline
find "$OUT/prof" -name "*kernel_stats*" -exec cp {} "$OUT/kernel_stats.csv" \; 2>/dev/null
PB=(python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --fast-steps 2 --fp32-steps 1)
step pmc_fetch 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- "${PB[@]}"
step pmc_write 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- "${PB[@]}"
python scripts/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json"
echo done | tee -a "$OUT/steps.log"
