#!/bin/bash
# GPU validation sequence for one gpurun call: parity tests -> smoke -> bench -> rocprofv3 stats.
# Every GPU step has its own time limit; a timeout / abort / segfault / kill ends the script
# (no further GPU work in this call); an ordinary test failure (exit 1) lets the later steps run.
#   usage: bash scripts/gpu_check.sh [tag]        (outputs under gpurun_out/<tag>/)
set -u
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
export HSA_ENABLE_IPC_MODE_LEGACY=0

step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  case $rc in
    0|1) return 0 ;;
    *) echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc ;;
  esac
}

step pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider -rf
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 600 python -u bench.py --steps 10 --warmup 3
cd /tmp && mkdir -p prof && cd - > /dev/null
step rocprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python bench.py --steps 3 --warmup 1 --no-cpu-baseline
find "$OUT/prof" -name "*stats*" -exec cp {} "$OUT/" \; 2>/dev/null
echo "done" | tee -a "$OUT/steps.log"
