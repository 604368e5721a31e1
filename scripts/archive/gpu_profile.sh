#!/bin/bash
# Round profile: kernel-trace stats + PMC passes of the default bench workload.
#   usage: bash scripts/gpu_profile.sh <tag>
set -u
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python bench.py --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/trace.log" 2>&1
rc=$?; echo "trace rc=$rc"
case $rc in 0|1) ;; *) exit $rc ;; esac
bash scripts/gpu_pmc.sh "$TAG"
