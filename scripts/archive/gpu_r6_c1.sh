#!/bin/bash
# Round-6 config-1 pass: the latency probe and the host-cost probe, then every GPU test. Each step has its own limit.
#   usage: bash scripts/gpu_r6_c1.sh [tag]
set -u
TAG=${1:-r6_c1}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -u scripts/probe_config1.py > "$OUT/probe.log" 2>&1 || exit 1
tail -1 "$OUT/probe.log"
timeout -k 10 150 python -u scripts/probe_config1_host.py > "$OUT/probe_host.log" 2>&1 || exit 2
tail -1 "$OUT/probe_host.log"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -rf \
  > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; exit $rc
