#!/bin/bash
# same-box A/B of the config-5 training step between the in-tree libdmip.so and variant builds (DMIP_LIB)
set -u
OUT=gpurun_out/${1:-abtrain}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do
  for lib in default "$@"; do
    n=$(basename "$lib" .so)_$r
    if [ "$lib" = default ]; then timeout -k 10 200 python scripts/bench_config5.py > "$OUT/$n.json" 2>&1 || exit 3
    else DMIP_LIB=$lib timeout -k 10 200 python scripts/bench_config5.py > "$OUT/$n.json" 2>&1 || exit 3; fi
    echo "$n $(tail -1 $OUT/$n.json)"
  done
done
