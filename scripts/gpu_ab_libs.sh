#!/bin/bash
# same-box A/B of the headline kernel between the in-tree libdmip.so and variant builds (DMIP_LIB), alternating
set -u
OUT=gpurun_out/${1:-ablibs}
shift
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
for r in 1 2; do
  for lib in default "$@"; do
    n=$(basename "$lib" .so)_$r
    if [ "$lib" = default ]; then timeout -k 10 300 "${B[@]}" > "$OUT/$n.log" 2>&1 || exit 3
    else DMIP_LIB=$lib timeout -k 10 300 "${B[@]}" > "$OUT/$n.log" 2>&1 || exit 3; fi
    python -c "import json;d=json.loads(open('$OUT/$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms', d.get('parity'))"
  done
done
