#!/bin/bash
# k-major fp32x3 engine: the product build vs the no-ring timing ablation (diagnostic library abv/diag/libdmip_diag.so, make diag; DMIP_X3_DIAG=1: no LDS-DMA, no
# ring barriers, stale weights -- timing only), alternating, same box
set -u
OUT=gpurun_out/${1:-x3knr}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
export DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3P=0
for v in prod:DMIP_X3_DIAG=0 noring:DMIP_X3_DIAG=1 prod2:DMIP_X3_DIAG=0 noring2:DMIP_X3_DIAG=1; do
  n=${v%%:*}
  env ${v#*:} timeout -k 10 300 "${B[@]}" > "$OUT/bench_$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$OUT/bench_$n.log"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/bench_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms')"
done
