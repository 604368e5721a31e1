#!/bin/bash
# the reference's evaluate pipeline at its own sizes (default precision fp32x3), then a same-box timing of
# the k-major engine's tiles-per-wave variants (NT = 3 default, 2, 1 = two waves per SIMD)
set -u
OUT=gpurun_out/${1:-evalnt}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u scripts/bench_evaluate_pipeline.py > "$OUT/evaluate.json" 2> "$OUT/evaluate.err" || { tail -5 "$OUT/evaluate.err"; exit 3; }
tail -c 800 "$OUT/evaluate.json"
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
for v in nt3:3 nt1:1 nt2:2 nt3b:3 nt1b:1; do
  n=${v%%:*}
  DMIP_X3K_NT=${v#*:} timeout -k 10 300 "${B[@]}" > "$OUT/bench_$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$OUT/bench_$n.log"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/bench_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms', d.get('parity'))"
done
