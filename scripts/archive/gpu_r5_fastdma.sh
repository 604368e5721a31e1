#!/bin/bash
# 16-bit engine with buffer LDS-DMA: its GPU tests, then fast_mode A/B against DMIP_LIB=$1 (alternating)
set -u
OUT=gpurun_out/${2:-r5fast}
BASE=$1
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 3; }
tail -1 "$OUT/pytest.log"
B=(python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-other-configs)
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export DMIP_LIB=$BASE DMIP_LIB_AB=1; else unset DMIP_LIB DMIP_LIB_AB; fi
    timeout -k 10 300 "${B[@]}" > "$OUT/b_${lib}_$r.json" 2> "$OUT/b_${lib}_$r.err" || { tail -5 "$OUT/b_${lib}_$r.err"; exit 3; }
    python -c "import json;d=json.loads(open('$OUT/b_${lib}_$r.json').read().strip().splitlines()[-1]);print('$lib $r fast', round(d['fast_mode']['launch_ms'],2), d['fast_mode']['parity'], 'x3k', round(d['roofline']['launch_ms'],2))"
  done
done
