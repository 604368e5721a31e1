#!/bin/bash
set -u
OUT=gpurun_out/r5mt
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2; do for mt in 2 3; do
  DMIP_MH_MT=$mt timeout -k 10 200 python -u scripts/bench_surrogate.py --no-cpu --reps 2 --rows 100 --steps 200 --eval-n 65536 > $OUT/mt${mt}_$r.json 2>$OUT/mt${mt}_$r.err || { tail -5 $OUT/mt${mt}_$r.err; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/mt${mt}_$r.json').read().strip().splitlines()[-1]);print('MT $mt', round(d['mh_fp32x3']['ms_per_launch'],2), 'f32', round(d['mh_ms_per_launch'],1))"
done; done
