#!/bin/bash
# spread LDS-DMA pieces in the fp32x3 DPS kernel: DPS tests, then a same-box A/B against the burst build (abv/burst)
set -u
OUT=gpurun_out/${1:-r5l}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_surrogate.py -m gpu -q --timeout 300 -k dps \
  --timeout-method thread -p no:cacheprovider -rf > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -6
case $rc in 0|1) ;; *) exit 3 ;; esac
for r in 1 2; do
  timeout -k 10 300 python -u scripts/bench_dps.py --reps 1 --gt-chains 2000 > "$OUT/new_$r.json" 2>/dev/null || exit 3
  python -c "import json; d=json.loads(open('$OUT/new_$r.json').read().strip().splitlines()[-1]); print('new', d['rank0_launch_ms'])"
  DMIP_LIB=abv/prev/libdmip.so DMIP_LIB_AB=1 timeout -k 10 300 python -u scripts/bench_dps.py --reps 1 --gt-chains 2000 > "$OUT/prev_$r.json" 2>/dev/null || exit 3
  python -c "import json; d=json.loads(open('$OUT/prev_$r.json').read().strip().splitlines()[-1]); print('prev', d['rank0_launch_ms'])"
done
