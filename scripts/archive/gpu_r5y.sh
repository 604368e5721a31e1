#!/bin/bash
# multi-tile MH kernel: bit-identity of DMIP_MH_MT=1|2|3, the MH tests (default), timing A/B of the three
set -u
OUT=gpurun_out/${1:-r5y}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for mt in 1 2 3; do
  DMIP_MH_MT=$mt timeout -k 10 120 python -u scripts/mh_mt_dump.py "$OUT/mt$mt.npz" > "$OUT/dump$mt.log" 2>&1 || { tail -5 "$OUT/dump$mt.log"; exit 3; }
done
python - "$OUT" <<'PY'
import numpy as np, sys
o = sys.argv[1]
d = {m: np.load(f"{o}/mt{m}.npz") for m in (1, 2, 3)}
for m in (2, 3):
    print("MT", m, {k: bool(np.array_equal(d[1][k], d[m][k])) for k in d[1].files},
          {k: float(np.abs(d[1][k] - d[m][k]).max()) for k in d[1].files})
PY
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py -k "mh or gt" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 3; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for mt in 1 2 3; do
    DMIP_MH_MT=$mt timeout -k 10 200 python -u scripts/bench_surrogate.py --no-cpu --reps 3 > "$OUT/mh_${mt}_$r.json" 2> "$OUT/mh_${mt}_$r.err" || { tail -5 "$OUT/mh_${mt}_$r.err"; exit 3; }
    python -c "import json;d=json.loads(open('$OUT/mh_${mt}_$r.json').read().strip().splitlines()[-1]);print('MT $mt rep $r', round(d['mh_fp32x3']['ms_per_launch'],2), 'ms; f32', round(d['mh_ms_per_launch'],1))"
  done
done
# DPS with the pinned range max against the unpinned build ($2, default abv/nopin/libdmip.so)
BASE=${2:-abv/nopin/libdmip.so}
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export DMIP_LIB=$BASE DMIP_LIB_AB=1; else unset DMIP_LIB DMIP_LIB_AB; fi
    timeout -k 10 200 python -u scripts/bench_dps.py --reps 3 > "$OUT/dps_${lib}_$r.json" 2> "$OUT/dps_${lib}_$r.err" || { tail -5 "$OUT/dps_${lib}_$r.err"; exit 3; }
    python -c "import json;d=json.loads(open('$OUT/dps_${lib}_$r.json').read().strip().splitlines()[-1]);print('dps $lib $r', round(d['rank0_launch_ms'],1), 'ms', d.get('quality',{}).get('KL2_vs_mcmc'))"
  done
done
unset DMIP_LIB DMIP_LIB_AB
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py -k "dps" > "$OUT/pytest_dps.log" 2>&1 || { tail -30 "$OUT/pytest_dps.log"; exit 3; }
tail -2 "$OUT/pytest_dps.log"
