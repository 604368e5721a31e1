#!/bin/bash
# same-box A/B of the DPS / MH fp32x3 kernels: in-tree library against DMIP_LIB=$1 (alternating), after the tests
set -u
OUT=gpurun_out/${2:-r5x}
BASE=$1
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py -k "dps or mh" > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 3; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export DMIP_LIB=$BASE DMIP_LIB_AB=1; else unset DMIP_LIB DMIP_LIB_AB; fi
    timeout -k 10 200 python -u scripts/bench_dps.py --reps 3 > "$OUT/dps_${lib}_$r.json" 2> "$OUT/dps_${lib}_$r.err" || { tail -5 "$OUT/dps_${lib}_$r.err"; exit 3; }
    timeout -k 10 200 python -u scripts/bench_surrogate.py --no-cpu --reps 3 > "$OUT/mh_${lib}_$r.json" 2> "$OUT/mh_${lib}_$r.err" || { tail -5 "$OUT/mh_${lib}_$r.err"; exit 3; }
    python - "$OUT" $lib $r <<'PY'
import json, sys
o, lib, r = sys.argv[1:]
d = json.loads(open(f"{o}/dps_{lib}_{r}.json").read().strip().splitlines()[-1])
m = json.loads(open(f"{o}/mh_{lib}_{r}.json").read().strip().splitlines()[-1])
print(lib, r, "dps", {k: v for k, v in d.items() if "ms" in k}, "mh_x3", round(m["mh_fp32x3"]["ms_per_launch"], 2))
PY
  done
done
