#!/bin/bash
# integer-bit relu / range max in the DPS and MH kernels: MT bit-identity, surrogate tests, same-box A/B against
# DMIP_LIB=$1 (the float-max build)
set -u
OUT=gpurun_out/${2:-r5z}
BASE=$1
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for mt in 1 2; do
  DMIP_MH_MT=$mt timeout -k 10 120 python -u scripts/mh_mt_dump.py "$OUT/mt$mt.npz" > "$OUT/dump$mt.log" 2>&1 || { tail -5 "$OUT/dump$mt.log"; exit 3; }
done
DMIP_LIB=$BASE DMIP_LIB_AB=1 timeout -k 10 120 python -u scripts/mh_mt_dump.py "$OUT/base.npz" > "$OUT/dumpb.log" 2>&1 || { tail -5 "$OUT/dumpb.log"; exit 3; }
python - "$OUT" <<'PY'
import numpy as np, sys
o = sys.argv[1]
d = {m: np.load(f"{o}/{m}.npz") for m in ("mt1", "mt2", "base")}
for m in ("mt2", "base"):
    print("mt1 vs", m, {k: bool(np.array_equal(d["mt1"][k], d[m][k])) for k in d["mt1"].files})
PY
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_surrogate.py > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 3; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export DMIP_LIB=$BASE DMIP_LIB_AB=1; else unset DMIP_LIB DMIP_LIB_AB; fi
    timeout -k 10 200 python -u scripts/bench_surrogate.py --no-cpu --reps 3 > "$OUT/mh_${lib}_$r.json" 2> "$OUT/mh_${lib}_$r.err" || { tail -5 "$OUT/mh_${lib}_$r.err"; exit 3; }
    timeout -k 10 200 python -u scripts/bench_dps.py --reps 3 > "$OUT/dps_${lib}_$r.json" 2> "$OUT/dps_${lib}_$r.err" || { tail -5 "$OUT/dps_${lib}_$r.err"; exit 3; }
    python - "$OUT" $lib $r <<'PY'
import json, sys
o, lib, r = sys.argv[1:]
d = json.loads(open(f"{o}/dps_{lib}_{r}.json").read().strip().splitlines()[-1])
m = json.loads(open(f"{o}/mh_{lib}_{r}.json").read().strip().splitlines()[-1])
print(lib, r, "dps", round(d["rank0_launch_ms"], 1), "KL2", d.get("quality", {}).get("KL2_vs_mcmc"), "mh_x3", round(m["mh_fp32x3"]["ms_per_launch"], 2))
PY
  done
done
