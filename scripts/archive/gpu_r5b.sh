#!/bin/bash
# x3k iteration: its tests (+ the A/B library's paired-engine tests), then a same-box A/B against the round-5
# base library and the phase stamps
set -u
OUT=gpurun_out/${1:-r5b}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3k.py tests/test_gpu_x3.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rf \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -12
case $rc in 0|1) ;; *) exit 3 ;; esac
for r in 1 2 3; do
  DMIP_LIB=abv/r5_base/libdmip.so DMIP_LIB_AB=1 timeout -k 10 200 python -u scripts/sweep.py --chains 100000 --rounds 2 > "$OUT/x3k_base_$r.json" 2>/dev/null || exit 3
  timeout -k 10 200 python -u scripts/sweep.py --chains 100000 --rounds 2 > "$OUT/x3k_new_$r.json" 2>/dev/null || exit 3
  python -c "import json;b=json.load(open('$OUT/x3k_base_$r.json'));n=json.load(open('$OUT/x3k_new_$r.json'));print('x3k base',b['v0_n100000']['ms_median'],'new',n['v0_n100000']['ms_median'])"
done
DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=2 DMIP_X3K_NT=3 timeout -k 10 200 python scripts/x3k_stamps.py > "$OUT/stamps_nt3.json" 2>&1 || { tail -5 "$OUT/stamps_nt3.json"; exit 3; }
tail -1 "$OUT/stamps_nt3.json"
echo done
