#!/bin/bash
# round 5, first box: the full GPU suite, the headline x3k A/B against the round-5 base library (same box,
# alternating processes) with phase stamps, the config-5 scratch swizzle A/B against round 4's library with
# its PMC passes, and one bench line
set -u
OUT=gpurun_out/r5a
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -rf \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -12
case $rc in 0|1) ;; *) exit 3 ;; esac
for r in 1 2 3; do
  DMIP_LIB=abv/r5_base/libdmip.so timeout -k 10 200 python -u scripts/sweep.py --chains 100000 --rounds 2 > "$OUT/x3k_base_$r.json" 2>/dev/null || exit 3
  timeout -k 10 200 python -u scripts/sweep.py --chains 100000 --rounds 2 > "$OUT/x3k_new_$r.json" 2>/dev/null || exit 3
  python -c "import json;b=json.load(open('$OUT/x3k_base_$r.json'));n=json.load(open('$OUT/x3k_new_$r.json'));print('x3k base',b['v0_n100000']['ms_median'],'new',n['v0_n100000']['ms_median'])"
done
DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=2 DMIP_X3K_NT=3 timeout -k 10 200 python scripts/x3k_stamps.py > "$OUT/stamps_nt3.json" 2>&1 || { tail -5 "$OUT/stamps_nt3.json"; exit 3; }
tail -1 "$OUT/stamps_nt3.json"
BASE=abv/x3k_r4c/libdmip.so
for r in 1 2; do
  timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/c5_new_$r.json" 2>/dev/null || exit 3
  DMIP_LIB=$BASE timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/c5_base_$r.json" 2>/dev/null || exit 3
  echo "c5 new  $(tail -1 $OUT/c5_new_$r.json)"; echo "c5 base $(tail -1 $OUT/c5_base_$r.json)"
done
P=(python scripts/bench_config5.py --steps 5)
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/pmc_2" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p2.log" 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc_1" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p1.log" 2>&1 || exit 3
timeout -k 10 600 python -u bench.py --steps 10 --warmup 3 > "$OUT/bench.log" 2>&1 || { tail -5 "$OUT/bench.log"; exit 3; }
tail -1 "$OUT/bench.log" | cut -c1-400
echo done
