#!/bin/bash
# The three width-512 x3 CDE tests on the in-tree library and two A/B variants (DMIP_LIB).
set -u
OUT=gpurun_out/r6_x3dbg
mkdir -p $OUT
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
K='test_x3_cde_sampler_vs_oracle and 512 or test_x3_balanced_schedule_matches_unsplit_runs'
for L in prod abv/noimm/libdmip.so abv/nohoist/libdmip.so; do
  E=""; [ $L != prod ] && E="DMIP_LIB=$L"
  env $E timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -rf \
    tests/test_gpu_x3.py -k "$K" > "$OUT/$(basename $(dirname $L))_$(basename $L).log" 2>&1
  rc=$?; echo "$L rc=$rc: $(tail -1 $OUT/$(basename $(dirname $L))_$(basename $L).log)"
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
