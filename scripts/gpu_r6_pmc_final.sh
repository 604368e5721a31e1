#!/bin/bash
# Round-6 closing PMC: the DPS kernel (dps_x3_kernel) and both config-5 kernels on the final tree, three counter
# groups each (one rocprofv3 run per group). Every GPU step has its own time limit; a failure ends the script.
#   usage: bash scripts/gpu_r6_pmc_final.sh [tag]
set -u
TAG=${1:-r6_pmc_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # step <name> <seconds> <cmd...>
  local name=$1 secs=$2
  shift 2
  echo "=== $name ($(date +%T))" | tee -a "$OUT/steps.log"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -2 "$OUT/$name.log"
  case $rc in 0) return 0 ;; *) echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc ;; esac
}
pmc3() {  # pmc3 <subdir> <cmd...>
  local sub=$1; shift
  step "${sub}_p1" 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/$sub/pmc_1" -o pmc --output-format csv -- "$@"
  step "${sub}_p2" 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM \
    SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/$sub/pmc_2" -o pmc --output-format csv -- "$@"
  step "${sub}_p3" 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
    -d "$OUT/$sub/pmc_3" -o pmc --output-format csv -- "$@"
}
pmc3 dps python scripts/bench_dps.py --samples 65536 --steps 200 --reps 1 --gt-chains 0
pmc3 c5 python scripts/bench_config5.py --steps 5
for s in dps:dps_x3_kernel c5:"loss_grad_kernel<3, 1>" c5:"loss_grad_kernel<3, 3>"; do
  sub=${s%%:*}; k=${s#*:}
  echo "### $sub $k"; python scripts/pmc_summary.py "$TAG/$sub" "$k"
done > "$OUT/summaries.txt" 2>&1
echo done | tee -a "$OUT/steps.log"
