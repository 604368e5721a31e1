#!/bin/bash
# Round-6 evidence pass on one GPU: the headline kernel's PMC (x3k_sampler_kernel), both config-5 kernels' PMC,
# and the width-512 one-tile engine (x3_sampler_kernel<CDE,512> / <POSTERIOR,512>): PMC plus the timing
# ablations of the diagnostic library (DMIP_X3_DIAG: 1 no ring, 2 no hidden activations, 4 no layer-1
# activation). Every GPU step has its own time limit; a failure ends the script.
#   usage: bash scripts/gpu_r6_evidence.sh [tag]
set -u
TAG=${1:-r6_evidence}
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
pmc3() {  # pmc3 <subdir> <cmd...>: three counter groups, one run each
  local sub=$1; shift
  step "${sub}_p1" 150 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/$sub/pmc_1" -o pmc --output-format csv -- "$@"
  step "${sub}_p2" 150 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM \
    SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/$sub/pmc_2" -o pmc --output-format csv -- "$@"
  step "${sub}_p3" 150 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE \
    -d "$OUT/$sub/pmc_3" -o pmc --output-format csv -- "$@"
}
step bench_headline 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-other-configs --no-fast --no-fp32
pmc3 x3k python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --no-fast --no-fp32
step c5_time 200 python -u scripts/bench_config5.py --steps 50
pmc3 c5 python scripts/bench_config5.py --steps 5
step w512_time 400 python -u scripts/bench_x3_rows.py --rows cde512,post512 --reps 2
pmc3 cde512 python scripts/bench_x3_rows.py --rows cde512 --reps 1 --steps 200
pmc3 post512 python scripts/bench_x3_rows.py --rows post512 --reps 1 --steps 200
for d in 0 1 2 4 6 7; do
  DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=$d step "diag512_$d" 200 python -u scripts/bench_x3_rows.py --rows cde512 --reps 2
done
for s in x3k:x3k_sampler_kernel c5:"loss_grad_kernel<3, 1>" c5:"loss_grad_kernel<3, 2>" cde512:x3_sampler_kernel post512:x3_sampler_kernel; do
  sub=${s%%:*}; k=${s#*:}
  echo "### $sub $k"; python scripts/pmc_summary.py "$TAG/$sub" "$k"
done > "$OUT/summaries.txt" 2>&1
echo done | tee -a "$OUT/steps.log"
