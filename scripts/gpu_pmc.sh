#!/bin/bash
# PMC counter passes for the sampler (one rocprofv3 call per pass, --kernel-trace only beside
# --pmc; no sys/runtime tracing). Outputs under gpurun_out/<tag>/pmc_<n>/.
#   usage: bash scripts/gpu_pmc.sh [tag] [extra bench args...]
set -u
TAG=${1:-pmc}
shift || true
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH=(python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@")

rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true

run_pass() {  # run_pass <n> <counters...>
  local n=$1
  shift
  echo "=== pass $n: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/pmc_$n" -o pmc --output-format csv -- "${BENCH[@]}" \
    > "$OUT/pmc_$n.log" 2>&1
  local rc=$?
  echo "=== pass $n rc=$rc" | tee -a "$OUT/steps.log"
  case $rc in
    0|1) return 0 ;;
    *) echo "fatal rc=$rc: stopping" | tee -a "$OUT/steps.log"; exit $rc ;;
  esac
}

run_pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
run_pass 2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT
run_pass 3 FETCH_SIZE
run_pass 4 WRITE_SIZE
run_pass 5 SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_SMEM
echo done | tee -a "$OUT/steps.log"
