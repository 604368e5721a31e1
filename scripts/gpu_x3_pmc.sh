#!/bin/bash
# x3 (fp32x3) sampler: timing ablations (DMIP_X3_DIAG) and PMC passes on the headline workload.
#   usage: bash scripts/gpu_x3_pmc.sh [tag]
set -u
TAG=${1:-x3pmc}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B=(python bench.py --precision fp32x3 --steps 3 --warmup 1 --no-cpu-baseline --no-fp32 --no-other-configs)
for d in 0 1 2 4 6 7; do
  DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=$d timeout -k 10 200 "${B[@]}" > "$OUT/diag_$d.log" 2>&1 || { echo "diag $d failed"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/diag_$d.log').read().strip().splitlines()[-1]);print('diag $d', round(d['roofline']['launch_ms'],2), 'ms')"
done
run_pass() {
  local n=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/pmc_$n" -o pmc --output-format csv -- "${B[@]}" > "$OUT/pmc_$n.log" 2>&1
  local rc=$?; echo "pass $n rc=$rc"
  case $rc in 0|1) return 0 ;; *) exit $rc ;; esac
}
run_pass 1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
run_pass 2 SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT
run_pass 3 SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_FLAT
python scripts/pmc_summary.py "$TAG" x3_sampler > "$OUT/summary.txt" 2>&1; cat "$OUT/summary.txt"
