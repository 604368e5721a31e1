#!/bin/bash
# PMC passes of the config-5 split training kernels (forward / reverse halves), one counter group per run
set -u
OUT=gpurun_out/${1:-pmc_split}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P=(python scripts/bench_config5.py --steps 5)
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc_1" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p1.log" 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/pmc_2" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p2.log" 2>&1 || exit 3
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/pmc_3" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p3.log" 2>&1 || exit 3
for k in "loss_grad_kernel<3, 1>" "loss_grad_kernel<3, 2>" "loss_grad_kernel<3, 3>"; do
  python scripts/pmc_summary.py "${1:-pmc_split}" "$k" --json "$OUT/summary_${k//[^0-9]/}.json"
done
