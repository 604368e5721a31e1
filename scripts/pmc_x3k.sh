#!/bin/bash
# PMC passes of the headline fp32x3 kernel (x3k_sampler_kernel): issue, waits, MFMA busy, LDS
set -u
TAG=${1:-pmc_x3k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P=(python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --no-fast --no-fp32)
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc_1" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p1.log" 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/pmc_2" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p2.log" 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/pmc_3" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p3.log" 2>&1 || exit 3
python scripts/pmc_summary.py "$TAG" x3k_sampler_kernel --json "$OUT/summary.json"
