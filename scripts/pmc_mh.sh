#!/bin/bash
# PMC passes of the multi-tile fp32x3 MH kernel (mh_x3_mt_kernel): issue, waits, MFMA busy,
# LDS, VMEM; 10 rows x 30k chains x 200 steps so each pass takes seconds
set -u
TAG=${1:-pmc_mh}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
P=(python scripts/bench_surrogate.py --no-cpu --steps 200 --reps 1 --eval-n 65536)
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc_1" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p1.log" 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS -d "$OUT/pmc_2" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p2.log" 2>&1 || exit 3
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d "$OUT/pmc_3" -o pmc --output-format csv -- "${P[@]}" > "$OUT/p3.log" 2>&1 || exit 3
python scripts/pmc_summary.py "$TAG" mh_x3_mt_kernel --json "$OUT/summary.json"
