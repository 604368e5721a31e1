#!/bin/bash
# Round-4 measurements: fresh PMC of the config-5 forward/reverse kernels (verdict r3 item 4), then the
# reference's linear configuration trained to completion and evaluated (verdict r3 item 3).
#   usage: bash scripts/gpu_r4m.sh [pmc|linear|all]
set -u
PART=${1:-all}
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/e2e
if [ "$PART" = pmc ] || [ "$PART" = all ]; then
  timeout -k 10 200 python -u scripts/bench_config5.py --steps 20 > gpurun_out/c5_bench.json 2> gpurun_out/c5_bench.err \
    || { tail -5 gpurun_out/c5_bench.err; exit 3; }
  tail -1 gpurun_out/c5_bench.json
  bash scripts/pmc_train_split.sh r4_pmc_c5 > gpurun_out/r4_pmc_c5.txt 2>&1 || { tail -5 gpurun_out/r4_pmc_c5.txt; exit 3; }
  tail -4 gpurun_out/r4_pmc_c5.txt
fi
if [ "$PART" = linear ] || [ "$PART" = all ]; then
  timeout -k 10 900 python -u scripts/bench_linear_e2e.py > gpurun_out/e2e/linear.json 2> gpurun_out/e2e/linear.err \
    || { tail -5 gpurun_out/e2e/linear.err; exit 3; }
  tail -1 gpurun_out/e2e/linear.json
fi
if [ "$PART" = fixture ] || [ "$PART" = all ]; then
  bash scripts/gpu_e2e_ref.sh fixture || exit 3
fi
