#!/bin/bash
# round-4 closing run: full validation (tests, smoke, bench, rocprof, traffic PMC), the linear fixture control,
# x3k phase stamps, and the headline's issue/MFMA PMC passes
set -u
bash scripts/gpu_round.sh r4c || exit 3
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/e2e
timeout -k 10 300 python -u scripts/bench_linear_e2e.py --fixture > gpurun_out/e2e/linear_fixture.json 2> gpurun_out/e2e/linear_fixture.err \
  || { tail -5 gpurun_out/e2e/linear_fixture.err; exit 3; }
tail -1 gpurun_out/e2e/linear_fixture.json
bash scripts/gpu_x3k_stamps.sh r4c_x3k_stamps || exit 3
bash scripts/pmc_x3k.sh r4c_pmc_x3k > gpurun_out/r4c_pmc_x3k.txt 2>&1 || { tail -5 gpurun_out/r4c_pmc_x3k.txt; exit 3; }
tail -25 gpurun_out/r4c_pmc_x3k.txt
