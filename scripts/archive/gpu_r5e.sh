#!/bin/bash
# round 5: DPS fp32x3 engine (surrogate/DPS tests, config-4 timing both engines, rocprof), then the config-5 step
set -u
OUT=gpurun_out/${1:-r5e}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_surrogate.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider -rf -s > "$OUT/pytest_sur.log" 2>&1
rc=$?; echo "pytest sur rc=$rc"; grep -E "FAILED|passed|failed|\[dps\]" "$OUT/pytest_sur.log" | tail -14
case $rc in 0|1) ;; *) exit 3 ;; esac
for p in fp32x3 fp32; do
  timeout -k 10 300 python -u scripts/bench_dps.py --precision $p --reps 2 > "$OUT/dps_$p.json" 2> "$OUT/dps_$p.err" || exit 3
  python -c "import json,sys; d=json.loads(open('$OUT/dps_$p.json').read().strip().splitlines()[-1]); print('$p', d['ms_per_call'], d['rank0_launch_ms'], d['quality']['KL2_vs_mcmc'], d['quality']['KL2_mcmc_vs_mcmc'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$OUT/prof_dps" -o run --output-format csv -- \
  python scripts/bench_dps.py --precision fp32x3 --reps 1 --gt-chains 2000 > "$OUT/prof_dps.log" 2>&1 || exit 3
find "$OUT/prof_dps" -name "*kernel_stats*" -exec cp {} "$OUT/dps_kernel_stats.csv" \;
cut -d, -f1-4 "$OUT/dps_kernel_stats.csv" | head -8 | cut -c1-150
bash scripts/gpu_r5d.sh "${1:-r5e}/c5"
