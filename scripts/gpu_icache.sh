#!/bin/bash
# instruction-cache counters of the fp32x3 sampler kernels (x3k NT = 3 / 2 and the one-tile engine)
set -u
OUT=gpurun_out/${1:-icache}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
B=(python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
for v in nt3:DMIP_X3K_NT=3 nt2:DMIP_X3K_NT=2 onetile:DMIP_X3K=0; do
  n=${v%%:*}
  env ${v#*:} timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_IFETCH GRBM_GUI_ACTIVE \
    -d "$OUT/$n" -o pmc --output-format csv -- "${B[@]}" > "$OUT/$n.log" 2>&1
  rc=$?; echo "$n rc=$rc"; case $rc in 0|1) ;; *) exit $rc ;; esac
  python scripts/pmc_summary.py "${1:-icache}/$n" "sampler_kernel" 2>&1 | grep -E "SQC|IFETCH|dispatch|clock" 
done
