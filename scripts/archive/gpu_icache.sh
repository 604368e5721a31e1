#!/bin/bash
# instruction-cache counters of the fp32x3 sampler kernels (paired x3p, k-major x3k) and the 16-bit engine
set -u
TAG=${1:-icache}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
for v in x3p:DMIP_X3P=1:fp32x3 x3k:DMIP_X3P=0:fp32x3 bf16:DMIP_X3P=0:bf16; do
  n=${v%%:*}; r=${v#*:}; e=${r%%:*}; prec=${r#*:}
  for pass in a b; do
    if [ $pass = a ]; then C="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE GRBM_GUI_ACTIVE"
    else C="SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES"; fi
    env $e timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C -d "$OUT/$n/pmc_$pass" -o pmc --output-format csv -- \
      python bench.py --steps 2 --warmup 1 --precision $prec --no-cpu-baseline --no-fp32 --no-fast --no-other-configs \
      > "$OUT/$n.$pass.log" 2>&1
    rc=$?; echo "$n $pass rc=$rc"; case $rc in 0|1) ;; *) exit $rc ;; esac
  done
  python scripts/pmc_summary.py "$TAG/$n" "sampler_kernel" 2>&1 | grep -E "SQC|IFETCH|WAVE_CYCLES|WAIT_INST|BUSY|dispatch|clock"
done
