#!/bin/bash
# Immediate-offset LDS-DMA pieces (x3k, x3, DPS) and the config-5 buffer-store records: the fp32x3 and training GPU
# tests, then the headline / width-512 rows / DPS / config-5 timings against the previous library (DMIP_LIB),
# alternating on one box.
#   usage: bash scripts/gpu_r6_imm.sh <tag> <previous.so>
set -u
TAG=$1; PREV=$2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf \
  tests/test_gpu_x3.py tests/test_gpu_x3k.py tests/test_gpu_surrogate.py tests/test_gpu_parity.py \
  tests/test_gpu_train_split.py tests/test_gpu_train_step.py > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest.log)"; case $rc in 0|1) ;; *) exit $rc ;; esac
B=(python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-other-configs --no-fast --no-fp32)
for r in 1 2; do
  for L in new $PREV; do
    n=new; E=""; [ $L != new ] && { n=prev; E="DMIP_LIB=$L"; }
    env $E timeout -k 10 200 "${B[@]}" > "$OUT/head_${n}_$r.log" 2>&1 || exit 3
    env $E timeout -k 10 300 python -u scripts/bench_x3_rows.py --rows cde512,post512 --reps 2 > "$OUT/rows_${n}_$r.log" 2>&1 || exit 3
    env $E timeout -k 10 200 python -u scripts/bench_dps.py --reps 2 --gt-chains 0 > "$OUT/dps_${n}_$r.log" 2>&1 || exit 3
    env $E timeout -k 10 120 python -u scripts/bench_config5.py --steps 50 > "$OUT/c5_${n}_$r.log" 2>&1 || exit 3
    echo "$n $r: head $(python -c "import json;d=json.loads(open('$OUT/head_${n}_$r.log').read().strip().splitlines()[-1]);print(round(d['roofline']['launch_ms'],2))") rows $(tail -1 $OUT/rows_${n}_$r.log) dps $(python -c "import json;d=json.loads(open('$OUT/dps_${n}_$r.log').read().strip().splitlines()[-1]);print(round(d['ms_per_call'],1))") c5 $(python -c "import json;d=json.loads(open('$OUT/c5_${n}_$r.log').read().strip().splitlines()[-1]);print(round(d['ms_device_step'],4))")"
  done
done
