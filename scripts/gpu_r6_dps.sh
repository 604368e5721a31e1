#!/bin/bash
# DPS (config 4): the DPS / MH GPU tests, then the in-tree library against A/B variant libraries (DMIP_LIB),
# alternating processes on one box (scripts/bench_dps.py, 262,144 chains x 1000 steps; KL2 vs a 30k-chain MH
# ground truth in the first pass only).
#   usage: [PYTEST_LIB=<variant.so>] bash scripts/gpu_r6_dps.sh <tag> <variant.so>...
# (PYTEST_LIB: the tests run on that library instead of the in-tree one)
set -u
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
env ${PYTEST_LIB:+DMIP_LIB=$PYTEST_LIB} timeout -k 10 600 python -u -m pytest -q --timeout 240 --timeout-method thread -p no:cacheprovider -rf -s \
  tests/test_gpu_surrogate.py -k "dps or mh" > "$OUT/pytest_dps.log" 2>&1
rc=$?; echo "pytest rc=$rc: $(tail -1 $OUT/pytest_dps.log)"; case $rc in 0|1) ;; *) exit $rc ;; esac
for r in 1 2; do
  G=0; [ $r = 1 ] && G=30000
  timeout -k 10 200 python -u scripts/bench_dps.py --reps 2 --gt-chains $G > "$OUT/new_$r.json" 2> "$OUT/new_$r.err" || exit 3
  echo "new $(python -c "import json;d=json.loads(open('$OUT/new_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_call'],1),'ms', (d.get('quality') or {}).get('KL2_vs_mcmc',''))")"
  for L in "$@"; do
    n=$(basename $(dirname $L))
    DMIP_LIB=$L timeout -k 10 200 python -u scripts/bench_dps.py --reps 2 --gt-chains 0 > "$OUT/${n}_$r.json" 2> "$OUT/${n}_$r.err" || exit 3
    echo "$n $(python -c "import json;d=json.loads(open('$OUT/${n}_$r.json').read().strip().splitlines()[-1]);print(round(d['ms_per_call'],1),'ms')")"
  done
done
