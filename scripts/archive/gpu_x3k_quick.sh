#!/bin/bash
# k-major fp32x3 engine: its GPU tests, then a same-box timing of NT = 3 / 2 and the one-tile engine.
set -u
TAG=${1:-x3kq}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_x3k.py -m gpu -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -8
case $rc in 0|1) ;; *) exit $rc ;; esac
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -k 10 300 "${B[@]}" > "$OUT/bench_$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$OUT/bench_$n.log"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/bench_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms', d.get('parity'))"
}
for v in ${VARIANTS:-nt3:DMIP_X3K_NT=3 nt2:DMIP_X3K_NT=2 onetile:DMIP_X3K=0}; do
  run "${v%%:*}" ${v#*:}
done
