#!/bin/bash
# 32x32-tile fp32x3 engine: its GPU tests (+ the x3k / x3 fp32x3 tests), then a same-box A/B of the engines
set -u
TAG=${1:-x3w}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3w.py tests/test_gpu_x3k.py tests/test_gpu_x3.py -m gpu -v -s -x \
  --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed|\[x3w\]" "$OUT/pytest.log" | tail -30
case $rc in 0) ;; *) exit 3 ;; esac
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -k 10 300 "${B[@]}" > "$OUT/bench_$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$OUT/bench_$n.log"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/bench_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms', d.get('parity'))"
}
run x3w DMIP_X3W=1
run x3k DMIP_X3W=0
run x3w2 DMIP_X3W=1
run x3k2 DMIP_X3W=0
