#!/bin/bash
# paired-tile 32x32 fp32x3 engine: its GPU tests, the x3 default-path tests, then a same-box timing against the
# 16x16 k-major engine (DMIP_X3P=0), alternating
set -u
TAG=${1:-x3p}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3p.py -m gpu -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider > "$OUT/pytest_x3p.log" 2>&1
rc=$?; echo "pytest x3p rc=$rc"; grep -E "FAILED|Error|passed|failed|\[x3p\]" "$OUT/pytest_x3p.log" | tail -30
case $rc in 0|1) ;; *) exit $rc ;; esac
[ "${SKIP_X3:-0}" = 1 ] || {
timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py -m gpu -v -s --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "trajectory or parity or handover or balanced or shards or default or snapshots or exact_f32" \
  > "$OUT/pytest_x3.log" 2>&1
rc=$?; echo "pytest x3 rc=$rc"; grep -E "FAILED|Error|passed|failed|\[x3\]" "$OUT/pytest_x3.log" | tail -30
case $rc in 0|1) ;; *) exit $rc ;; esac
}
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -k 10 300 "${B[@]}" > "$OUT/bench_$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$OUT/bench_$n.log"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/bench_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms', d.get('parity'))"
}
for r in 1 2; do
  run "x3p_$r" DMIP_X3P=1
  run "x3k_$r" DMIP_X3P=0
done
