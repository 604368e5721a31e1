#!/bin/bash
# k-major fp32x3 engine: GPU tests (x3k + x3 + corrector), then a same-box A/B of the engines.
set -u
TAG=${1:-x3k}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3k.py tests/test_gpu_x3.py tests/test_gpu_parity.py tests/test_gpu_f32.py \
  -m gpu -k "x3 or corrector" -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed|\[x3k\]" "$OUT/pytest.log" | tail -30
case $rc in 0|1) ;; *) exit $rc ;; esac
B=(python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-fp32 --no-fast --no-other-configs)
run() {  # run <name> <env...>
  local n=$1; shift
  env "$@" timeout -k 10 300 "${B[@]}" > "$OUT/bench_$n.log" 2>&1 || { echo "bench $n failed"; tail -5 "$OUT/bench_$n.log"; exit 3; }
  python -c "import json;d=json.loads(open('$OUT/bench_$n.log').read().strip().splitlines()[-1]);print('$n', round(d['value']), round(d['roofline']['launch_ms'],2), 'ms', d.get('parity'))"
}
run nt3 DMIP_X3K_NT=3
run nt2 DMIP_X3K_NT=2
run onetile DMIP_X3K=0
run nt3_noring DMIP_X3K_NT=3 DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=1
run nt2_noring DMIP_X3K_NT=2 DMIP_LIB=abv/diag/libdmip_diag.so DMIP_X3_DIAG=1
timeout -k 10 200 python scripts/bench_config5.py > "$OUT/config5.json" 2>&1 || { echo "config5 failed"; tail -5 "$OUT/config5.json"; exit 3; }
tail -1 "$OUT/config5.json"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "loss_grad or config5 or train_epoch" -v -s --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest_train.log" 2>&1
rc=$?; echo "pytest train rc=$rc"; grep -E "FAILED|passed|failed|G5|ragged|config5" "$OUT/pytest_train.log" | tail -40
