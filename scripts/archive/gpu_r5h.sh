#!/bin/bash
# round 5: the SiLU chain (new tests) + the exact-f32 engine's tests (the ACT template) + the surrogate/DPS tests
set -u
OUT=gpurun_out/${1:-r5h}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_silu.py tests/test_gpu_f32.py tests/test_gpu_surrogate.py -m gpu -v \
  --timeout 300 --timeout-method thread -p no:cacheprovider -rf > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|passed|failed" "$OUT/pytest.log" | tail -14
