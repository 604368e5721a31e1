#!/bin/bash
# x3k with the fp16-range check on each segment's final state: tests (x3k, range, hand-over), same-box A/B
# against the round-3 build, FETCH/WRITE PMC passes of the headline
set -u
OUT=gpurun_out/${1:-r4rng}
BASE=${2:-abv/x3k_r3/libdmip.so}
mkdir -p "$OUT"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_x3k.py tests/test_gpu_x3.py tests/test_gpu_x3p.py -m gpu -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|Error|passed|failed" "$OUT/pytest.log" | tail -8
case $rc in 0) ;; *) exit 3 ;; esac
bash scripts/gpu_ab_libs.sh "${1:-r4rng}/ab" "$BASE" || exit 3
PB=(python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-other-configs --fast-steps 2 --fp32-steps 1)
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o pmc --output-format csv -- "${PB[@]}" > "$OUT/pf.log" 2>&1 || exit 3
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/pmc_write" -o pmc --output-format csv -- "${PB[@]}" > "$OUT/pw.log" 2>&1 || exit 3
python scripts/pmc_traffic.py "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json"
