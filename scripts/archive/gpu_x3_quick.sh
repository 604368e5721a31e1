set -u
mkdir -p gpurun_out/x3a
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest tests/test_gpu_x3.py -x -v -s --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/x3a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "\[x3\]|PASS|FAIL|Error|error" gpurun_out/x3a/pytest.log | tail -60
case $rc in 0|1) ;; *) exit $rc ;; esac
for p in fp32x3 bf16; do
timeout -k 10 300 python bench.py --precision $p --steps 3 --warmup 1 --no-cpu-baseline --no-fp32 --no-other-configs > gpurun_out/x3a/bench_$p.log 2>&1 || exit 3
python -c "import json;d=json.loads(open('gpurun_out/x3a/bench_$p.log').read().strip().splitlines()[-1]);print('$p', d['value'], d['roofline']['launch_ms'], d['roofline']['frac'], d.get('parity'))"
done
