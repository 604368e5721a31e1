set -u
mkdir -p gpurun_out/r6_x3s
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 150 python -u scripts/probe_config1.py > gpurun_out/r6_x3s/probe_split.log 2>&1 || { echo probe rc=$?; tail -5 gpurun_out/r6_x3s/probe_split.log; exit 1; }
tail -1 gpurun_out/r6_x3s/probe_split.log
DMIP_X3_SPLIT=0 timeout -k 10 150 python -u scripts/probe_config1.py > gpurun_out/r6_x3s/probe_onetile.log 2>&1 || exit 2
tail -1 gpurun_out/r6_x3s/probe_onetile.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_x3.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -rf > gpurun_out/r6_x3s/pytest_x3.log 2>&1; rc=$?
tail -3 gpurun_out/r6_x3s/pytest_x3.log; exit $rc
