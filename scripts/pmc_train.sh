# PMC passes of the fused bf16 training kernel (config 5), one counter group per rocprofv3 run.
#   bash scripts/pmc_train.sh <tag>   -> gpurun_out/<tag>/pmc*/
set -e
TAG=${1:-pmc_train}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "loss_grad or train" > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u scripts/bench_train.py --no-cpu --steps 20 > $OUT/bench_train.json 2> $OUT/bench_train.err
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python scripts/bench_train.py --no-cpu --steps 5 > $OUT/trace.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS -d $OUT/pmc1 -o run --output-format csv -- python scripts/bench_train.py --no-cpu --steps 3 > $OUT/pmc1.log 2>&1
