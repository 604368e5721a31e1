# second PMC pass group of the config-5 training kernel (dependency / LDS / memory waits)
set -e
OUT=gpurun_out/pmc_train2
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES -d $OUT/p1 -o run --output-format csv -- python scripts/bench_train.py --no-cpu --steps 3 > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $OUT/p2 -o run --output-format csv -- python scripts/bench_train.py --no-cpu --steps 3 > $OUT/p2.log 2>&1
