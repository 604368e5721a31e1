# A/B timing of the in-tree libdmip.so against another build (DMIP_LIB) on one box, alternating
# processes: bash scripts/ab_lib.sh <other.so> [variants...]
set -e
OTHER=$1; shift
V=${@:-0}
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  DMIP_LIB=$OTHER timeout -k 10 200 python -u scripts/sweep.py --variants $V --chains 65536 100000 --rounds 2 > gpurun_out/ab/other_$r.json 2>/dev/null
  timeout -k 10 200 python -u scripts/sweep.py --variants $V --chains 65536 100000 --rounds 2 > gpurun_out/ab/new_$r.json 2>/dev/null
done
