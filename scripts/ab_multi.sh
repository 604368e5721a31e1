# Same-box A/B of the in-tree libdmip.so against several other builds (DMIP_LIB), alternating
# processes round by round: bash scripts/ab_multi.sh <a.so> <b.so> ...   -> gpurun_out/abm/<tag>_<round>.json
set -e
mkdir -p gpurun_out/abm
for r in 1 2 3; do
  timeout -k 10 200 python -u scripts/sweep.py --variants 0 --chains 65536 100000 --rounds 2 > gpurun_out/abm/intree_$r.json 2>/dev/null
  for lib in "$@"; do
    tag=$(basename "$lib" .so)
    DMIP_LIB=$lib timeout -k 10 200 python -u scripts/sweep.py --variants 0 --chains 65536 100000 --rounds 2 > gpurun_out/abm/${tag}_$r.json 2>/dev/null
  done
done
