#!/bin/bash
# Round-6 A/B of the config-5 record stores' cache policy (abv/c5aux<a>: -DDMIP_TRAIN_REC_AUX=a) against the product
# library: rocprofv3 kernel stats of scripts/bench_config5.py, alternating, two rounds; prints both halves' averages.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/c5aux; mkdir -p $OUT
for r in 1 2; do
  for v in prod "$@"; do
    L=""; [ $v != prod ] && L="DMIP_LIB=abv/$v/libdmip.so DMIP_LIB_AB=1"
    env $L timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $OUT/${v}_$r -o run --output-format csv -- \
      python scripts/bench_config5.py --steps 50 > $OUT/${v}_$r.log 2>&1 || exit 1
    f=$(find $OUT/${v}_$r -name "*kernel_stats.csv" | head -1)
    python - "$f" "$v" "$r" <<'PY'
import csv, sys
st = {r[0]: float(r[3]) / 1e3 for r in csv.reader(open(sys.argv[1])) if r[0].startswith('"') or 'loss_grad' in r[0]}
fw = [v for k, v in st.items() if "loss_grad_kernel<3, 1>" in k]
rv = [v for k, v in st.items() if "loss_grad_kernel<3, 3>" in k]
print(sys.argv[2], sys.argv[3], "forward %.1f us" % fw[0], "reverse %.1f us" % rv[0], flush=True)
PY
  done
done
