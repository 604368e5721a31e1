export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 100 python -u scripts/probe_config1.py > gpurun_out/t8k_base_$r.log 2>&1 || exit 1
  DMIP_LIB=abv/x3s8k/libdmip.so DMIP_LIB_AB=1 timeout -k 10 100 python -u scripts/probe_config1.py > gpurun_out/t8k_new_$r.log 2>&1 || exit 2
done
for f in gpurun_out/t8k_*.log; do echo "$f $(tail -1 $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["chains_at_200"])')"; done
