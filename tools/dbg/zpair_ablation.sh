# V_ZPAIR ablation (diag build): the generators idle (WCSDE_ZGEN_OFF=1, wrong results) vs the product
export TMPDIR=/tmp PYTHONPATH=. WCSDE_LIB_OVERRIDE=$PWD/nremmodfc_amd/libwcsde_diag.so
mkdir -p gpurun_out/r06j
for r in 1 2; do
  timeout -k 10 200 python tools/time_shard.py 5000,4100 > gpurun_out/r06j/prod$r.log 2>&1 || exit 1
  WCSDE_ZGEN_OFF=1 timeout -k 10 200 python tools/time_shard.py 5000,4100 > gpurun_out/r06j/genoff$r.log 2>&1 || exit 1
  echo "product: $(grep B= gpurun_out/r06j/prod$r.log | cut -c1-40 | tr '\n' ' ')"
  echo "gen off: $(grep B= gpurun_out/r06j/genoff$r.log | cut -c1-40 | tr '\n' ' ')"
done
