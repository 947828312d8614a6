# kZK (steps per V_ZMEM/V_ZPAIR launch) A/B: 1000 (product) vs blocks small enough that the
# double-buffered normals stay in the 256 MB MALL.  time_shard also checks bit-identity vs WCSDE_ZMEM=0.
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/r06k
for r in 1 2; do
  for v in prod zk2000 zk4000; do
    if [ $v = prod ]; then unset WCSDE_LIB_OVERRIDE; else export WCSDE_LIB_OVERRIDE=$PWD/tools/dbg/libwc_sde_$v.so; fi
    timeout -k 10 200 python tools/time_shard.py 5000,4100,2500 > gpurun_out/r06k/$v$r.log 2>&1 || exit 1
    echo "$v: $(grep B= gpurun_out/r06k/$v$r.log | cut -d' ' -f1-3,13- | tr '\n' ' ')"
  done
done
