#!/bin/bash
# noise-server wave for five-group workgroups (V_NSRV): bit-compare against the same build without it
# (tools/dbg/libwcsde_nonsrv.so), shard rates, the SDE GPU tests, and the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/ns
mkdir -p $OUT
for v in nonsrv prod; do
  L=$PWD/tools/dbg/libwcsde_nonsrv.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/cmp_libs.py save $OUT/sde_$v.npz > $OUT/sde_$v.log 2>&1 || { tail -5 $OUT/sde_$v.log; exit 1; }
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/time_shard.py 20000,16000 > $OUT/shard_$v.log 2>&1 || { tail -5 $OUT/shard_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/sde_$v.log | grep "N=90"; grep -v amdgpu.ids $OUT/shard_$v.log
done
python tools/cmp_libs.py cmp $OUT/sde_nonsrv.npz $OUT/sde_prod.npz; echo "== cmp rc=$?"
rm -f $OUT/*.npz
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sde_gpu.py > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep -v amdgpu.ids $OUT/bench.log | cut -c1-200; grep -o '"kernel_ms": {[^}]*}' $OUT/bench.log
