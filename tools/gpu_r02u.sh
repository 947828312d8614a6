#!/bin/bash
# half-tile waves for five groups per CU (V_HALF): bit-compare + timing against the same build
# without it, then the integrator GPU tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/u
mkdir -p $OUT
for v in nohalf prod; do
  L=$PWD/tools/dbg/libwcsde_nohalf.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L CMP_TIME=1 timeout -k 10 300 python -u tools/cmp_libs.py save $OUT/sde_$v.npz > $OUT/sde_$v.log 2>&1 || { tail -5 $OUT/sde_$v.log; exit 1; }
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/time_shard.py 20000,16500,18000 > $OUT/shard_$v.log 2>&1 || { tail -5 $OUT/shard_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/sde_$v.log | grep "chunk\|N=90 B=20000"; grep -v amdgpu.ids $OUT/shard_$v.log
done
python tools/cmp_libs.py cmp $OUT/sde_nohalf.npz $OUT/sde_prod.npz > $OUT/cmp.log; echo "== cmp rc=$?"; grep -c identical $OUT/cmp.log; grep DIFFER $OUT/cmp.log | head
rm -f $OUT/*.npz
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sde_gpu.py tests/test_fullsize_gpu.py > $OUT/t.log 2>&1; rc=$?
tail -2 $OUT/t.log; exit $rc
