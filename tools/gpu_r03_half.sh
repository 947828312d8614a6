#!/bin/bash
# The half-tile normals-block kernel (tools/dbg/libwc_sde_half.so, V_HALF2) against the product at
# the small strong-scaling shards: rates and bit-identity with the plain kernel (tools/time_shard.py),
# then the precomputed-normals tests on the variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/half; mkdir -p $OUT
for v in product half product half; do
  L=$PWD/nremmodfc_amd/libwcsde.so; [ $v != product ] && L=$PWD/tools/dbg/libwc_sde_$v.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/time_shard.py ${SHARDS:-2500,1250,3500} > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  echo "== $v"; grep us/step $OUT/$v.log
done
WCSDE_LIB_OVERRIDE=$PWD/tools/dbg/libwc_sde_half.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_sde_gpu.py -k "precomputed or small" > $OUT/t.log 2>&1; echo "tests rc=$?"; tail -2 $OUT/t.log
