#!/bin/bash
# A C5 persistent-kernel variant build (tools/dbg/libwc_sde_large_<name>.so) against the product:
# bit comparison and µs per step at the C5 shard, interleaved twice (tools/cmp_c5.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
V=$1
OUT=gpurun_out/c5v; mkdir -p $OUT
for r in 1 2; do
  for v in product $V; do
    L=$PWD/nremmodfc_amd/libwcsde.so; [ $v != product ] && L=$PWD/tools/dbg/libwc_sde_large_$v.so
    WCSDE_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/cmp_c5.py save /tmp/c5v_$v.npz > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
    echo "$v: $(grep us/step $OUT/$v.log)"
  done
done
python tools/cmp_c5.py cmp /tmp/c5v_product.npz /tmp/c5v_$V.npz
