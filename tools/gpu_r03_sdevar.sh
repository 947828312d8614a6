#!/bin/bash
# An SDE variant build (tools/dbg/libwc_sde_<name>.so) against the product at the small strong-scaling
# shards (tools/time_shard.py; its bit-identity column compares each build's ZMEM path with its plain
# kernel), interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
V=$1
OUT=gpurun_out/sdev; mkdir -p $OUT
for r in 1 2; do
  for v in product $V; do
    L=$PWD/nremmodfc_amd/libwcsde.so; [ $v != product ] && L=$PWD/tools/dbg/libwc_sde_$v.so
    WCSDE_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/time_shard.py ${SHARDS:-2500,1250} > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
    echo "== $v"; grep us/step $OUT/$v.log
  done
done
