#!/bin/bash
# A Welch variant build (tools/dbg/libwelch_<name>.so, tools/dbg/welch_variants.sh) against the
# product: bit-compare the PSD/peaks on a seeded ring and time the C3 segment, interleaved twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
V=$1
OUT=gpurun_out/wv; mkdir -p $OUT
for r in 1 2; do
  for v in product $V; do
    L=$PWD/nremmodfc_amd/libwcsde.so; [ $v != product ] && L=$PWD/tools/dbg/libwelch_$v.so
    WCSDE_LIB_OVERRIDE=$L timeout -k 10 120 python -u tools/cmp_welch.py save $OUT/$v.npz > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
    echo "$v: $(grep ms $OUT/$v.log)"
  done
done
python tools/cmp_welch.py cmp $OUT/product.npz $OUT/$V.npz
