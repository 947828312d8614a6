#!/bin/bash
# Welch ablation on the GPU box: the product kernel, without the next-column loads, and loads +
# stage 1 only (tools/dbg/welch_variants.sh builds the variants), each at C3's 20,000 x 90.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for v in product ${WELCH_VARIANTS:-noload nofft}; do
  L=$PWD/nremmodfc_amd/libwcsde.so; [ $v != product ] && L=$PWD/tools/dbg/libwelch_$v.so
  for r in 1 2; do
    WCSDE_LIB_OVERRIDE=$L timeout -k 10 120 python tools/time_welch.py 20000 > gpurun_out/wa_$v.log 2>&1 || { tail -5 gpurun_out/wa_$v.log; exit 1; }
    echo "$v: $(grep ms gpurun_out/wa_$v.log)"
  done
done
