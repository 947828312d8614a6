#!/bin/bash
# Welch kernel change vs the HEAD build of wc_welch.hip (tools/dbg/libwcsde_welchhead.so): bit-compare + timing, the
# signal GPU tests, and the bench line of the new build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/wl
mkdir -p $OUT
for v in base prod; do
  L=$PWD/tools/dbg/libwcsde_welchhead.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/cmp_welch.py save $OUT/welch_$v.npz > $OUT/welch_$v.log 2>&1 || { tail -5 $OUT/welch_$v.log; exit 1; }
  echo "== welch $v"; grep -v amdgpu.ids $OUT/welch_$v.log
done
python tools/cmp_welch.py cmp $OUT/welch_base.npz $OUT/welch_prod.npz; echo "== cmp welch rc=$?"
rm -f $OUT/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_signal_gpu.py > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep -v amdgpu.ids $OUT/bench.log | cut -c1-300; grep -o '"kernel_ms": {[^}]*}' $OUT/bench.log
