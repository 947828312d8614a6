#!/bin/bash
# BOLD table through scalar loads: bit-compare + timing against the session-start build, the
# signal GPU tests, and the bench line of the new build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/p
mkdir -p $OUT
for v in base prod; do
  L=$PWD/tools/dbg/libwcsde_base.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/cmp_bold.py save $OUT/bold_$v.npz > $OUT/bold_$v.log 2>&1 || { tail -5 $OUT/bold_$v.log; exit 1; }
  echo "== bold $v"; grep -v amdgpu.ids $OUT/bold_$v.log
done
python tools/cmp_bold.py cmp $OUT/bold_base.npz $OUT/bold_prod.npz; echo "== cmp bold rc=$?"
rm -f $OUT/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_signal_gpu.py > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep -v amdgpu.ids $OUT/bench.log | cut -c1-300; grep -o '"kernel_ms": {[^}]*}' $OUT/bench.log
