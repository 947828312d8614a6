#!/bin/bash
# Welch as two 1000-point halves (12 columns in flight per CU): the Welch GPU tests first, then
# PSD difference + timing against the session-start build, then the bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/r
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_signal_gpu.py -k "welch" > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for v in base prod; do
  L=$PWD/tools/dbg/libwcsde_base.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/cmp_welch.py save $OUT/welch_$v.npz > $OUT/welch_$v.log 2>&1 || { tail -5 $OUT/welch_$v.log; exit 1; }
  echo "== welch $v"; grep -v amdgpu.ids $OUT/welch_$v.log
done
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/r/welch_base.npz"), np.load("gpurun_out/r/welch_prod.npz")
d = np.abs(a["psd"] - b["psd"]) / np.abs(a["psd"]).max(axis=1, keepdims=True)
print("psd max rel diff (vs row max)", d.max(), "peaks equal", np.array_equal(a["peak"], b["peak"]))
PY
rm -f $OUT/*.npz
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_signal_gpu.py tests/test_stats_gpu.py > $OUT/t2.log 2>&1 || { tail -30 $OUT/t2.log; exit 1; }
tail -2 $OUT/t2.log
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
grep -o '"value": [0-9.e+]*' $OUT/bench.log; grep -o '"kernel_ms": {[^}]*}' $OUT/bench.log
