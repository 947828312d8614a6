#!/bin/bash
# The two-waves-per-column Welch kernel (tools/dbg/libwelch_pair.so) against the product build:
# PSD/peak difference on a seeded ring, C3 segment time, and the Welch GPU tests on the variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/wp; mkdir -p $OUT
for v in product pair; do
  L=$PWD/nremmodfc_amd/libwcsde.so; [ $v != product ] && L=$PWD/tools/dbg/libwelch_$v.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 120 python -u tools/cmp_welch.py save $OUT/$v.npz > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  echo "$v: $(grep ms $OUT/$v.log)"
done
python tools/cmp_welch.py cmp $OUT/product.npz $OUT/pair.npz
python - <<'PY'
import numpy as np
a, b = np.load("gpurun_out/wp/product.npz"), np.load("gpurun_out/wp/pair.npz")
print("psd rel", np.abs(a["psd"] - b["psd"]).max() / np.abs(a["psd"]).max(), "peaks equal", np.array_equal(a["peak"], b["peak"]))
PY
WCSDE_LIB_OVERRIDE=$PWD/tools/dbg/libwelch_pair.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_signal_gpu.py -k welch > $OUT/t.log 2>&1; echo "tests rc=$?"; tail -3 $OUT/t.log
