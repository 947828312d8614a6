# fp64 Welch: the wave-per-column kernel -- tests first, then timing against the LDS-Stockham kernel
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_signal_gpu.py -x -q -s -k "welch" --timeout 120 --timeout-method thread > gpurun_out/r05h_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "TOL|passed|failed|Error" gpurun_out/r05h_tests.log | tail -12; [ $rc -eq 0 ] || exit 1
for r in 1 2; do
  for L in nremmodfc_amd/libwcsde.so tools/dbg/libwelch_twtab.so; do
    echo "$L: $(WCSDE_LIB_OVERRIDE=$PWD/$L timeout -k 10 120 python tools/time_welch64.py 20000 2>&1 | grep ms)" || exit 1
  done
done | tee gpurun_out/r05h_w64.log
