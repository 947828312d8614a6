set -u
export TMPDIR=/tmp PYTHONPATH=.
timeout -k 10 400 python -u -m pytest tests/test_sde_large_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r05_p4_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r05_p4_tests.log
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
bash tools/ab_multi.sh tools/cmp_c5.py 2 nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_large_w8.so > gpurun_out/r05_ab_p4.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05_ab_p4.log
python tools/cmp_c5.py cmp gpurun_out/abm/libwcsde.npz gpurun_out/abm/libwc_sde_large_w8.npz
WCSDE_LIB_OVERRIDE=nremmodfc_amd/libwcsde_diag.so timeout -k 10 200 python tools/time_c5.py --steps 4000 --reps 1 WCSDE_PERSISTENT=1 WCSDE_PERSISTENT=3 WCSDE_PERSISTENT=4 WCSDE_PERSISTENT=5 > gpurun_out/r05_p4_abl.log 2>&1; echo "abl rc=$?"; cat gpurun_out/r05_p4_abl.log
rm -f gpurun_out/abm/*.npz
for L in nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_pregs0.so nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_pregs0.so; do
  WCSDE_LIB_OVERRIDE=$PWD/$L timeout -k 10 200 python bench.py --precision f64 --steps 1 --warmup 1 --sde-only --no-cpu-baseline > gpurun_out/f64b.log 2>&1 || { echo "f64 bench failed $L"; tail -5 gpurun_out/f64b.log; exit 1; }
  echo "$L: $(python -c "import json;d=json.loads([l for l in open('gpurun_out/f64b.log') if l.startswith('{')][0]);print(d['kernel_ms'], d['value'])")"
done
timeout -k 10 600 python -u -m pytest tests/test_sde_gpu.py -x -q -k "f64 or replay" --timeout 300 --timeout-method thread > gpurun_out/r05_f64_tests.log 2>&1; echo "f64 tests rc=$?"; tail -3 gpurun_out/r05_f64_tests.log
