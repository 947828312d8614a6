set -u
export TMPDIR=/tmp PYTHONPATH=.
bash tools/ab_multi.sh tools/cmp_c5.py 2 tools/dbg/libwc_base_r05c.so nremmodfc_amd/libwcsde.so > gpurun_out/r05_ab_stage.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05_ab_stage.log
python tools/cmp_c5.py cmp gpurun_out/abm/libwc_base_r05c.npz gpurun_out/abm/libwcsde.npz
rm -f gpurun_out/abm/*.npz
for L in tools/dbg/libwc_base_r05c.so nremmodfc_amd/libwcsde.so tools/dbg/libwc_base_r05c.so nremmodfc_amd/libwcsde.so; do
  WCSDE_LIB_OVERRIDE=$PWD/$L timeout -k 10 200 python bench.py --precision f64 --steps 1 --warmup 1 --sde-only --no-cpu-baseline > gpurun_out/f64b.log 2>&1 || { echo "f64 bench failed $L"; tail -5 gpurun_out/f64b.log; exit 1; }
  echo "$L: $(python -c "import json;d=json.loads([l for l in open('gpurun_out/f64b.log') if l.startswith('{')][0]);print(d['kernel_ms'], d['value'])")"
done
timeout -k 10 600 python -u -m pytest tests/test_sde_large_gpu.py tests/test_f64m_gpu.py tests/test_sde_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r05_c_tests.log 2>&1; echo "tests rc=$?"; grep TOL gpurun_out/r05_c_tests.log; tail -2 gpurun_out/r05_c_tests.log
