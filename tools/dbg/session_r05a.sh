set -u
export TMPDIR=/tmp PYTHONPATH=.
bash tools/profile_c5_all.sh > gpurun_out/r05_pmc_all.log 2>&1; echo "pmc rc=$?"; tail -6 gpurun_out/r05_pmc_all.log
bash tools/ab_multi.sh tools/cmp_c5.py 2 nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_large_zearly.so > gpurun_out/r05_ab_zearly.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05_ab_zearly.log
for L in nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_sg1.so nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_sg1.so; do
  WCSDE_LIB_OVERRIDE=$PWD/$L timeout -k 10 200 python bench.py --precision f64 --steps 1 --warmup 1 --sde-only --no-cpu-baseline > gpurun_out/f64b.log 2>&1 || { echo "f64 bench failed $L"; tail -5 gpurun_out/f64b.log; exit 1; }
  echo "$L: $(python -c "import json;d=json.loads([l for l in open('gpurun_out/f64b.log') if l.startswith('{')][0]);print(d['kernel_ms'], d['value'])")"
done
timeout -k 10 600 python -u -m pytest tests/test_sde_gpu.py tests/test_fullsize_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r05_sde_tests.log 2>&1; echo "sde tests rc=$?"; tail -3 gpurun_out/r05_sde_tests.log
