# fp64 integrator: tail launch, normals-first variants and ablations (A/B, one box), then parity tests
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
f64() {
  WCSDE_LIB_OVERRIDE=$PWD/$1 timeout -k 10 200 python bench.py --precision f64 --steps 1 --warmup 1 --sde-only --no-cpu-baseline > gpurun_out/f64b.log 2>&1 || { echo "f64 bench failed $1"; tail -5 gpurun_out/f64b.log; return 1; }
  echo "$1: $(python -c "import json;d=json.loads([l for l in open('gpurun_out/f64b.log') if l.startswith('{')][0]);print(d['kernel_ms'])")"
}
for r in 1 2; do
  for L in nremmodfc_amd/libwcsde.so tools/dbg/libwc_sde_notail.so tools/dbg/libwc_sde_z1.so tools/dbg/libwc_sde_z2.so tools/dbg/libwc_sde_nomfma.so tools/dbg/libwc_sde_norng.so; do
    f64 $L || exit 1
  done
done 2>&1 | tee gpurun_out/r05d_f64.log
timeout -k 10 600 python -u -m pytest tests/test_f64m_gpu.py tests/test_sde_gpu.py tests/test_sde_large_gpu.py -x -q -s --timeout 300 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1; echo "tests rc=$?"; grep TOL gpurun_out/r05d_tests.log; tail -2 gpurun_out/r05d_tests.log
