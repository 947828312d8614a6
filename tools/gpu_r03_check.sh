set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sde_gpu.py tests/test_hma_gpu.py tests/test_facades_gpu.py tests/test_sde_large_gpu.py tests/test_large_n_gpu.py "tests/test_sweep.py::test_many_seeds_main_n1000_short" -q -rA -s --timeout 300 --timeout-method thread > gpurun_out/g2_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "TOL|passed|failed|Error" gpurun_out/g2_pytest.log | tail -40
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/g2_c5.log 2>&1; echo "c5 rc=$?"; tail -c 1500 gpurun_out/g2_c5.log
