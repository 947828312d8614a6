#!/bin/bash
# round-2 iteration: new tests (N > 96 epilogue, drivers, ABI), observed fp32 tolerances,
# small-batch kernel variants, fp32 FC SSIM over the full schedule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_large_n_gpu.py tests/test_sweep.py tests/test_abi.py > gpurun_out/t_large.log 2>&1; rc=$?
tail -15 gpurun_out/t_large.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 $PT -s tests/test_sde_gpu.py tests/test_sde_large_gpu.py > gpurun_out/t_sde.log 2>&1; rc=$?
grep "TOL\|passed\|failed" gpurun_out/t_sde.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/time_small.py > gpurun_out/small.log 2>&1; rc=$?
cat gpurun_out/small.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/fc_ssim_f32.py 32 > gpurun_out/fcssim.log 2>&1; rc=$?
tail -3 gpurun_out/fcssim.log; exit $rc
