#!/bin/bash
# round-2 iteration b: tightened tolerances, bench contract, full-size invariance with the 6-wave
# small-batch kernel, small-batch variant timings, shard rates, fp32 FC SSIM over the full schedule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT -s tests/test_sde_gpu.py tests/test_sde_large_gpu.py tests/test_fullsize_gpu.py tests/test_bench.py > gpurun_out/t_b.log 2>&1; rc=$?
grep -E "TOL|passed|failed|Error" gpurun_out/t_b.log | tail -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/time_small.py 27,31,32,35 > gpurun_out/small.log 2>&1; rc=$?
cat gpurun_out/small.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
PYTHONPATH=. timeout -k 10 200 python -u tools/time_shard.py 20000,10000,5000,2500,1250 > gpurun_out/shard.log 2>&1; rc=$?
cat gpurun_out/shard.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 python -u tools/fc_ssim_f32.py 32 > gpurun_out/fcssim.log 2>&1; rc=$?
tail -3 gpurun_out/fcssim.log; exit $rc
