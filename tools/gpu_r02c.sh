#!/bin/bash
# round-2 iteration c: BOLD kernel with fewer fp64 operations (signal tests, statistics vs the
# shipped tables, timing), config-2 full-size run, fp32 FC SSIM over the full schedule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $PT -s tests/test_signal_gpu.py tests/test_facades_gpu.py tests/test_large_n_gpu.py tests/test_stats_gpu.py tests/test_sweep.py > gpurun_out/t_c.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed|max \|z\||C2 full" gpurun_out/t_c.log | tail -70; [ $rc -ne 0 ] && exit $rc
PYTHONPATH=. timeout -k 10 200 python -u tools/time_bold.py 20000 > gpurun_out/tb.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tb.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u tools/fc_ssim_f32.py 32 > gpurun_out/fcssim.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/fcssim.log | tail -4; exit $rc
