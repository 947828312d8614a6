#!/bin/bash
# persistent C5 kernel: bit-exactness vs the step kernel, N > 96 suites, timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $PT tests/test_sde_large_gpu.py tests/test_large_n_gpu.py > gpurun_out/t_f.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed|assert" gpurun_out/t_f.log | tail -30; [ $rc -ne 0 ] && exit $rc
PYTHONPATH=. timeout -k 10 200 python -u tools/time_large.py 1000 2500,2048,1280 > gpurun_out/tl.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tl.log; [ $rc -ne 0 ] && exit $rc
WCSDE_PERSISTENT=0 PYTHONPATH=. timeout -k 10 200 python -u tools/time_large.py 1000 2500 > gpurun_out/tl0.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/tl0.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log | cut -c1-300; exit $rc
