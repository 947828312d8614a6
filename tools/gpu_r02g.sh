#!/bin/bash
# persistent kernel as the C5 default: N > 96 suites, C5 bench + kernel stats, C5 PMC
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c5k
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 600 $PT tests/test_sde_large_gpu.py tests/test_large_n_gpu.py > gpurun_out/t_g.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed|assert" gpurun_out/t_g.log | tail -30; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5k -o k -- python3 bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/prof_c5k/bench.log 2>&1; rc=$?
tail -1 gpurun_out/prof_c5k/bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 bash tools/profile_c5.sh > gpurun_out/pc5.log 2>&1; rc=$?
tail -3 gpurun_out/pc5.log; exit $rc
