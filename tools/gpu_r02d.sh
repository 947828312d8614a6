#!/bin/bash
# round-2 evidence d: the whole GPU suite, smoke, C3 bench, rocprof kernel trace + PMC passes,
# C5 bench + PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
grep -E "passed|failed|FAILED|Error|FC SSIM" gpurun_out/pytest_gpu.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
bash tools/profile_bench.sh > gpurun_out/pb.log 2>&1; rc=$?; tail -2 gpurun_out/pb.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
bash tools/profile_c5.sh > gpurun_out/pc5.log 2>&1; rc=$?; tail -1 gpurun_out/pc5.log | cut -c1-300; exit $rc
