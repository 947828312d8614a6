#!/bin/bash
# C5 with two K chunks per barrier: bench line + rocprofv3 kernel stats, C5 PMC bytes, C5 SQ counters
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_c5k
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/bench_c5.log 2>&1; rc=$?
tail -1 gpurun_out/bench_c5.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5k -o k -- python3 bench.py --config c5 --steps 2 --warmup 1 > gpurun_out/prof_c5k/bench.log 2>&1; rc=$?
tail -1 gpurun_out/prof_c5k/bench.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 bash tools/profile_c5.sh > gpurun_out/pc5.log 2>&1; rc=$?
tail -3 gpurun_out/pc5.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 700 bash tools/profile_c5_sq.sh > gpurun_out/pc5sq.log 2>&1; rc=$?
tail -2 gpurun_out/pc5sq.log; exit $rc
