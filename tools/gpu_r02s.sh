#!/bin/bash
# round-2 final evidence on the final build: GPU suite, smoke, bench, kernel trace + PMC passes
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
STEPS="tests smoke bench" bash tools/gpu_check.sh > gpurun_out/gc.log 2>&1; rc=$?
grep -E "rc=|passed|failed|smoke ok" gpurun_out/gc.log | head; [ $rc -ne 0 ] && exit $rc
bash tools/profile_bench.sh > gpurun_out/pb.log 2>&1; rc=$?; tail -2 gpurun_out/pb.log | cut -c1-200; exit $rc
