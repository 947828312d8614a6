#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/zprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/zprof -o z -- python3 tools/time_shard.py 2500 > gpurun_out/zprof/log.txt 2>&1; echo rc=$?
grep "B=" gpurun_out/zprof/log.txt
find gpurun_out/zprof -name "*kernel_stats.csv" -exec cut -c1-250 {} \;
