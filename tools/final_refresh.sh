#!/bin/bash
# Round-end evidence in one GPU session: full GPU suite, smoke, bench + kernel trace, PMC passes,
# C5 bench, SC optimiser with kernel trace. Stops at the first failure (run from the repo root).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_check.sh > gpurun_out/gc.log 2>&1 || exit $?
bash tools/profile_bench.sh > gpurun_out/pb.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5.log 2>&1 || exit $?
mkdir -p gpurun_out/opt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/opt -o o -- \
    python3 -m nremmodfc_amd.optimize_sc --iters 100 --out gpurun_out/opt > gpurun_out/opt/log.jsonl 2>&1 || exit $?
echo done
