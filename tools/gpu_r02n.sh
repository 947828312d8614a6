#!/bin/bash
# shard rates of the current build + the long SC optimiser run (convergence towards the shipped SC)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/n
mkdir -p $OUT
timeout -k 10 200 python -u tools/time_shard.py > $OUT/shard.log 2>&1 || { cat $OUT/shard.log; exit 1; }
grep -v amdgpu.ids $OUT/shard.log
timeout -k 10 600 python -u tools/sc_converge.py 3000 100 > $OUT/sc_converge.jsonl 2>&1 || { tail -5 $OUT/sc_converge.jsonl; exit 1; }
grep -v amdgpu.ids $OUT/sc_converge.jsonl | cut -c1-250
