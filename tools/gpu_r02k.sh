#!/bin/bash
# config 5 end to end with the persistent integrator: rank 3 of 8 of the 1000-node sweep, full schedule
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
SLURM_ARRAY_TASK_ID=3 SLURM_ARRAY_TASK_MAX=7 timeout -k 10 700 python -u -m nremmodfc_amd.sweep homo --nodes 1000 \
    --out gpurun_out/c5 --tag c5_n1000 > gpurun_out/c5/log.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c5/log.txt | tail -3 | cut -c1-600; exit $rc
