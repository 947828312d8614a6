#!/bin/bash
# persistent C5 kernel iteration: bit-exactness vs the step kernel, then us per step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PT="python -u -m pytest -x -v --timeout 200 --timeout-method thread"
timeout -k 10 300 $PT tests/test_sde_large_gpu.py -k "persistent or large_vs_oracle" > gpurun_out/t_h.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|passed|failed|assert" gpurun_out/t_h.log | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u tools/time_pmap.py 2500 ${PMAPS:-0,8} > gpurun_out/pmap.log 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/pmap.log; exit $rc
