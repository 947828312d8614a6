#!/bin/bash
# SDE kernel change on the GPU box: the integrator's GPU tests, then the bench line (no CPU leg)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sde_gpu.py -q -s --timeout 200 --timeout-method thread > gpurun_out/sde_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "TOL|passed|failed" gpurun_out/sde_pytest.log | tail -14
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/sde_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/sde_bench.log; exit 1; }
grep -v amdgpu.ids gpurun_out/sde_bench.log | cut -c1-300; grep -o '"kernel_ms": {[^}]*}' gpurun_out/sde_bench.log
