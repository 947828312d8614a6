#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_fc_ssim_gpu.py "tests/test_signal_gpu.py::test_pipeline_fc_ssim_vs_oracle" "tests/test_facades_gpu.py" -q -s -rA --timeout 400 --timeout-method thread > gpurun_out/fc_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "TOL|passed|failed|Error" gpurun_out/fc_pytest.log | tail -12
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep -v amdgpu.ids
