#!/bin/bash
# small-shard normals path: bit-identity test, then the shard timing table (with the plain path beside it)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sde_gpu.py -k "precomputed or grouped or homogeneous" -q -rA --timeout 200 --timeout-method thread > gpurun_out/zm_pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error|assert" gpurun_out/zm_pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/time_shard.py ${SHARDS:-20000,10000,5000,2500,1250} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/zm_shard.log
