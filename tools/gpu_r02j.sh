#!/bin/bash
# packed fp32 cell update (C3 kernel): bit-compare against the previous build, time both
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
WCSDE_LIB_OVERRIDE=$PWD/nremmodfc_amd/libwcsde_prev.so CMP_TIME=1 timeout -k 10 200 python -u tools/cmp_libs.py save gpurun_out/prev.npz 2>&1 | grep -v amdgpu.ids; [ ${PIPESTATUS[0]} -ne 0 ] && exit 1
CMP_TIME=1 timeout -k 10 200 python -u tools/cmp_libs.py save gpurun_out/new.npz 2>&1 | grep -v amdgpu.ids; [ ${PIPESTATUS[0]} -ne 0 ] && exit 1
python tools/cmp_libs.py cmp gpurun_out/prev.npz gpurun_out/new.npz; rc=$?
rm -f gpurun_out/prev.npz gpurun_out/new.npz
exit $rc
