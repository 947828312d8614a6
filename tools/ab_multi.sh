#!/bin/bash
# Interleaved timing of several builds of libwcsde.so with one cmp tool (round-robin, R rounds):
#   bash tools/ab_multi.sh <cmp tool> <rounds> lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
CMP=$1 R=$2; shift 2
mkdir -p gpurun_out/abm
for r in $(seq $R); do
  for L in "$@"; do
    WCSDE_LIB_OVERRIDE=$PWD/$L CMP_TIME=1 timeout -k 10 300 python -u $CMP save gpurun_out/abm/$(basename $L .so).npz > gpurun_out/abm/t.log 2>&1 || { tail -5 gpurun_out/abm/t.log; exit 1; }
    echo "round $r $L: $(grep -v amdgpu.ids gpurun_out/abm/t.log | tr '\n' ' ')"
  done
done
