#!/bin/bash
# Interleaved A/B timing of one command against two builds of libwcsde.so on the GPU box:
# ROUNDS x (base build, product build), each run under its own time limit; stops at the
# first failure.  Output: gpurun_out/ab_cmd/<round>_<base|prod>.log, echoed as it goes.
#
#   bash tools/ab_cmd.sh <base .so> <rounds> <command ...>
#   e.g. bash tools/ab_cmd.sh tools/dbg/libwcsde_base.so 2 python -u tools/time_shard.py 2500,1250
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
BASE=$1 ROUNDS=$2
shift 2
OUT=gpurun_out/ab_cmd
mkdir -p $OUT
for r in $(seq 1 $ROUNDS); do
  for v in base prod; do
    L=$PWD/$BASE; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
    WCSDE_LIB_OVERRIDE=$L timeout -k 10 ${AB_TIMEOUT:-300} "$@" > $OUT/${r}_$v.log 2>&1 || { echo "FAIL $r $v"; tail -5 $OUT/${r}_$v.log; exit 1; }
    echo "== round $r $v"; grep -v amdgpu.ids $OUT/${r}_$v.log
  done
done
