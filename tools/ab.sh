#!/bin/bash
# A/B of a kernel change on the GPU box (the entry point that replaced round 2's per-session
# gpu_r02*.sh scripts): bit-compare and time the BASE build of libwcsde.so against the product
# build, then run the GPU tests of the touched stage.
#
#   bash tools/ab.sh <stage> <base .so> [pytest file] [candidate .so, default the product build]
#     stage: sde (tools/cmp_libs.py), bold (tools/cmp_bold.py), welch (tools/cmp_welch.py), c5 (tools/cmp_c5.py)
#
# The base build is made beforehand on the CPU: stash the change, `python -m nremmodfc_amd._build`,
# copy nremmodfc_amd/libwcsde.so to tools/dbg/libwcsde_base.so, unstash, rebuild.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
STAGE=$1 BASE=$2 TESTS=${3:-} CAND=${4:-nremmodfc_amd/libwcsde.so}
case $STAGE in sde) CMP=tools/cmp_libs.py ;; bold) CMP=tools/cmp_bold.py ;; welch) CMP=tools/cmp_welch.py ;; c5) CMP=tools/cmp_c5.py ;;
  *) echo "unknown stage $STAGE"; exit 2 ;; esac
OUT=gpurun_out/ab_$STAGE
mkdir -p $OUT
for v in base prod; do
  L=$PWD/$BASE; [ $v = prod ] && L=$PWD/$CAND
  WCSDE_LIB_OVERRIDE=$L CMP_TIME=1 timeout -k 10 300 python -u $CMP save $OUT/$v.npz > $OUT/$v.log 2>&1 || { tail -5 $OUT/$v.log; exit 1; }
  echo "== $STAGE $v"; grep -v amdgpu.ids $OUT/$v.log
done
python $CMP cmp $OUT/base.npz $OUT/prod.npz; echo "== cmp $STAGE rc=$?"
rm -f $OUT/*.npz
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread $TESTS > $OUT/t.log 2>&1 || { tail -20 $OUT/t.log; exit 1; }
  tail -2 $OUT/t.log
fi
