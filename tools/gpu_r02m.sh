#!/bin/bash
# A/B of the round-2 instruction cuts against the build at the start of the session:
# SDE with E kept in 2^-10 units (bit-exact claim) and the 2-op a_ie increment (WC_INC2),
# BOLD with three-address Horner fmas (bit-exact claim); then the GPU suite on the product
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/m
mkdir -p $OUT
D=$PWD/tools/dbg
for v in base es inc2; do
  WCSDE_LIB_OVERRIDE=$D/libwcsde_$v.so CMP_TIME=1 timeout -k 10 300 python -u tools/cmp_libs.py save $OUT/sde_$v.npz > $OUT/sde_$v.log 2>&1 || { tail -5 $OUT/sde_$v.log; exit 1; }
  echo "== sde $v"; grep -v amdgpu.ids $OUT/sde_$v.log
done
python tools/cmp_libs.py cmp $OUT/sde_base.npz $OUT/sde_es.npz > $OUT/cmp_es.log 2>&1; echo "== cmp base es rc=$?"; cat $OUT/cmp_es.log
python tools/cmp_libs.py cmp $OUT/sde_base.npz $OUT/sde_inc2.npz > $OUT/cmp_inc2.log 2>&1; echo "== cmp base inc2 rc=$?"; cat $OUT/cmp_inc2.log
for v in base prod; do
  L=$D/libwcsde_$v.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/cmp_bold.py save $OUT/bold_$v.npz > $OUT/bold_$v.log 2>&1 || { tail -5 $OUT/bold_$v.log; exit 1; }
  echo "== bold $v"; grep -v amdgpu.ids $OUT/bold_$v.log
done
python tools/cmp_bold.py cmp $OUT/bold_base.npz $OUT/bold_prod.npz; echo "== cmp bold rc=$?"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; exit $rc
