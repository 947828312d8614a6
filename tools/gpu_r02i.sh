#!/bin/bash
# persistent C5 kernel ablations (diag build): 1 product, 2 no MFMA, 3 no epilogue, 4 no K loads, 5 no waits
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/abl.log
for v in 1 2 3 4 5; do
  WCSDE_LIB_OVERRIDE=$PWD/nremmodfc_amd/libwcsde_diag.so WCSDE_PERSISTENT=$v REPS=1 timeout -k 10 120 python -u tools/time_pmap.py 2500 0 > gpurun_out/abl_$v.log 2>&1 || { cat gpurun_out/abl_$v.log; exit 1; }
  echo "variant $v: $(grep us/step gpurun_out/abl_$v.log)" | tee -a gpurun_out/abl.log
done
