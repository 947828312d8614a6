#!/bin/bash
# All C5 PMC passes (fetch, write, sqa, sqb, tcc) of tools/c5_pmc_run.py in ONE gpurun call: the
# persistent kernel is launched as an ordinary launch (WCSDE_COOP=0, same grid, one workgroup per CU
# on the idle GPU), which avoids the runtime's teardown fault after a cooperative launch under
# rocprofv3.  Each pass is its own rocprofv3 run; the script stops at the first
# failing pass.  Then tools/profile_c5_summary.py on the CPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp WCSDE_COOP=0
for P in ${PASSES:-fetch write writering sqa sqb tcc}; do
  bash tools/profile_c5_pass.sh $P || { echo "pass $P failed"; exit 1; }
done
# the summaries here (they also land in gpurun_out/prof_c5/), then drop the per-dispatch CSVs, which
# would push gpurun_out past what a call returns
python3 tools/profile_c5_summary.py ${SUMMARIES:-hbm sq tcc} > gpurun_out/prof_c5/summary.log 2>&1 || { tail -5 gpurun_out/prof_c5/summary.log; exit 1; }
find gpurun_out/prof_c5 -name "*counter_collection.csv" -delete
