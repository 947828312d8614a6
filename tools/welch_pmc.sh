#!/bin/bash
# PMC passes over tools/time_welch.py (Welch segment kernel alone at C3's 20,000 x 90 columns)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_welch}  # (WCSDE_LIB_OVERRIDE selects another build, e.g. an ablation)
mkdir -p $OUT
export PYTHONPATH=.
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o p -- python3 tools/time_welch.py 20000 > $OUT/a.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES --output-format csv -d $OUT/b -o p -- python3 tools/time_welch.py 20000 > $OUT/b.log 2>&1 || exit $?
rm -f $OUT/a/*/*agent_info.csv $OUT/b/*/*agent_info.csv
python3 tools/pmc_summary.py $OUT/a welch_wave > $OUT/sum_a.json
python3 tools/pmc_summary.py $OUT/b welch_wave > $OUT/sum_b.json
cat $OUT/sum_a.json $OUT/sum_b.json
