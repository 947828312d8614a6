#!/bin/bash
# SQ-counter passes over the C5 persistent integrator (tools/c5_pmc_run.py, one 400-step dispatch):
# instruction mix, MFMA busy, VALU issue and the wave-cycle split (issuing / issue-stalled / parked)
# -> gpurun_out/prof_c5sq/pmc_c5_sq.json (copy to profiles/ afterwards)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_c5sq
mkdir -p $OUT
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $OUT/a -o p -- python3 tools/c5_pmc_run.py 400 > $OUT/a.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/b -o p -- python3 tools/c5_pmc_run.py 400 > $OUT/b.log 2>&1
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import summary
(ka, a), = summary("gpurun_out/prof_c5sq/a", "persist_kernel").items()
(_, b), = summary("gpurun_out/prof_c5sq/b", "persist_kernel").items()
STEPS, WAVES = 400, 256 * 8
act = a["GRBM_GUI_ACTIVE"] / 8 * 1024
d = {"kernel": ka, "steps": STEPS, "waves": WAVES,
     "per_wave_step": {k: a[k] / (WAVES * STEPS) for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD")},
     "salu_per_wave_step": b["SQ_INSTS_SALU"] / (WAVES * STEPS),
     "mfma_busy_frac": a["SQ_VALU_MFMA_BUSY_CYCLES"] / act,
     "valu_issue_busy_frac": 4 * a["SQ_ACTIVE_INST_VALU"] / act,
     "lds_bank_conflict_frac": b["SQ_LDS_BANK_CONFLICT"] / max(1.0, b["SQ_LDS_IDX_ACTIVE"]),
     "wave_cycle_split": {k: b[k] / b["SQ_WAVE_CYCLES"] for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS")},
     "note": "rocprofv3 --pmc passes of tools/c5_pmc_run.py 400 (one persist_kernel dispatch of 400 Euler steps at the "
             "C5 shard, 2,500 x 1000, 8 waves per CU on 256 CUs). Busy fractions over GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs."}
json.dump(d, open("gpurun_out/prof_c5sq/pmc_c5_sq.json", "w"), indent=1)
print(json.dumps(d))
PY
