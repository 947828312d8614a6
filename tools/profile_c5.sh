#!/bin/bash
# HBM-traffic evidence for `bench.py --config c5` (run on the GPU box from the repo root):
# FETCH_SIZE and WRITE_SIZE in separate --pmc passes over a 400-step run of the bench's C5 shard
# (tools/c5_pmc_run.py: one persist_kernel dispatch of 400 Euler steps), divided per step and scaled
# to the 20,000-step chunk that bench.py's roofline calls one "launch"
# -> gpurun_out/prof_c5/pmc_sde_c5.json (copy to profiles/ afterwards).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof_c5
mkdir -p $OUT
STEPS=${C5STEPS:-400}
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 tools/c5_pmc_run.py $STEPS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 tools/c5_pmc_run.py $STEPS > $OUT/write.log 2>&1
python3 - <<'PY'
import json, os, sys
sys.path.insert(0, "tools")
from pmc_summary import summary
(kf, vf), = summary("gpurun_out/prof_c5/fetch", "persist_kernel").items()
(kw, vw), = summary("gpurun_out/prof_c5/write", "persist_kernel").items()
B, N, STEPS = 2500, 1000, 20000
RUN = int(os.environ.get("C5STEPS", "400"))  # one persist_kernel launch integrates RUN steps
fetch = 2 * vf["FETCH_SIZE"] * 1024.0 / RUN
write = vw["WRITE_SIZE"] * 1024.0 / RUN
d = {"kernel": kf, "B": B, "N": N, "euler_steps": STEPS, "precision": "f32",
     "fetch_bytes_per_step": fetch, "write_bytes_per_step": write,
     "fetch_bytes_per_launch": fetch * STEPS, "write_bytes_per_launch": write * STEPS,
     "hbm_bytes_per_launch": (fetch + write) * STEPS, "dispatches": vf["dispatches"],
     "state_bytes_per_step": B * N * 36, "connectome_bytes_per_step": 1024 * 1024 * 2 * 2,
     "algorithmic_bytes_per_launch": B * N * (STEPS // 20 * 4 + 2 * 3 * 8 + 2 * 8),
     "note": "rocprofv3 --pmc passes of `python3 tools/c5_pmc_run.py 400` (tools/profile_c5.sh): one persist_kernel "
             "dispatch of 400 Euler steps, divided by 400 and scaled by 20,000 to bench.py's per-chunk 'launch'. FETCH_SIZE x2 (gfx950), KB -> B; the "
             "counters include Infinity-Cache (MALL) hits; the state stays in registers, so the bytes are the "
             "per-step operand stream (connectome rows and the E image)."}
json.dump(d, open("gpurun_out/prof_c5/pmc_sde_c5.json", "w"), indent=1)
print(json.dumps(d))
PY
