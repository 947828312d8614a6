#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of a short bench run  -> gpurun_out/prof/bench_kernel_stats.csv
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: they do not fit one pass)
#   3. profiles/pmc_sde.json: HBM bytes per wc_sde_kernel launch (FETCH_SIZE doubled for gfx950, KB -> B)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps ${PSTEPS:-4} --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 bench.py $ARGS > $OUT/write.log 2>&1
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import summary
f = summary("gpurun_out/prof/fetch", "wc_sde_kernel")
w = summary("gpurun_out/prof/write", "wc_sde_kernel")
(kf, vf), = f.items()
(kw, vw), = w.items()
fetch = 2 * vf["FETCH_SIZE"] * 1024.0
write = vw["WRITE_SIZE"] * 1024.0
d = {"kernel": kf, "B": 20000, "N": 90, "euler_steps": 20000, "precision": "f32",
     "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
     "hbm_bytes_per_launch": fetch + write, "dispatches": vf["dispatches"],
     "note": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes; FETCH_SIZE x2 (gfx950 16-B/lane "
             "reads tallied at half), KB -> B; Infinity-Cache hits are included by these counters"}
json.dump(d, open("profiles/pmc_sde.json", "w"), indent=1)
print(json.dumps(d))
PY
cp $OUT/bench_kernel_stats.csv profiles/ 2>/dev/null || true
tail -1 $OUT/trace.log
