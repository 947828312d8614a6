#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats of a short bench run        -> profiles/r01_bench_kernel_stats.csv
#   2. FETCH_SIZE and WRITE_SIZE in separate --pmc passes (MI355X_MICROARCH.md: they do not fit one pass)
#   3. one SQ pass (instruction mix, MFMA busy, wave cycles) + GRBM_GUI_ACTIVE
#   4. profiles/pmc_sde.json: HBM bytes per wc_sde_kernel launch (FETCH_SIZE doubled for gfx950, KB -> B)
#      and the instruction / utilisation counters of the same kernel
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
ARGS="--steps ${PSTEPS:-4} --warmup 1 --no-cpu-baseline"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import summary
f = summary("gpurun_out/prof/fetch", "wc_sde_kernel")
w = summary("gpurun_out/prof/write", "wc_sde_kernel")
q = summary("gpurun_out/prof/sq", "wc_sde_kernel")
(kf, vf), = f.items()
(kw, vw), = w.items()
(kq, vq), = q.items()
fetch = 2 * vf["FETCH_SIZE"] * 1024.0
write = vw["WRITE_SIZE"] * 1024.0
B, N, STEPS = 20000, 90, 20000
node_steps = B * N * STEPS
wave_steps = (B // 16) * 3 * STEPS  # 16 simulations x 3 waves (2 node tiles each) per group
simds = 256 * 4
d = {"kernel": kf, "B": B, "N": N, "euler_steps": STEPS, "precision": "f32",
     "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
     "hbm_bytes_per_launch": fetch + write, "dispatches": vf["dispatches"],
     "algorithmic_bytes_per_launch": B * N * (STEPS // 20 * 4 + 2 * 3 * 8 + 2 * 8),
     "sq": {k: vq[k] for k in vq if k != "dispatches"},
     "valu_insts_per_wave_step": vq["SQ_INSTS_VALU"] / wave_steps,
     "mfma_insts_per_wave_step": vq["SQ_INSTS_MFMA"] / wave_steps,
     "trans_insts_per_wave_step": vq["SQ_INSTS_VALU_TRANS_F32"] / wave_steps,
     "mfma_busy_frac": vq["SQ_VALU_MFMA_BUSY_CYCLES"] / (vq["GRBM_GUI_ACTIVE"] / 8 * simds),
     "valu_issue_busy_frac": 4 * vq["SQ_ACTIVE_INST_VALU"] / (vq["GRBM_GUI_ACTIVE"] / 8 * simds),
     "note": "rocprofv3 --pmc passes of `python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline` "
             "(tools/profile_bench.sh), averaged per wc_sde_kernel dispatch. FETCH_SIZE x2 (gfx950), KB -> B; "
             "HBM counters include Infinity-Cache traffic. A wave-step = one Euler step of one wave "
             "(16 simulations x 2 node tiles of 16; 3 waves per group of 16 simulations). mfma_busy_frac = SQ_VALU_MFMA_BUSY_CYCLES / "
             "(GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)."}
json.dump(d, open("profiles/pmc_sde.json", "w"), indent=1)
json.dump(d, open("gpurun_out/prof/pmc_sde.json", "w"), indent=1)  # gpurun merges gpurun_out/ back only
print(json.dumps(d))
PY
cp $OUT/bench_kernel_stats.csv profiles/r02_bench_kernel_stats.csv 2>/dev/null || true
# on the GPU box only gpurun_out/ travels back: copy gpurun_out/prof/pmc_sde.json and
# gpurun_out/prof/bench_kernel_stats.csv into profiles/ afterwards
tail -1 $OUT/trace.log
