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
ARGS="--steps ${PSTEPS:-4} --warmup 1 --no-cpu-baseline --secondary-steps 0"
STAMP=$(sha256sum nremmodfc_amd/libwcsde.so | cut -d' ' -f1)  # the library every pass below runs
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o bench -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o p -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o p -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VALU_TRANS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o p -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o p -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1
for d in $OUT/fetch $OUT/write $OUT/sq $OUT/sq2; do mkdir -p $d && echo $STAMP > $d/lib.sha256; done
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import lib_stamp, summary
stamp = lib_stamp("gpurun_out/prof/fetch", "gpurun_out/prof/write", "gpurun_out/prof/sq", "gpurun_out/prof/sq2")
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
d = {"kernel": kf, "lib_sha256": stamp, "B": B, "N": N, "euler_steps": STEPS, "precision": "f32",
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
q2 = summary("gpurun_out/prof/sq2", "wc_sde_kernel")
(_, v2), = q2.items()
d["wave_cycle_split"] = {k: v2[k] / v2["SQ_WAVE_CYCLES"] for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")}
json.dump(d, open("profiles/pmc_sde.json", "w"), indent=1)
# the two signal kernels of the bench step: instruction counts per unit of work, issue and wait split
sig = {"lib_sha256": stamp, "note": "rocprofv3 --pmc passes of the same bench run (tools/profile_bench.sh), averaged per dispatch. "
               "Busy fractions: 4 x SQ_ACTIVE_INST_* quad-cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); "
               "wave_cycle_split: SQ_WAIT_ANY (parked on s_waitcnt/barrier), SQ_WAIT_INST_ANY (issue stall), "
               "SQ_ACTIVE_INST_ANY (issuing), fractions of SQ_WAVE_CYCLES."}
C = 20000 * 90
for name, sub, units, per in (("bold_steady_copy", "bold_chunk_kernel<float, true, true, true>", C * 2000.0 / 64, "wave-sample"),  # (one pass per 2000 samples)
                              ("welch", "welch_wave_kernel", 2.0 * C, "column-segment")):  # (two segments per launch)
    a = summary("gpurun_out/prof/sq", sub)
    b = summary("gpurun_out/prof/sq2", sub)
    fe = summary("gpurun_out/prof/fetch", sub)
    wr = summary("gpurun_out/prof/write", sub)
    if not (a and b and fe and wr):
        continue
    (ka, va), = a.items(); (_, vb), = b.items(); (_, vf2), = fe.items(); (_, vw2), = wr.items()
    act = va["GRBM_GUI_ACTIVE"] / 8 * simds
    sig[name] = {"kernel": ka, "unit": per,
                 "valu_insts_per_unit": va["SQ_INSTS_VALU"] / units,
                 "lds_insts_per_unit": vb["SQ_INSTS_LDS"] / units,
                 "valu_issue_busy_frac": 4 * va["SQ_ACTIVE_INST_VALU"] / act,
                 "lds_bank_conflict_frac": vb["SQ_LDS_BANK_CONFLICT"] / max(1.0, vb["SQ_LDS_IDX_ACTIVE"]),
                 "wave_cycle_split": {k: vb[k] / vb["SQ_WAVE_CYCLES"] for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")},
                 "hbm_bytes_per_dispatch": 2 * vf2["FETCH_SIZE"] * 1024.0 + vw2["WRITE_SIZE"] * 1024.0,
                 "dispatches": va["dispatches"]}
json.dump(sig, open("profiles/pmc_signal.json", "w"), indent=1)
json.dump(sig, open("gpurun_out/prof/pmc_signal.json", "w"), indent=1)
json.dump(d, open("gpurun_out/prof/pmc_sde.json", "w"), indent=1)  # gpurun merges gpurun_out/ back only
print(json.dumps(d))
PY
cp $OUT/bench_kernel_stats.csv gpurun_out/prof/r03_bench_kernel_stats.csv 2>/dev/null || true
# on the GPU box only gpurun_out/ travels back: copy gpurun_out/prof/pmc_sde.json and
# gpurun_out/prof/bench_kernel_stats.csv into profiles/ afterwards
tail -1 $OUT/trace.log
# per-dispatch CSVs stay on the box (a call returns at most 64 MiB of gpurun_out/)
find $OUT -name "*counter_collection.csv" -delete
find $OUT -name "*kernel_trace.csv" -delete
