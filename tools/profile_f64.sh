#!/bin/bash
# PMC of the reference-precision integrator (wc_sde_kernel<double, ...>, bench.py --precision f64):
# kernel trace + two SQ passes of one --sde-only step (two 20,000-step launches), each pass its own
# rocprofv3 run; summary -> gpurun_out/prof64/pmc_sde_f64.json (copied to profiles/ by hand).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/prof64
mkdir -p $OUT
STAMP=$(sha256sum nremmodfc_amd/libwcsde.so | cut -d' ' -f1)
ARGS="--precision f64 --steps 1 --warmup 0 --sde-only --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o f64 -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sqa -o p -- python3 bench.py $ARGS > $OUT/sqa.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --output-format csv -d $OUT/sqb -o p -- python3 bench.py $ARGS > $OUT/sqb.log 2>&1 || exit $?
for d in $OUT/sqa $OUT/sqb; do echo $STAMP > $d/lib.sha256; done
python3 - <<'PY'
import collections, json, sys
sys.path.insert(0, "tools")
from pmc_summary import lib_stamp, summary
stamp = lib_stamp("gpurun_out/prof64/sqa", "gpurun_out/prof64/sqb")
# a launch may be two dispatches (the full two-group rounds + the one-group tail, WC_F64_TAIL):
# per-launch totals are the sums of the per-dispatch averages of every wc_sde_kernel<double> form
def total(s):
    out = collections.Counter()
    for v in s.values():
        out.update({c: x for c, x in v.items() if c != "dispatches"})
    return out
sa, sb = summary("gpurun_out/prof64/sqa", "wc_sde_kernel"), summary("gpurun_out/prof64/sqb", "wc_sde_kernel")
a, b = total(sa), total(sb)
B, STEPS = 20000, 20000
waves = -(-B // 16) * 6  # fp64: six one-tile waves per group of 16 simulations
ws = waves * STEPS
act = a["GRBM_GUI_ACTIVE"] / 8 * 1024
d = {"kernel": " + ".join(sorted(sa)), "lib_sha256": stamp, "B": B, "N": 90, "euler_steps": STEPS, "precision": "f64",
     "per_wave_step": {c: a[c] / ws for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS")}
                      | {"SQ_INSTS_VMEM_RD": b["SQ_INSTS_VMEM_RD"] / ws},
     "mfma_busy_frac": a["SQ_VALU_MFMA_BUSY_CYCLES"] / act,
     "valu_issue_busy_frac": 4 * a["SQ_ACTIVE_INST_VALU"] / act,
     "wave_cycle_split": {c: b[c] / b["SQ_WAVE_CYCLES"] for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY")},
     "gpu_active_cycles_per_launch": a["GRBM_GUI_ACTIVE"] / 8,
     "note": "rocprofv3 --pmc passes of `bench.py --precision f64 --steps 1 --warmup 0 --sde-only` (tools/profile_f64.sh): "
             "per-launch sums over the wc_sde_kernel<double> dispatches of one 20,000-step launch of 20,000 simulations "
             "(two-group rounds + one-group tail); a wave-step = one Euler step of one wave (six waves per group of 16)."}
json.dump(d, open("gpurun_out/prof64/pmc_sde_f64.json", "w"), indent=1)
print(json.dumps(d))
PY
find gpurun_out/prof64 -name "*counter_collection.csv" -delete
find gpurun_out/prof64 -name "*kernel_trace.csv" -delete
