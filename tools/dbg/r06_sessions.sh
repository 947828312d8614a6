#!/bin/bash
# Round 6's one-off GPU A/B sessions, one case each (logs under gpurun_out/r06<x>, kept in profiles/r06/):
#   bash tools/dbg/r06_sessions.sh zpair_genoff   V_ZPAIR with its generator waves idle (diag build, wrong
#                                                 normals) vs the product: 5,000 / 4,100 simulations
#   bash tools/dbg/r06_sessions.sh zpair_pmc      PMC passes over the V_ZPAIR integrator at the 4-GPU C3 shard
#   bash tools/dbg/r06_sessions.sh zk             steps per V_ZMEM/V_ZPAIR launch, 1000 (product) vs the
#                                                 variants built by `tools/dbg/variants.sh wc_sde zk<K>=-DWC_ZK=<K>`
#                                                 (a WC_ZK macro around kZK in wc_sde.hip; not in the product source)
#   bash tools/dbg/r06_sessions.sh coop           C5 persistent grid, cooperative vs ordinary launch, no profiler
# The closing evidence runs are `STEPS="tests smoke bench trace" bash tools/gpu_check.sh`.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONPATH=.
case "${1:-}" in
  zpair_genoff)
    O=gpurun_out/r06j; mkdir -p $O
    export WCSDE_LIB_OVERRIDE=$PWD/nremmodfc_amd/libwcsde_diag.so
    for r in 1 2; do
      timeout -k 10 200 python tools/time_shard.py 5000,4100 > $O/prod$r.log 2>&1 || exit 1
      WCSDE_ZGEN_OFF=1 timeout -k 10 200 python tools/time_shard.py 5000,4100 > $O/genoff$r.log 2>&1 || exit 1
      echo "product: $(grep B= $O/prod$r.log | cut -c1-40 | tr '\n' ' ')"
      echo "gen off: $(grep B= $O/genoff$r.log | cut -c1-40 | tr '\n' ' ')"
    done ;;
  zpair_pmc)
    O=gpurun_out/r06zp; mkdir -p $O
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 tools/zpair_pmc_run.py 4000 > $O/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/sqa -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/sqa.log 2>&1 || { echo "sqa rc=$?"; exit 1; }
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sqb -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/sqb.log 2>&1 || { echo "sqb rc=$?"; exit 1; }
    python3 - "$O" <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import summary
O = sys.argv[1]
out = {}
for p in ("fetch", "write", "sqa", "sqb"):
    for k, v in summary(f"{O}/{p}", "wc_sde_kernel").items():
        out.setdefault(k, {}).update(v)
print(json.dumps(out, indent=1))
json.dump(out, open(f"{O}/zpair_pmc.json", "w"), indent=1)
PY
    find $O -name "*counter_collection.csv" -size +5M -delete ;;
  zk)
    O=gpurun_out/r06k; mkdir -p $O
    for r in 1 2; do
      for v in prod ${ZK_VARIANTS:-zk60 zk100 zk200 zk2000 zk4000}; do
        if [ $v = prod ]; then unset WCSDE_LIB_OVERRIDE; else export WCSDE_LIB_OVERRIDE=$PWD/tools/dbg/libwc_sde_$v.so; fi
        timeout -k 10 200 python tools/time_shard.py 5000,4100,2500 > $O/$v$r.log 2>&1 || exit 1
        echo "$v: $(grep B= $O/$v$r.log | cut -d' ' -f1-3,13- | tr '\n' ' ')"
      done
    done ;;
  coop)
    O=gpurun_out/r06l; mkdir -p $O
    for r in 1 2 3; do
      timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/coop$r.log 2>&1 || exit 1
      WCSDE_COOP=0 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > $O/plain$r.log 2>&1 || exit 1
      for v in coop plain; do
        python - $O/$v$r.log $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "ms_per_step", d["ms_per_step"], "kernel_ms", d.get("kernel_ms"))
PY
      done
    done ;;
  *) echo "usage: $0 zpair_genoff|zpair_pmc|zk|coop"; exit 2 ;;
esac
