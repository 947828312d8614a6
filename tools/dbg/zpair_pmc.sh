# PMC passes over the V_ZPAIR integrator at the 4-GPU C3 shard (tools/zpair_pmc_run.py), one counter set per run
export TMPDIR=/tmp
O=gpurun_out/r06zp
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 tools/zpair_pmc_run.py 4000 > $O/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/fetch.log 2>&1 || { echo "fetch rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/write.log 2>&1 || { echo "write rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $O/sqa -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/sqa.log 2>&1 || { echo "sqa rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sqb -o p -- python3 tools/zpair_pmc_run.py 4000 > $O/sqb.log 2>&1 || { echo "sqb rc=$?"; exit 1; }
python3 - <<'PY'
import json, sys
sys.path.insert(0, "tools")
from pmc_summary import summary
O = "gpurun_out/r06zp"
out = {}
for p in ("fetch", "write", "sqa", "sqb"):
    for k, v in summary(f"{O}/{p}", "wc_sde_kernel").items():
        out.setdefault(k, {}).update(v)
print(json.dumps(out, indent=1))
json.dump(out, open(f"{O}/zpair_pmc.json", "w"), indent=1)
PY
find $O -name "*counter_collection.csv" -size +5M -delete
