# fp64 Welch (welch_kernel<double>) ablations: twiddle loads, segment loads, both; plus one SQ pass
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for r in 1 2; do
  for L in nremmodfc_amd/libwcsde.so tools/dbg/libwelch_w64notw.so tools/dbg/libwelch_w64noload.so tools/dbg/libwelch_w64both.so; do
    echo "$L: $(WCSDE_LIB_OVERRIDE=$PWD/$L timeout -k 10 120 python tools/time_welch64.py 20000 2>&1 | grep ms)" || exit 1
  done
done | tee gpurun_out/r05g_w64.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_w64 -o p -- python3 tools/time_welch64.py 20000 > gpurun_out/prof_w64.log 2>&1 || { echo "pmc rc=$?"; exit 1; }
python3 tools/pmc_summary.py gpurun_out/prof_w64 welch_kernel
find gpurun_out/prof_w64 -name "*counter_collection.csv" -delete
