#!/bin/bash
# ONE rocprofv3 --pmc pass over tools/c5_pmc_run.py (the C5 persistent integrator, one 400-step
# dispatch), per gpurun call.  (Round 4's passes segfaulted in process teardown after "tool
# finalization"; tools/c5_pmc_run.py writes /proc/self/maps at exit to $OUT/<pass>.maps so that the
# frames of such a fault map to library + offset.)
#   PASS = fetch | write | writering | sqa | sqb | tcc (L2 hits and misses)  -> gpurun_out/prof_c5/<pass>/ ; then tools/profile_c5_summary.py
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
P=$1
OUT=gpurun_out/prof_c5
mkdir -p $OUT
case $P in
  fetch) C="FETCH_SIZE" ;;
  write) C="WRITE_SIZE" ;;
  writering) C="WRITE_SIZE"; export C5_RING=1 ;;  # the round-5 harness's node-major ring records
  sqa) C="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE" ;;
  tcc) C="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum" ;;
  sqb) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE" ;;
  *) echo "unknown pass $P"; exit 2 ;;
esac
export C5_MAPS_OUT=$OUT/$P.maps
mkdir -p $OUT/$P && sha256sum nremmodfc_amd/libwcsde.so | cut -d' ' -f1 > $OUT/$P/lib.sha256  # the library this pass runs
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/$P -o p -- python3 tools/c5_pmc_run.py 400 > $OUT/$P.log 2>&1
rc=$?
grep -q "persist_kernel" $OUT/$P/p_counter_collection.csv && echo "pass $P: counters written (rocprofv3 rc=$rc)"
exit $rc
