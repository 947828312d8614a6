# PMC of the fp64 Welch wave-pair kernel (tools/time_welch64.py: one-segment launches at 20,000 x 90)
set -u
export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/prof_w64b
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d $O/a -o p -- python3 tools/time_welch64.py 20000 > $O/a.log 2>&1 || { echo "a rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/b -o p -- python3 tools/time_welch64.py 20000 > $O/b.log 2>&1 || { echo "b rc=$?"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o p -- python3 tools/time_welch64.py 20000 > $O/f.log 2>&1 || { echo "f rc=$?"; exit 1; }
sha256sum nremmodfc_amd/libwcsde.so | cut -d' ' -f1 > $O/lib.sha256
python3 tools/pmc_summary.py $O/a welch_wave64 > $O/sum_a.json && python3 tools/pmc_summary.py $O/b welch_wave64 > $O/sum_b.json && python3 tools/pmc_summary.py $O/f welch_wave64 > $O/sum_f.json
find $O -name "*counter_collection.csv" -delete
cat $O/sum_a.json $O/sum_b.json $O/sum_f.json
