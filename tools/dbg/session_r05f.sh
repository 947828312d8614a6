# Welch floor: timing of the product kernel and its ablations (no next-column loads = FFT alone;
# no stages 2-4 = loads + stage 1 alone), then SQ/LDS PMC passes of the product and the FFT-alone build
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
for r in 1 2; do
  for L in nremmodfc_amd/libwcsde.so tools/dbg/libwelch_noload.so tools/dbg/libwelch_nofft.so; do
    echo "$L: $(WCSDE_LIB_OVERRIDE=$PWD/$L timeout -k 10 120 python tools/time_welch.py 20000 2>&1 | grep ms)" || exit 1
  done
done | tee gpurun_out/r05f_welch_ab.log
bash tools/welch_pmc.sh gpurun_out/prof_welch_prod > gpurun_out/r05f_pmc_prod.log 2>&1 || { echo "pmc prod rc=$?"; exit 1; }
WCSDE_LIB_OVERRIDE=$PWD/tools/dbg/libwelch_noload.so bash tools/welch_pmc.sh gpurun_out/prof_welch_noload > gpurun_out/r05f_pmc_noload.log 2>&1 || { echo "pmc noload rc=$?"; exit 1; }
WCSDE_LIB_OVERRIDE=$PWD/tools/dbg/libwelch_nofft.so bash tools/welch_pmc.sh gpurun_out/prof_welch_nofft > gpurun_out/r05f_pmc_nofft.log 2>&1 || { echo "pmc nofft rc=$?"; exit 1; }
find gpurun_out/prof_welch_* -name "*counter_collection.csv" -size +20M -delete
echo done
