# C5: E image three pairs ahead and rows two, interleaved timing + bits
set -u
export TMPDIR=/tmp PYTHONPATH=.
D=tools/dbg
bash tools/ab_multi.sh tools/cmp_c5.py 3 nremmodfc_amd/libwcsde.so $D/libwc_sde_large_e3r2.so > gpurun_out/r05j_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05j_ab.log
echo "e3r2 vs base: $(python tools/cmp_c5.py cmp gpurun_out/abm/libwcsde.npz gpurun_out/abm/libwc_sde_large_e3r2.npz | tr '\n' ' ')"
rm -f gpurun_out/abm/*.npz
