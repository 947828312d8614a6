# C5 persistent kernel: SGPR-offset buffer loads, SGPR-spill fixes (laundered per-step offsets, cell
# constants in VGPRs) and a third pair of E-image lead; interleaved timing + bit comparison against
# the round-5 build (c5base)
set -u
export TMPDIR=/tmp PYTHONPATH=.
D=tools/dbg
bash tools/ab_multi.sh tools/cmp_c5.py 2 $D/libwc_sde_large_c5base.so $D/libwc_sde_large_so.so $D/libwc_sde_large_sok.so $D/libwc_sde_large_sokl.so $D/libwc_sde_large_sokl3.so > gpurun_out/r05e_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05e_ab.log
for v in so sok sokl sokl3; do echo "$v vs base: $(python tools/cmp_c5.py cmp gpurun_out/abm/libwc_sde_large_c5base.npz gpurun_out/abm/libwc_sde_large_$v.npz | tr '\n' ' ')"; done
rm -f gpurun_out/abm/*.npz
