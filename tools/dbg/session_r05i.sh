# C5: the normals of the first 1-2 simulation tiles drawn during the K loop's first remote pairs
set -u
export TMPDIR=/tmp PYTHONPATH=.
D=tools/dbg
bash tools/ab_multi.sh tools/cmp_c5.py 2 nremmodfc_amd/libwcsde.so $D/libwc_sde_large_zk1.so $D/libwc_sde_large_zk2.so > gpurun_out/r05i_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/r05i_ab.log
for v in zk1 zk2; do echo "$v vs base: $(python tools/cmp_c5.py cmp gpurun_out/abm/libwcsde.npz gpurun_out/abm/libwc_sde_large_$v.npz | tr '\n' ' ')"; done
rm -f gpurun_out/abm/*.npz
