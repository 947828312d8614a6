#!/bin/bash
# mixed-tile waves for three groups per CU (V_MIX): bit-compare against the same build without it,
# shard rates, the GPU suite, and the map sweep validated against the shipped table
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/t
mkdir -p $OUT
for v in nomix prod; do
  L=$PWD/tools/dbg/libwcsde_nomix.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/cmp_libs.py save $OUT/sde_$v.npz > $OUT/sde_$v.log 2>&1 || { tail -5 $OUT/sde_$v.log; exit 1; }
  WCSDE_LIB_OVERRIDE=$L timeout -k 10 200 python -u tools/time_shard.py 20000,10000,9000,12000 > $OUT/shard_$v.log 2>&1 || { tail -5 $OUT/shard_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/sde_$v.log | grep "N=90"; grep -v amdgpu.ids $OUT/shard_$v.log
done
python tools/cmp_libs.py cmp $OUT/sde_nomix.npz $OUT/sde_prod.npz; echo "== cmp rc=$?"
rm -f $OUT/*.npz
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m nremmodfc_amd.sweep maps --map-ids 1 1 --out $OUT/maps > $OUT/maps.log 2>&1 || { tail -5 $OUT/maps.log; exit 1; }
grep -v amdgpu.ids $OUT/maps.log | tail -1 | cut -c1-300
f=$(ls $OUT/maps/*.txt | head -1)
timeout -k 10 300 python tools/validate_stats.py "$f" maps $OUT/maps_stats.json > $OUT/maps_val.log 2>&1 || exit 1
tail -3 $OUT/maps_val.log
