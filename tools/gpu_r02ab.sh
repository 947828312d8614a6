#!/bin/bash
# C5 own-block-first K order with the hand-off wait after the own chunks (WC_OWNFIRST): us/step against the session-start build,
# the N > 96 suites (bit-exact persistent vs step kernel), then the C5 bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/of
mkdir -p $OUT
for v in noown prod; do
  L=$PWD/tools/dbg/libwcsde_noown.so; [ $v = prod ] && L=$PWD/nremmodfc_amd/libwcsde.so
  REPS=2 WCSDE_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/time_pmap.py 2500 4 > $OUT/pmap_$v.log 2>&1 || { tail -5 $OUT/pmap_$v.log; exit 1; }
  echo "== pmap $v"; grep -v amdgpu.ids $OUT/pmap_$v.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_sde_large_gpu.py tests/test_large_n_gpu.py > $OUT/t.log 2>&1 || { tail -30 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 > $OUT/bench_c5.log 2>&1 || { tail -5 $OUT/bench_c5.log; exit 1; }
grep -v amdgpu.ids $OUT/bench_c5.log | cut -c1-250; grep -o '"kernel_ms": {[^}]*}' $OUT/bench_c5.log
