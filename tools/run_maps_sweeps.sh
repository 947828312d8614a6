#!/bin/bash
# Full-length map and shuffled heterogeneity sweeps (whole_sweep_both_maps.py, map ids 1 1 and 2 2) on one
# GPU, each validated cell by cell against the reference's shipped tables (tools/validate_stats.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mapsw
mkdir -p $OUT
for ids in "1 1" "2 2"; do
  kind=$([ "$ids" = "1 1" ] && echo maps || echo shuf)
  timeout -k 10 400 python -m nremmodfc_amd.sweep maps --map-ids $ids --out $OUT/$kind > $OUT/$kind.log 2>&1 || exit $?
  tail -1 $OUT/$kind.log | cut -c1-300
  f=$(ls $OUT/$kind/*.txt | head -1)
  timeout -k 10 300 python tools/validate_stats.py "$f" $kind $OUT/${kind}_stats.json > $OUT/${kind}_val.log 2>&1 || exit $?
  tail -16 $OUT/${kind}_val.log
done
