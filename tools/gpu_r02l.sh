#!/bin/bash
# round-2 sweep evidence on the final build: strong-scaling shard rates, the full homogeneous C3 sweep
# and the map / shuffled sweeps, each validated cell by cell against the shipped tables
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/sw
mkdir -p $OUT
PYTHONPATH=. timeout -k 10 200 python -u tools/time_shard.py > $OUT/shard.log 2>&1 || { cat $OUT/shard.log; exit 1; }
grep -v amdgpu.ids $OUT/shard.log
timeout -k 10 400 python -u -m nremmodfc_amd.sweep homo --out $OUT/homo > $OUT/homo.log 2>&1 || { tail -5 $OUT/homo.log; exit 1; }
grep -v amdgpu.ids $OUT/homo.log | tail -1 | cut -c1-400
f=$(ls $OUT/homo/*.txt | head -1)
timeout -k 10 300 python tools/validate_stats.py "$f" homo $OUT/homo_stats.json > $OUT/homo_val.log 2>&1 || exit 1
tail -16 $OUT/homo_val.log
for ids in "1 1" "2 2"; do
  kind=$([ "$ids" = "1 1" ] && echo maps || echo shuf)
  timeout -k 10 400 python -u -m nremmodfc_amd.sweep maps --map-ids $ids --out $OUT/$kind > $OUT/$kind.log 2>&1 || exit 1
  grep -v amdgpu.ids $OUT/$kind.log | tail -1 | cut -c1-300
  f=$(ls $OUT/$kind/*.txt | head -1)
  timeout -k 10 300 python tools/validate_stats.py "$f" $kind $OUT/${kind}_stats.json > $OUT/${kind}_val.log 2>&1 || exit 1
  tail -3 $OUT/${kind}_val.log
done
