#!/bin/bash
# final-build whole sweeps: the homogeneous C3 sweep and the shuffled-map sweep, each validated
# cell by cell against the shipped tables
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/v
mkdir -p $OUT
timeout -k 10 400 python -u -m nremmodfc_amd.sweep homo --out $OUT/homo > $OUT/homo.log 2>&1 || { tail -5 $OUT/homo.log; exit 1; }
grep -v amdgpu.ids $OUT/homo.log | tail -1 | cut -c1-300
f=$(ls $OUT/homo/*.txt | head -1)
timeout -k 10 300 python tools/validate_stats.py "$f" homo $OUT/homo_stats.json > $OUT/homo_val.log 2>&1 || exit 1
tail -16 $OUT/homo_val.log
gzip -c "$f" > $OUT/homo_sweep.txt.gz
timeout -k 10 400 python -u -m nremmodfc_amd.sweep maps --map-ids 2 2 --out $OUT/shuf > $OUT/shuf.log 2>&1 || { tail -5 $OUT/shuf.log; exit 1; }
grep -v amdgpu.ids $OUT/shuf.log | tail -1 | cut -c1-300
f=$(ls $OUT/shuf/*.txt | head -1)
timeout -k 10 300 python tools/validate_stats.py "$f" shuf $OUT/shuf_stats.json > $OUT/shuf_val.log 2>&1 || exit 1
tail -3 $OUT/shuf_val.log
rm -rf $OUT/homo $OUT/shuf
