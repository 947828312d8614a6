#!/bin/bash
# Round-3 final evidence on one box: the whole GPU suite, smoke, then the full homogeneous C3 sweep
# (whole_sweep_both.py on the shipped grid, 20,000 x 90, 1001 s) validated cell by cell against the
# reference's shipped table. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/final; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -m nremmodfc_amd.sweep homo --out $OUT/homo > $OUT/homo.log 2>&1 || { echo "sweep failed"; tail -5 $OUT/homo.log; exit 1; }
tail -1 $OUT/homo.log | cut -c1-300
f=$(ls $OUT/homo/*.txt | head -1)
timeout -k 10 300 python tools/validate_stats.py "$f" homo $OUT/homo_stats.json > $OUT/homo_val.log 2>&1 || { echo "validate failed"; tail -5 $OUT/homo_val.log; exit 1; }
tail -16 $OUT/homo_val.log
