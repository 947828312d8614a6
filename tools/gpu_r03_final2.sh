#!/bin/bash
# Round-3 closing evidence on one box: the GPU suite, smoke, PMC passes of the bench (profile_bench.sh,
# which also writes profiles/pmc_*.json for the bench line that follows), the bench line with its CPU
# baseline, and a rocprofv3 kernel trace of a short bench run. Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/final2; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/profile_bench.sh > $OUT/pb.log 2>&1 || { echo "profile_bench failed"; tail -5 $OUT/pb.log; exit 1; }
cp profiles/pmc_sde.json profiles/pmc_signal.json $OUT/
timeout -k 10 600 python bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -c 300 $OUT/bench.log
