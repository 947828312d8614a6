#!/bin/bash
# checkpoint of the tree as committed: the whole GPU suite, smoke(), the default bench line
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/y
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1; rc=$?
tail -1 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py > $OUT/bench.log 2>&1; rc=$?
grep -v amdgpu.ids $OUT/bench.log | tail -1 | cut -c1-300; exit $rc
