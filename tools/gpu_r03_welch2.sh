#!/bin/bash
# Two-segment Welch launches: their tests, the pipeline/statistics tests that run through them, and
# the bench line (Welch per segment).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/w2; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_signal_gpu.py tests/test_stats_gpu.py tests/test_fullsize_gpu.py tests/test_large_n_gpu.py tests/test_sweep.py > $OUT/t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $OUT/t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail -5 $OUT/bench.log; exit 1; }
python -c "
import json;d=json.loads([l for l in open('$OUT/bench.log') if l.startswith('{')][-1]);print(d['value'], d['ms_per_step'], d['kernel_ms'])"
