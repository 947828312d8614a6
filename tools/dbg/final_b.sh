# Closing check of the round: the whole GPU suite, smoke and the default bench as the driver runs them
set -u
export TMPDIR=/tmp
O=gpurun_out/r06fb
mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -5 $O/bench.log; exit 1; }
grep '^{' $O/bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])
for k,v in d['secondary'].items(): print(k, v['value'], v['ms_per_step'], v['kernel_ms'], v['roofline']['frac'])"
