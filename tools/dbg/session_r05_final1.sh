# Round-5 final evidence, part 1: GPU test suite, smoke, the three bench lines (C3 with its CPU
# baseline, C5 with its N = 1000 CPU baseline, fp64) and the kernel traces of the same commands
set -u
export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/r05f1
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -5 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 600 python bench.py --config c5 > $O/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -5 $O/bench_c5.log; exit 1; }
timeout -k 10 600 python bench.py --precision f64 --no-cpu-baseline > $O/bench_f64.log 2>&1 || { echo "bench f64 failed"; tail -5 $O/bench_f64.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o b -- python3 bench.py --no-cpu-baseline > $O/trace_c3.log 2>&1 || { echo "trace c3 rc=$?"; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_f64 -o b -- python3 bench.py --precision f64 --no-cpu-baseline > $O/trace_f64.log 2>&1 || { echo "trace f64 rc=$?"; exit 1; }
WCSDE_COOP=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o b -- python3 bench.py --config c5 --no-cpu-baseline > $O/trace_c5.log 2>&1 || { echo "trace c5 rc=$?"; exit 1; }
find $O -name "*kernel_trace.csv" -size +10M -delete
for f in bench_c3 bench_c5 bench_f64; do echo "$f: $(grep '^{' $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernel_ms'], d['roofline']['frac'])")"; done
