set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
[ -n "$SKIPT" ] || timeout -k 10 300 python -u -m pytest tests/test_signal_gpu.py tests/test_facades_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sig.log 2>&1; rc=$?; tail -5 gpurun_out/t_sig.log; [ $rc -ne 0 ] && exit $rc
PYTHONPATH=. timeout -k 10 120 python tools/time_bold.py 20000 > gpurun_out/tb.log 2>&1 && cat gpurun_out/tb.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; tail -1 gpurun_out/bench.log | cut -c1-300; grep -o '"kernel_ms.*' gpurun_out/bench.log; exit $rc
