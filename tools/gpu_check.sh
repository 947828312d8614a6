#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprof kernel trace; optionally the
# reference-precision bench (bench64), the full homogeneous sweep with its statistics against the
# shipped table (sweep) and the CPU baseline against core count (cpu).
#   STEPS="tests smoke bench prof bench64 sweep many cpu" bash tools/gpu_check.sh
# OUT (default gpurun_out) names the output directory; TESTS selects the pytest targets.
# Stops at the first crash/timeout (exit codes other than 0/1 from pytest).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
mkdir -p $OUT
STEPS="${STEPS:-tests smoke bench prof}"
fatal() { local rc=$1; [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -q -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
      echo "pytest gpu rc=$rc"; tail -25 $OUT/pytest_gpu.log
      if fatal $rc; then echo "STOP after tests"; exit $rc; fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
      echo "smoke rc=$rc"; tail -5 $OUT/smoke.log
      if [ $rc -ne 0 ]; then echo "STOP after smoke"; exit $rc; fi ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; rc=$?
      echo "bench rc=$rc"; tail -5 $OUT/bench.log
      if [ $rc -ne 0 ]; then echo "STOP after bench"; exit $rc; fi ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o sde -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1; rc=$?
      echo "prof rc=$rc"; tail -3 $OUT/prof.log; find $OUT/prof -name "*stats*" | head
      if [ $rc -ne 0 ]; then echo "STOP after prof"; exit $rc; fi ;;
    bench64)
      # the reference-precision line (fp64 throughout) with its kernel trace
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof64 -o f64 -- python3 bench.py --precision f64 --steps ${STEPS64:-2} --warmup 1 --no-cpu-baseline > $OUT/bench64.log 2>&1; rc=$?
      echo "bench64 rc=$rc"; tail -3 $OUT/bench64.log
      if [ $rc -ne 0 ]; then echo "STOP after bench64"; exit $rc; fi ;;
    sweep)
      timeout -k 10 600 python -m nremmodfc_amd.sweep homo --out $OUT/homo > $OUT/homo.log 2>&1; rc=$?
      echo "sweep rc=$rc"; tail -1 $OUT/homo.log | cut -c1-300
      if [ $rc -ne 0 ]; then echo "STOP after sweep"; exit $rc; fi
      f=$(ls $OUT/homo/*.txt | head -1)
      timeout -k 10 300 python tools/validate_stats.py "$f" homo $OUT/homo_stats.json > $OUT/homo_val.log 2>&1 || { echo "validate failed"; tail -5 $OUT/homo_val.log; exit 1; }
      tail -16 $OUT/homo_val.log ;;
    many)
      # run_many_seeds.py (C2): 50 seeds x 4 states with device HMA -> the pickle the consumers read
      timeout -k 10 300 python -m nremmodfc_amd.sweep many --modality ${MODALITY:-homo} --out $OUT/many > $OUT/many.log 2>&1; rc=$?
      echo "many rc=$rc"; tail -1 $OUT/many.log | cut -c1-300
      if [ $rc -ne 0 ]; then echo "STOP after many"; exit $rc; fi ;;
    cpu)
      timeout -k 10 300 python -u tools/cpu_scaling.py > $OUT/cpu_scaling.log 2>&1; rc=$?
      echo "cpu rc=$rc"; cat $OUT/cpu_scaling.log
      if [ $rc -ne 0 ]; then echo "STOP after cpu"; exit $rc; fi ;;
  esac
done
