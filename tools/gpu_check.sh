#!/bin/bash
# One GPU session: parity tests, smoke, short bench, rocprof kernel trace; optionally the
# reference-precision bench (bench64), the full homogeneous sweep with its statistics against the
# shipped table (sweep) and the CPU baseline against core count (cpu).
#   STEPS="tests smoke bench prof trace pmc bench64 sweep many shards c4shards c5sweep cpu" bash tools/gpu_check.sh
#   trace: kernel trace + stats of the default bench command (C3 + its C5 and fp64 secondary lines;
#          the C5 kernel as an ordinary launch, WCSDE_COOP=0: rocprofv3's teardown faults after a
#          cooperative one)
#   pmc:   every counter set bench.py attaches (tools/profile_bench.sh, profile_f64.sh, profile_c5_all.sh),
#          copied into profiles/ stamped with this library
#   shards / c4shards: the whole-pipeline shard projections of the C3 sweep and the C4 job
#   c5sweep: one 8-GPU rank's C5 shard (2,500 x 1000, full schedule)
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
    trace)
      WCSDE_COOP=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1; rc=$?
      echo "trace rc=$rc"; grep '^{' $OUT/trace.log | cut -c1-200
      find $OUT/trace -name "*kernel_trace.csv" -size +10M -delete
      if [ $rc -ne 0 ]; then echo "STOP after trace"; exit $rc; fi ;;
    pmc)
      bash tools/profile_bench.sh > $OUT/pmc_bench.log 2>&1 || { echo "profile_bench rc=$?"; tail -5 $OUT/pmc_bench.log; exit 1; }
      bash tools/profile_f64.sh > $OUT/pmc_f64.log 2>&1 || { echo "profile_f64 rc=$?"; tail -5 $OUT/pmc_f64.log; exit 1; }
      bash tools/profile_c5_all.sh > $OUT/pmc_c5.log 2>&1 || { echo "profile_c5 rc=$?"; tail -5 $OUT/pmc_c5.log; exit 1; }
      for f in pmc_sde.json pmc_signal.json; do cp gpurun_out/prof/$f profiles/; done
      cp gpurun_out/prof64/pmc_sde_f64.json profiles/
      for f in pmc_sde_c5.json pmc_c5_sq.json pmc_c5_tcc.json; do cp gpurun_out/prof_c5/$f profiles/; done
      mkdir -p $OUT/pmc && cp profiles/pmc_*.json $OUT/pmc/ && echo "pmc ok" ;;
    shards)
      WS="1 2 4 8" OUT=$OUT/shards_homo bash tools/shard_projection.sh > $OUT/shards_homo.log 2>&1; rc=$?
      echo "shards rc=$rc"; tail -4 $OUT/shards_homo.log
      if [ $rc -ne 0 ]; then echo "STOP after shards"; exit $rc; fi ;;
    c4shards)
      MODE="maps --map-ids 1 1 2 2 --seeds 50 --seed0 0" WS="1 2 4 8" OUT=$OUT/shards_c4 bash tools/shard_projection.sh > $OUT/shards_c4.log 2>&1; rc=$?
      echo "c4 shards rc=$rc"; tail -4 $OUT/shards_c4.log
      if [ $rc -ne 0 ]; then echo "STOP after c4shards"; exit $rc; fi ;;
    c5sweep)
      SLURM_ARRAY_TASK_ID=3 SLURM_ARRAY_TASK_MAX=7 timeout -k 10 400 python -u -m nremmodfc_amd.sweep homo --nodes 1000 --out $OUT/c5 > $OUT/c5_shard_sweep.log 2>&1; rc=$?
      echo "c5sweep rc=$rc"; tail -1 $OUT/c5_shard_sweep.log | cut -c1-250
      if [ $rc -ne 0 ]; then echo "STOP after c5sweep"; exit $rc; fi ;;
    cpu)
      timeout -k 10 300 python -u tools/cpu_scaling.py > $OUT/cpu_scaling.log 2>&1; rc=$?
      echo "cpu rc=$rc"; cat $OUT/cpu_scaling.log
      if [ $rc -ne 0 ]; then echo "STOP after cpu"; exit $rc; fi ;;
  esac
done
