#!/bin/bash
# Samples the GPU's power and shader clock (rocm-smi, read-only) while a short bench runs, to see
# whether the integrator runs at the peak clock or below it (power / current limit).
#   bash tools/clock_sample.sh   -> gpurun_out/clock.log (one "t power sclk" line per sample)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/clock.log
: > $OUT
timeout -k 10 300 python3 bench.py --steps 40 --warmup 2 --no-cpu-baseline > gpurun_out/clock_bench.log 2>&1 &
BP=$!
while kill -0 $BP 2>/dev/null; do
  S=$(timeout 10 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Package Power|sclk clock level" | tr -s ' \t' ' ' | tr '\n' ' ')
  echo "$(date +%s.%N) $S" >> $OUT
done
wait $BP
echo "bench rc=$?" >> $OUT
