#!/bin/bash
# Round-3 evidence refresh from one build: C3 PMC (profile_bench.sh), C5 PMC (HBM + SQ passes),
# then the C5 and C3 bench lines that read those profiles (bench.py takes roofline.traffic and the
# C5 SQ figures from profiles/). Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/refresh
bash tools/profile_bench.sh > gpurun_out/refresh/pb.log 2>&1 || { echo "profile_bench rc=$?"; tail -5 gpurun_out/refresh/pb.log; exit 1; }
echo "profile_bench ok"
bash tools/profile_c5.sh > gpurun_out/refresh/pc5.log 2>&1 || { echo "profile_c5 rc=$?"; tail -5 gpurun_out/refresh/pc5.log; exit 1; }
cp gpurun_out/prof_c5/pmc_sde_c5.json profiles/
bash tools/profile_c5_sq.sh > gpurun_out/refresh/pc5sq.log 2>&1 || { echo "profile_c5_sq rc=$?"; tail -5 gpurun_out/refresh/pc5sq.log; exit 1; }
cp gpurun_out/prof_c5sq/pmc_c5_sq.json profiles/
echo "c5 profiles ok"
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/refresh/bench_c5.log 2>&1 || { echo "c5 bench failed"; tail -5 gpurun_out/refresh/bench_c5.log; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/refresh/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/refresh/bench.log; exit 1; }
cp profiles/pmc_sde.json profiles/pmc_signal.json profiles/pmc_sde_c5.json profiles/pmc_c5_sq.json gpurun_out/refresh/
echo done
