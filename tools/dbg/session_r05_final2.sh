# Round-5 final evidence, part 2: PMC of the three bench lines on the library the bench loads
set -u
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out
bash tools/profile_bench.sh > gpurun_out/r05_prof_bench.log 2>&1 || { echo "profile_bench rc=$?"; tail -5 gpurun_out/r05_prof_bench.log; exit 1; }
bash tools/profile_f64.sh > gpurun_out/r05_prof_f64.log 2>&1 || { echo "profile_f64 rc=$?"; tail -5 gpurun_out/r05_prof_f64.log; exit 1; }
bash tools/profile_c5_all.sh > gpurun_out/r05_prof_c5.log 2>&1 || { echo "profile_c5 rc=$?"; tail -5 gpurun_out/r05_prof_c5.log; exit 1; }
echo done; ls gpurun_out/prof gpurun_out/prof64 gpurun_out/prof_c5
