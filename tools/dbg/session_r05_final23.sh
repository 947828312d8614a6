# Round-5 final evidence, parts 2 + 3 in one call: PMC of the three bench lines on the library the
# bench loads, then the three bench lines again with those counters attached
set -u
export TMPDIR=/tmp PYTHONPATH=.
bash tools/dbg/session_r05_final2.sh || exit 1
for f in pmc_sde.json pmc_signal.json; do cp gpurun_out/prof/$f profiles/; done
cp gpurun_out/prof64/pmc_sde_f64.json profiles/
for f in pmc_sde_c5.json pmc_c5_sq.json pmc_c5_tcc.json; do cp gpurun_out/prof_c5/$f profiles/; done
O=gpurun_out/r05f3
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 600 python bench.py --config c5 > $O/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -5 $O/bench_c5.log; exit 1; }
timeout -k 10 600 python bench.py --precision f64 > $O/bench_f64.log 2>&1 || { echo "bench f64 failed"; tail -5 $O/bench_f64.log; exit 1; }
for f in bench_c3 bench_c5 bench_f64; do echo "$f: $(grep '^{' $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['kernel_ms'], r['frac'], r.get('pmc_lib_sha256'), r.get('pmc_refused'), (d.get('cpu_baseline') or {}).get('value'))")"; done
