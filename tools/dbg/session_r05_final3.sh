# Round-5 final evidence, part 3: the three bench lines with the refreshed PMC attached (and the fp64
# line with its CPU baseline), then the C4 maps sweep's whole-pipeline shard projection (W = 1, 2, 4, 8)
set -u
export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/r05f3
mkdir -p $O
timeout -k 10 600 python bench.py > $O/bench_c3.log 2>&1 || { echo "bench c3 failed"; tail -5 $O/bench_c3.log; exit 1; }
timeout -k 10 600 python bench.py --config c5 > $O/bench_c5.log 2>&1 || { echo "bench c5 failed"; tail -5 $O/bench_c5.log; exit 1; }
timeout -k 10 600 python bench.py --precision f64 > $O/bench_f64.log 2>&1 || { echo "bench f64 failed"; tail -5 $O/bench_f64.log; exit 1; }
for f in bench_c3 bench_c5 bench_f64; do echo "$f: $(grep '^{' $O/$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['kernel_ms'], r['frac'], r.get('pmc_lib_sha256'), r.get('pmc_refused'), (d.get('cpu_baseline') or {}).get('value'))")"; done
MODE="maps --map-ids 1 1" WS="1 2 4 8" OUT=gpurun_out/shards_maps bash tools/shard_projection.sh > $O/shards_maps.log 2>&1; echo "maps shards rc=$?"; tail -5 $O/shards_maps.log
