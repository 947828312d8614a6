# C5 persistent kernel: cooperative launch (the product) vs the ordinary launch of the same grid the
# PMC passes use (WCSDE_COOP=0), alternated, no profiler: the ms per 20,000-step launch of each
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/r06l
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06l/coop$r.log 2>&1 || exit 1
  WCSDE_COOP=0 timeout -k 10 300 python bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r06l/plain$r.log 2>&1 || exit 1
  for v in coop plain; do
    python - gpurun_out/r06l/$v$r.log $v <<'PY'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[2], "ms_per_step", d["ms_per_step"], "kernel_ms", d.get("kernel_ms"))
PY
  done
done
