export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/r06i
for zs in 0 1; do
  WCSDE_ZSELF=$zs timeout -k 10 200 python tools/time_shard.py 5000,4100,5700 > gpurun_out/r06i/zself$zs.log 2>&1 || { echo "zself $zs rc=$?"; exit 1; }
  echo "ZSELF=$zs"; grep B= gpurun_out/r06i/zself$zs.log
done
WCSDE_ZSELF=1 timeout -k 10 300 python -u -m pytest tests/test_sde_gpu.py -k "precomputed_normals" -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06i/pytest.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/r06i/pytest.log
