# Pipeline A/B: BOLD + Welch of chunk k on a second stream beside the integrator's chunk k + 1
# (WCSDE_PIPE_OVERLAP=1, default) vs one stream; whole-pipeline shard walls, bit-identical tables
export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fullsize_gpu.py tests/test_signal_gpu.py tests/test_sweep.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
for ov in 1 0; do
  WCSDE_PIPE_OVERLAP=$ov WS="1 4 8" OUT=$O/homo$ov bash tools/shard_projection.sh > $O/homo$ov.log 2>&1 || { echo "homo $ov failed"; exit 1; }
  WCSDE_PIPE_OVERLAP=$ov MODE="maps --map-ids 1 1 2 2 --seeds 50 --seed0 0" WS="8" OUT=$O/c4$ov bash tools/shard_projection.sh > $O/c4$ov.log 2>&1 || { echo "c4 $ov failed"; exit 1; }
  echo "overlap=$ov"; grep '"W"' $O/homo$ov.log | cut -c1-75; grep '"W"' $O/c4$ov.log | cut -c1-75
done
for W in 1 4 8; do
  a=$(ls $O/homo1/w$W/*.txt); b=$(ls $O/homo0/w$W/*.txt); cmp -s "$a" "$b" && echo "W=$W tables identical" || echo "W=$W tables DIFFER"
done
