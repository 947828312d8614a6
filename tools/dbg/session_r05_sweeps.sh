# Round-5 end-to-end sweeps on the final library: one 8-GPU rank's C5 shard (2,500 x 1000, full
# schedule) and the full C3 homogeneous sweep, each with its per-cell table kept
set -u
export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/r05sw
mkdir -p $O
SLURM_ARRAY_TASK_ID=3 SLURM_ARRAY_TASK_MAX=7 timeout -k 10 400 python -u -m nremmodfc_amd.sweep homo --nodes 1000 --out $O/c5 > $O/c5_shard_sweep.log 2>&1 || { echo "c5 rc=$?"; tail -5 $O/c5_shard_sweep.log; exit 1; }
tail -1 $O/c5_shard_sweep.log | cut -c1-250
timeout -k 10 300 python -u -m nremmodfc_amd.sweep homo --out $O/homo > $O/homo_sweep.log 2>&1 || { echo "homo rc=$?"; tail -5 $O/homo_sweep.log; exit 1; }
tail -1 $O/homo_sweep.log | cut -c1-250
f=$(ls $O/homo/*.txt | head -1)
timeout -k 10 300 python tools/validate_stats.py "$f" homo $O/homo_stats.json > $O/homo_val.log 2>&1; echo "validate rc=$?"; tail -6 $O/homo_val.log
ls $O/c5
