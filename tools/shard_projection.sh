#!/bin/bash
# Whole-pipeline strong-scaling projection of the C3 sweep (whole_sweep_both.py:60-64's round robin),
# measured on ONE GPU: for W = 1, 2, 4, 8 (and 16) the full homogeneous sweep's rank-0 shard
# (20,000 / W simulations, the full 1001 s schedule, BOLD / band-pass / Welch / FC / metrics
# included) runs as SLURM-array task 0 of W; each task prints its wall time (the perf JSON line).
# The W-GPU sweep time is the slowest shard's time (the shards are equal to one simulation), so
# the projected speed-up at W is t(1) / t(W).  Not a SCALE run: one GPU, one shard at a time.
# MODE="maps --map-ids 1 1" (or "2 2") projects the C4 heterogeneity sweeps the same way.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
MODE=${MODE:-homo}
OUT=${OUT:-gpurun_out/shards}
export OUT
mkdir -p $OUT
for W in ${WS:-1 2 4 8 16}; do
  rm -rf $OUT/w$W
  SLURM_ARRAY_TASK_ID=0 SLURM_ARRAY_TASK_MAX=$((W - 1)) timeout -k 10 300 \
    python -m nremmodfc_amd.sweep $MODE --out $OUT/w$W > $OUT/w$W.log 2>&1
  rc=$?
  echo "W=$W rc=$rc $(grep -h '"wall_s"' $OUT/w$W.log | tail -1 | cut -c1-200)"
  [ $rc -ne 0 ] && exit $rc
done
python3 - <<'PY'
import json, glob, os
rows = []
out = os.environ["OUT"]
for f in sorted(glob.glob(os.path.join(out, "w*.log")), key=lambda p: int(p.split("w")[-1].split(".")[0])):
    W = int(f.split("w")[-1].split(".")[0])
    d = [json.loads(l) for l in open(f) if l.startswith("{") and '"wall_s"' in l][-1]
    rows.append((W, d["sims"], d["wall_s"], d["node_steps_per_s"]))
t1 = rows[0][2] if rows and rows[0][0] == 1 else None
for W, sims, wall, rate in rows:
    sp = t1 / wall if t1 else float("nan")
    print(json.dumps({"W": W, "shard_sims": sims, "shard_wall_s": round(wall, 3), "per_gpu_node_steps_per_s": rate,
                      "projected_W_gpu_node_steps_per_s": rate * W, "projected_speedup": round(sp, 3),
                      "efficiency": round(sp / W, 3)}))
PY
