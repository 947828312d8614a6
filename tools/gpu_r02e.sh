#!/bin/bash
# round-2 evidence e: config 5 end to end (one 8-GPU rank's shard of the 1000-node sweep, full
# schedule, through the SLURM-array path), config 2 at full size, the strong-scaling bench path
# rehearsed with two gloo ranks on the one GPU
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5 gpurun_out/c2
SLURM_ARRAY_TASK_ID=3 SLURM_ARRAY_TASK_MAX=7 timeout -k 10 700 python -u -m nremmodfc_amd.sweep homo --nodes 1000 \
    --out gpurun_out/c5 --tag c5_n1000 > gpurun_out/c5/log.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c5/log.txt | tail -3 | cut -c1-600; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m nremmodfc_amd.sweep many --modality map --out gpurun_out/c2 --tag c2_map > gpurun_out/c2/log.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/c2/log.txt | tail -2 | cut -c1-400; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --scaling strong --dist-backend gloo --steps 3 --warmup 1 > gpurun_out/strong2.log 2>&1; rc=$?
grep '^{' gpurun_out/strong2.log | cut -c1-500; exit $rc
