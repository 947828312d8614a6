#!/bin/bash
# Full-horizon fixed-seed FC parity on the GPU box: fp64, fp64 perturbed, fp32 pipelines on the 32 keys of
# tests/golden/ref_replay_full.npz -> gpurun_out/fc_horizon_gpu.npz (report: tools/fc_horizon_report.py, here)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python -u tools/fc_horizon_gpu.py gpurun_out/fc_horizon_gpu.npz
