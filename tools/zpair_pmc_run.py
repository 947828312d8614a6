#!/usr/bin/env python3
"""The 4-GPU C3 shard (5,000 simulations = 313 groups: the V_ZPAIR integrator) for rocprofv3 --pmc passes:
STEPS Euler steps recording every 20th time-major, as the sweep pipeline does (2 launches of 1000 steps
for STEPS = 2000, after one warm-up block).

  rocprofv3 --pmc <counters> -- python3 tools/zpair_pmc_run.py 2000"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, driver_params  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    B = int(os.environ.get("ZP_B", "5000"))
    G, S, keys = bench.sweep_batch(0)
    bt = Batch(datasets.load_sc(), G[:B], S[:B], keys[:B], driver_params(), precision="f32")
    rec = torch.empty((steps // 20, B, 90), dtype=torch.float32, device="cuda")
    bt.integrate(steps, 2.0, 20, rec)
    torch.cuda.synchronize()
    print("ok", B, steps)


if __name__ == "__main__":
    main()
