"""Integrator rate at the per-GPU shard sizes of an N-GPU strong-scaling C3 sweep
(20,000 simulations / N): B = 20000, 10000, 5000, 2500, recording every 20 steps."""
import sys
import time

import torch

from bench import sweep_batch
from nremmodfc_amd import datasets
from nremmodfc_amd.model import Batch, driver_params

sc = datasets.load_sc()
G, S, keys = sweep_batch(0)
for B in [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "20000,10000,5000,2500".split(","))]:
    bt = Batch(sc, G[:B], S[:B], keys[:B], driver_params(), precision="f32")
    rec = torch.empty((1000, B, 90), dtype=torch.float32, device="cuda")
    bt.integrate(2000, 2.0, 20, rec[:100])
    torch.cuda.synchronize()
    t = time.perf_counter()
    bt.integrate(20000, 2.0, 20, rec)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    print(f"B={B}: {dt / 20000 * 1e6:.2f} us/step, {B * 90 * 20000 / dt:.3e} node-steps/s", flush=True)
