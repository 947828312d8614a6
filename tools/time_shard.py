"""Integrator rate at the per-GPU shard sizes of an N-GPU strong-scaling C3 sweep
(20,000 simulations / N): B = 20000, 10000, 5000, 2500, 1250, recording every 20 steps.
Small shards run with the normals precomputed on the idle CUs (V_ZMEM) unless WCSDE_ZMEM=0;
each shard is also run with WCSDE_ZMEM=0 and the two trajectories are compared bit for bit.

  PYTHONPATH=. python tools/time_shard.py [B,B,...]"""
import os
import sys
import time

import torch

from bench import sweep_batch
from nremmodfc_amd import datasets
from nremmodfc_amd.model import Batch, driver_params

sc = datasets.load_sc()
G, S, keys = sweep_batch(0)
for B in [int(x) for x in (sys.argv[1].split(",") if len(sys.argv) > 1 else "20000,10000,5000,2500,1250".split(","))]:
    res = {}
    for zm in ("1", "0"):
        os.environ["WCSDE_ZMEM"] = zm
        bt = Batch(sc, G[:B], S[:B], keys[:B], driver_params(), precision="f32")
        rec = torch.empty((1000, B, 90), dtype=torch.float32, device="cuda")
        bt.integrate(2000, 2.0, 20, rec[:100])
        torch.cuda.synchronize()
        best = 1e9
        for _ in range(2):
            t = time.perf_counter()
            bt.integrate(20000, 2.0, 20, rec)
            torch.cuda.synchronize()
            best = min(best, time.perf_counter() - t)
        res[zm] = (best, rec.clone(), bt.E.clone())
        del bt, rec
    (d1, r1, e1), (d0, r0, e0) = res["1"], res["0"]
    same = torch.equal(r1, r0) and torch.equal(e1, e0)
    print(f"B={B}: {d1 / 20000 * 1e6:.3f} us/step ({B * 90 * 20000 / d1:.3e} node-steps/s); WCSDE_ZMEM=0 "
          f"{d0 / 20000 * 1e6:.3f} us/step; bit-identical: {same}", flush=True)
os.environ.pop("WCSDE_ZMEM", None)
