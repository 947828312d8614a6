"""C5 shard (2,500 x 1000) persistent integrator: us per step with E recorded every 20 steps into a
node-major ring, into a time-major buffer (the pipeline's fp32 layout), and with no records."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, sim_keys  # noqa: E402


def main():
    N, B, steps = 1000, 2500, 4000
    sc = datasets.synthetic_sc(N)
    rng = np.random.default_rng(0)
    G = 0.16 + rng.uniform(-0.1, 0.3, B)
    S = 7.68 + rng.uniform(-0.2, 0.2, B)
    keys = sim_keys(np.arange(B) % 50, np.arange(B) // 50)
    ring = torch.empty(B * N * (steps // 20), dtype=torch.float32, device="cuda")
    tmaj = torch.empty((steps // 20, B, N), dtype=torch.float32, device="cuda")
    for rep in range(2):
        for mode in ("ring", "tmaj", "none"):
            b = Batch(sc, G, S, keys, precision="f32")
            b.integrate(20, 0.05)
            torch.cuda.synchronize()
            t = time.perf_counter()
            if mode == "ring":
                b.integrate(steps, 2.0, 20, ring, rec_ld=steps // 20)
            elif mode == "tmaj":
                b.integrate(steps, 2.0, 20, tmaj)
            else:
                b.integrate(steps, 2.0)
            torch.cuda.synchronize()
            print(f"rep {rep} {mode}: {(time.perf_counter() - t) / steps * 1e6:.2f} us/step", flush=True)


if __name__ == "__main__":
    main()
