"""Bit-compare and time the N > 96 persistent integrator of two builds of libwcsde.so (one process per
library, WCSDE_LIB_OVERRIDE selects it) at the C5 shard (2,500 x 1000, ring records every 20 steps).
python tools/cmp_c5.py save OUT.npz | cmp A.npz B.npz"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(out):
    import torch
    from nremmodfc_amd import datasets
    from nremmodfc_amd.model import Batch, sim_keys
    N, B, steps = 1000, 2500, 4000
    sc = datasets.synthetic_sc(N)
    rng = np.random.default_rng(0)
    G = 0.16 + rng.uniform(-0.1, 0.3, B)
    S = 7.68 + rng.uniform(-0.2, 0.2, B)
    keys = sim_keys(np.arange(B) % 50, np.arange(B) // 50)
    ring = torch.empty(B * N * (steps // 20), dtype=torch.float32, device="cuda")
    times = []
    for rep in range(3):
        b = Batch(sc, G, S, keys, precision="f32")
        b.integrate(20, 0.05)
        torch.cuda.synchronize()
        t = time.perf_counter()
        b.integrate(steps, 2.0, 20, ring, rec_ld=steps // 20)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
    print(f"C5 shard: {min(times) / steps * 1e6:.2f} us/step (runs {', '.join(f'{x / steps * 1e6:.2f}' for x in times)})",
          flush=True)
    np.savez(out, E=b.E.cpu().numpy(), I=b.I.cpu().numpy(), A=b.A.cpu().numpy(),
             ring=ring.view(B * N, -1)[::97].cpu().numpy())


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in x.files:
        same = np.array_equal(x[k], y[k])
        print(k, "identical" if same else f"DIFFER max|d| {np.nanmax(np.abs(x[k] - y[k])):.3e}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3])
