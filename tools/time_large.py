"""Time the N > 96 integrator (wc_sde_large.hip) on the C5 shape: node-steps/s."""
import sys
import time

import numpy as np
import torch

from nremmodfc_amd import datasets
from nremmodfc_amd.model import Batch, sim_keys


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    Bs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else (2500, 5000, 20000)
    for B in Bs:
        sc = datasets.synthetic_sc(N)
        rng = np.random.default_rng(0)
        G = 0.16 + rng.uniform(-0.1, 0.3, B)
        S = 7.68 + rng.uniform(-0.2, 0.2, B)
        b = Batch(sc, G, S, sim_keys(np.arange(B) % 50, np.arange(B) // 50), precision="f32")
        b.integrate(20, 0.05)
        steps = 400 if B <= 5000 else 100
        ring = torch.empty(B * N * 64, dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        t = time.perf_counter()
        b.integrate(steps, 2.0, 20, ring, rec_ld=64)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        flops = 2 * N + 35
        print(f"N={N} B={B}: {dt / steps * 1e6:.1f} us/step, {B * N * steps / dt:.3e} node-steps/s, "
              f"{B * N * steps * flops / dt / 1e12:.1f} TFLOP/s algorithmic", flush=True)
        assert torch.isfinite(b.E).all()


if __name__ == "__main__":
    main()
