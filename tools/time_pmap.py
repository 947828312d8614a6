"""Persistent C5 integrator: us per step for each XCD placement (WCSDE_PMAP = node blocks per XCD;
0 = plain order), and the final state must not depend on the placement."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, sim_keys  # noqa: E402


def main():
    N, B = 1000, int(sys.argv[1]) if len(sys.argv) > 1 else 2500
    steps = 4000
    sc = datasets.synthetic_sc(N)
    rng = np.random.default_rng(0)
    G = 0.16 + rng.uniform(-0.1, 0.3, B)
    S = 7.68 + rng.uniform(-0.2, 0.2, B)
    keys = sim_keys(np.arange(B) % 50, np.arange(B) // 50)
    ring = torch.empty(B * N * (steps // 20), dtype=torch.float32, device="cuda")
    ref = None
    for rep in range(int(os.environ.get("REPS", "2"))):
        for pm in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,4,8").split(","):
            os.environ["WCSDE_PMAP"] = pm
            b = Batch(sc, G, S, keys, precision="f32")
            b.integrate(20, 0.05)
            torch.cuda.synchronize()
            t = time.perf_counter()
            b.integrate(steps, 2.0, 20, ring, rec_ld=steps // 20)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            st = torch.stack([b.E, b.I, b.A])
            same = ref is None or torch.equal(st, ref)
            ref = st if ref is None else ref
            print(f"rep {rep} pmap {pm}: {dt / steps * 1e6:.2f} us/step, {B * N * steps / dt:.3e} node-steps/s, "
                  f"same={same}", flush=True)
            assert same or os.environ.get("WCSDE_PERSISTENT", "1") != "1"  # 2..5: diag-build ablations


if __name__ == "__main__":
    main()
