"""C5 shard (2,500 x 1000) integrator: us per step under environment variants, interleaved.

Each argument is one variant, a comma-separated list of VAR=VALUE settings applied for its runs
(e.g. WCSDE_PERSISTENT=2 with the diag build selects an ablation; WCSDE_PMAP=4 an XCD placement).
E is recorded every 20 steps time-major, as the fp32 pipeline does.  Variants that run product
arithmetic (no WCSDE_PERSISTENT=2..5) must give the first such variant's state bit for bit.

  PYTHONPATH=. python tools/time_c5.py [--steps S] [--reps R] VAR=V[,VAR=V] ...
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, sim_keys  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--B", type=int, default=2500)
    ap.add_argument("variants", nargs="*", default=["WCSDE_PERSISTENT=1"])
    args = ap.parse_args()
    N, B, steps = 1000, args.B, args.steps
    sc = datasets.synthetic_sc(N)
    rng = np.random.default_rng(0)
    G = 0.16 + rng.uniform(-0.1, 0.3, B)
    S = 7.68 + rng.uniform(-0.2, 0.2, B)
    keys = sim_keys(np.arange(B) % 50, np.arange(B) // 50)
    tmaj = torch.empty((steps // 20, B, N), dtype=torch.float32, device="cuda")
    ref = None
    for rep in range(args.reps):
        for var in args.variants:
            env = dict(kv.split("=", 1) for kv in var.split(",") if kv)
            old = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            b = Batch(sc, G, S, keys, precision="f32")
            b.integrate(20, 0.05)
            torch.cuda.synchronize()
            t = time.perf_counter()
            b.integrate(steps, 2.0, 20, tmaj)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t
            product = env.get("WCSDE_PERSISTENT", "1") in ("0", "1")
            same = ""
            if product:
                st = torch.stack([b.E, b.I, b.A])
                if ref is None:
                    ref = (st, tmaj.clone())
                same = f", bit-identical={torch.equal(st, ref[0]) and torch.equal(tmaj, ref[1])}"
            print(f"rep {rep} [{var}]: {dt / steps * 1e6:.2f} us/step, {B * N * steps / dt:.3e} node-steps/s{same}",
                  flush=True)
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            del b


if __name__ == "__main__":
    main()
