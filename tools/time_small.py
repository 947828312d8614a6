#!/usr/bin/env python3
"""Small-batch (strong-scaling shard) integrator variants of the diag build:
us per Euler step at B = 20,000 / N_gpus for several kernel configurations, with
time-major records every 20 steps (the pipeline's layout), interleaved rounds.

  python tools/time_small.py [variants] [batches]      (needs libwcsde_diag.so)
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from tools.diag_variants import diag  # noqa: E402  (sets WCSDE_LIB_OVERRIDE to the diag build)
import oracle  # noqa: E402
from bench import sweep_batch  # noqa: E402
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, driver_params  # noqa: E402


def main():
    variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "27,31,32,33,34,35,36").split(",")]
    batches = [int(b) for b in (sys.argv[2] if len(sys.argv) > 2 else "1250,2500,5000,10000").split(",")]
    steps = int(os.environ.get("DIAG_STEPS", "4000"))
    sc = datasets.load_sc()
    p = driver_params()
    G, S, keys = sweep_batch(0)
    # correctness of each variant vs the oracle (37 sims)
    ob = oracle.OracleBatch(sc, G[:37], S[:37], keys[:37], p)
    ob.integrate(300, 0.05)
    orec = ob.integrate(600, 2.0, 20)
    err = {}
    for v in variants:
        bt = Batch(sc, G[:37], S[:37], keys[:37], p, precision="f32")
        diag(bt, v, 300, 0.05)
        # diag variants >= 20 record node-major [B*N][ld], ld = records rounded up to 4 (wc_diag_integrate)
        rec = torch.empty((37 * 90, 32), dtype=torch.float32, device="cuda")
        diag(bt, v, 600, 2.0, 20, rec)
        torch.cuda.synchronize()
        got = rec[:, :30].reshape(37, 90, 30).permute(0, 2, 1)
        err[v] = float(np.abs(got.double().cpu().numpy() - orec).max())
    for B in batches:
        bt = Batch(sc, G[:B], S[:B], keys[:B], p, precision="f32")
        rec = torch.empty((B * 90, (steps // 20 + 3) // 4 * 4), dtype=torch.float32, device="cuda")
        diag(bt, variants[0], 200, 0.05)
        times = {v: [] for v in variants}
        for _ in range(3):
            for v in variants:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                diag(bt, v, steps, 2.0, 20, rec)
                e1.record()
                torch.cuda.synchronize()
                times[v].append(e0.elapsed_time(e1))
        for v in variants:
            ms = min(times[v])
            print(json.dumps({"B": B, "variant": v, "us_per_step": ms * 1e3 / steps,
                              "node_steps_per_s": B * 90 * steps / (ms * 1e-3), "max_err_vs_oracle": err[v]}),
                  flush=True)


if __name__ == "__main__":
    main()
