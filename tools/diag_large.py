#!/usr/bin/env python3
"""Ablation of the N > 96 step kernel (wc_diag_integrate variants 100..103):
100 product, 101 no chunk fetch, 102 no MFMA, 103 no epilogue state traffic,
104 3 stages + epilogue state prefetched, 105 2 stages + prefetch, 106 3 stages,
107 nontemporal epilogue state loads/stores.
Times us/step at N (default 1000) and B (default 2500); interleaved rounds."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nremmodfc_amd import _lib, datasets  # noqa: E402
from nremmodfc_amd.model import Batch, sim_keys  # noqa: E402
from tools.diag_variants import diag  # noqa: E402


def main():
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2500
    steps = 200
    sc = datasets.synthetic_sc(N)
    rng = np.random.default_rng(0)
    bt = Batch(sc, 0.16 + rng.uniform(-0.1, 0.3, B), 7.68 + rng.uniform(-0.2, 0.2, B),
               sim_keys(np.arange(B), np.zeros(B, dtype=np.int64)), precision="f32")
    variants = [int(v) for v in os.environ.get("DIAG_VARIANTS", "100,101,102,103,104,105,106,107").split(",")]
    times = {v: [] for v in variants}
    for r in range(3):
        for v in variants:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            diag(bt, v, steps, 2.0)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    for v in variants:
        ms = min(times[v])
        print(f"variant {v}: {ms * 1e3 / steps:.1f} us/step, {B * N * steps / (ms * 1e-3):.3e} node-steps/s")


if __name__ == "__main__":
    main()
