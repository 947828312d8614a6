"""Bit-compare the integrator of two builds of libwcsde.so on the same inputs (one process per
library: WCSDE_LIB_OVERRIDE selects it).  python tools/cmp_libs.py save OUT.npz | cmp A.npz B.npz"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CASES = [(90, 20000, True), (90, 20000, False), (90, 10000, False), (90, 2500, True), (90, 60, False), (60, 700, False), (30, 100, False)]


def save(out):
    import torch
    from nremmodfc_amd import datasets
    from nremmodfc_amd.model import Batch, sim_keys
    res = {}
    for N, B, ring in CASES:
        sc = datasets.load_sc() if N == 90 else datasets.synthetic_sc(N)
        rng = np.random.default_rng(N + B)
        G = 0.16 + rng.uniform(-0.1, 0.3, B)
        S = 7.68 + rng.uniform(-0.2, 0.2, B)
        bt = Batch(sc, G, S, sim_keys(np.arange(B) % 50, np.arange(B) // 50), precision="f32")
        bt.integrate(100, 0.05)
        steps = 2000
        if N == 90 and B == 20000 and os.environ.get("CMP_TIME"):
            big = torch.empty(B * N * 1000, dtype=torch.float32, device="cuda")
            for rep in range(3):
                torch.cuda.synchronize()
                t = time.perf_counter()
                bt.integrate(20000, 2.0, 20, big)  # time-major, as the fp32 pipeline and bench.py record
                torch.cuda.synchronize()
                dt = time.perf_counter() - t
                print(f"  20000-step chunk: {dt * 1e3:.2f} ms, {dt / 20000 * 1e6:.3f} us/step", flush=True)
            del big
        if ring:
            rec = torch.zeros(B * N * (steps // 20), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            t = time.perf_counter()
            bt.integrate(steps, 2.0, 20, rec, rec_ld=steps // 20)
        else:
            rec = torch.zeros((steps // 20, B, N), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            t = time.perf_counter()
            bt.integrate(steps, 2.0, 20, rec)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t
        print(f"N={N} B={B}: {dt / steps * 1e6:.3f} us/step {B * N * steps / dt:.3e} node-steps/s", flush=True)
        key = f"{N}_{B}"
        res[key + "_E"] = bt.E.cpu().numpy()
        res[key + "_I"] = bt.I.cpu().numpy()
        res[key + "_A"] = bt.A.cpu().numpy()
        res[key + "_rec"] = rec.cpu().numpy()
    np.savez(out, **res)


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in x.files:
        same = np.array_equal(x[k], y[k])
        d = np.abs(x[k].astype(np.float64) - y[k].astype(np.float64)).max()
        print(k, "identical" if same else f"DIFFER max|d| {d:.3e}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3])
