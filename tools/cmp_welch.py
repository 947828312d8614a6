"""Bit-compare the Welch accumulator of two builds of libwcsde.so (one process per library:
WCSDE_LIB_OVERRIDE selects it) on the same seeded ring, and time one C3 segment.
python tools/cmp_welch.py save OUT.npz | cmp A.npz B.npz"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(out):
    import torch
    from nremmodfc_amd.sigchain import WelchAccumulator
    g = torch.Generator(device="cuda").manual_seed(11)
    B, N, ld = 300, 90, 4000
    E = 0.2 + 0.1 * torch.rand(B * N * ld, dtype=torch.float32, device="cuda", generator=g)
    wa = WelchAccumulator(B, N)
    for k in range(3):
        wa.accumulate(E, ld, 1000, 4, 2000 * k)
    peak, psd = wa.peak(want_psd=True)
    res = {"peak": peak.cpu().numpy(), "psd": psd.cpu().numpy()}
    B3 = 20000
    E3 = torch.rand(B3 * N * ld, dtype=torch.float32, device="cuda", generator=g)
    w3 = WelchAccumulator(B3, N)
    w3.accumulate(E3, ld, 1000, 4, 0)
    times = []
    for k in range(6):
        torch.cuda.synchronize()
        t = time.perf_counter()
        w3.accumulate(E3, ld, 1000, 4, 2000 * (k % 2))
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
    dt = min(times)
    print(f"C3 Welch segment: {dt * 1e3:.3f} ms (median {np.median(times) * 1e3:.3f}), "
          f"{B3 * N * ld * 4 / dt / 1e12:.2f} TB/s of segment data", flush=True)
    np.savez(out, **res)


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in x.files:
        same = np.array_equal(x[k], y[k])
        print(k, "identical" if same else f"DIFFER max|d| {np.abs(x[k] - y[k]).max():.3e}")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3])
