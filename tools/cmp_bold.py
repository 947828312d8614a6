"""Bit-compare the streamed BOLD/filtfilt chain of two builds of libwcsde.so (one process per
library: WCSDE_LIB_OVERRIDE selects it) on the same seeded E input, over a whole short
schedule (head, steady chunks, tail), and time one steady chunk at the C3 shape.
python tools/cmp_bold.py save OUT.npz | cmp A.npz B.npz"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def save(out):
    import torch
    from nremmodfc_amd.sigchain import BoldStream
    g = torch.Generator(device="cuda").manual_seed(7)
    C, n_total = 20_000, 40_000
    bs = BoldStream(C, n_total, 2000, 1000, 0.04, "cuda")
    for _ in range(n_total // 1000):
        E = 0.2 + 0.1 * torch.rand(1000 * C, dtype=torch.float32, device="cuda", generator=g)
        bs.feed(E, 1000)
    res = {"bold": bs.finish().cpu().numpy()}
    # timing: one steady chunk (time-major input + node-major copy) at the C3 column count
    C3 = 20_000 * 90
    tm = 0.2 + 0.1 * torch.rand(1000 * C3, dtype=torch.float32, device="cuda", generator=g)
    nm = torch.empty(C3 * 4000, dtype=torch.float32, device="cuda")
    big = BoldStream(C3, 300_000, 2000, 1000, 0.04, "cuda")
    for _ in range(3):
        big.feed(tm, 1000)
    times = []
    for _ in range(5):
        torch.cuda.synchronize()
        t = time.perf_counter()
        big.feed(tm, 1000, copy=nm, copy_ld=4000, copy_offset=1000)
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t)
    print(f"C3 steady chunk with copy: {min(times) * 1e3:.3f} ms (median {np.median(times) * 1e3:.3f})", flush=True)
    np.savez(out, **res)


def cmp(a, b):
    x, y = np.load(a), np.load(b)
    bad = 0
    for k in x.files:
        same = np.array_equal(x[k], y[k])
        d = np.abs(x[k] - y[k]).max()
        print(k, "identical" if same else f"DIFFER max|d| {d:.3e} (max|x| {np.abs(x[k]).max():.3e})")
        bad += not same
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3])
