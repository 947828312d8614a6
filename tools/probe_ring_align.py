"""BOLD steady chunk (C3 shape, time-major E in, node-major copy out) timed against the Welch
ring's slot offset and column stride: the bench trace shows odd chunks ~0.6 ms slower than even
ones, and the 6000-sample ring puts odd slots 32 B off a 128-B line.  Also times the two
time-major input buffers the pipeline alternates between.

  PYTHONPATH=. python tools/probe_ring_align.py"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nremmodfc_amd.sigchain import BoldStream  # noqa: E402


def main():
    C3 = 20_000 * 90
    g = torch.Generator(device="cuda").manual_seed(7)
    tms = [0.2 + 0.1 * torch.rand(1000 * C3, dtype=torch.float32, device="cuda", generator=g) for _ in range(2)]
    big = BoldStream(C3, 300_000, 2000, 1000, 0.04, "cuda")
    for _ in range(3):
        big.feed(tms[0], 1000)

    def t_feed(tm, ring, ld, off, reps=4):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t = time.perf_counter()
            big.feed(tm, 1000, copy=ring, copy_ld=ld, copy_offset=off)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return min(ts) * 1e3, float(np.median(ts)) * 1e3

    for ld, slot in ((6000, 1000), (6144, 1024), (6016, 1000)):
        ring = torch.empty(C3 * ld, dtype=torch.float32, device="cuda")
        for s in range(6):
            off = s * slot
            mn, md = t_feed(tms[s & 1], ring, ld, off)
            print(f"ld {ld} slot {s} offset {off:5d} (byte offset mod 128 = {(off * 4) % 128:3d}), input {s & 1}: "
                  f"min {mn:.3f} ms, median {md:.3f} ms", flush=True)
        for s in range(2):
            mn, md = t_feed(tms[1 - (s & 1)], ring, ld, s * slot)
            print(f"ld {ld} slot {s} with the other input buffer: min {mn:.3f} ms, median {md:.3f} ms", flush=True)
        del ring
        torch.cuda.empty_cache()
    ts = []
    for _ in range(4):
        torch.cuda.synchronize()
        t = time.perf_counter()
        big.feed(tms[0], 1000)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t)
    print(f"no copy: min {min(ts) * 1e3:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
