"""Time wc_welch_accumulate on an fp64 ring (the reference-precision pipeline's Welch, the LDS-Stockham
welch_kernel<double>): one 4000-sample segment of every column at the sweep shape."""
import sys
import time

import torch

from nremmodfc_amd.sigchain import WelchAccumulator


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    N, ld = 90, 4000
    E = torch.rand(B * N * ld, dtype=torch.float64, device="cuda")
    wa = WelchAccumulator(B, N)
    wa.accumulate(E, ld, 1000, 4, 0)
    torch.cuda.synchronize()
    reps = 4
    t = time.perf_counter()
    for k in range(reps):
        wa.accumulate(E, ld, 1000, 4, 0)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(f"B={B} N={N} fp64: {dt * 1e3:.2f} ms per segment, {B * N * 4000 * 8 / 1e9 / dt:.0f} GB/s of segment data")


if __name__ == "__main__":
    main()
