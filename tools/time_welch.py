"""Time wc_welch_accumulate (one 4000-sample segment of every column) at the sweep shape."""
import sys
import time

import torch

from nremmodfc_amd.sigchain import WelchAccumulator


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    N = 90
    ld = 4000
    E = torch.rand(B * N * ld, dtype=torch.float32, device="cuda")
    wa = WelchAccumulator(B, N)
    for _ in range(2):
        wa.accumulate(E, ld, 1000, 4, 0)
    torch.cuda.synchronize()
    reps = 10
    t = time.perf_counter()
    for k in range(reps):
        wa.accumulate(E, ld, 1000, 4, 2000 * (k % 2))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    gb = B * N * 4000 * 4 / 1e9
    print(f"B={B} N={N}: {dt * 1e3:.2f} ms per segment, {gb / dt:.0f} GB/s of segment data")


if __name__ == "__main__":
    main()
