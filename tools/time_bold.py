"""Time wc_bold_chunk (one 1000-sample chunk of every column) at the sweep shape."""
import sys
import time

import torch

from nremmodfc_amd.sigchain import BoldStream


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    C = B * 90
    ld = 4000
    E = (0.2 + 0.1 * torch.rand(C * ld, dtype=torch.float32, device="cuda"))
    bs = BoldStream(C, 300_000, 2000, 1000, 0.04, "cuda")
    bs.feed(E, 1000, e_ld=ld, offset=0)
    torch.cuda.synchronize()
    reps = 10
    t = time.perf_counter()
    for k in range(reps):
        bs.feed(E, 1000, e_ld=ld, offset=1000 * (k % 4))
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / reps
    print(f"B={B} C={C}: {dt * 1e3:.2f} ms per 1000-sample chunk, {C * 1000 / dt:.3e} column-samples/s, "
          f"{C * 1000 * 4 / dt / 1e9:.0f} GB/s of E")


if __name__ == "__main__":
    main()
