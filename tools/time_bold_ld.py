"""Time one steady BOLD chunk with the node-major copy at the C3 shape for several ring row
strides (copy_ld, floats): does the stride of the copy's 128-B row stores matter?
python tools/time_bold_ld.py [B] [ld ...]"""
import sys
import time

import torch

from nremmodfc_amd.sigchain import BoldStream


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    lds = [int(x) for x in sys.argv[2:]] or [6000, 6016, 6032, 6064, 6128, 6144, 6160]
    C = B * 90
    tm = 0.2 + 0.1 * torch.rand(1000 * C, dtype=torch.float32, device="cuda")
    ring = torch.empty(C * max(lds), dtype=torch.float32, device="cuda")
    bs = BoldStream(C, 300_000, 2000, 1000, 0.04, "cuda")
    for _ in range(3):  # past Neq and the head: the timed chunks are steady state
        bs.feed(tm, 1000)
    for rnd in range(2):
        for ld in lds:
            bs.feed(tm, 1000, copy=ring, copy_ld=ld, copy_offset=1000)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(4):
                bs.feed(tm, 1000, copy=ring, copy_ld=ld, copy_offset=1000)
            torch.cuda.synchronize()
            print(f"round {rnd} copy_ld {ld}: {(time.perf_counter() - t) / 4 * 1e3:.2f} ms per chunk", flush=True)


if __name__ == "__main__":
    main()
