"""Time wc_bold_chunk (one 1000-sample chunk of every column) at the sweep shape:
node-major input, time-major input, time-major input + node-major copy."""
import sys
import time

import torch

from nremmodfc_amd.sigchain import BoldStream


def run(bs, fn, reps=6):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
    C = B * 90
    ld = 4000
    nm = 0.2 + 0.1 * torch.rand(C * ld, dtype=torch.float32, device="cuda")
    tm = 0.2 + 0.1 * torch.rand(1000 * C, dtype=torch.float32, device="cuda")
    bs = BoldStream(C, 300_000, 2000, 1000, 0.04, "cuda")
    for _ in range(3):  # past Neq and the head: the timed chunks are steady state
        bs.feed(tm, 1000)
    for name, fn in (("node-major", lambda: bs.feed(nm, 1000, e_ld=ld, offset=0)),
                     ("time-major", lambda: bs.feed(tm, 1000)),
                     ("time-major+copy", lambda: bs.feed(tm, 1000, copy=nm, copy_ld=ld, copy_offset=1000))):
        dt = run(bs, fn)
        print(f"B={B} {name}: {dt * 1e3:.2f} ms per chunk", flush=True)


if __name__ == "__main__":
    main()
