"""Welch at C3's 20,000 x 90: K consecutive segments (argv[2], default 2) as K launches (nseg = 1)
against one launch of all K (nseg = K) over a ring of 4000 + 2000 (K - 1) samples, interleaved, and
the PSDs of the two forms compared."""
import sys
import time

import torch

from nremmodfc_amd.sigchain import WelchAccumulator


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    N, ld = 90, 4000 + 2000 * (K - 1)
    E = torch.rand(B * N * ld, dtype=torch.float32, device="cuda")
    res = {}
    for rep in range(3):
        for mode in (1, K):
            wa = WelchAccumulator(B, N)
            torch.cuda.synchronize()
            t = time.perf_counter()
            for k in range(10 // K):
                s0 = 4000 * (k % 2)  # (the group at 0, or at 4000, which wraps)
                if mode == 1:
                    for j in range(K):
                        wa.accumulate(E, ld, 1000, ld // 1000, s0 + 2000 * j)
                else:
                    wa.accumulate(E, ld, 1000, ld // 1000, s0, nseg=K)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t) / (10 // K * K)
            res[mode] = wa
            print(f"rep {rep} nseg={mode}: {dt * 1e3:.2f} ms per segment, {B * N * 4000 * 4 / dt / 1e9:.0f} GB/s of "
                  f"segment data", flush=True)
    p1, _ = res[1].peak(want_psd=True)
    p2, _ = res[K].peak(want_psd=True)
    a1, a2 = res[1].acc, res[K].acc
    print(f"acc max rel diff {((a1 - a2).abs().max() / a1.abs().max()).item():.2e}, peaks equal {torch.equal(p1, p2)}")


if __name__ == "__main__":
    main()
