#!/usr/bin/env python3
"""Short C5 integrator run for rocprofv3 --pmc passes (tools/profile_c5_pass.sh): the bench's C5 shard
(2,500 simulations of the (G, sigma) grid on the 1000-node synthetic connectome), STEPS Euler steps
recording every 20th time-major, as bench.py and the fp32 sweep pipeline record (C5_RING=1: into a
node-major ring with ld = STEPS / 20, the round-5 harness, whose 4-B record stores at an 80-B stride
cost partial-line writes)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, driver_params  # noqa: E402


def _dump_maps():
    """/proc/self/maps at Python exit (before the C-level exit handlers), so that the frames of a
    fault during process teardown can be mapped to library + offset."""
    out = os.environ.get("C5_MAPS_OUT")
    if out:
        with open("/proc/self/maps") as f, open(out, "w") as g:
            g.write(f.read())


def main():
    import atexit
    atexit.register(_dump_maps)
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 400
    sc = datasets.synthetic_sc(1000)
    G, S, keys = bench.sweep_batch(0)
    G, S, keys = G[:2500], S[:2500], keys[:2500]
    bt = Batch(sc, G, S, keys, driver_params(), precision="f32")
    if os.environ.get("C5_RING") == "1":
        ring = torch.empty(2500 * 1000 * (steps // 20), dtype=bt.rec_dtype, device="cuda")
        bt.integrate(steps, 2.0, 20, ring, rec_ld=steps // 20)
    else:
        tmaj = torch.empty((steps // 20, 2500, 1000), dtype=bt.rec_dtype, device="cuda")
        bt.integrate(steps, 2.0, 20, tmaj)
    torch.cuda.synchronize()
    print("ok", steps)


if __name__ == "__main__":
    main()
