#!/usr/bin/env python3
"""Fixed-seed FC parity at the reference's full horizon, GPU side (run on the GPU box).

For the 32 (seed, stream) keys of tests/golden/ref_replay_full.npz (cell (0, 0), the keys of
oracle_pin_cell.json) this runs the product pipeline over the full 1001 s schedule
(whole_sweep_both.py:43-95: 298 BOLD samples) and saves every simulation's FC (strict upper
triangle) and 16 metric columns:

  f64        the fp64 parity path;
  f64+eps    the same keys with run()'s initial E of node 0 scaled by (1 + eps), eps = 1e-15,
             1e-12, 1e-9, 1e-6 (how far a perturbation of a given size carries at 1001 s);
  f32        the fp32 product path.

tools/fc_horizon_report.py compares them with the reference's own run() (the fixture's fc_ref,
made by tools/fc_horizon_ref.py) and with the oracle (fc_orc) -> profiles/r03_fc_horizon.json.

  python tools/fc_horizon_gpu.py OUT.npz
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from nremmodfc_amd import datasets, sweep  # noqa: E402
from nremmodfc_amd.model import Schedule, driver_params  # noqa: E402
from nremmodfc_amd.pipeline import run_sweep  # noqa: E402

EPS = (1e-15, 1e-12, 1e-9, 1e-6)


def flat(fc):
    iu = np.triu_indices(fc.shape[-1], 1)
    return fc[:, iu[0], iu[1]]


def main():
    out = sys.argv[1]
    fx = np.load(os.path.join(ROOT, "tests", "golden", "ref_replay_full.npz"))
    keys = fx["keys"].astype(np.uint64)
    K, N = len(keys), 90
    sc = datasets.load_sc()
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    p = driver_params()
    G, S = np.full(K, sweep.BASE_G), np.full(K, sweep.BASE_SIGMA)
    res = {}
    t0 = time.perf_counter()
    # fp64: unperturbed + one copy per eps, in one batch
    nv = 1 + len(EPS)
    E0 = np.full((nv * K, N), p.E0)
    for i, e in enumerate(EPS):
        E0[(i + 1) * K:(i + 2) * K, 0] *= 1 + e
    r = run_sweep(sc, np.tile(G, nv), np.tile(S, nv), np.tile(keys, nv), emp, Schedule(), precision="f64",
                  want_fc=True, init_state={"E": E0})
    cols = r.columns()
    cm = np.stack([cols[c] for c in sweep.METRIC_COLS], axis=1)
    res["fc_f64"], res["m_f64"] = flat(r.fc[:K]), cm[:K]
    for i, e in enumerate(EPS):
        res[f"fc_f64_eps{e:.0e}"] = flat(r.fc[(i + 1) * K:(i + 2) * K])
        res[f"m_f64_eps{e:.0e}"] = cm[(i + 1) * K:(i + 2) * K]
    t64 = time.perf_counter() - t0
    print(f"f64 x {nv} variants: {t64:.1f} s", flush=True)
    t0 = time.perf_counter()
    r = run_sweep(sc, G, S, keys, emp, Schedule(), precision="f32", want_fc=True)
    cols = r.columns()
    res["fc_f32"], res["m_f32"] = flat(r.fc), np.stack([cols[c] for c in sweep.METRIC_COLS], axis=1)
    print(f"f32: {time.perf_counter() - t0:.1f} s", flush=True)
    np.savez_compressed(out, keys=keys, eps=np.array(EPS), columns=np.array(sweep.METRIC_COLS), **res)
    print("wrote", out)


if __name__ == "__main__":
    main()
