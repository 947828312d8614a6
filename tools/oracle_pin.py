#!/usr/bin/env python3
"""Pin the CPU oracle's run() restatement to the reference's shipped tables.

The reference's hot loop has no fixed-seed fixtures (its numba RNG is seeded from
os.urandom); its only outputs are the published sweep tables
output/sweep_delta_*.txt.  This runs the ORACLE (oracle/wc_oracle.c, fp64, the
restatement of netwWilsonCowanPlastic.py:77-137, and oracle/sigchain.py for
simBOLD / corrcoef / get_all_metrics / kuramoto / Welch, whole_sweep_both.py:79-95)
over the FULL 1001 s schedule for SEEDS seeds of the shipped grid cell
(dG, dsigma) = (0, 0) -- the W optimum, identical in all three shipped files -- and
writes every simulation's 16 metric columns with the cell's z-scores against the
shipped homogeneous table (tests/golden/shipped_cell_stats.npz) to
tests/golden/oracle_pin_cell.json.

  python tools/oracle_pin.py [SEEDS] [THREADS]     (~10 s of oracle time per sim-core)

tests/test_oracle_pin.py checks the committed file (fast) and, with WCSDE_SLOW=1,
recomputes two of its simulations bit for bit.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle  # noqa: E402
import oracle.sigchain as osg  # noqa: E402
from nremmodfc_amd import datasets, sweep  # noqa: E402
from nremmodfc_amd.model import Schedule, driver_params, sim_keys  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "oracle_pin_cell.json")
CELL = (0.0, 0.0)


def cell_sims(n_seeds):
    return [s for s in sweep.homogeneous(n_seeds, 0) if (round(s.dG, 4), round(s.dsigma, 4)) == CELL]


def oracle_rows(sims, threads, schedule=None):
    """Full-schedule oracle runs -> list of {column: value}."""
    sch = schedule or Schedule()
    sc = datasets.load_sc()
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    p = driver_params()
    rows = []
    for b0 in range(0, len(sims), threads):
        part = sims[b0:b0 + threads]
        ob = oracle.OracleBatch(sc, np.stack([s.G for s in part]), np.stack([s.sigma for s in part]),
                                sim_keys([s.seed for s in part], [s.stream for s in part]), p)
        ob.integrate(sch.n_trans1, sch.tau_ip[0], nthreads=threads)
        ob.integrate(sch.n_trans2, sch.tau_ip[1], nthreads=threads)
        rec = ob.integrate(sch.n_sim, sch.tau_ip[2], sch.rec_every, nthreads=threads)
        for b in range(len(part)):
            m, _, _ = osg.sim_metrics(rec[b], emp)
            rows.append({c: float(m[c]) for c in sweep.METRIC_COLS})
        del rec
        print(f"{b0 + len(part)}/{len(sims)} simulations", flush=True)
    return rows


def zscores(rows):
    st = np.load(os.path.join(ROOT, "tests", "golden", "shipped_cell_stats.npz"))
    cols = list(st["columns"])
    k = [tuple(np.round(c, 4)) for c in st["homo_cells"]].index(CELL)
    vals = np.array([[r[c] for c in cols] for r in rows])
    n = len(rows)
    se = np.sqrt(vals.std(axis=0, ddof=1) ** 2 / n + st["homo_std"][k] ** 2 / st["homo_count"][k])
    d = vals.mean(axis=0) - st["homo_mean"][k]
    z = np.where(se > 0, d / np.where(se > 0, se, 1), np.where(d == 0, 0.0, np.inf))
    return dict(zip(cols, z.tolist()))


def main():
    n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    threads = int(sys.argv[2]) if len(sys.argv) > 2 else min(8, len(os.sched_getaffinity(0)))
    sims = cell_sims(n_seeds)
    t0 = time.perf_counter()
    rows = oracle_rows(sims, threads)
    wall = time.perf_counter() - t0
    z = zscores(rows)
    out = {"what": "oracle (wc_oracle.c fp64 + oracle/sigchain.py), full 1001 s schedule, shipped homogeneous "
                   "grid cell (dG, dsigma) = (0, 0), Philox keys sim_keys(seed, stream)",
           "cell": CELL, "seeds": [s.seed for s in sims], "streams": [s.stream for s in sims],
           "columns": sweep.METRIC_COLS, "rows": [[r[c] for c in sweep.METRIC_COLS] for r in rows],
           "z_vs_shipped_homo": z, "max_abs_z": max(abs(v) for v in z.values()),
           "median_abs_z": float(np.median(np.abs(list(z.values())))), "wall_s": wall, "threads": threads}
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: out[k] for k in ("max_abs_z", "median_abs_z", "wall_s")}))
    print(json.dumps(z))


if __name__ == "__main__":
    main()
