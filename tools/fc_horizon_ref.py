#!/usr/bin/env python3
"""Fixed-seed parity at the reference's full horizon, on the CPU (build container only).

For K simulations of the shipped W-optimum cell (dG, dsigma) = (0, 0) -- the 32 (seed, stream)
keys of tests/golden/oracle_pin_cell.json -- this runs

  * the REFERENCE's own run() (/root/reference/netwWilsonCowanPlastic.py:86-137, numba
    decorators as identities, np.random.normal replaying the Philox stream: see
    tests/golden/make_ref_replay.py) over the full 1001 s driver schedule
    (whole_sweep_both.py:43-50), and
  * the build's C oracle (oracle/wc_oracle.c) on the same key,

both fp64 and fed bit-identical noise, so they differ only in the rounding of np.dot
(BLAS) / np.exp against the C loop's sequential dot / libm exp.  Both E_t go through the
same epilogue (oracle.sigchain.sim_metrics: BOLD, filtfilt, FC, metrics, Kuramoto, Welch).

Writes tests/golden/ref_replay_full.npz: per key the reference's and the oracle's FC (strict
upper triangles), their 16 metric columns, and the pathwise divergence max_n |E_ref - E_orc|
per second of recorded time.  tests/test_fc_parity_cpu.py and the GPU horizon tests read it.

  OPENBLAS_NUM_THREADS=1 python tools/fc_horizon_ref.py [K] [PROCS]    (~7 min per 8 keys)
"""
import json
import os
import sys
import time
from multiprocessing import Pool

os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("OMP_NUM_THREADS", "1")

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
OUT = os.path.join(ROOT, "tests", "golden", "ref_replay_full.npz")


def one(args):
    seed, stream = args
    import make_ref_replay as mr
    import oracle
    import oracle.sigchain as osg
    from nremmodfc_amd import datasets, sweep
    from nremmodfc_amd.model import Schedule, driver_params, sim_keys
    sch = Schedule()
    if os.environ.get("WCSDE_HORIZON_TEST"):  # smoke-test the tool on a short schedule
        sch = Schedule(n_trans2=1000, n_sim=1_100_000)
    mr.STEPS = (sch.n_trans1, sch.n_trans2, sch.n_sim)
    sc = datasets.load_sc()
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    key = int(sim_keys([seed], [stream])[0])
    G, S = sweep.BASE_G, sweep.BASE_SIGMA
    t0 = time.perf_counter()
    wc = mr.load_reference()
    Y = mr.run_case(wc, sc, G, S, key)
    E_ref = np.ascontiguousarray(Y[:, 0, :])
    del Y
    t_ref = time.perf_counter() - t0
    t0 = time.perf_counter()
    ob = oracle.OracleBatch(sc, G, S, [key], driver_params())
    ob.integrate(sch.n_trans1, sch.tau_ip[0])
    ob.integrate(sch.n_trans2, sch.tau_ip[1])
    E_orc = ob.integrate(sch.n_sim, sch.tau_ip[2], sch.rec_every)[0]
    t_orc = time.perf_counter() - t0
    div = np.abs(E_ref - E_orc).max(axis=1).reshape(-1, 500).max(axis=1)  # per second of record
    m_ref, _, fc_ref = osg.sim_metrics(E_ref, emp)
    m_orc, _, fc_orc = osg.sim_metrics(E_orc, emp)
    cols = sweep.METRIC_COLS
    return {"seed": seed, "stream": stream, "key": key,
            "fc_ref": osg.flat_fc(fc_ref), "fc_orc": osg.flat_fc(fc_orc),
            "m_ref": np.array([m_ref[c] for c in cols]), "m_orc": np.array([m_orc[c] for c in cols]),
            "div": div, "ssim": osg.ssim(fc_ref, fc_orc, 1.0), "t_ref": t_ref, "t_orc": t_orc}


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    procs = int(sys.argv[2]) if len(sys.argv) > 2 else min(8, len(os.sched_getaffinity(0)))
    pin = json.load(open(os.path.join(ROOT, "tests", "golden", "oracle_pin_cell.json")))
    jobs = list(zip(pin["seeds"], pin["streams"]))[:K]
    t0 = time.perf_counter()
    res = []
    with Pool(procs) as pool:
        for r in pool.imap(one, jobs):
            res.append(r)
            print(json.dumps({"seed": r["seed"], "ssim_ref_vs_oracle": r["ssim"],
                              "div_at_s": {s: float(r["div"][s]) for s in (0, 1, 5, 10, 30, 100, 300, 599)
                                           if s < len(r["div"])},
                              "t_ref": round(r["t_ref"], 1), "t_orc": round(r["t_orc"], 1)}), flush=True)
    out = OUT if not os.environ.get("WCSDE_HORIZON_TEST") else "/tmp/ref_replay_test.npz"
    np.savez_compressed(
        out, seeds=np.array([r["seed"] for r in res]), streams=np.array([r["stream"] for r in res]),
        keys=np.array([r["key"] for r in res], dtype=np.uint64),
        fc_ref=np.stack([r["fc_ref"] for r in res]), fc_orc=np.stack([r["fc_orc"] for r in res]),
        m_ref=np.stack([r["m_ref"] for r in res]), m_orc=np.stack([r["m_orc"] for r in res]),
        div=np.stack([r["div"] for r in res]), columns=np.array(list(__import__(
            "nremmodfc_amd.sweep", fromlist=["METRIC_COLS"]).METRIC_COLS)),
        wall_s=np.array(time.perf_counter() - t0), procs=np.array(procs))
    ss = np.array([r["ssim"] for r in res])
    print(json.dumps({"K": len(res), "ssim_ref_vs_oracle_mean": ss.mean(), "min": ss.min(), "max": ss.max(),
                      "wall_s": time.perf_counter() - t0}))


if __name__ == "__main__":
    main()
