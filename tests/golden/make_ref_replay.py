#!/usr/bin/env python3
"""Bit-level pin of the oracle's run() to the reference's OWN source (build container only).

SURVEY.md 7.1(a) / 8(c): /root/reference/netwWilsonCowanPlastic.py runs as plain NumPy once
its numba decorators are identities (numba's JIT does not change the arithmetic of
wc:72-137; the module imports BOLDModel at wc:10 but run() never calls it).  Its noise is
one call per Euler step, ``np.random.normal(0, sqdtD, size=N)`` (wc:80).  Replacing that
call by a replay of the build's Philox stream -- ``0 + sqdtD * z`` with z =
oracle.step_normals(key, step, N), the exact loc + scale * z numpy computes -- makes the
reference's own run() produce the trajectory the build's oracle and GPU path must
reproduce for the same key.

Writes tests/golden/ref_replay.npz: for each case, Y_t [n_rec][3][N] exactly as the
reference's run() returns it (state BEFORE every 20th step of the last phase, wc:128-130),
plus the inputs (G, sigmaE vectors, key, step counts).  Only data is committed; the
reference source is read from /root/reference at generation time and never copied.

Usage: python tests/golden/make_ref_replay.py
"""
import importlib.util
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

# (phase-1, phase-2, phase-3) Euler steps; the reference's tau_ip 0.05 / 1 / 2 (wc:101,111,118)
STEPS = (100, 100, 2000)
REC = 20


def _identity_numba():
    """numba stand-in: decorators return the Python function (``run.recompile()`` a no-op)."""
    nb = types.ModuleType("numba")

    def _dec(*a, **k):
        if len(a) == 1 and callable(a[0]) and not k:
            f = a[0]
            f.recompile = lambda: None
            return f

        def wrap(f):
            f.recompile = lambda: None
            return f
        return wrap

    nb.njit = nb.jit = nb.vectorize = _dec
    nb.float64 = lambda *a: None
    core = types.ModuleType("numba.core")
    errors = types.ModuleType("numba.core.errors")
    errors.NumbaPerformanceWarning = type("NumbaPerformanceWarning", (Warning,), {})
    core.errors = errors
    nb.core = core
    return {"numba": nb, "numba.core": core, "numba.core.errors": errors,
            "BOLDModel": types.ModuleType("BOLDModel")}


def load_reference():
    sys.modules.update(_identity_numba())
    spec = importlib.util.spec_from_file_location("ref_wc", os.path.join(REF, "netwWilsonCowanPlastic.py"))
    wc = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(wc)
    return wc


class Replay:
    """np.random.normal replacement: step s of the run returns loc + scale * z(key, s)."""

    def __init__(self, key, N):
        import oracle
        self.key, self.N, self.step, self.z = int(key), N, 0, oracle.step_normals

    def __call__(self, loc=0.0, scale=1.0, size=None):
        assert size == self.N
        z = self.z(self.key, self.step, self.N)
        self.step += 1
        return loc + scale * z


def run_case(wc, sc, G, sigmaE, key):
    from nremmodfc_amd.model import driver_params
    p = driver_params()
    N = sc.shape[0]
    # driver configuration (whole_sweep_both.py:39-52): P, rhoE, CM; lengths of the time grids
    wc.P, wc.rhoE, wc.CM, wc.N, wc.nnodes = p.P, p.rhoE, sc.copy(), N, N
    wc.G, wc.sigmaE = G, sigmaE
    wc.timeTrans1 = np.arange(STEPS[0]) * wc.dtSim
    wc.timeTrans2 = np.arange(STEPS[1]) * wc.dtSim
    wc.timeSim = np.arange(STEPS[2]) * wc.dtSim
    wc.time = np.arange(STEPS[2] // REC) * wc.dt
    rep = Replay(key, N)
    saved = np.random.normal
    np.random.normal = rep
    try:
        wc.run.recompile()
        Y = wc.run()
    finally:
        np.random.normal = saved
    assert rep.step == sum(STEPS)
    return Y


def main():
    from nremmodfc_amd import datasets
    from nremmodfc_amd.model import sim_keys
    wc = load_reference()
    sc = datasets.load_sc()
    N = sc.shape[0]
    mach = datasets.load_map(datasets.MAPNAMES_ACH[1])
    mna = datasets.load_map(datasets.MAPNAMES_NA[1])
    cases = {
        # homogeneous cell (dG, dsigma) = (0.04, 0.1): scalars, as whole_sweep_both.py:68-72 sets them
        "homo": (0.16 + 0.04, 7.68 + 0.1, int(sim_keys([3], [17])[0])),
        # maps cell (dG, dsigma) = (0.2, -0.1): per-node vectors (whole_sweep_both_maps.py:104-108)
        "maps": (0.16 + 0.2 * mach, 7.68 + (-0.1) * mna, int(sim_keys([11], [203])[0])),
    }
    out = {"steps": np.array(STEPS), "rec_every": np.array(REC)}
    for name, (G, S, key) in cases.items():
        Y = run_case(wc, sc, G, S, key)
        out[f"{name}_Y"] = Y
        out[f"{name}_G"] = np.broadcast_to(np.asarray(G, dtype=np.float64), (N,)).copy()
        out[f"{name}_sigmaE"] = np.broadcast_to(np.asarray(S, dtype=np.float64), (N,)).copy()
        out[f"{name}_key"] = np.array(key, dtype=np.uint64)
        print(name, Y.shape, float(Y[-1, 0].mean()), float(Y[-1, 2].mean()))
    np.savez_compressed(os.path.join(HERE, "ref_replay.npz"), **out)
    print("wrote", os.path.join(HERE, "ref_replay.npz"))


if __name__ == "__main__":
    main()
