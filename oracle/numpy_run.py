"""CPU ORACLE (test infrastructure / the bench's cpu_baseline leg, never the product path):
the reference's hot loop restated operation for operation in NumPy.

netwWilsonCowanPlastic.py runs run() under numba; without numba (absent here and on the GPU
box) the same NumPy operations are what the reference's own code executes.  This module
repeats them in the same order -- S (wc:72-74), wilsonCowan (wc:77-83: np.random.normal,
np.dot(CM, E), np.vstack), the three Euler loops and the storage of run() (wc:99-137) -- so
that, fed the same normals, it reproduces the reference's Y_t bit for bit
(tests/test_oracle_numpy_run.py against tests/golden/ref_replay.npz, which the reference's
own source produced), and its timing is the reference's per-step NumPy cost (bench.py's
cpu_baseline, SURVEY.md 8(d): one single-threaded process per core, truncated horizon).
"""
import numpy as np


def S(x, sigma, mu):
    """wc:72-74."""
    return 1 / (1 + np.exp(-(x - mu) * sigma))


def make_wilson_cowan(p, CM, N, normal):
    """wilsonCowan of wc:77-83 closed over the driver's globals (p: WCParams-like; normal(loc,
    scale, size) draws the noise, np.random.normal in the reference)."""
    a_ee, a_ei, a_ii, tauE, tauI = p.a_ee, p.a_ei, p.a_ii, p.tauE, p.tauI
    P, rhoE, rE, rI, sigmaI, sqdtD = p.P, p.rhoE, p.rE, p.rI, p.sigmaI, p.sqdtD

    def wilsonCowan(t, X, sigmaE, mu, tau_ip, G):
        E, I, a_ie = X
        noise = normal(0, sqdtD, size=N)
        return np.vstack(((-E + (1 - rE * E) * S(a_ee * E - a_ie * I + G * np.dot(CM, E) + P + noise, sigmaE, mu)) / tauE,
                          (-I + (1 - rI * I) * S(a_ei * E - a_ii * I, sigmaI, mu)) / tauI,
                          (I * (E - rhoE)) / tau_ip))
    return wilsonCowan


def run(p, CM, G, sigmaE, n1, n2, n3, rec_every=20, normal=np.random.normal, mu=1):
    """run() of wc:86-137 with phase lengths n1, n2, n3 -> Y_t [n3 // rec_every][3][N]."""
    CM = np.asarray(CM, dtype=np.float64)
    N = CM.shape[0]
    wilsonCowan = make_wilson_cowan(p, CM, N, normal)
    dtSim = p.dtSim
    Var = np.array([p.E0, p.I0, p.a_ie_0]).reshape(3, 1) * np.ones((1, N))
    tau_ip = 0.05
    for i, t in enumerate(np.arange(n1) * dtSim):
        Var += dtSim * wilsonCowan(t, Var, sigmaE, mu, tau_ip, G)
    tau_ip = 1
    for i, t in enumerate(np.arange(n2) * dtSim):
        Var += dtSim * wilsonCowan(t, Var, sigmaE, mu, tau_ip, G)
    tau_ip = 2
    downsamp = rec_every
    Y_t = np.zeros((n3 // downsamp, 3, N))
    for i, t in enumerate(np.arange(n3) * dtSim):
        if i % downsamp == 0:
            Y_t[i // downsamp] = Var
        Var += dtSim * wilsonCowan(t, Var, sigmaE, mu, tau_ip, G)
    return Y_t


def timed_sample(steps, seed=0, nodes=90):
    """One simulation of the C3 cell (0.16, 7.68) for `steps` recorded-phase steps on the
    90-node connectome (nodes = 1000: the C5 synthetic connectome, datasets.synthetic_sc, where
    np.dot(CM, E) of wc:81 is a BLAS gemv of 1e6 multiply-adds per step), numpy's own normal
    draws (the reference's RNG call): -> seconds."""
    import time
    import types

    from nremmodfc_amd import datasets
    # the reference's constants (wc:20-57) with the drivers' P, rhoE (whole_sweep_both.py:39-40); a
    # plain namespace so a worker imports numpy only (nremmodfc_amd.model would import torch)
    p = types.SimpleNamespace(a_ee=3.5, a_ie_0=2.5, a_ei=3.75, a_ii=0, tauE=0.010, tauI=0.020, P=0.4, rhoE=0.18,
                              rE=0.5, rI=0.5, sigmaI=4, sqdtD=0.002 / np.sqrt(0.0001), dtSim=0.0001, E0=0.1, I0=0.1)
    sc = datasets.load_sc() if nodes == 90 else datasets.synthetic_sc(nodes)
    np.random.seed(seed)
    t0 = time.perf_counter()
    run(p, sc, 0.16, 7.68, 0, 0, steps, 20)
    return time.perf_counter() - t0


if __name__ == "__main__":  # worker of bench.py's cpu_baseline: python -m oracle.numpy_run STEPS SEED [NODES]
    import sys
    print(timed_sample(int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 90), flush=True)
