"""SC optimiser: drop-in for optimize_SC_Hopf.py.

Same algorithm, constants and outputs as optimize_SC_Hopf.py:9-106: starting
from the Deco AAL connectome, for `iters` iterations simulate the Hopf network
(G = 0.6) once per seed, band-pass the x signals (Bessel order 3, 0.01-0.1 Hz,
filtfilt), cut 60 s at both ends, average the Pearson FC over the seeds, compare
it with the empirical wake FC (mean difference, Kolmogorov-Smirnov distance,
Euclidean distance, Pearson correlation) and move the homotopic SC entries by
epsilon * (empirical - simulated); clip at 0, keep the strongest 30% of links and
restore the total weight.

Every simulation of an iteration runs in one device launch (wc_hopf_integrate),
the band-pass in one more (wc_filtfilt) and the FCs in three more
(wc_corrcoef, split over time blocks); the per-iteration SC update is O(N^2) host bookkeeping, as in
the reference.

    python -m nremmodfc_amd.optimize_sc [--iters 100] [--seeds 10] [--out DIR]

writes all_SCs.npy [N][N][iters], fitting.npy [4][iters] and SC_opti.txt (the
final C: the reference's commented-out np.savetxt, optimize_SC_Hopf.py:106).
"""
import argparse
import ctypes
import functools
import json
import os
import time

import numpy as np
import torch

from . import Hopf_model_multi as HM
from . import _lib, datasets, graph_utils, sigchain

N_AAL = 90
HOMOTOPIC = np.array([(i, N_AAL - (i + 1)) for i in range(N_AAL)])  # optimize_SC_Hopf.py:10


def configure(sc):
    """optimize_SC_Hopf.py:15-40: model, simulation and network parameters."""
    HM.a = 0
    HM.w = 0.05 * 2 * np.pi
    HM.beta = 0.032
    HM.dt = 1e-1
    HM.teq = 60
    HM.tmax = 600 + HM.teq * 2
    HM.downsamp = 1
    HM.M = sc
    HM.norm = np.mean(np.sum(HM.M, 0))
    HM.nnodes = len(HM.M)
    HM.ones_vector = np.ones(HM.nnodes).reshape((1, HM.nnodes))
    HM.G = 0.6
    HM.seed = 0


@functools.lru_cache(maxsize=8)
def band(resolution, fmin=0.01, fmax=0.1):
    """signal.bessel(3, [2 res Fmin, 2 res Fmax], 'bandpass') (optimize_SC_Hopf.py:62-64) and
    lfilter_zi: SciPy's own design routines (seven coefficients, host); the
    order-6 band-pass is ill-conditioned in (b, a) form, so the exact SciPy
    coefficients are used rather than a restatement (1e-15 coefficient changes
    move the filtered signal by ~1e-5)."""
    from scipy import signal
    b, a = signal.bessel(3, [2 * resolution * fmin, 2 * resolution * fmax], btype="bandpass")
    return b, a, signal.lfilter_zi(b, a)


def simulated_fc(seeds, device="cuda"):
    """Mean over seeds of corrcoef(filtfilt(x)[cut0:cut1].T) (optimize_SC_Hopf.py:50-71)."""
    L = _lib.lib()
    x = HM.sim_batch(seeds, device=device)  # [Nmax][B][N]
    T, B, N = x.shape
    res = HM.dt * HM.downsamp
    b, a, zi = band(res)
    dp = lambda v: (ctypes.c_double * len(v))(*[float(t) for t in v])  # noqa: E731
    y = torch.empty_like(x)
    rc = L.wc_filtfilt(len(a) - 1, dp(b), dp(a), dp(zi), T, B * N, _lib.ptr(x), _lib.ptr(y), _lib.stream_handle())
    _lib.check(rc, "wc_filtfilt")
    cut0, cut1 = int(60 / res), int((HM.tmax - 60) / res)
    fc = sigchain.corrcoef(y[cut0:cut1], B, N)  # split over time blocks: 10 series fill the GPU
    return fc.mean(dim=0).cpu().numpy()


def ks_2samp(x, y):
    """Two-sample Kolmogorov-Smirnov statistic D (scipy.stats.ks_2samp(...)[0])."""
    x, y = np.sort(x), np.sort(y)
    allv = np.concatenate([x, y])
    cdf1 = np.searchsorted(x, allv, side="right") / len(x)
    cdf2 = np.searchsorted(y, allv, side="right") / len(y)
    return float(np.max(np.abs(cdf1 - cdf2)))


def fitting_measures(objective, dist_sim):
    """optimize_SC_Hopf.py:77-85."""
    return np.array([np.mean(objective) - np.mean(dist_sim), ks_2samp(objective, dist_sim),
                     np.linalg.norm(objective - dist_sim), np.corrcoef(objective, dist_sim)[0, 1]])


def update_sc(C, objective, dist_sim, epsilon, original_sum, threshold=0.3, lock_sum=True):
    """optimize_SC_Hopf.py:89-101: homotopic step, clip, 30% density, total weight.

    threshold=0 / lock_sum=False skip the two steps the reference marks optional
    (:96); the shipped SC_opti_25julio.txt differs from the Deco SC only at the
    homotopic entries, i.e. it was produced without them."""
    C = C.copy()
    h0, h1 = HOMOTOPIC[:, 0], HOMOTOPIC[:, 1]
    C[h0, h1] += graph_utils.matrix_recon(epsilon * (objective - dist_sim))[h0, h1]
    C[C < 0] = 0
    if threshold:
        C = graph_utils.thresholding(C, threshold)
    return C * original_sum / np.sum(C) if lock_sum else C


def optimize(iters=100, seeds=10, epsilon=0.03, sc=None, empfc=None, device="cuda", log=None, threshold=0.3,
             lock_sum=True):
    """The optimisation loop; returns (C, all_SCs [N][N][iters], fitting [4][iters])."""
    sc = datasets.load_deco_sc() if sc is None else np.asarray(sc, dtype=np.float64)
    empfc = datasets.load_empfc("W") if empfc is None else empfc
    configure(sc)
    objective = graph_utils.get_uptri(empfc)
    C = np.copy(HM.M)
    n = HM.nnodes
    all_scs = np.zeros((n, n, iters))
    fitting = np.zeros((4, iters))
    original_sum = np.sum(sc)
    for i in range(iters):
        t0 = time.perf_counter()
        all_scs[:, :, i] = C
        dist_sim = graph_utils.get_uptri(simulated_fc(range(seeds), device))
        fitting[:, i] = fitting_measures(objective, dist_sim)
        C = update_sc(C, objective, dist_sim, epsilon, original_sum, threshold, lock_sum)
        HM.M = C
        HM.norm = np.mean(np.sum(HM.M, 0))
        if log:
            log({"iter": i, "fitting": fitting[:, i].tolist(), "sum": float(np.sum(C)),
                 "links": int(np.sum(C > 0)), "s": time.perf_counter() - t0})
    return C, all_scs, fitting


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--seeds", type=int, default=10)
    ap.add_argument("--epsilon", type=float, default=0.03)
    ap.add_argument("--threshold", type=float, default=0.3, help="link density kept per iteration (0: skip)")
    ap.add_argument("--no-lock-sum", action="store_true", help="skip the total-weight normalisation")
    ap.add_argument("--out", default="output")
    args = ap.parse_args(argv)
    os.makedirs(args.out, exist_ok=True)
    t0 = time.perf_counter()
    C, all_scs, fitting = optimize(args.iters, args.seeds, args.epsilon, log=lambda d: print(json.dumps(d), flush=True),
                                   threshold=args.threshold, lock_sum=not args.no_lock_sum)
    np.save(os.path.join(args.out, "all_SCs.npy"), all_scs)
    np.save(os.path.join(args.out, "fitting.npy"), fitting)
    np.savetxt(os.path.join(args.out, "SC_opti.txt"), C)
    print(json.dumps({"iters": args.iters, "seeds": args.seeds, "wall_s": time.perf_counter() - t0}))


if __name__ == "__main__":
    main()
