"""CPU oracle of the SC optimiser's Hopf network and the optimiser's host logic (no GPU).

The reference Hopf_model_multi.py needs numba and networkx (absent), so the
restatement is pinned by the analytic noise-free solution of the Stuart-Landau
oscillator (a = 0: r' = -r^3, theta' = w) -- first-order convergence of the Euler
loop -- and by the SciPy routines the reference calls (filtfilt, ks_2samp,
pearsonr) for the rest of the loop.
"""
import numpy as np
import pytest
from scipy import signal, stats

import oracle
from nremmodfc_amd import graph_utils
from nremmodfc_amd.optimize_sc import HOMOTOPIC, band, fitting_measures, ks_2samp, update_sc
from oracle import sigchain as osg


def _uncoupled(dt, T):
    x = np.array([[0.5, 0.2, 0.9, 0.05]])
    y = np.array([[0.1, 0.3, 0.0, 0.6]])
    r0, th0 = np.hypot(x, y), np.arctan2(y, x)
    p = dict(a=0.0, w=0.05 * 2 * np.pi, beta=0.0, dt=dt, G=0.0, norm=1.0)
    oracle.hopf_integrate(p, np.zeros((4, 4)), [1], x, y, 0, T)
    t = T * dt
    r = r0 / np.sqrt(1 + 2 * r0 ** 2 * t)
    return np.abs(np.hypot(x, y) - r).max(), np.abs(np.angle(np.exp(1j * (np.arctan2(y, x) - th0 - p["w"] * t)))).max()


def test_hopf_oracle_converges_to_analytic_solution():
    e1 = _uncoupled(1e-3, 2000)
    e2 = _uncoupled(5e-4, 4000)
    assert e1[0] < 1e-4 and e1[1] < 1e-3
    assert 1.8 < e1[0] / e2[0] < 2.2 and 1.8 < e1[1] / e2[1] < 2.2  # Euler: error ~ dt


def test_hopf_oracle_synchronous_state_has_no_coupling():
    """Identical initial states stay identical without noise (sum_j M_ij (x_j - x_i) = 0)."""
    rng = np.random.default_rng(0)
    M = rng.uniform(size=(6, 6))
    x = np.full((1, 6), 0.4)
    y = np.full((1, 6), -0.2)
    p = dict(a=0.0, w=0.3, beta=0.0, dt=0.1, G=0.6, norm=np.mean(M.sum(0)))
    oracle.hopf_integrate(p, M, [3], x, y, 0, 500)
    assert np.ptp(x) == 0 and np.ptp(y) == 0


def test_hopf_oracle_noise_is_the_philox_pair_stream():
    """Node i's (x, y) noise = Box-Muller pair (2i, 2i+1) of the simulation's stream:
    with a zero drift (a = w = G = 0, x = y = 0), one step adds beta sqrt(dt) z."""
    N = 7
    x, y = np.zeros((1, N)), np.zeros((1, N))
    p = dict(a=0.0, w=0.0, beta=0.5, dt=0.04, G=0.0, norm=1.0)
    oracle.hopf_integrate(p, np.zeros((N, N)), [11], x, y, 5, 1)
    z = np.zeros(2 * N + 2)
    lib = oracle.lib()
    import ctypes
    zz = np.zeros(2 * N)
    lib.orc_step_normals(11, 5, 2 * N, zz.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    np.testing.assert_allclose(x[0], 0.5 * 0.2 * zz[0::2], rtol=0, atol=1e-15)
    np.testing.assert_allclose(y[0], 0.5 * 0.2 * zz[1::2], rtol=0, atol=1e-15)
    del z


def test_filtfilt_order6_oracle_matches_scipy():
    b, a, _ = band(0.1)
    x = np.random.default_rng(1).standard_normal((7200, 4)).cumsum(0) * 0.01
    np.testing.assert_array_equal(osg.filtfilt(b, a, x), signal.filtfilt(b, a, x, axis=0))


def test_graph_utils_match_reference_semantics():
    rng = np.random.default_rng(2)
    m = rng.uniform(size=(9, 9))
    m = m + m.T
    loop = [m[r, c] for r in range(8) for c in range(r + 1, 9)]  # graph_utils.py:100-103
    np.testing.assert_array_equal(graph_utils.get_uptri(m), loop)
    rec = graph_utils.matrix_recon(graph_utils.get_uptri(m))
    np.testing.assert_array_equal(rec, m - np.diag(np.diag(m)))
    t = graph_utils.thresholding(m.copy(), 0.3)
    k = int(36 * 0.3)
    assert (graph_utils.get_uptri(t) > 0).sum() == k
    np.testing.assert_array_equal(np.sort(graph_utils.get_uptri(t))[-k:], np.sort(loop)[-k:])
    assert (t == t.T).all() and (np.diag(t) == 0).all()


def test_fitting_measures_match_scipy():
    rng = np.random.default_rng(3)
    o, s = rng.uniform(size=4005), rng.uniform(size=4005) * 0.8 + 0.1
    f = fitting_measures(o, s)
    assert f[0] == np.mean(o) - np.mean(s)
    assert ks_2samp(o, s) == stats.ks_2samp(o, s)[0]
    np.testing.assert_allclose(f[2], np.linalg.norm(o - s), rtol=1e-15)
    np.testing.assert_allclose(f[3], stats.pearsonr(o, s)[0], rtol=1e-13)


def test_update_sc_follows_the_reference_steps():
    """optimize_SC_Hopf.py:89-101 restated line by line against update_sc."""
    rng = np.random.default_rng(4)
    C = rng.uniform(size=(90, 90)) * (rng.uniform(size=(90, 90)) < 0.4)
    C = np.triu(C, 1) + np.triu(C, 1).T
    obj, sim = rng.uniform(size=4005), rng.uniform(size=4005)
    osum = C.sum() * 1.1
    ref = C.copy()
    ref[HOMOTOPIC[:, 0], HOMOTOPIC[:, 1]] += graph_utils.matrix_recon(0.03 * (obj - sim))[HOMOTOPIC[:, 0], HOMOTOPIC[:, 1]]
    ref[ref < 0] = 0
    ref = graph_utils.thresholding(ref, 0.3)
    ref = ref * osum / np.sum(ref)
    np.testing.assert_array_equal(update_sc(C, obj, sim, 0.03, osum), ref)
