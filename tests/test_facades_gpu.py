"""Drop-in module facades (netwWilsonCowanPlastic, utils) used the reference's way.

Tolerances: wc.run() fp64 vs the oracle 1e-9 (same as test_sde_gpu); simBOLD
1e-7 relative (filtfilt conditioning, see test_signal_gpu); utils against the
reference's own utils.py outputs (golden_utils.npz) rtol 1e-9.
"""
import os

import numpy as np
import pytest

import oracle
import oracle.sigchain as osg
from nremmodfc_amd import datasets
from tests.golden.make_golden import inputs

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_utils_get_all_metrics_golden(cuda):
    from nremmodfc_amd import utils
    gu = np.load(os.path.join(G, "golden_utils.npz"))
    emps = [datasets.load_empfc(s) for s in datasets.STATES]
    fcs = inputs()["fcs"] + [emps[0], emps[3]]
    for i, fc in enumerate(fcs):
        for j, e in enumerate(emps):
            got = utils.get_all_metrics(fc, e, data_range=1)
            np.testing.assert_allclose(got, gu["metrics"][i, j], rtol=1e-9, atol=1e-12)


def test_utils_kuramoto_golden(cuda):
    from nremmodfc_amd import utils
    gu = np.load(os.path.join(G, "golden_utils.npz"))
    for i, k in enumerate(inputs()["kur"]):
        np.testing.assert_allclose(utils.kuramoto(k), gu["kuramoto"][i], rtol=1e-9)


def test_wc_run_like_reference_driver(cuda, sc90):
    """whole_sweep_both.py:39-78 style: set module globals, recompile, run, simBOLD."""
    from nremmodfc_amd import netwWilsonCowanPlastic as wc
    from nremmodfc_amd.model import driver_params, sim_keys
    wc.P, wc.rhoE, wc.CM = 0.4, 0.18, sc90
    wc.precision = "f64"
    wc.tTrans1, wc.tTrans2, tstop = 0.02, 0.2, 2.0
    wc.timeTrans1 = np.arange(0, wc.tTrans1, wc.dtSim)
    wc.timeTrans2 = np.arange(0, wc.tTrans2, wc.dtSim)
    wc.tstop = tstop
    wc.timeSim = np.arange(0, tstop, wc.dtSim)
    wc.time = np.arange(0, tstop, wc.dt)
    wc.G, wc.sigmaE, wc.sid = 0.16, 7.68, 3
    wc.run.recompile()
    tray = wc.run()
    assert tray.shape == (len(wc.time), 3, 90) and tray.dtype == np.float64

    ob = oracle.OracleBatch(sc90, 0.16, 7.68, sim_keys([3], [0]), driver_params())
    ob.integrate(len(wc.timeTrans1), 0.05)
    ob.integrate(len(wc.timeTrans2), 1.0)
    rec = ob.integrate(len(wc.timeSim), 2.0, wc.downsamp)[0]
    np.testing.assert_allclose(tray[:, 0, :], rec, rtol=0, atol=1e-9)
    np.testing.assert_allclose(tray[-1, 2, :], ob.A[0], rtol=0, atol=1e-3)  # a_ie: last record is <20 steps before the end
    assert np.isfinite(tray).all()

    E = np.tile(tray[:, 0, :], (7, 1))  # 7000 samples: past the 2000-sample BOLD transient
    bold = wc.simBOLD(E, nnodes=90)
    want = osg.sim_bold(E, bold_downsamp=1000)
    assert bold.shape == want.shape
    assert np.abs(bold - want).max() <= 1e-7 * np.abs(want).max()


def test_wc_run_checks_globals(cuda):
    from nremmodfc_amd import netwWilsonCowanPlastic as wc
    n = wc.N
    wc.N = n + 1
    try:
        with pytest.raises(ValueError):
            wc.run()
    finally:
        wc.N = n
    with pytest.raises(ValueError):
        wc.wilsonCowan(0.0, np.zeros((3, n + 1)), 7.68, 1, 2, 0.16)


def test_wilsonCowan_single_evaluation(cuda, sc90):
    """wc.wilsonCowan(t, X, sigmaE, mu, tau_ip, G) (wc:77-83) on the device: the reference's
    expression in numpy with the same normals (Philox step k of key (sid, RHS_STREAM) on the k-th
    call for that sid; independent of run()'s stream 0 and counted per sid)."""
    from nremmodfc_amd import netwWilsonCowanPlastic as wc
    from nremmodfc_amd.model import sim_keys
    old = {k: getattr(wc, k) for k in ("CM", "P", "rhoE", "sid")}
    try:
        wc.CM, wc.P, wc.rhoE, wc.sid = sc90, 0.4, 0.18, 21
        wc._rhs_steps.clear()
        rng = np.random.default_rng(3)
        X = np.stack([rng.uniform(0.05, 0.4, 90), rng.uniform(0.05, 0.4, 90), rng.uniform(2.3, 2.7, 90)])
        ach = datasets.load_map("DIST_VAChT_feobv_hc18_aghourian")
        key = int(sim_keys([21], [wc.RHS_STREAM])[0])
        S = lambda x, s, m: 1 / (1 + np.exp(-(x - m) * s))  # noqa: E731
        for k, (G, sig, mu, tau) in enumerate([(0.16, 7.68, 1, 2), (0.16 + 0.1 * ach, 7.5, 1.1, 0.05)]):
            got = wc.wilsonCowan(0.0, X, sig, mu, tau, G)
            E, I, A = X
            noise = wc.sqdtD * oracle.step_normals(key, k, 90)
            want = np.vstack(((-E + (1 - wc.rE * E) * S(wc.a_ee * E - A * I + G * np.dot(sc90, E) + wc.P + noise,
                                                            sig, mu)) / wc.tauE,
                              (-I + (1 - wc.rI * I) * S(wc.a_ei * E - wc.a_ii * I, wc.sigmaI, mu)) / wc.tauI,
                              (I * (E - wc.rhoE)) / tau))
            assert got.shape == (3, 90)
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
        assert wc._rhs_steps == {21: 2}
    finally:
        for k, v in old.items():
            setattr(wc, k, v)


def test_cortex_run_flow(cuda, sc90):
    """cortex_run.py:69-135 style: per-node G / sigmaE maps assigned to the module
    globals, wilsonCowan.recompile(), run(), simBOLD at BOLD_downsamp=10, Kuramoto of
    both the BOLD and the raw E_t, and the metrics against an empirical FC."""
    from nremmodfc_amd import netwWilsonCowanPlastic as wc
    from nremmodfc_amd import utils
    from nremmodfc_amd.model import sim_keys
    ach = datasets.load_map("DIST_VAChT_feobv_hc18_aghourian")
    na = datasets.load_map("DIST_LC_proj")
    G, S = 0.16 + 0.1 * ach, 7.68 - 0.12 * na
    old = {k: getattr(wc, k) for k in ("CM", "G", "sigmaE", "rhoE", "P", "tTrans1", "tTrans2", "tstop", "timeTrans1",
                                       "timeTrans2", "timeSim", "time", "sid", "precision")}
    try:
        wc.sigmaE, wc.G, wc.CM, wc.rhoE, wc.P = S, G, sc90, 0.14, 0.4
        wc.precision = "f64"
        wc.tTrans1, wc.tTrans2, tstop = 0.01, 0.1, 10.0
        wc.timeTrans1 = np.arange(0, wc.tTrans1, wc.dtSim)
        wc.timeTrans2 = np.arange(0, wc.tTrans2, wc.dtSim)
        wc.tstop = tstop
        wc.timeSim = np.arange(0, tstop, wc.dtSim)
        wc.time = np.arange(0, tstop, wc.dt)
        wc.sid = 11
        wc.wilsonCowan.recompile()
        tray = wc.run()
        assert tray.shape == (len(wc.time), 3, 90)

        ob = oracle.OracleBatch(sc90, G, S, sim_keys([11], [0]), wc._params())
        ob.integrate(len(wc.timeTrans1), 0.05)
        ob.integrate(len(wc.timeTrans2), 1.0)
        rec = ob.integrate(len(wc.timeSim), 2.0, wc.downsamp)[0]
        np.testing.assert_allclose(tray[:, 0, :], rec, rtol=0, atol=1e-9)

        E_t = tray[:, 0, :]
        bold = wc.simBOLD(E_t, nnodes=90, BOLD_downsamp=10)
        want = osg.sim_bold(E_t, bold_downsamp=10)
        assert bold.shape == want.shape == ((len(wc.time) - 2000 + 9) // 10, 90)
        assert np.abs(bold - want).max() <= 1e-7 * np.abs(want).max()

        np.testing.assert_allclose(utils.kuramoto(bold), osg.kuramoto(bold), rtol=1e-9)
        np.testing.assert_allclose(utils.kuramoto(E_t), osg.kuramoto(E_t), rtol=1e-9)
        sfc = np.corrcoef(bold.T)
        got = utils.get_all_metrics(sfc, datasets.load_empfc("W"), data_range=1)
        assert np.isfinite(got).all() and -1 <= got[0] <= 1
    finally:
        for k, v in old.items():
            setattr(wc, k, v)
