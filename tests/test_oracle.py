"""The CPU oracle pinned against known answers (no GPU)."""
import numpy as np
import pytest

import oracle
from nremmodfc_amd.model import WCParams, driver_params, sim_keys

# Random123 known-answer vectors for philox4x32-10 (kat_vectors, Salmon et al. SC'11)
KAT = [
    ([0, 0, 0, 0], [0, 0], [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]),
    ([0xffffffff] * 4, [0xffffffff] * 2, [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]),
    ([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0],
     [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]),
]


@pytest.mark.parametrize("ctr,key,want", KAT)
def test_philox_kat(ctr, key, want):
    assert oracle.philox(ctr, key) == want


def test_normals_distribution():
    # 200 steps x 1000 nodes of one stream: N(0,1) moments
    z = np.concatenate([oracle.step_normals(12345, s, 1000) for s in range(200)])
    assert abs(z.mean()) < 0.01
    assert abs(z.std() - 1.0) < 0.01
    assert abs(np.mean(z ** 3)) < 0.03
    assert abs(np.mean(z ** 4) - 3.0) < 0.06


def test_normals_distinct_streams():
    a = oracle.step_normals(1, 0, 90)
    b = oracle.step_normals(2, 0, 90)
    c = oracle.step_normals(1, 1, 90)
    assert not np.allclose(a, b) and not np.allclose(a, c)
    # partial quads: N=90 is a prefix of N=92
    assert np.array_equal(oracle.step_normals(7, 3, 92)[:90], oracle.step_normals(7, 3, 90))


def test_deterministic_fixed_point(sc90):
    """With no noise and sigma=0 the E sigmoid is 1/2: E* solves -E + (1-rE E)/2 = 0."""
    p = driver_params(D=0.0)
    ob = oracle.OracleBatch(sc90, 0.16, 0.0, sim_keys([0], [0]), p)
    ob.integrate(20000, 0.05)
    e_star = 1.0 / (2.0 + p.rE)  # -E + (1 - rE E)/2 = 0
    np.testing.assert_allclose(ob.E, e_star, rtol=1e-9)


def test_euler_step_by_hand(sc90):
    """One Euler step equals a direct numpy evaluation of wc:77-83."""
    p = driver_params()
    N = 90
    G, sig = 0.16, 7.68
    ob = oracle.OracleBatch(sc90, G, sig, sim_keys([3], [5]), p)
    key = int(sim_keys([3], [5])[0])
    E, I, A = ob.E[0].copy(), ob.I[0].copy(), ob.A[0].copy()
    ob.integrate(1, 1.0)
    z = oracle.step_normals(key, 0, N)
    S = lambda x, s, m: 1 / (1 + np.exp(-(x - m) * s))
    dE = (-E + (1 - p.rE * E) * S(p.a_ee * E - A * I + G * (sc90 @ E) + p.P + p.sqdtD * z, sig, p.mu)) / p.tauE
    dI = (-I + (1 - p.rI * I) * S(p.a_ei * E - p.a_ii * I, p.sigmaI, p.mu)) / p.tauI
    dA = I * (E - p.rhoE) / 1.0
    np.testing.assert_allclose(ob.E[0], E + p.dtSim * dE, rtol=1e-13)
    np.testing.assert_allclose(ob.I[0], I + p.dtSim * dI, rtol=1e-13)
    np.testing.assert_allclose(ob.A[0], A + p.dtSim * dA, rtol=1e-13)


def test_record_semantics(sc90):
    """Samples are the state BEFORE every rec_every-th update (wc:124-125)."""
    p = driver_params()
    keys = sim_keys([0, 1], [0, 0])
    a = oracle.OracleBatch(sc90, 0.16, 7.68, keys, p)
    rec = a.integrate(100, 2.0, rec_every=20)
    b = oracle.OracleBatch(sc90, 0.16, 7.68, keys, p)
    for k in range(5):
        np.testing.assert_array_equal(rec[:, k, :], b.E)
        b.integrate(20, 2.0)
    np.testing.assert_array_equal(a.E, b.E)
