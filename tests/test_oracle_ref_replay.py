"""The oracle's run() pinned to the REFERENCE's own source at fixed noise (no GPU).

tests/golden/ref_replay.npz holds Y_t as /root/reference/netwWilsonCowanPlastic.py:86-137
itself returns it (numba decorators as identities, np.random.normal replaying the build's
Philox stream; tests/golden/make_ref_replay.py) for a homogeneous and a maps-mode parameter
vector over 100 + 100 + 2000 Euler steps.  The oracle fed the same normals must reproduce
E, I and a_ie at every recorded step.  They differ only in rounding: np.dot (BLAS order)
and numpy's exp against the C loop's sequential sum and libm (observed max 3.1e-15).
"""
import os

import numpy as np
import pytest

import oracle
from nremmodfc_amd import datasets
from nremmodfc_amd.model import driver_params

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_replay.npz")


def oracle_Y(d, name):
    """Y_t [n_rec][3][N] of the oracle for one fixture case (state BEFORE every 20th step)."""
    n1, n2, n3 = (int(x) for x in d["steps"])
    R = int(d["rec_every"])
    ob = oracle.OracleBatch(datasets.load_sc(), d[f"{name}_G"][None], d[f"{name}_sigmaE"][None],
                            [int(d[f"{name}_key"])], driver_params())
    ob.integrate(n1, 0.05)
    ob.integrate(n2, 1.0)
    rows = []
    for _ in range(n3 // R):
        rows.append(np.stack([ob.E[0], ob.I[0], ob.A[0]]))
        ob.integrate(R, 2.0)
    return np.array(rows)


@pytest.mark.parametrize("name", ["homo", "maps"])
def test_oracle_matches_reference_run(name):
    d = np.load(GOLD)
    Y = d[f"{name}_Y"]
    assert Y.shape == (100, 3, 90)
    diff = np.abs(oracle_Y(d, name) - Y)
    print(f"TOL ref-replay-{name} max={diff.max():.3e} exact={np.mean(diff == 0):.3f}")
    assert diff.max() <= 1e-13, diff.max(axis=(0, 2))
    # the replay is not vacuous: the noise moves the trajectory by far more than the bound
    assert np.abs(np.diff(Y[:, 0, :], axis=0)).max() > 1e-3


def test_replay_fixture_is_sensitive_to_the_noise():
    """A different key gives a different trajectory: the fixture pins the noise replay too."""
    d = np.load(GOLD)
    e = dict(d)
    e["homo_key"] = np.array(int(d["homo_key"]) + 1, dtype=np.uint64)
    diff = np.abs(oracle_Y(e, "homo") - d["homo_Y"])
    assert diff.max() > 1e-4
