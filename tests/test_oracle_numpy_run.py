"""oracle/numpy_run.py (the bench's reference-shaped CPU leg) is the reference's NumPy loop:
fed the replayed Philox normals it reproduces the Y_t that the reference's own source produced
(tests/golden/ref_replay.npz, make_ref_replay.py) bit for bit (no GPU)."""
import os

import numpy as np
import pytest

import oracle
from nremmodfc_amd import datasets
from nremmodfc_amd.model import driver_params
from oracle import numpy_run

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_replay.npz")


@pytest.mark.parametrize("name", ["homo", "maps"])
def test_numpy_restatement_is_the_reference_loop(name):
    d = np.load(GOLD)
    key, N = int(d[f"{name}_key"]), 90
    step = [0]

    def normal(loc, scale, size):
        z = oracle.step_normals(key, step[0], size)
        step[0] += 1
        return loc + scale * z

    G, S = d[f"{name}_G"], d[f"{name}_sigmaE"]
    if name == "homo":  # the homogeneous driver sets scalars (whole_sweep_both.py:68-72)
        G, S = float(G[0]), float(S[0])
    n1, n2, n3 = (int(x) for x in d["steps"])
    Y = numpy_run.run(driver_params(), datasets.load_sc(), G, S, n1, n2, n3, int(d["rec_every"]), normal=normal)
    assert step[0] == n1 + n2 + n3
    np.testing.assert_array_equal(Y, d[f"{name}_Y"])
