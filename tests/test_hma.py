"""nremmodfc_amd.HMA vs the reference HMA.py outputs (tests/golden/golden_hma.npz), no GPU."""
import os

import numpy as np

from nremmodfc_amd import HMA, datasets
from tests.golden.make_golden import inputs

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_hma.npz")


def test_hma_matches_reference():
    g = np.load(G)
    emps = [datasets.load_empfc(s) for s in ("W", "N1", "N2", "N3")]
    fcs = inputs()["fcs"] + emps
    assert int(g["n"]) == len(fcs)
    for i, fc in enumerate(fcs):
        f = fc.copy()
        cn, cs, h_all = HMA.Functional_HP(f)
        np.testing.assert_array_equal(np.array(cn), g[f"clus_num{i}"])
        np.testing.assert_array_equal(f, g[f"clipped{i}"])  # in-place clip, as HMA.py:55
        hin, hse = HMA.Balance(f, cn, cs)
        hin_n, hse_n = HMA.nodal_measures(f, cn, cs)
        np.testing.assert_allclose(hin, g[f"hin{i}"], rtol=1e-13)
        np.testing.assert_allclose(hse, g[f"hse{i}"], rtol=1e-13)
        np.testing.assert_allclose(hin_n, g[f"hin_node{i}"], rtol=1e-12, atol=1e-16)
        np.testing.assert_allclose(hse_n, g[f"hse_node{i}"], rtol=1e-12, atol=1e-16)
        assert len(h_all) == fc.shape[0] - 1


def test_integration_segregation_dict_keys():
    d = HMA.integration_segregation(datasets.load_empfc("W").copy())
    assert set(d) == {"Hin_sim", "Hse_sim", "Hin_node_sim", "Hse_node_sim", "sFC"}
    assert (d["sFC"] >= 0).all()
