"""Device HMA (wc_hma) vs the reference HMA.py outputs (golden_hma.npz) and vs the
host facade nremmodfc_amd.HMA on random FC-like matrices, odd N included."""
import os

import numpy as np
import pytest
import torch

from nremmodfc_amd import HMA, datasets, sigchain
from tests.golden.make_golden import inputs

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_hma.npz")


def _fc_like(rng, B, N, T=298):
    """corrcoef of correlated random series: one large mode plus structure, as simulated FC."""
    out = []
    for _ in range(B):
        common = rng.standard_normal((T, 1))
        mods = rng.standard_normal((T, 4))[:, rng.integers(0, 4, N)]
        x = 0.6 * common + 0.5 * mods + rng.standard_normal((T, N))
        out.append(np.corrcoef(x.T))
    return np.stack(out)


def test_hma_matches_reference_golden(cuda):
    g = np.load(G)
    emps = [datasets.load_empfc(s) for s in ("W", "N1", "N2", "N3")]
    fcs = np.stack(inputs()["fcs"] + emps)
    t = torch.from_numpy(fcs.copy()).to(cuda)
    r = sigchain.hma(t, want_clus_num=True)
    cn = r["clus_num"].cpu().numpy()
    for i in range(len(fcs)):
        np.testing.assert_array_equal(cn[i], g[f"clus_num{i}"])
        np.testing.assert_allclose(r["hin"][i].item(), g[f"hin{i}"], rtol=1e-12)
        np.testing.assert_allclose(r["hse"][i].item(), g[f"hse{i}"], rtol=1e-12)
        np.testing.assert_allclose(r["hin_node"][i].cpu().numpy(), g[f"hin_node{i}"], rtol=1e-10, atol=1e-15)
        np.testing.assert_allclose(r["hse_node"][i].cpu().numpy(), g[f"hse_node{i}"], rtol=1e-10, atol=1e-15)
        np.testing.assert_array_equal(t[i].cpu().numpy(), g[f"clipped{i}"])  # in-place clip (HMA.py:55)


@pytest.mark.parametrize("N,B", [(90, 40), (89, 7), (17, 5), (96, 3), (3, 2)])
def test_hma_matches_host_facade(cuda, N, B):
    rng = np.random.default_rng(N * 100 + B)
    fcs = _fc_like(rng, B, N)
    r = sigchain.hma(torch.from_numpy(fcs.copy()).to(cuda), want_clus_num=True)
    for b in range(B):
        f = fcs[b].copy()
        cn, cs, _ = HMA.Functional_HP(f)
        hin, hse = HMA.Balance(f, cn, cs)
        hin_n, hse_n = HMA.nodal_measures(f, cn, cs)
        np.testing.assert_array_equal(r["clus_num"][b].cpu().numpy(), cn)
        np.testing.assert_allclose(r["hin"][b].item(), hin, rtol=1e-12)
        np.testing.assert_allclose(r["hse"][b].item(), hse, rtol=1e-11)
        np.testing.assert_allclose(r["hin_node"][b].cpu().numpy(), hin_n, rtol=1e-10, atol=1e-15)
        np.testing.assert_allclose(r["hse_node"][b].cpu().numpy(), hse_n, rtol=1e-9, atol=1e-15)
        sv = np.linalg.svd(np.where(fcs[b] < 0, 0, fcs[b]), compute_uv=False)
        np.testing.assert_allclose(r["sv"][b].cpu().numpy(), sv, rtol=1e-11, atol=1e-13)


@pytest.mark.parametrize("N,B", [(97, 3), (150, 2), (301, 2)])
def test_hma_large_n_matches_host_facade(cuda, N, B):
    """N > 96 (HMA.py has no N cap): the device eigensolver + wc_hma_modes vs the host facade
    (the reference's algorithm, numpy SVD)."""
    rng = np.random.default_rng(N * 7 + B)
    fcs = _fc_like(rng, B, N)
    t = torch.from_numpy(fcs.copy()).to(cuda)
    r = sigchain.hma(t, want_clus_num=True)
    for b in range(B):
        f = fcs[b].copy()
        cn, cs, _ = HMA.Functional_HP(f)
        hin, hse = HMA.Balance(f, cn, cs)
        hin_n, hse_n = HMA.nodal_measures(f, cn, cs)
        np.testing.assert_array_equal(r["clus_num"][b].cpu().numpy(), cn)
        np.testing.assert_allclose(r["hin"][b].item(), hin, rtol=1e-11)
        np.testing.assert_allclose(r["hse"][b].item(), hse, rtol=1e-10)
        np.testing.assert_allclose(r["hin_node"][b].cpu().numpy(), hin_n, rtol=1e-9, atol=1e-14)
        np.testing.assert_allclose(r["hse_node"][b].cpu().numpy(), hse_n, rtol=1e-8, atol=1e-14)
        np.testing.assert_array_equal(t[b].cpu().numpy(), f)  # clipped in place, as HMA.py:55


def test_hma_batch_is_order_independent(cuda):
    rng = np.random.default_rng(5)
    fcs = _fc_like(rng, 6, 90)
    a = sigchain.hma(torch.from_numpy(fcs.copy()).to(cuda))
    b = sigchain.hma(torch.from_numpy(fcs[::-1].copy()).to(cuda))
    assert torch.equal(a["hin"], b["hin"].flip(0)) and torch.equal(a["hse_node"], b["hse_node"].flip(0))
