"""BASELINE config 5 end to end: the N > 96 epilogue (wc_fc_large.hip) and the sweep
pipeline on the 1000-node synthetic connectome.

* FC / get_all_metrics / mean / Kuramoto at N = 97 ... 1000 vs the oracle
  (np.corrcoef, oracle.sigchain = the reference's utils.py restated; utils.py:34-50).
* wc_corrcoef at N > 96 (the SC optimiser's long series) vs np.corrcoef.
* run_sweep at N = 1000 vs the oracle signal chain applied to the same fp64 trajectory
  (the integrator itself is pinned to the oracle in test_sde_large_gpu.py).
* Full size (the C5 shard: 2,500 simulations x 1000 nodes per GPU), where the oracle
  cannot run: permutation, round-robin shard and launch-chunking invariance, bit for bit.
"""
import numpy as np
import pytest
import torch

import oracle.sigchain as osg
from bench import sweep_batch
from nremmodfc_amd import datasets
from nremmodfc_amd import sigchain as wsg
from nremmodfc_amd.model import Batch, Schedule, driver_params, sim_keys
from nremmodfc_amd.pipeline import run_sweep

pytestmark = pytest.mark.gpu


def _series(M, B, N, seed):
    """BOLD-like series with a shared component (FC entries spread over [-1, 1])."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((M, B, N)) + 0.8 * rng.standard_normal((M, B, 1)) * rng.uniform(-1, 1, (1, B, N))
    return x + rng.standard_normal((1, B, N))


def _emp(N, K, seed):
    rng = np.random.default_rng(seed)
    return np.stack([np.corrcoef(rng.standard_normal((3 * N // 2, N)).T + 0.3 * k) for k in range(K)])


@pytest.mark.parametrize("N,B,M,K", [(97, 3, 298, 2), (130, 2, 298, 4), (257, 1, 40, 1), (1000, 2, 298, 2)])
def test_fc_metrics_large_vs_oracle(cuda, N, B, M, K):
    x = _series(M, B, N, N + B)
    emp = _emp(N, K, N)
    xt = torch.from_numpy(x).cuda()
    fc, met, extra = wsg.fc_metrics(xt, B, N, emp, kuramoto=True, want_fc=True)
    _, met2, extra2 = wsg.fc_metrics(xt, B, N, emp, kuramoto=True, want_fc=False)  # FC in the workspace
    torch.cuda.synchronize()
    assert torch.equal(met, met2) and torch.equal(extra, extra2)
    fc, met, extra = fc.cpu().numpy(), met.cpu().numpy(), extra.cpu().numpy()
    for b in range(B):
        sfc = np.corrcoef(x[:, b, :].T)
        np.testing.assert_allclose(fc[b], sfc, rtol=0, atol=1e-12)
        for k in range(K):
            np.testing.assert_allclose(met[b, k], osg.get_all_metrics(sfc, emp[k], 1), rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(extra[b, 0], np.mean(sfc), rtol=1e-12)
        np.testing.assert_allclose(extra[b, 1:], osg.kuramoto(x[:, b, :]), rtol=1e-9)


def test_fc_in_large_vs_oracle(cuda):
    """fc_in mode (precomputed FCs) at N = 400 against the reference's get_all_metrics."""
    N, K = 400, 3
    emp = _emp(N, K, 5)
    fcs = np.stack([_emp(N, 1, 100 + i)[0] for i in range(2)] + [emp[1]])
    _, met, extra = wsg.fc_metrics(fc_in=torch.from_numpy(fcs).cuda(), empfc=emp)
    met, extra = met.cpu().numpy(), extra.cpu().numpy()
    for b in range(len(fcs)):
        for k in range(K):
            np.testing.assert_allclose(met[b, k], osg.get_all_metrics(fcs[b], emp[k], 1), rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(extra[b, 0], fcs[b].mean(), rtol=1e-12)
    assert abs(met[2, 1, 0] - 1.0) < 1e-14 and met[2, 1, 1] == 0.0  # identical matrices


@pytest.mark.parametrize("M,B,N", [(6000, 2, 200), (300, 1, 1000), (5, 3, 97)])
def test_corrcoef_large_vs_numpy(cuda, M, B, N):
    rng = np.random.default_rng(M + B + N)
    x = rng.standard_normal((M, B, N)).cumsum(0) * 0.01 + rng.standard_normal((1, B, N))
    fc = wsg.corrcoef(torch.from_numpy(x).cuda(), B, N).cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(fc[b], np.corrcoef(x[:, b, :].T), rtol=0, atol=1e-12)


def test_pipeline_n1000_vs_oracle_chain(cuda):
    """run_sweep on the 1000-node synthetic connectome (fp64): BOLD, FC, gof vs two
    synthetic 'empirical' FCs, Kuramoto, mean and the Welch peak equal the oracle's
    epilogue (whole_sweep_both.py:79-95 restated) applied to the same trajectory."""
    N, B = 1000, 2
    sc = datasets.synthetic_sc(N)
    sch = Schedule(n_trans1=20, n_trans2=200, n_sim=80_000)  # T = 4000 samples: one Welch segment
    G = np.array([0.16, 0.26])
    S = np.array([7.68, 7.58])
    keys = sim_keys([0, 1], [3, 17])
    emp = dict(zip(("W", "N1"), _emp(N, 2, 9)))
    res = run_sweep(sc, G, S, keys, emp, sch, precision="f64", bold_downsamp=100, want_fc=True, want_bold=True)
    bt = Batch(sc, G, S, keys, driver_params(), precision="f64")
    bt.integrate(sch.n_trans1, 0.05)
    bt.integrate(sch.n_trans2, 1.0)
    rec = torch.empty((sch.n_sim // 20, B, N), dtype=torch.float64, device="cuda")
    bt.integrate(sch.n_sim, 2.0, 20, rec)
    rec = rec.cpu().numpy()
    cols = res.columns()
    for b in range(B):
        want, wbold, wfc = osg.sim_metrics(rec[:, b, :], emp, bold_downsamp=100)
        assert np.abs(res.bold[:, b, :] - wbold).max() <= 1e-7 * np.abs(wbold).max()
        assert np.abs(res.fc[b] - wfc).max() <= 1e-6
        for name, v in want.items():
            if name == "peakfreq":
                assert cols[name][b] == v, (name, cols[name][b], v)
            else:
                np.testing.assert_allclose(cols[name][b], v, rtol=1e-6, atol=1e-8, err_msg=name)


def _c5_shard():
    """The C5 per-GPU shard: 2,500 simulations of the (G, sigma) x seed grid (bench.py --config c5)."""
    G, S, keys = sweep_batch(0)
    return G[:2500], S[:2500], keys[:2500]


def _state(bt):
    return torch.stack([bt.E, bt.I, bt.A]).cpu().numpy()


def test_c5_full_shard_permutation_shard_chunking(cuda):
    sc = datasets.synthetic_sc(1000)
    G, S, keys = _c5_shard()
    B = len(keys)
    p = driver_params()
    full = Batch(sc, G, S, keys, p, precision="f32")
    full.integrate(200, 0.05)
    full.integrate(200, 2.0)
    ref = _state(full)
    perm = np.random.default_rng(1).permutation(B)
    pb = Batch(sc, G[perm], S[perm], keys[perm], p, precision="f32")
    pb.integrate(200, 0.05)
    pb.integrate(200, 2.0)
    assert np.array_equal(_state(pb), ref[:, perm])
    shard = np.arange(B)[np.arange(B) % 8 == 3]  # 313 simulations: ragged sim tiles
    sb = Batch(sc, G[shard], S[shard], keys[shard], p, precision="f32")
    for n in (1, 150, 49):
        sb.integrate(n, 0.05)
    sb.integrate(200, 2.0)
    assert np.array_equal(_state(sb), ref[:, shard])


def test_c5_full_shard_pipeline_rows(cuda):
    """The whole chain for the 2,500 x 1000 shard on a short schedule: every output is
    finite, and a round-robin sub-shard run on its own reproduces its rows exactly."""
    sc = datasets.synthetic_sc(1000)
    G, S, keys = _c5_shard()
    sch = Schedule(n_trans1=200, n_trans2=2000, n_sim=100_000)  # T = 5000
    full = run_sweep(sc, G, S, keys, {}, sch, bold_downsamp=100)
    shard = np.arange(len(keys))[np.arange(len(keys)) % 8 == 5]
    part = run_sweep(sc, G[shard], S[shard], keys[shard], {}, sch, bold_downsamp=100)
    fc = full.columns()
    for k, v in part.columns().items():
        assert np.array_equal(v, fc[k][shard]), k
    for k in ("sync", "meta", "mean", "peakfreq"):
        assert np.isfinite(fc[k]).all(), k
    assert (fc["peakfreq"] > 0).all() and (np.abs(fc["mean"]) <= 1).all()
