"""HIP signal chain (libwcsde.so) vs the CPU oracle and the golden vectors.

Tolerances:
  * simBOLD (BOLD ODE + filtfilt + decimation), fp64: |d| <= 1e-7 * max|BOLD|.
    The band-pass's DF2T recursion is ill-conditioned (companion matrix with
    |A^1000| ~ 3e7): SciPy's own filtfilt sits 4e-9 from an extended-precision
    evaluation, two association orders of the same fp64 recursion differ by
    ~6e-9, and a 1-ulp change of the BOLD input (exp(log v / alpha) vs pow)
    moves the output by 2-6e-8;
  * FC: 1e-12; get_all_metrics, kuramoto, mean(FC): rtol 1e-9;
  * Welch PSD: rtol 1e-9 (fp64 input), 2e-4 (fp32 input); peak frequency exact.
"""
import os

import numpy as np
import pytest
import torch

import oracle
import oracle.sigchain as osg
from nremmodfc_amd import datasets
from nremmodfc_amd import sigchain as wsg
from tests.golden.make_golden import inputs

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _e_like(T, C, seed):
    rng = np.random.default_rng(seed)
    t = np.arange(T) / 500.0
    return (0.2 + 0.1 * np.sin(2 * np.pi * 4.8 * t)[:, None] * rng.uniform(0.5, 1.5, C)
            + 0.03 * rng.standard_normal((T, C))).astype(np.float64)


@pytest.mark.parametrize("T,dec,C", [(20_000, 1000, 6), (12_345, 1000, 3), (5_000, 10, 4), (300_000, 1000, 2)])
def test_sim_bold_matches_oracle(cuda, T, dec, C):
    E = _e_like(T, C, T + dec)
    want = osg.sim_bold(E, bold_downsamp=dec)
    got = wsg.sim_bold(torch.from_numpy(E).cuda(), bold_downsamp=dec).cpu().numpy()
    assert got.shape == want.shape
    assert np.abs(got - want).max() <= 1e-7 * np.abs(want).max(), np.abs(got - want).max() / np.abs(want).max()


def test_bold_chunking_is_exact(cuda):
    T, C = 9_000, 5
    E = torch.from_numpy(_e_like(T, C, 7)).cuda()
    one = wsg.sim_bold(E, bold_downsamp=1000)
    bs = wsg.BoldStream(C, T, dec=1000)
    for a, b in ((0, 17), (17, 2000), (2000, 2001), (2001, 5555), (5555, T)):
        bs.feed(E[a:b].contiguous())
    assert torch.equal(one, bs.finish())
    # node-major ring-slot input (e_ld) gives the same
    nm = E.t().contiguous()
    bs2 = wsg.BoldStream(C, T, dec=1000)
    bs2.feed(nm, T, e_ld=T)
    assert torch.equal(one, bs2.finish())


@pytest.mark.parametrize("C", [5, 300, 700])
def test_bold_copy_transposes_into_ring(cuda, C):
    """wc_bold_chunk's copy output: the fp32 time-major chunk lands node-major in
    the ring slot (ragged chunk lengths and column counts), and the BOLD result is
    unchanged."""
    T = 6_000
    E = torch.from_numpy(_e_like(T, C, C)).float().cuda()
    ref = wsg.BoldStream(C, T, dec=1000)
    ref.feed(E)
    want = ref.finish()
    ld = 4000
    ring = torch.full((C * ld,), float("nan"), dtype=torch.float32, device="cuda")
    bs = wsg.BoldStream(C, T, dec=1000)
    t = 0
    for n in (1000, 37, 963, 1000, 1000, 1000, 1000, 1000 - 0):
        n = min(n, T - t)
        if n <= 0:
            break
        slot_off = (t % ld)
        if slot_off + n > ld:  # keep each chunk inside the ring (test layout only)
            n = ld - slot_off
        bs.feed(E[t:t + n].contiguous(), copy=ring, copy_ld=ld, copy_offset=slot_off)
        got = ring.view(C, ld)[:, slot_off:slot_off + n]
        assert torch.equal(got, E[t:t + n].t()), (t, n)
        t += n
    while t < T:  # the rest without copies
        bs.feed(E[t:T].contiguous())
        t = T
    assert torch.equal(bs.finish(), want)


def test_fc_metrics_vs_oracle(cuda):
    rng = np.random.default_rng(3)
    B, N, M = 5, 90, 298
    bold = rng.standard_normal((M, B, N)).cumsum(0) + rng.standard_normal((M, B, 1))
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    fc, met, extra = wsg.fc_metrics(torch.from_numpy(bold).cuda(), B, N, np.stack(list(emp.values())),
                                    want_fc=True)
    fc, met, extra = fc.cpu().numpy(), met.cpu().numpy(), extra.cpu().numpy()
    for b in range(B):
        sfc = np.corrcoef(bold[:, b, :].T)
        np.testing.assert_allclose(fc[b], sfc, rtol=0, atol=1e-12)
        for k, s in enumerate(emp):
            np.testing.assert_allclose(met[b, k], osg.get_all_metrics(sfc, emp[s], 1), rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(extra[b, 0], np.mean(sfc), rtol=1e-12)
        np.testing.assert_allclose(extra[b, 1:], osg.kuramoto(bold[:, b, :]), rtol=1e-9)


def test_gof_vs_reference_utils_golden(cuda):
    """fc_in mode against the reference's own utils.get_all_metrics outputs."""
    inp = inputs()
    gu = np.load(os.path.join(G, "golden_utils.npz"))
    emps = np.stack([datasets.load_empfc(s) for s in ("W", "N1", "N2", "N3")])
    fcs = np.stack(inp["fcs"] + [emps[0], emps[3]])
    _, met, _ = wsg.fc_metrics(fc_in=torch.from_numpy(fcs).cuda(), empfc=emps)
    np.testing.assert_allclose(met.cpu().numpy(), gu["metrics"], rtol=1e-9, atol=1e-12)


def test_kuramoto_vs_reference_utils_golden(cuda):
    inp = inputs()
    gu = np.load(os.path.join(G, "golden_utils.npz"))
    for i, k in enumerate(inp["kur"]):
        M, N = k.shape
        _, _, extra = wsg.fc_metrics(torch.from_numpy(k).cuda(), 1, N, None)
        np.testing.assert_allclose(extra[0, 1:].cpu().numpy(), gu["kuramoto"][i], rtol=1e-9)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_welch_vs_oracle(cuda, dtype):
    B, N, T = 3, 7, 20_000
    E = _e_like(T, B * N, 11).reshape(T, B, N)
    Et = torch.from_numpy(E).to("cuda", dtype)
    peak, psd = wsg.welch_peak(Et, want_psd=True)
    Eh = Et.double().cpu().numpy()
    for b in range(B):
        f, P = osg.welch_psd(Eh[:, b, :].T, 500.0, 4000)
        mp = P.mean(axis=0)
        rt = 1e-9 if dtype == torch.float64 else 2e-4
        np.testing.assert_allclose(psd[b].cpu().numpy(), mp, rtol=rt, atol=rt * mp.max())
        assert peak[b].item() == osg.welch_peak(Eh[:, b, :])


@pytest.mark.parametrize("B,N", [(5, 1), (2, 3), (4, 9)])
def test_welch_f32_ring_wrap_and_small_n(cuda, B, N):
    """fp32 product kernel: a segment that wraps the 4-slot ring (ld padded past
    slot * nslots) gives the same accumulator bits as the same samples read from a
    contiguous column; N < 4 leaves waves idle; odd B leaves half a workgroup empty.
    Each simulation's PSD also matches the oracle."""
    T = 6000
    X = torch.from_numpy(_e_like(T, B * N, B * 10 + N).T.copy()).to("cuda", torch.float32)  # [C][T]
    slot, nslots, ld = 1000, 4, 4096
    ring = torch.zeros((B * N, ld), dtype=torch.float32, device="cuda")
    for t0 in range(2000, T, slot):  # samples [2000, 6000) into slots (t // slot) % 4
        q = (t0 // slot) % nslots
        ring[:, q * slot:(q + 1) * slot] = X[:, t0:t0 + slot]
    a = wsg.WelchAccumulator(B, N)
    a.accumulate(ring.reshape(-1), ld, slot, nslots, 2000)  # runs: slots 2, 3, 0, 1
    c = wsg.WelchAccumulator(B, N)
    c.accumulate(X.reshape(-1), T, T, 1, 2000)
    torch.cuda.synchronize()
    assert torch.equal(a.acc, c.acc)
    _, psd = a.peak(want_psd=True)
    Xh = X.double().cpu().numpy().reshape(B, N, T)
    for b in range(B):
        f, P = osg.welch_psd(Xh[b][:, 2000:], 500.0, 4000)
        mp = P.mean(axis=0)
        np.testing.assert_allclose(psd[b].cpu().numpy(), mp, rtol=2e-4, atol=2e-4 * mp.max())


@pytest.mark.parametrize("B,N,K", [(5, 1, 2), (3, 2, 2), (4, 9, 2), (2, 90, 2), (3, 3, 4), (2, 90, 4)])
def test_welch_f32_two_segments_per_launch(cuda, B, N, K):
    """nseg = K (2: the pipeline's form; 4): one launch of K overlapping segments over a ring of
    4000 + 2000 (K - 1) samples, wrapping, equals the K segments launched one by one to fp32
    summation order (the waves group the per-lane sums differently), with the same peaks; and the
    PSD matches the oracle.  Small N leaves some waves of a simulation idle."""
    span = 4000 + 2000 * (K - 1)
    T = 4000 + span
    X = torch.from_numpy(_e_like(T, B * N, B * 20 + N).T.copy()).to("cuda", torch.float32)  # [C][T]
    slot = 1000
    nslots = span // slot
    ld = nslots * slot + 144
    ring = torch.zeros((B * N, ld), dtype=torch.float32, device="cuda")
    for t0 in range(4000, T, slot):  # samples [4000, T) into slots (t // slot) % nslots
        q = (t0 // slot) % nslots
        ring[:, q * slot:(q + 1) * slot] = X[:, t0:t0 + slot]
    two = wsg.WelchAccumulator(B, N)
    two.accumulate(ring.reshape(-1), ld, slot, nslots, 4000, nseg=K)  # [4000 + 2000 k, 8000 + 2000 k)
    one = wsg.WelchAccumulator(B, N)
    for k in range(K):
        one.accumulate(ring.reshape(-1), ld, slot, nslots, 4000 + 2000 * k)
    assert two.nseg == one.nseg == K
    p2, psd2 = two.peak(want_psd=True)
    p1, _ = one.peak(want_psd=True)
    torch.cuda.synchronize()
    rel = ((two.acc - one.acc).abs().max() / one.acc.abs().max()).item()
    assert rel <= 2e-6, rel
    assert torch.equal(p1, p2)
    Xh = X.double().cpu().numpy().reshape(B, N, T)
    for b in range(B):
        f, P = osg.welch_psd(Xh[b][:, 4000:], 500.0, 4000)
        mp = P.mean(axis=0)
        np.testing.assert_allclose(psd2[b].cpu().numpy(), mp, rtol=2e-4, atol=2e-4 * mp.max())


@pytest.mark.parametrize("B,N", [(5, 1), (2, 3), (4, 9), (2, 90)])
def test_welch_f64_wave_kernel_ring_wrap(cuda, B, N):
    """fp64 rings: the wave-per-column kernel (even ld, slot, seg0) reading a segment that wraps
    the 4-slot ring against the LDS-Stockham welch_kernel<double> (an odd ld selects it) on the same
    samples: the same PSD to 1e-12 (the mean and the window are formed in another order), the same
    peaks; and the oracle's PSD within 1e-9.  N < 4 leaves waves of the workgroup idle."""
    T = 6000
    X = torch.from_numpy(_e_like(T, B * N, B * 30 + N).T.copy()).to("cuda", torch.float64)  # [C][T]
    slot, nslots, ld = 1000, 4, 4096
    ring = torch.zeros((B * N, ld), dtype=torch.float64, device="cuda")
    for t0 in range(2000, T, slot):  # samples [2000, 6000) into slots (t // slot) % 4
        q = (t0 // slot) % nslots
        ring[:, q * slot:(q + 1) * slot] = X[:, t0:t0 + slot]
    a = wsg.WelchAccumulator(B, N)
    a.accumulate(ring.reshape(-1), ld, slot, nslots, 2000)  # runs: slots 2, 3, 0, 1
    odd = torch.zeros((B * N, 4001), dtype=torch.float64, device="cuda")
    odd[:, :4000] = X[:, 2000:]
    c = wsg.WelchAccumulator(B, N)
    c.accumulate(odd.reshape(-1), 4001, 4000, 1, 0)  # odd ld: welch_kernel<double>
    pa, psd = a.peak(want_psd=True)
    pc, _ = c.peak(want_psd=True)
    torch.cuda.synchronize()
    rel = ((a.acc - c.acc).abs().max() / c.acc.abs().max()).item()
    print(f"TOL welch-f64-wave-vs-lds-{B}-{N} rel={rel:.3e}")
    assert rel <= 1e-12
    assert torch.equal(pa, pc)
    Xh = X.cpu().numpy().reshape(B, N, T)
    for b in range(B):
        f, P = osg.welch_psd(Xh[b][:, 2000:], 500.0, 4000)
        mp = P.mean(axis=0)
        np.testing.assert_allclose(psd[b].cpu().numpy(), mp, rtol=1e-9, atol=1e-9 * mp.max())


def test_welch_golden_full_length(cuda):
    """300,000-sample input of the SciPy golden: node-mean PSD and peak."""
    inp = inputs()
    gs = np.load(os.path.join(G, "golden_scipy.npz"))
    E = torch.from_numpy(inp["e_t"]).cuda()[:, None, :]  # [T][1][3]
    peak, psd = wsg.welch_peak(E, want_psd=True)
    mp = gs["welch_P"].mean(axis=0)
    np.testing.assert_allclose(psd[0].cpu().numpy(), mp, rtol=1e-9, atol=1e-9 * mp.max())
    assert peak[0].item() == gs["welch_f"][np.argmax(mp)]


def test_pipeline_short_schedule_vs_oracle(cuda, sc90):
    """run_sweep end to end (fp64) vs the oracle's run() + sim_metrics per simulation."""
    from nremmodfc_amd.model import Schedule, driver_params, sim_keys
    from nremmodfc_amd.pipeline import run_sweep
    sch = Schedule(n_trans1=200, n_trans2=2000, n_sim=200_000)  # T = 10,000 samples
    G = np.array([0.16, 0.10, 0.22, 0.16, 0.30])
    S = np.array([7.68, 7.50, 7.80, 7.88, 7.68])
    keys = sim_keys([0, 1, 2, 3, 4], [0, 5, 9, 11, 3])
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    res = run_sweep(sc90, G, S, keys, emp, sch, precision="f64", want_fc=True, want_bold=True)
    p = driver_params()
    ob = oracle.OracleBatch(sc90, G, S, keys, p)
    ob.integrate(sch.n_trans1, 0.05)
    ob.integrate(sch.n_trans2, 1.0)
    rec = ob.integrate(sch.n_sim, 2.0, 20)  # [B][T][N]
    cols = res.columns()
    for b in range(len(keys)):
        want, wbold, wfc = osg.sim_metrics(rec[b], emp)
        scale = np.abs(wbold).max()
        assert np.abs(res.bold[:, b, :] - wbold).max() <= 1e-7 * scale
        assert np.abs(res.fc[b] - wfc).max() <= 1e-6
        for name, v in want.items():
            if name == "peakfreq":
                assert cols[name][b] == v, (name, cols[name][b], v)
            else:
                np.testing.assert_allclose(cols[name][b], v, rtol=1e-6, atol=1e-8, err_msg=name)


@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_pipeline_chunk_length_invariance(cuda, sc90, prec):
    """The recorded phase in 1000- or 2000-sample chunks (the default; ring slots 8000 B apart) gives
    the same outputs bit for bit: the integrator is launch-chunking invariant, BOLD is fed in
    either length, Welch takes the same segment pairs from a 6-slot or a 3-slot ring."""
    from nremmodfc_amd.model import Schedule, sim_keys
    from nremmodfc_amd.pipeline import run_sweep
    sch = Schedule(n_trans1=200, n_trans2=2000, n_sim=200_000)  # T = 10,000 samples
    G = np.array([0.16, 0.10, 0.22, 0.16, 0.30])
    S = np.array([7.68, 7.50, 7.80, 7.88, 7.68])
    keys = sim_keys([0, 1, 2, 3, 4], [0, 5, 9, 11, 3])
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    r1 = run_sweep(sc90, G, S, keys, emp, sch, precision=prec, chunk_samples=1000, want_bold=True)
    r2 = run_sweep(sc90, G, S, keys, emp, sch, precision=prec, chunk_samples=2000, want_bold=True)
    assert np.array_equal(r1.bold, r2.bold)
    for name, v in r1.columns().items():
        assert np.array_equal(v, r2.columns()[name]), name


def test_pipeline_fc_ssim_vs_oracle(cuda, sc90):
    """Pathwise FC parity of the fp64 pipeline with the oracle while the two trajectories are still
    coherent: 2,200 transient + 400,000 recorded steps (18 BOLD samples), utils.py:48's
    data_range = 1.  Beyond tens of seconds of model time two fp64 implementations that round
    differently decorrelate (the oracle against the reference's own run() under the same noise
    included); the full 1001 s horizon is tested against the reference's run() itself in
    tests/test_fc_ssim_gpu.py."""
    from nremmodfc_amd.model import Schedule, driver_params, sim_keys
    from nremmodfc_amd.pipeline import run_sweep
    sch = Schedule(n_trans1=200, n_trans2=2000, n_sim=400_000)  # 18 BOLD samples
    G = np.array([0.16, 0.10, 0.22, 0.16])
    S = np.array([7.68, 7.50, 7.80, 7.88])
    keys = sim_keys([0, 1, 2, 3], [0, 5, 9, 11])
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    res = run_sweep(sc90, G, S, keys, emp, sch, precision="f64", want_fc=True)
    ob = oracle.OracleBatch(sc90, G, S, keys, driver_params())
    ob.integrate(sch.n_trans1, 0.05)
    ob.integrate(sch.n_trans2, 1.0)
    rec = ob.integrate(sch.n_sim, 2.0, 20)
    for b in range(len(keys)):
        _, _, wfc = osg.sim_metrics(rec[b], emp)
        assert osg.ssim(res.fc[b], wfc, data_range=1.0) >= 0.999999


@pytest.mark.parametrize("M,B,N", [(6000, 10, 90), (777, 3, 90), (65, 1, 7), (3, 2, 2), (6000, 300, 96)])
def test_corrcoef_split_vs_numpy(cuda, M, B, N):
    """wc_corrcoef (time-block split) vs np.corrcoef, incl. one block, tiny M and a batch past the split."""
    rng = np.random.default_rng(M + B + N)
    x = rng.standard_normal((M, B, N)).cumsum(0) * 0.01 + rng.standard_normal((1, B, N))
    fc = wsg.corrcoef(torch.from_numpy(x).cuda(), B, N).cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(fc[b], np.corrcoef(x[:, b, :].T), rtol=0, atol=1e-12)


@pytest.mark.parametrize("M", [6000, 777])
def test_fc_long_series_vs_numpy(cuda, M):
    """wc_fc_metrics' corrcoef over long series (the SC optimiser's 6000-sample window)."""
    rng = np.random.default_rng(M)
    B, N = 3, 90
    x = rng.standard_normal((M, B, N)).cumsum(0) * 0.01 + rng.standard_normal((1, B, N))
    fc, _, _ = wsg.fc_metrics(torch.from_numpy(x).cuda(), B, N, None, kuramoto=False, want_fc=True)
    fc = fc.cpu().numpy()
    for b in range(B):
        np.testing.assert_allclose(fc[b], np.corrcoef(x[:, b, :].T), rtol=0, atol=1e-12)
