"""N > 96 integrator (wc_sde_large.hip: one GEMM-shaped launch per Euler step)
vs the CPU oracle, same Philox stream as the N <= 96 path.

Tolerances: fp64 max |dE| <= 1e-9; fp32 (fp16x3 22-bit coupling, fp32 state,
compensated a_ie) max 3e-5 / rms 3e-6 over these 120-200-step horizons, about 10x
the deviation observed on MI355X (max 3.4e-6, rms 2.8e-7).
Sizes cover BASELINE config 5 (N = 1000 synthetic connectome) and ragged tails
(B and N not multiples of the 64 x 64 workgroup tile).
"""
import numpy as np
import pytest
import torch

import oracle
from nremmodfc_amd import datasets
from nremmodfc_amd.model import Batch, driver_params, sim_keys
from tests.test_sde_gpu import observed, run_pair, tol

pytestmark = pytest.mark.gpu


def _sc(N, seed):
    return datasets.synthetic_sc(N, seed=seed)


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("N,B", [(97, 3), (200, 70), (1000, 5)])
def test_large_vs_oracle(cuda, prec, N, B):
    sc = _sc(N, N)
    rng = np.random.default_rng(B)
    G = 0.16 + rng.uniform(-0.1, 0.3, B)
    S = 7.68 + rng.uniform(-0.2, 0.2, B)
    keys = sim_keys(list(range(B)), [N] * B)
    n = 200 if N < 1000 else 120
    g, o, gb, ob, _ = run_pair(sc, G, S, keys, n // 2, n // 2, n, 7, prec)
    mx, rms = tol(prec, (3e-5, 3e-6))  # observed f32: max <= 3.4e-6, rms <= 2.8e-7
    d = np.abs(g - o)
    observed(d, f"large-{prec}-{N}-{B}")
    assert d.max() <= mx and np.sqrt(np.mean(d ** 2)) <= rms, (d.max(), np.sqrt(np.mean(d ** 2)))
    for x, y in ((gb.E, ob.E), (gb.I, ob.I), (gb.A, ob.A)):
        assert np.abs(x.cpu().numpy() - y).max() <= mx


def test_large_maps_mode(cuda):
    """Per-node G and sigmaE (maps mode) at N = 1000."""
    N, B = 1000, 4
    sc = _sc(N, 7)
    m = datasets.synthetic_map(N)
    G = np.stack([0.16 + d * m for d in (-0.1, 0.0, 0.1, 0.28)])
    S = np.stack([7.68 + d * m for d in (0.18, -0.2, 0.0, 0.1)])
    keys = sim_keys([9] * B, list(range(B)))
    g, o, *_ = run_pair(sc, G, S, keys, 40, 40, 80, 20, "f64")
    assert np.abs(g - o).max() <= 1e-9


def test_large_chunking_and_ring_layout(cuda):
    """Chunked calls equal one call (fp64 bit-exact); node-major ring records
    (rec_ld > 0, the sweep pipeline's layout) equal the time-major ones."""
    N, B = 130, 3
    sc = _sc(N, 3)
    keys = sim_keys([1, 2, 3], [0, 0, 0])
    a = Batch(sc, 0.16, 7.68, keys, precision="f64")
    rec = torch.empty((10, B, N), dtype=torch.float64, device="cuda")
    a.integrate(100, 2.0, 10, rec)
    b = Batch(sc, 0.16, 7.68, keys, precision="f64")
    ld = 16
    ring = torch.zeros(B * N * ld, dtype=torch.float64, device="cuda")
    b.integrate(50, 2.0, 10, ring, rec_ld=ld)
    b.integrate(50, 2.0, 10, ring[5:], rec_ld=ld)
    torch.cuda.synchronize()
    assert torch.equal(a.E, b.E) and torch.equal(a.I, b.I) and torch.equal(a.A, b.A)
    nm = ring.view(B, N, ld)[:, :, :10].permute(2, 0, 1)
    assert torch.equal(nm, rec)


def test_large_f32_tracks_f64_statistics(cuda):
    N, B = 1000, 8
    sc = _sc(N, 11)
    keys = sim_keys(list(range(B)), [0] * B)
    out = {}
    for prec in ("f32", "f64"):
        b = Batch(sc, 0.16, 7.68, keys, precision=prec)
        b.integrate(2000, 0.05)
        rec = torch.empty((200, B, N), dtype=b.rec_dtype, device="cuda")
        b.integrate(4000, 2.0, 20, rec)
        out[prec] = rec.double().mean(0).cpu().numpy()
    observed(np.abs(out["f32"] - out["f64"]), "large-f32-vs-f64-mean")
    assert np.abs(out["f32"] - out["f64"]).max() < 3e-5  # observed 2.7e-6 (6000 steps)


def _both_paths(sc, G, S, keys, steps, rec_every=20, rec_ld=0, chunks=None):
    """The same integration through the default path (the persistent kernel wherever it is
    resident) and through the one-launch-per-step kernel (WCSDE_PERSISTENT=0): final state and records."""
    import os
    out = {}
    for flag in ("default", "0"):
        os.environ.pop("WCSDE_PERSISTENT", None)
        if flag != "default":
            os.environ["WCSDE_PERSISTENT"] = flag
        try:
            b = Batch(sc, G, S, keys, precision="f32")
            b.integrate(60, 0.05)
            n_rec = -(-steps // rec_every)
            if rec_ld:
                rec = torch.zeros((b.B * b.N * rec_ld,), dtype=torch.float32, device="cuda")
                b.integrate(steps, 2.0, rec_every, rec, rec_ld=rec_ld)
            else:
                rec = torch.empty((n_rec, b.B, b.N), dtype=torch.float32, device="cuda")
                done = 0
                for n in (chunks or [steps]):
                    b.integrate(n, 2.0, rec_every, rec[done // rec_every:])
                    done += n
            b.check()  # wc_integrate_status: no wait of the last call timed out (and the state is finite)
            out[flag] = (b.E.clone(), b.I.clone(), b.A.clone(), rec)
        finally:
            os.environ.pop("WCSDE_PERSISTENT", None)
    return out["default"], out["0"]


@pytest.mark.parametrize("N,B", [(1000, 2500), (700, 170), (250, 170), (97, 1)])
def test_persistent_matches_step_kernel(cuda, N, B):
    """Round 2's persistent kernel (state in registers, in-launch E-image hand-off between the
    node-block workgroups of a simulation block) gives the step kernel's bits: same MFMA order,
    same epilogue arithmetic.  C5 shard; N = 700 runs the runtime-loop variant (NRP_T = -1) over ten
    remote chunk pairs, so the 3-stage LDS ring wraps several times; ragged tiles (3 x 2
    workgroups); a single simulation."""
    sc = _sc(N, 21)
    rng = np.random.default_rng(N)
    G = 0.16 + rng.uniform(-0.1, 0.3, B)
    S = 7.68 + rng.uniform(-0.2, 0.2, B)
    keys = sim_keys(np.arange(B) % 50, np.arange(B) // 50 + 7)
    p, s = _both_paths(sc, G, S, keys, 300)
    for name, x, y in zip(("E", "I", "A", "rec"), p, s):
        d = (x.double() - y.double()).abs()
        if not torch.equal(x, y):
            first = int(torch.nonzero(d.reshape(d.shape[0], -1).amax(1) if name == "rec" else d.reshape(-1))[0, 0])
            print(f"{name}: max |d| {d.max().item():.3e}, {int((d > 0).sum())} of {d.numel()} differ, first {first}")
    for x, y in zip(p, s):
        assert torch.equal(x, y)
    assert torch.isfinite(p[0]).all()


def test_persistent_maps_ring_and_chunks(cuda):
    """Per-node G and sigma (maps mode), node-major ring records, and chunked calls."""
    N, B = 1000, 90
    sc = _sc(N, 5)
    m = datasets.synthetic_map(N)
    G = np.stack([0.16 + d * m for d in np.linspace(-0.1, 0.28, B)])
    S = np.stack([7.68 + d * m[::-1] for d in np.linspace(-0.2, 0.18, B)])
    keys = sim_keys([3] * B, list(range(B)))
    p, s = _both_paths(sc, G, S, keys, 200, rec_every=20, rec_ld=12)
    for x, y in zip(p, s):
        assert torch.equal(x, y)
    p, s = _both_paths(sc, G, S, keys, 200, rec_every=20, chunks=[40, 100, 60])
    for x, y in zip(p, s):
        assert torch.equal(x, y)


def test_integrate_status_is_stream_ordered(cuda):
    """ABI 7: wc_integrate returns without waiting (the persistent path keeps no host word and does
    not synchronise); wc_integrate_status waits for the stream and reads the last call's status word
    from the workspace.  A call on a side stream is still running when wc_integrate returns."""
    from nremmodfc_amd import _lib
    N, B = 1000, 2500
    sc = _sc(N, 3)
    keys = sim_keys(np.arange(B) % 50, np.arange(B) // 50)
    b = Batch(sc, 0.16, 7.68, keys, precision="f32")
    s = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        b.integrate(20000, 2.0, stream=s)  # ~0.36 s of persistent work: far longer than the host's return
        ev = torch.cuda.Event()
        ev.record(s)
    assert not ev.query(), "wc_integrate waited for its stream"
    L = _lib.lib()
    assert L.wc_integrate_status(_lib.ptr(b.ws), B, N, _lib.WC_F32, _lib.stream_handle(s)) == 0
    assert ev.query()
    assert torch.isfinite(b.E).all()
