"""Size-independent properties at the BASELINE full batch (C3: 20,000 simulations x 90
nodes on one GPU), where the oracle cannot run: every simulation is independent, so
results must not depend on where a simulation sits in the batch, on how the batch is
sharded across ranks (the 8-GPU round robin of whole_sweep_both.py:63-64) or on the
launch chunking -- bit for bit, since every kernel is column-independent."""
import numpy as np
import pytest
import torch

from bench import sweep_batch
from nremmodfc_amd import datasets
from nremmodfc_amd.model import Batch, Schedule, driver_params
from nremmodfc_amd.pipeline import run_sweep

pytestmark = pytest.mark.gpu


def _state(bt):
    return torch.stack([bt.E, bt.I, bt.A]).cpu().numpy()


def test_full_batch_permutation_and_shard_invariance(cuda, sc90):
    G, S, keys = sweep_batch(0)
    B = len(keys)
    assert B == 20_000
    p = driver_params()
    full = Batch(sc90, G, S, keys, p, precision="f32")
    full.integrate(300, 0.05)
    full.integrate(300, 2.0)
    ref = _state(full)
    perm = np.random.default_rng(0).permutation(B)
    pb = Batch(sc90, G[perm], S[perm], keys[perm], p, precision="f32")
    pb.integrate(300, 0.05)
    pb.integrate(300, 2.0)
    assert np.array_equal(_state(pb), ref[:, perm])
    # rank 3 of 8 in the reference's round robin (sim % threads == rank): a 2,500-simulation
    # batch, which runs the register-resident kernel instead of the grouped one
    shard = np.arange(B)[np.arange(B) % 8 == 3]
    sb = Batch(sc90, G[shard], S[shard], keys[shard], p, precision="f32")
    sb.integrate(300, 0.05)
    sb.integrate(300, 2.0)
    assert np.array_equal(_state(sb), ref[:, shard])
    # rank 1 of 4: 5,000 simulations, the two-groups-per-workgroup kernel
    shard = np.arange(B)[np.arange(B) % 4 == 1]
    sb = Batch(sc90, G[shard], S[shard], keys[shard], p, precision="f32")
    sb.integrate(300, 0.05)
    sb.integrate(300, 2.0)
    assert np.array_equal(_state(sb), ref[:, shard])


def test_full_batch_launch_chunking(cuda, sc90):
    G, S, keys = sweep_batch(1)
    p = driver_params()
    a = Batch(sc90, G, S, keys, p, precision="f32")
    a.integrate(1000, 2.0)
    b = Batch(sc90, G, S, keys, p, precision="f32")
    for n in (1, 399, 600):
        b.integrate(n, 2.0)
    assert np.array_equal(_state(a), _state(b))


def test_full_pipeline_shard_invariance(cuda, sc90):
    """The whole per-simulation chain (integrator, BOLD/filtfilt, Welch, FC, metrics,
    Kuramoto) for 20,000 simulations on a short schedule: a round-robin shard run on
    its own reproduces its rows of the full run exactly."""
    G, S, keys = sweep_batch(0)
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    sch = Schedule(n_trans1=200, n_trans2=2000, n_sim=200_000)
    full = run_sweep(sc90, G, S, keys, emp, sch)
    shard = np.arange(len(keys))[np.arange(len(keys)) % 8 == 5]
    part = run_sweep(sc90, G[shard], S[shard], keys[shard], emp, sch)
    for k, v in part.columns().items():
        assert np.array_equal(v, full.columns()[k][shard]), k
    assert np.isfinite(full.metrics).all() and (full.peakfreq > 0).all()


def test_f64_full_batch_tail_launch_invariance(cuda, sc90):
    """The fp64 integrator at the full batch runs two launches (the two-group rounds over the first
    2 x 256 x 2 groups of 16, then one-group workgroups for the rest, wc_sde.hip launch_f64_nt6):
    a simulation gives the same bits wherever it sits -- in a small batch (one-group workgroups
    only), in the main launch or in the tail one of the full batch."""
    G, S, keys = sweep_batch(0)
    B = len(keys)
    p = driver_params()
    full = Batch(sc90, G, S, keys, p, precision="f64")
    full.integrate(40, 0.05)
    full.integrate(40, 2.0)
    ref = _state(full)
    # sims from the main launch's first and last groups and from the tail
    pick = np.r_[0:16, 16 * 1023:16 * 1025, B - 40:B]
    sb = Batch(sc90, G[pick], S[pick], keys[pick], p, precision="f64")
    sb.integrate(40, 0.05)
    sb.integrate(40, 2.0)
    assert np.array_equal(_state(sb), ref[:, pick])
