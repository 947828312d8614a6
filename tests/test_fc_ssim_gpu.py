"""north_star: "FC SSIM >= 0.999 vs reference at fixed seed", measured at the reference's real
horizon: the full 1001 s schedule, 298 BOLD samples, utils.py:48's data_range = 1.

The reference at fixed seed is the reference's OWN run() (netwWilsonCowanPlastic.py:86-137 executed
with np.random.normal replaying the build's Philox stream; tools/fc_horizon_ref.py ->
tests/golden/ref_replay_full.npz, 32 keys of the W-optimum cell).  The same fixture holds the fp64
C oracle fed the SAME normals: the two differ only in the rounding of np.dot / np.exp against a
sequential C loop, and their FCs agree to SSIM 0.865 (0.82-0.91), not 0.999.  Their trajectories are
fully decorrelated long before the recorded phase (max |dE| ~0.55 in its first second); a 1e-15
perturbation of the initial state does the same (profiles/r03_fc_horizon.json).  So pathwise
SSIM >= 0.999 at this horizon is reachable only by reproducing the reference's float operations bit
for bit -- not by fp64, not by any fp32 path.  What holds, and is asserted here on 16 keys:
  * the device pipeline, fp64 AND the fp32 product, is as close to the reference at the same seed
    as the reference's own fp64 restatement is (same-noise floor ~0.866, far above the 0.771
    between-seed floor);
  * the seed-averaged FC matches the reference's at its own split-half sampling floor;
  * every metric column's mean over seeds matches the reference's.
This test therefore has NO pathwise power: any implementation with the right noise mapping lands at
the ~0.866 same-noise floor (a coupling off by 2^-11 would pass it).  The pathwise gates are the
short-horizon ones (test_sde_gpu.py: the reference-run replay and test_f32_gate_detects_coupling_error).
"""
import os

import numpy as np
import pytest

import oracle.sigchain as osg
from nremmodfc_amd import datasets, sweep
from nremmodfc_amd.model import Schedule
from nremmodfc_amd.pipeline import run_sweep

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_replay_full.npz")
K = 16


def _full(flat, n=90):
    fc = np.eye(n)
    iu = np.triu_indices(n, 1)
    fc[iu] = flat
    fc[iu[1], iu[0]] = flat
    return fc


def test_fc_same_seed_full_horizon_vs_reference_run(cuda, sc90):
    fx = np.load(GOLD)
    keys = fx["keys"][:K].astype(np.uint64)
    ref = np.stack([_full(f) for f in fx["fc_ref"][:K]])
    orc = np.stack([_full(f) for f in fx["fc_orc"][:K]])
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    G, S = np.full(K, sweep.BASE_G), np.full(K, sweep.BASE_SIGMA)
    ss = lambda A, B: np.array([osg.ssim(a, b, 1.0) for a, b in zip(A, B)])  # noqa: E731
    floor_same = ss(orc, ref)                       # the reference's own fp64 restatement
    floor_between = ss(ref, np.roll(ref, 1, axis=0))
    half = osg.ssim(ref[:K // 2].mean(0), ref[K // 2:].mean(0), 1.0)
    for prec in ("f64", "f32"):
        r = run_sweep(sc90, G, S, keys, emp, Schedule(), precision=prec, want_fc=True)
        same = ss(r.fc, ref)
        mean_fc = osg.ssim(r.fc.mean(0), ref.mean(0), 1.0)
        print(f"TOL fc-horizon-{prec}: same-seed SSIM vs reference {same.mean():.4f} (oracle's {floor_same.mean():.4f}, "
              f"between seeds {floor_between.mean():.4f}); seed-mean FC {mean_fc:.4f} (split-half floor {half:.4f})")
        assert same.mean() >= floor_same.mean() - 0.03          # observed: f64 0.867, f32 0.867 vs 0.865 (32 keys)
        assert same.mean() >= floor_between.mean() + 0.05
        assert mean_fc >= half - 0.005
        cols = r.columns()
        m = np.stack([cols[c] for c in sweep.METRIC_COLS], axis=1)
        mref = fx["m_ref"][:K]
        se = np.sqrt(2.0 / K) * mref.std(0, ddof=1)
        z = np.abs(m.mean(0) - mref.mean(0)) / np.where(se > 0, se, 1)
        assert z.max() < 4.0, dict(zip(sweep.METRIC_COLS, z.round(2)))
