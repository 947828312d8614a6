"""north_star: "FC SSIM >= 0.999 vs reference at fixed seed" for the fp32 PRODUCT path over
the real horizon -- the full 1001 s schedule, 298 BOLD samples, utils.py:48's data_range = 1.

The fixed-seed reference is the fp64 pipeline: it follows the oracle (the restated
reference loop, itself pinned to the shipped tables: test_oracle_pin.py) to <= 1e-9 on
short horizons and to FC SSIM >= 0.999999 at 400k steps (test_pipeline_fc_ssim_vs_oracle).
Over 1001 s the SDE is chaotic, so the fp32 and fp64 realisations of one seed decorrelate
(a 1e-7 difference grows ~1e4-fold per second of model time): pathwise 0.999 is NOT
reachable by any fp32 path.  Measured on MI355X (32 seeds at cell (0, 0),
profiles/r02_fc_ssim_f32.json): same-seed SSIM(fp32 FC, fp64 FC) 0.861 (0.830-0.901),
between-seed floor SSIM(fp64 seed s, fp64 seed s+1) 0.771; seed-averaged FCs fp32 vs fp64
0.994 against a split-half fp64 floor of 0.979.  This test re-measures those numbers on
16 seeds and checks what does hold: same-seed SSIM above the between-seed floor (the fp32
path follows the same noise realisation) and the seed-averaged FC matching fp64 at the
level of the fp64 split-half sampling floor.
"""
import numpy as np
import pytest

import oracle.sigchain as osg
from nremmodfc_amd import datasets, sweep
from nremmodfc_amd.model import Schedule, sim_keys
from nremmodfc_amd.pipeline import run_sweep

pytestmark = pytest.mark.gpu


def test_f32_fc_ssim_full_schedule(cuda, sc90):
    B = 16
    sims = [s for s in sweep.homogeneous(B, 0) if (round(s.dG, 4), round(s.dsigma, 4)) == (0.0, 0.0)]
    G = np.stack([s.G for s in sims])
    S = np.stack([s.sigma for s in sims])
    keys = sim_keys([s.seed for s in sims], [s.stream for s in sims])
    emp = {s: datasets.load_empfc(s) for s in datasets.STATES}
    fc = {p: run_sweep(sc90, G, S, keys, emp, Schedule(), precision=p, want_fc=True).fc for p in ("f32", "f64")}
    assert fc["f32"].shape == (B, 90, 90)
    same = np.array([osg.ssim(fc["f32"][b], fc["f64"][b], 1.0) for b in range(B)])
    floor = np.array([osg.ssim(fc["f64"][b], fc["f64"][(b + 1) % B], 1.0) for b in range(B)])
    mean_fc = osg.ssim(fc["f32"].mean(0), fc["f64"].mean(0), 1.0)
    half = osg.ssim(fc["f64"][:B // 2].mean(0), fc["f64"][B // 2:].mean(0), 1.0)
    print(f"FC SSIM fp32 vs fp64, same seed: mean {same.mean():.4f} (min {same.min():.4f}); between seeds "
          f"{floor.mean():.4f}; seed-mean FCs {mean_fc:.4f} (fp64 split-half floor {half:.4f})")
    assert same.mean() > floor.mean() + 0.03
    assert mean_fc >= half - 0.005
