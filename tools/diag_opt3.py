"""Hopf FC conditioning probe (GPU box): the device trajectories of three seeds against the oracle's,
then both trajectories through the same scipy filtfilt + corrcoef, so the FC difference that
trajectory-level agreement leaves is separated from the device FC chain's own error (the band
filter near Nyquist turns 1e-16 input differences into ~1e-7 FC differences; DESIGN §4,
tests/test_hopf_gpu.py).  Test infrastructure: imports the oracle as the checker."""
import numpy as np
from scipy import signal
import oracle
from nremmodfc_amd import Hopf_model_multi as HM
from nremmodfc_amd import datasets, optimize_sc

optimize_sc.configure(datasets.load_deco_sc())
seeds = [0, 1, 2]
fc_dev = optimize_sc.simulated_fc(seeds)
gx = HM.sim_batch(seeds).cpu().numpy()
p = dict(a=0.0, w=0.05 * 2 * np.pi, beta=0.032, dt=0.1, G=0.6, norm=np.mean(HM.M.sum(0)))
ics = [HM.initial_conditions(s, 90) for s in seeds]
x = np.stack([c[0] for c in ics]); y = np.stack([c[1] for c in ics])
oracle.hopf_integrate(p, HM.M, seeds, x, y, 0, 600)
rec = oracle.hopf_integrate(p, HM.M, seeds, x, y, 600, 7200, 1)
print("traj", np.abs(gx.transpose(1, 0, 2) - rec).max())
b, a, _ = optimize_sc.band(0.1)
fo = sum(np.corrcoef(signal.filtfilt(b, a, rec[s], axis=0)[600:6600].T) for s in range(3)) / 3
fg = sum(np.corrcoef(signal.filtfilt(b, a, gx[:, s, :], axis=0)[600:6600].T) for s in range(3)) / 3
print("fc orc-traj vs gpu-traj (both scipy)", np.abs(fo - fg).max(), "dev vs gpu-traj/scipy", np.abs(fc_dev - fg).max())
print("norm", p["norm"], HM.norm, HM.tmax, HM.teq, HM.dt)
