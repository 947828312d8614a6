"""Device vs oracle Hopf trajectories over the optimiser's full 7800-step run:
max |dx| at checkpoints (how fast fp64 rounding differences grow)."""
import numpy as np
import torch  # noqa: F401

import oracle
from nremmodfc_amd import Hopf_model_multi as HM
from nremmodfc_amd import datasets, optimize_sc

optimize_sc.configure(datasets.load_deco_sc())
seeds = [0, 1, 2]
gx = HM.sim_batch(seeds).cpu().numpy()  # [7200][B][N]
p = dict(a=HM.a, w=HM.w, beta=HM.beta, dt=HM.dt, G=HM.G, norm=HM.norm)
ics = [HM.initial_conditions(s, 90) for s in seeds]
x, y = np.stack([c[0] for c in ics]), np.stack([c[1] for c in ics])
oracle.hopf_integrate(p, HM.M, seeds, x, y, 0, 600)
rec = oracle.hopf_integrate(p, HM.M, seeds, x, y, 600, 7200, 1)
d = np.abs(gx.transpose(1, 0, 2) - rec).max(axis=(0, 2))
for k in (0, 100, 1000, 3000, 7199):
    print(k, d[k], np.abs(rec[:, k]).max())
