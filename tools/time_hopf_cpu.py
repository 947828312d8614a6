"""CPU baseline for one SC-optimiser iteration: the oracle's Hopf loop (10 seeds x 7800
steps, OpenMP over seeds) + SciPy filtfilt + np.corrcoef, on this host's cores."""
import json
import os
import time

import numpy as np
from scipy import signal

import oracle
from nremmodfc_amd import Hopf_model_multi as HM
from nremmodfc_amd import datasets, optimize_sc

optimize_sc.configure(datasets.load_deco_sc())
seeds = list(range(10))
p = dict(a=HM.a, w=HM.w, beta=HM.beta, dt=HM.dt, G=HM.G, norm=HM.norm)
t0 = time.perf_counter()
ics = [HM.initial_conditions(s, 90) for s in seeds]
x = np.stack([c[0] for c in ics]); y = np.stack([c[1] for c in ics])
oracle.hopf_integrate(p, HM.M, seeds, x, y, 0, 600)
rec = oracle.hopf_integrate(p, HM.M, seeds, x, y, 600, 7200, 1)
t1 = time.perf_counter()
b, a, _ = optimize_sc.band(0.1)
fc = sum(np.corrcoef(signal.filtfilt(b, a, rec[s], axis=0)[600:6600].T) for s in range(10)) / 10
t2 = time.perf_counter()
print(json.dumps({"kind": "oracle C loop + scipy", "cores": len(os.sched_getaffinity(0)),
                  "sde_s": t1 - t0, "post_s": t2 - t1, "iteration_s": t2 - t0}))
