"""The ctypes stub INTEGRATION.md section 3 shows a maintainer (run() replaced through the
C ABI) runs as written and matches the package's own batch API, so the document stays
true to include/wcsde.h."""
import os
import re

import numpy as np
import pytest
import torch

from nremmodfc_amd import datasets
from nremmodfc_amd.model import Batch, driver_params

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _stub_source():
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", doc, flags=re.S)
    src = [b for b in blocks if "def run_gpu" in b]
    assert len(src) == 1
    return src[0]


def test_integration_stub_runs_and_matches_batch(cuda, monkeypatch):
    monkeypatch.chdir(ROOT)  # the stub loads nremmodfc_amd/libwcsde.so by relative path
    p = driver_params()
    sc = datasets.load_sc()
    N = sc.shape[0]
    ns = dict(vars(p))
    ns.update(CM=sc, N=N, G=0.2, sigmaE=7.5, a_ie_0=2.5, dt=p.dt, dtSim=p.dtSim, sqdtD=p.sqdtD,
              timeTrans1=np.arange(0, 0.005, p.dtSim), timeTrans2=np.arange(0, 0.01, p.dtSim),
              timeSim=np.arange(0, 0.04, p.dtSim))
    ns["time"] = np.arange(0, len(ns["timeSim"]) * p.dtSim, p.dt)
    exec(_stub_source(), ns)
    Y = ns["run_gpu"](seed_key=5)
    assert Y.shape == (len(ns["time"]), 3, N)
    bt = Batch(sc, np.array([0.2]), np.array([7.5]), np.array([5], dtype=np.uint64), p, precision="f64")
    bt.integrate(len(ns["timeTrans1"]), 0.05)
    bt.integrate(len(ns["timeTrans2"]), 1.0)
    rec = torch.empty((len(ns["time"]), 1, N), dtype=torch.float64, device="cuda")
    bt.integrate(len(ns["timeSim"]), 2.0, int(p.dt / p.dtSim), rec)
    torch.cuda.synchronize()
    assert np.array_equal(Y[:, 0, :], rec[:, 0, :].cpu().numpy())
