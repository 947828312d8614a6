"""Time wc_hma on the run_many_seeds batch (200 FC matrices, N = 90) vs the host facade."""
import json
import time

import numpy as np
import torch

from nremmodfc_amd import HMA, sigchain

rng = np.random.default_rng(0)
fcs = []
for _ in range(200):
    x = 0.6 * rng.standard_normal((298, 1)) + 0.5 * rng.standard_normal((298, 4))[:, rng.integers(0, 4, 90)] \
        + rng.standard_normal((298, 90))
    fcs.append(np.corrcoef(x.T))
fcs = np.stack(fcs)
t = torch.from_numpy(fcs.copy()).cuda()
sigchain.hma(t.clone())
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
sigchain.hma(t)
e1.record()
torch.cuda.synchronize()
dev_ms = e0.elapsed_time(e1)
t0 = time.perf_counter()
for f in fcs[:20]:
    HMA.integration_segregation(f.copy())
host_ms = (time.perf_counter() - t0) / 20 * 200 * 1e3
print(json.dumps({"B": 200, "N": 90, "device_ms": dev_ms, "host_facade_ms_for_200": host_ms}))
