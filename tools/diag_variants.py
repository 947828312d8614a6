#!/usr/bin/env python3
"""On-GPU ablation of the integrator's compile-time variants (wc_diag_integrate).

For each variant: correctness vs the CPU oracle on a small batch (fp32
tolerance of tests/test_sde_gpu.py), then time per Euler step on the C3 bench
workload (20,000 sims x 90 nodes, recording every 20 steps).  Interleaved rounds
in one process (cdna_hip_programming.md rule 24).
"""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the ablation entry point lives in the diag build only (python -m nremmodfc_amd._build --diag)
os.environ.setdefault("WCSDE_LIB_OVERRIDE", os.path.join(ROOT, "nremmodfc_amd", "libwcsde_diag.so"))
import oracle  # noqa: E402
from bench import sweep_batch  # noqa: E402
from nremmodfc_amd import _lib, datasets  # noqa: E402
from nremmodfc_amd.model import Batch, driver_params  # noqa: E402

L = _lib.lib()
L.wc_diag_integrate.restype = ctypes.c_int
c_vp, c_i64 = ctypes.c_void_p, ctypes.c_int64
L.wc_diag_integrate.argtypes = [ctypes.c_int, ctypes.POINTER(_lib.WCParamsC), ctypes.c_int, ctypes.c_int,
                                c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_i64, c_i64, ctypes.c_double,
                                c_i64, c_vp, c_vp, ctypes.c_size_t, c_vp]


def diag(bt, variant, nsteps, tau, rec_every=0, rec=None):
    rc = L.wc_diag_integrate(variant, ctypes.byref(bt._pc), bt.B, bt.N, _lib.ptr(bt.sc), _lib.ptr(bt.G),
                             _lib.ptr(bt.sigmaE), _lib.ptr(bt.keys), _lib.ptr(bt.E), _lib.ptr(bt.I),
                             _lib.ptr(bt.A), bt.step, nsteps, tau, rec_every, _lib.ptr(rec),
                             _lib.ptr(bt.ws), bt.ws.numel(), _lib.stream_handle())
    _lib.check(rc, f"diag variant {variant}")
    bt.step += nsteps


def main():
    variants = [int(v) for v in (sys.argv[1].split(",") if len(sys.argv) > 1 else range(16))]
    steps = int(os.environ.get("DIAG_STEPS", "2000"))
    rounds = int(os.environ.get("DIAG_ROUNDS", "3"))
    sc = datasets.load_sc()
    p = driver_params()
    G, S, keys = sweep_batch(0)
    # correctness (ablation variants 6/7 are expected to fail)
    ok = {}
    first = {}  # the first variant's records: bit-identity of the others against it
    sG, sS, sk = G[:37], S[:37], keys[:37]
    ob = oracle.OracleBatch(sc, sG, sS, sk, p)
    ob.integrate(300, 0.05)
    orec = ob.integrate(600, 2.0, 20)
    for v in variants:
        bt = Batch(sc, sG, sS, sk, p, precision="f32")
        diag(bt, v, 300, 0.05)
        if 20 <= v < 38:  # node-major [B*N][32] records
            rec = torch.empty((37 * 90, 32), dtype=torch.float32, device="cuda")
            diag(bt, v, 600, 2.0, 20, rec)
            got = rec[:, :30].reshape(37, 90, 30).permute(0, 2, 1)
        else:
            rec = torch.empty((30, 37, 90), dtype=torch.float32, device="cuda")
            diag(bt, v, 600, 2.0, 20, rec)
            got = rec.permute(1, 0, 2)
        torch.cuda.synchronize()
        g = got.double().cpu().numpy()
        d = np.abs(g - orec)
        ok[v] = (float(d.max()), float(np.sqrt((d ** 2).mean())), bool(np.array_equal(g, first.setdefault("g", g))))
    # timing (DIAG_B: batch size, default the C3 batch)
    nb = int(os.environ.get("DIAG_B", len(keys)))
    G, S, keys = G[:nb], S[:nb], keys[:nb]
    bt = Batch(sc, G, S, keys, p, precision="f32")
    rec = torch.empty((-(-steps // 20), bt.B, bt.N), dtype=torch.float32, device="cuda")
    recn = torch.empty((bt.B * bt.N, (-(-steps // 20) + 3) // 4 * 4), dtype=torch.float32, device="cuda")
    diag(bt, variants[0], 500, 0.05)
    times = {v: [] for v in variants}
    for r in range(rounds):
        for v in variants:
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            rec_every = int(os.environ.get("DIAG_REC", "20"))
            diag(bt, v, steps, 2.0, rec_every, (recn if 20 <= v < 38 else rec) if rec_every else None)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1))
    res = []
    for v in variants:
        ms = min(times[v])
        ns = bt.B * bt.N * steps / (ms * 1e-3)
        res.append({"variant": v, "ms": ms, "us_per_step": ms * 1e3 / steps, "node_steps_per_s": ns,
                    "tflops_215": ns * 215 / 1e12, "max_err": ok[v][0], "rms_err": ok[v][1],
                    "bits_equal_first_variant": ok[v][2]})
        print(json.dumps(res[-1]), flush=True)


if __name__ == "__main__":
    main()
