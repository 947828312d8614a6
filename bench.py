#!/usr/bin/env python3
"""Benchmark: node-timesteps/s of the (G, sigma) x 50-seed Wilson-Cowan sweep.

Workload (BASELINE.json configs[2], the metric's config, one GPU): the full
homogeneous sweep of whole_sweep_both.py -- 50 seeds x 20 dG x 20 dsigma =
20,000 simulations of the 90-node AAL connectome (SC_opti_25julio), G = 0.16 +
dG, sigmaE = 7.68 + dsigma on the shipped grid (whole_sweep_both_maps.py:92-93).
One bench "step" = one chunk of `--chunk` Euler steps of the recorded phase
(tau_ip = 2, E stored every 20 steps, wc:118-135) for every simulation of the
batch, state and inputs resident in HBM.  With --gpus N (torchrun, one rank per
GPU) each rank runs its own 20,000-simulation shard (seeds 50r..50r+49):
weak scaling, no data-path collective.

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from nremmodfc_amd import datasets  # noqa: E402
from nremmodfc_amd.model import Batch, driver_params, sim_keys  # noqa: E402

PEAK_FP32_TFLOPS = 157.3   # MI355X FP32 vector = FP32 matrix (MI355X_MICROARCH.md)
PEAK_FP64_TFLOPS = 78.6


def flops_per_node_step(N):
    """2N coupling flops + 35 elementwise ops per node-step."""
    return 2 * N + 35


def sweep_batch(rank, n_seeds=50, nG=20, nS=20):
    dG = np.linspace(-0.1, 0.3, nG, endpoint=False)
    dS = np.linspace(-0.2, 0.2, nS, endpoint=False)
    seeds = np.arange(n_seeds) + rank * n_seeds
    s, g, q = np.meshgrid(seeds, np.arange(nG), np.arange(nS), indexing="ij")  # product(seeds, dG, ds)
    s, g, q = s.ravel(), g.ravel(), q.ravel()
    G = 0.16 + dG[g]
    S = 7.68 + dS[q]
    keys = sim_keys(s, g * nS + q)
    return G, S, keys


def cpu_baseline(sc, seconds=15.0, steps=2000):
    """The oracle's C restatement of run() on the host cores (kind 'port')."""
    import oracle
    try:
        ncores = len(os.sched_getaffinity(0))
    except AttributeError:
        ncores = os.cpu_count()
    ncores = max(1, min(ncores, 16))   # the box's CPU share for one GPU
    G, S, keys = sweep_batch(0)
    p = driver_params()
    B = 2 * ncores
    ob = oracle.OracleBatch(sc, G[:B], S[:B], keys[:B], p)
    ob.integrate(200, 2.0, 20, nthreads=ncores)  # warm
    total, t0, n = 0, time.perf_counter(), 0
    while True:
        ob.integrate(steps, 2.0, 20, nthreads=ncores)
        n += 1
        total = time.perf_counter() - t0
        if total >= seconds:
            break
    ns = B * sc.shape[0] * steps * n
    return {"value": ns / total, "unit": "node-timesteps/sec", "cores": ncores, "kind": "port",
            "sample": f"{B} sims x {steps * n} Euler steps of the C3 grid (tau_ip=2, E recorded every "
                      f"20 steps), oracle/wc_oracle.c fp64, OpenMP over simulations, {total:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chunk", type=int, default=10_000, help="Euler steps per bench step")
    ap.add_argument("--precision", default="f32", choices=("f32", "f64"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    sc = datasets.load_sc()
    N = sc.shape[0]
    G, S, keys = sweep_batch(rank)
    B = len(keys)
    p = driver_params()
    bt = Batch(sc, G, S, keys, p, precision=args.precision, device=f"cuda:{local}")
    R = 20
    n_rec = -(-args.chunk // R)
    rec = torch.empty((n_rec, B, N), dtype=bt.rec_dtype, device=bt.device)
    # reach the recorded phase's operating point cheaply: a short transient
    bt.integrate(2000, 0.05)

    def step():
        bt.integrate(args.chunk, 2.0, R, rec)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps  # device time per launch pair (prep + SDE kernel)
    if dist:
        t = torch.tensor([elapsed], device=bt.device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    node_steps = B * N * args.chunk * args.steps * world
    value = node_steps / elapsed
    per_launch_ns = B * N * args.chunk
    fl = flops_per_node_step(N)
    peak = PEAK_FP32_TFLOPS if args.precision == "f32" else PEAK_FP64_TFLOPS
    achieved = per_launch_ns * fl / (kern_ms * 1e-3) / 1e12
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_sde.json")
    if os.path.exists(pmc):
        try:
            d = json.load(open(pmc))
            if d.get("B") == B and d.get("N") == N and d.get("chunk") == args.chunk and \
                    d.get("precision") == args.precision:
                traffic = d.get("hbm_bytes_per_launch")
        except (ValueError, OSError):
            traffic = None
    out = {
        "metric": "node-timesteps/sec (90-node WC, (G,sigma)x50-seed sweep) at 1/2/4/8 GPUs",
        "value": value,
        "unit": "node-timesteps/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "f32" else "f64",
        "data": "synthetic noise (Philox), real 90-node SC_opti_25julio connectome",
        "config": {"workload": "C3: full homogeneous (G,sigma) sweep x 50 seeds (whole_sweep_both.py) "
                               "per GPU, recorded phase tau_ip=2",
                   "sims_per_gpu": B, "nodes": N, "euler_steps_per_step": args.chunk,
                   "record_every": R, "parallelism": f"sims sharded x{world}"},
        "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                     "frac": achieved / peak, "traffic": traffic,
                     "kernel_ms_per_launch": kern_ms,
                     "flops_per_node_step": fl},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(sc, seconds=args.cpu_seconds)
    elif rank == 0:
        out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
