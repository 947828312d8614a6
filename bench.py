#!/usr/bin/env python3
"""Benchmark: node-timesteps/s of the (G, sigma) x 50-seed Wilson-Cowan sweep.

Workload (BASELINE.json configs[2], the metric's config, one GPU): the full
homogeneous sweep of whole_sweep_both.py -- 50 seeds x 20 dG x 20 dsigma =
20,000 simulations of the 90-node AAL connectome (SC_opti_25julio), G = 0.16 +
dG, sigmaE = 7.68 + dsigma on the shipped grid (whole_sweep_both_maps.py:92-93).
One bench "step" = 2000 recorded samples of every simulation of the batch: two
chunks of 20,000 Euler steps of the recorded phase (tau_ip = 2, E stored every
20 steps, wc:118-135), each followed by the streamed BOLD / band-pass stage
(which also transposes the chunk into the 6-slot Welch ring), plus one
4000-sample Welch segment (a launch of the last two every other step) -- the steady state of
the sweep pipeline (nremmodfc_amd/pipeline.py); inputs and state resident in
HBM.  --sde-only times the integrator alone.  With --gpus N (torchrun, one rank per
GPU) the ONE 20,000-simulation C3 sweep north_star names is split over the ranks
with the reference's round robin (simulation i on rank i % N,
whole_sweep_both.py:63-64; strong scaling, the default, no data-path
collective); the weak-scaling job (every rank its own 20,000-simulation sweep,
seeds 50r..50r+49) is timed after it and reported as `weak_scaling`
(--scaling weak makes it the headline instead).

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
PEAK_HBM_GBPS = 8000.0     # MI355X HBM3E (MI355X_MICROARCH.md)
PEAK_F16_TFLOPS = 2500.0   # dense fp16 MFMA (MI355X_MICROARCH.md); the fp16x3 coupling runs on it
PEAK_IC_GATHER_GBPS = 8600.0  # rows gathered from the Infinity Cache into the CUs, chip-wide (MI355X_MICROARCH.md)
PEAK_L2_GATHER_GBPS = 18800.0  # L2-resident rows gathered into the CUs, chip-wide (the guide's 16.8-18.8 TB/s)


def flops_per_node_step(N):
    """2N coupling flops + 35 elementwise ops per node-step."""
    return 2 * N + 35


def issued_mfma_flops_per_node_step(N):
    """MFMA flops the f32 kernels actually issue per node-step: the coupling runs as three fp16
    products (fp16x3) over nodes padded to 16 (N <= 96) or 64 (N > 96) on both sides."""
    pad = 16 if N <= 96 else 64
    Np = -(-N // pad) * pad
    return 3 * 2 * Np * Np / N


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


def loaded_lib_sha256():
    """sha256 of the libwcsde.so this process loads (nremmodfc_amd/_build.py LIB_LOAD): the stamp a
    profiles/pmc_*.json must carry for its counters to be attached to the bench line."""
    import hashlib
    from nremmodfc_amd import _build
    with open(_build.LIB_LOAD, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


CPU_SHARE = 16  # host cores one GPU's job may use on the GPU box (its OMP_NUM_THREADS / MAX_JOBS)


def _cores():
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = os.cpu_count()
    return avail, max(1, min(avail, CPU_SHARE))


def cpu_baseline_numpy(steps=150_000, nodes=90):
    """The reference's own hot loop as NumPy executes it (oracle/numpy_run.py: wc:72-137 operation
    for operation, bit-identical to the reference's run() under the same normals), one
    single-threaded process per core as the reference's SLURM array runs it,
    truncated horizon (per-step cost is constant).  Workers are child processes started with
    subprocess (numpy only, OPENBLAS/OMP/MKL_NUM_THREADS=1)."""
    import subprocess
    avail, ncores = _cores()
    env = dict(os.environ, OPENBLAS_NUM_THREADS="1", OMP_NUM_THREADS="1", MKL_NUM_THREADS="1")
    t0 = time.perf_counter()
    procs = [subprocess.Popen([sys.executable, "-m", "oracle.numpy_run", str(steps), str(i), str(nodes)], cwd=ROOT, env=env,
                              stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True) for i in range(ncores)]
    secs = []
    for pr in procs:
        out, _ = pr.communicate()
        if pr.returncode != 0:
            raise RuntimeError("cpu_baseline_numpy: a worker failed")
        secs.append(float(out.strip().splitlines()[-1]))
    wall = time.perf_counter() - t0
    per_core = [nodes * steps / s for s in secs]
    value = nodes * steps * ncores / max(secs)  # every worker's node-steps over the slowest worker's loop time
    net = "N=90" if nodes == 90 else f"N={nodes} (datasets.synthetic_sc: np.dot(CM, E) a BLAS gemv per step)"
    return {"value": value, "unit": "node-timesteps/sec", "cores": ncores, "kind": "port",
            "cores_available": avail, "cores_cap": CPU_SHARE,
            "per_core": {"mean": float(np.mean(per_core)), "min": float(min(per_core))},
            "sample": f"{ncores} processes x 1 sim x {steps} Euler steps of the C3 cell (0.16, 7.68), {net}: the "
                      f"reference's NumPy loop (oracle/numpy_run.py, bit-identical to netwWilsonCowanPlastic.py's "
                      f"run() under replayed noise), numpy's normal draws, 1 BLAS thread each; {wall:.1f} s wall",
            "note": "cores capped at one GPU's host share on the box (CPU_SHARE)"}


def cpu_baseline_compiled(sc, seconds=8.0, steps=2000):
    """The oracle's compiled C restatement of run() (oracle/wc_oracle.c), OpenMP over simulations:
    the per-step cost of a compiled loop, as numba gives the reference (kind 'port')."""
    import oracle
    avail, ncores = _cores()
    G, S, keys = sweep_batch(0)
    p = driver_params()
    B = 2 * ncores
    ob = oracle.OracleBatch(sc, G[:B], S[:B], keys[:B], p)
    ob.integrate(min(200, steps), 2.0, 20, nthreads=ncores)  # warm
    total, t0, n = 0, time.perf_counter(), 0
    while True:
        ob.integrate(steps, 2.0, 20, nthreads=ncores)
        n += 1
        total = time.perf_counter() - t0
        if total >= seconds:
            break
    ns = B * sc.shape[0] * steps * n
    return {"value": ns / total, "unit": "node-timesteps/sec", "cores": ncores, "kind": "port",
            "cores_available": avail, "cores_cap": CPU_SHARE,
            "per_core": ns / total / ncores,
            "sample": f"{B} sims x {steps * n} Euler steps of the C3 grid on N={sc.shape[0]} (tau_ip=2, E recorded "
                      f"every 20 steps), oracle/wc_oracle.c fp64 (the compiled loop numba gives the reference; "
                      f"its CM.E is a scalar dot loop), OpenMP over simulations, {ncores} threads, {total:.1f} s",
            "note": "cores capped at one GPU's host share on the box (CPU_SHARE = 16 of the affinity mask's "
                    "cores_available); profiles/r04_cpu_scaling.log has the per-core rate at 1..16 cores"}


def cpu_baseline(sc, seconds=8.0, steps=2000, numpy_leg=True):
    """N = 90: the reported baseline is the compiled port (oracle/wc_oracle.c): the reference
    decorates run() and wilsonCowan with numba's @njit (netwWilsonCowanPlastic.py:77,86) and cannot
    be imported without numba, so as shipped its loop always runs compiled.  The interpreted NumPy
    restatement (the same loop without the JIT) is reported beside it as `numpy_interpreted`.

    N = 1000 (C5): the step is dominated by np.dot(CM, E) (wc:81), a 1e6-MAC gemv, which numba and
    NumPy both hand to BLAS; the NumPy loop then runs at the compiled rate and the C port's scalar
    dot loop is slower.  Both legs run; the faster is `value` (the other beside it), so the GPU is
    compared against the better of the two CPU forms.  `seconds` sizes each leg."""
    N = sc.shape[0]
    if N == 90:
        out = cpu_baseline_compiled(sc, seconds, steps)
        if numpy_leg:
            out["numpy_interpreted"] = cpu_baseline_numpy(steps=max(2000, int(seconds * 20_000)))
            out["numpy_interpreted"]["kind"] = "interpreted"
        return out
    comp = cpu_baseline_compiled(sc, seconds, steps=max(20, int(steps * (90 / N) ** 2)))
    nump = cpu_baseline_numpy(steps=max(200, int(seconds * 2_000_000 / N)), nodes=N)
    best, other, oname = (nump, comp, "compiled_port") if nump["value"] >= comp["value"] else (comp, nump, "numpy_interpreted")
    best = dict(best)
    best[oname] = other
    best["note"] = (f"N={N}: the faster of the reference's NumPy loop (BLAS gemv for np.dot(CM, E), wc:81) and the "
                    f"compiled C port; " + best.get("note", ""))
    return best


def run_workload(sc, G, S, keys, p, args, dev, dist, steps, warmup):
    """Time `steps` bench steps of one batch after `warmup` untimed ones; a barrier and a device
    synchronisation on both sides, the maximum over ranks.  -> (seconds, mean ms per kernel)."""
    from nremmodfc_amd.sigchain import NEQ, BoldStream, WelchAccumulator

    N = sc.shape[0]
    B = len(keys)
    C = B * N
    bt = Batch(sc, G, S, keys, p, precision=args.precision, device=dev)
    R, CH = 20, 1000                     # record every 20 steps; 1000-sample integrator chunks (20,000 Euler steps)
    WELCH_SEG = 4000                     # nperseg (whole_sweep_both.py:90), hop WELCH_SEG / 2
    CHUNKS = 2                           # chunks per bench step (one Welch segment per step: a launch of two
                                         # overlapping segments every other step, as the sweep pipeline runs them)
    SLOT, NSLOT = CH * CHUNKS, 3         # the 6000-sample Welch ring in 2000-sample slots: one BOLD pass per step
    LD = SLOT * NSLOT                    # (slots start 8000 B apart, a multiple of 64 B: 1000-sample slots put every
                                         # other one 32 B off a line and its node-major rows cost ~0.55 ms more per
                                         # chunk, profiles/r04_ab/ring_align.log)
    EULER = CH * R                       # Euler steps per chunk
    n_total = (warmup + steps) * CHUNKS * CH + NEQ
    ring = torch.empty(C * LD, dtype=bt.rec_dtype, device=dev)
    # fp32 + consumers: the integrator writes each step's two chunks time-major, the BOLD pass transposes
    # them into the node-major Welch ring (the sweep pipeline's layout, nremmodfc_amd/pipeline.py)
    # (--sde-only records the same way, time-major, so it times exactly the pipeline's integrator work)
    tmaj = torch.empty(SLOT * C, dtype=bt.rec_dtype, device=dev) if args.precision == "f32" else None
    bold = welch = None
    if not args.sde_only:
        bold = BoldStream(C, max(n_total, 300_000), NEQ, 1000, p.dt * p.downsamp, dev)
        welch = WelchAccumulator(B, N, dev)
    # (no separate transient launch: every wc_sde_kernel launch of the run is one 20,000-step chunk,
    # so the rocprofv3 average of the kernel equals the per-launch time reported here)
    state = {"k": 0, "timed": False, "pending": False}
    ev = {"sde": [], "bold": [], "welch": [], "welch1": []}

    def timed(name, fn):
        if not state["timed"]:
            return fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        ev[name].append((e0, e1))

    def step():
        """2000 recorded samples (40,000 Euler steps) of every simulation: integrate two 1000-sample
        chunks, stream BOLD over the 2000 samples into their ring slot, one 4000-sample Welch segment
        (every other step one launch of the last two segments, as nremmodfc_amd/pipeline.py does)."""
        slot = (state["k"] // CHUNKS) % NSLOT
        for h in range(CHUNKS):
            if tmaj is not None:
                timed("sde", lambda: bt.integrate(EULER, 2.0, R, tmaj[h * CH * C:]))
            else:
                timed("sde", lambda: bt.integrate(EULER, 2.0, R, ring[slot * SLOT + h * CH:], rec_ld=LD))
        if bold is not None:
            if tmaj is not None:
                timed("bold", lambda: bold.feed(tmaj, SLOT, e_ld=0, copy=ring, copy_ld=LD, copy_offset=slot * SLOT))
            else:
                timed("bold", lambda: bold.feed(ring, SLOT, e_ld=LD, offset=slot * SLOT))
        state["k"] += CHUNKS
        # the segment ending at this step's last sample: held for one step and launched with the next
        # one (two per launch, as the pipeline does); flush_welch() launches a held one alone
        if welch is not None and state["k"] * CH >= WELCH_SEG:
            if state["pending"]:
                k = state["k"]
                timed("welch", lambda: welch.accumulate(ring, LD, SLOT, NSLOT, k * CH - WELCH_SEG - WELCH_SEG // 2, nseg=2))
            state["pending"] = not state["pending"]

    def flush_welch():
        if welch is not None and state["pending"]:
            k = state["k"]
            timed("welch1", lambda: welch.accumulate(ring, LD, SLOT, NSLOT, k * CH - WELCH_SEG))
            state["pending"] = False

    for _ in range(warmup):
        step()
    flush_welch()
    bt.check()  # (its first call loads torch's kernels: outside the timed region)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    state["timed"] = True
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    flush_welch()  # (an odd step count: the last segment alone, inside the timed region)
    bt.check()  # waits for the stream; raises if an integrator call failed on the device
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern = {k: (sum(a.elapsed_time(b) for a, b in v) / len(v) if v else None) for k, v in ev.items()}
    if kern["welch"] is not None:
        kern["welch"] /= 2  # ms per segment (each launch takes two)
    if kern["bold"] is not None:
        kern["bold"] /= CHUNKS  # ms per 1000-sample chunk (each pass takes a step's two)
    kern.pop("welch1")  # (a lone last segment of an odd step count: timed in the step, not reported)
    return elapsed, kern


def measure(args, world, rank, local, dist, cpu_seconds=None, cpu_numpy=True):
    """One bench line for args.config / args.precision: time the workload, attach the roofline, and
    (rank 0 of a one-GPU run, cpu_seconds given) the CPU baseline of the same workload."""
    if args.scaling is None:  # c3: the ONE sweep north_star names, split over the ranks (identical at N = 1)
        args.scaling = "strong" if args.config == "c3" else "weak"
    if args.scaling == "strong":  # one sweep, the reference's round robin (whole_sweep_both.py:63-64)
        G, S, keys = sweep_batch(0)
        if args.config == "c5":  # the C5 job: 20,000 sims over 8 GPUs; strong scaling of 1/8 of it per GPU at N=8
            G, S, keys = G[:2500 * 8], S[:2500 * 8], keys[:2500 * 8]
        mine = np.arange(len(keys)) % world == rank
        G, S, keys = G[mine], S[mine], keys[mine]
        sc = datasets.synthetic_sc(1000) if args.config == "c5" else datasets.load_sc()
    elif args.config == "c5":
        sc = datasets.synthetic_sc(1000)
        G, S, keys = sweep_batch(rank)
        lo = rank * 2500 % len(keys)
        G, S, keys = G[lo:lo + 2500], S[lo:lo + 2500], keys[lo:lo + 2500]
    else:
        sc = datasets.load_sc()
        G, S, keys = sweep_batch(rank)
    N = sc.shape[0]
    B = len(keys)
    p = driver_params()
    dev = torch.device("cuda", local)
    elapsed, kern = run_workload(sc, G, S, keys, p, args, dev, dist, args.steps, args.warmup)
    weak = None
    if dist and args.scaling == "strong" and args.config == "c3" and args.weak_steps > 0:
        # the weak-scaling aggregate beside it: every rank its own 20,000-simulation sweep (seeds 50r..)
        torch.cuda.empty_cache()
        Gw, Sw, kw = sweep_batch(rank)
        ew, kern_w = run_workload(sc, Gw, Sw, kw, p, args, dev, dist, args.weak_steps, 1)
        nsw = len(kw) * world * N * 20 * 1000 * 2 * args.weak_steps
        weak = {"value": nsw / ew, "ms_per_step": ew / args.weak_steps * 1e3, "steps": args.weak_steps,
                "sims_per_gpu": len(kw), "sims_total": len(kw) * world, "kernel_ms": kern_w}
    EULER, CHUNKS, R = 20 * 1000, 2, 20
    B_all = B
    if dist:  # strong scaling: shards may differ by one simulation
        t = torch.tensor([B], device=dev if args.dist_backend == "nccl" else "cpu", dtype=torch.int64)
        dist.all_reduce(t)
        B_all = int(t.item())
    else:
        B_all = B * world
    node_steps = B_all * N * EULER * CHUNKS * args.steps
    value = node_steps / elapsed
    fl = flops_per_node_step(N)
    per_launch_ns = B * N * EULER
    t_launch = kern["sde"] * 1e-3
    pmc_d = {}
    pmc_refused = []
    stamp = loaded_lib_sha256()

    def stamped(path):
        """profiles/pmc_*.json, only if its counters were taken on the library this process runs."""
        try:
            d = json.load(open(path)) if os.path.exists(path) else {}
        except (ValueError, OSError):
            return {}
        if d and d.get("lib_sha256") != stamp:
            pmc_refused.append({"file": os.path.relpath(path, ROOT), "stamp": d.get("lib_sha256"), "loaded": stamp})
            return {}
        return d
    pmc = os.path.join(ROOT, "profiles", "pmc_sde_c5.json" if args.config != "c3" else
                       "pmc_sde.json" if args.precision == "f32" else "pmc_sde_f64.json")
    d = stamped(pmc)
    if d.get("B") == B and d.get("N") == N and d.get("euler_steps") == EULER and \
            d.get("precision") == args.precision and \
            (N <= 96 or ("persist" in d.get("kernel", "")) == (os.environ.get("WCSDE_PERSISTENT") != "0")):
        pmc_d = d
    traffic = pmc_d.get("hbm_bytes_per_launch")
    util = {k: pmc_d[k] for k in ("valu_insts_per_wave_step", "mfma_insts_per_wave_step", "mfma_busy_frac")
            if k in pmc_d}
    if N > 96 and pmc_d:
        # the persistent kernel's SQ counters come from their own PMC passes (tools/profile_c5_pass.sh sqa / sqb, tools/profile_c5_summary.py)
        q = stamped(os.path.join(ROOT, "profiles", "pmc_c5_sq.json"))
        if q.get("kernel") == pmc_d.get("kernel"):
            util.update({k: q[k] for k in ("mfma_busy_frac", "valu_issue_busy_frac", "salu_per_wave_step") if k in q})
            util.update({f"{k.lower()}_per_wave_step": v for k, v in q.get("per_wave_step", {}).items()})
            util["wave_cycle_split"] = q.get("wave_cycle_split")
    if args.precision == "f64" and pmc_d:
        # the fp64 integrator's SQ passes (tools/profile_f64.sh)
        util.update({k: pmc_d[k] for k in ("mfma_busy_frac", "valu_issue_busy_frac", "wave_cycle_split") if k in pmc_d})
        util.update({f"{k.lower()}_per_wave_step": v for k, v in pmc_d.get("per_wave_step", {}).items()})
    sq = pmc_d.get("sq", {})
    if sq.get("SQ_ACTIVE_INST_VALU") and sq.get("GRBM_GUI_ACTIVE"):
        # SQ_ACTIVE_INST_VALU counts quad-cycles per SIMD; GRBM_GUI_ACTIVE sums the 8 XCDs' clocks
        util["valu_issue_busy_frac"] = 4 * sq["SQ_ACTIVE_INST_VALU"] / (sq["GRBM_GUI_ACTIVE"] / 8 * 1024)
    issued = None
    if args.precision == "f32":
        ifl = issued_mfma_flops_per_node_step(N)
        issued = {"dtype": "f16", "flops_per_node_step": ifl, "tflops": per_launch_ns * ifl / t_launch / 1e12,
                  "peak": PEAK_F16_TFLOPS, "util": per_launch_ns * ifl / t_launch / 1e12 / PEAK_F16_TFLOPS}
    if N <= 96 and args.precision == "f64":
        # the fp64 parity integrator (wc_sde_kernel<double>): per SIMD the fp64 VALU work and the fp64 MFMA
        # coupling take turns (ablations, DESIGN.md 5: no MFMA -105 ms, no normals -77 ms of 293), so the
        # bound is their summed issue time: 4 cycles per fp64 VALU instruction, 64 per v_mfma_f64_16x16x4
        # (78.6 TFLOP/s over 1024 SIMDs at 2.4 GHz), over the wave-steps of the launch
        achieved = per_launch_ns * fl / t_launch / 1e12
        roof = {"bound": "valu+mfma (fp64)", "achieved": achieved, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_FP64_TFLOPS, "traffic": traffic,
                "traffic_algorithmic": B * N * (EULER // R * 8 + 2 * 3 * 8 + 2 * 8),
                "kernel": "wc_sde_kernel<double> (one launch = %d Euler steps of %d sims; the full two-group "
                          "rounds and the one-group tail are two dispatches)" % (EULER, B),
                "algorithmic_flops_per_node_step": fl,
                "issued_fp64_mfma_flops_per_node_step": 2 * 96 * 96 / N if N > 80 else None,
                "note": "frac = algorithmic flops / fp64 vector peak (78.6 TFLOP/s, = the fp64 MFMA peak on MI355X); "
                        "issue_model prices the instructions the kernel issues (PMC) at the fp64 pipe rates"}
        pws = pmc_d.get("per_wave_step", {})
        if pws.get("SQ_INSTS_VALU") and pws.get("SQ_INSTS_MFMA"):
            wave_steps = -(-B // 16) * 6 * EULER
            cyc = 4 * pws["SQ_INSTS_VALU"] + 64 * pws["SQ_INSTS_MFMA"]
            t_model = wave_steps * cyc / 1024 / 2.4e9
            roof["issue_model"] = {"cycles_per_wave_step": cyc, "wave_steps": wave_steps,
                                   "ms_all_simds_busy": t_model * 1e3, "frac": t_model / t_launch}
    elif N <= 96:
        # C3 (wc_sde_kernel): state in registers for the whole launch; PMC: VALU-issue-bound (MFMA busy ~15 %).
        # SURVEY 8(d)'s algorithmic work F(N) = 2N + 35 flops per node-step against the fp32 VECTOR (VALU) peak.
        peak = PEAK_FP32_TFLOPS if args.precision == "f32" else PEAK_FP64_TFLOPS
        achieved = per_launch_ns * fl / t_launch / 1e12
        roof = {"bound": "valu", "achieved": achieved, "peak": peak, "unit": "TFLOP/s", "frac": achieved / peak,
                "traffic": traffic, "traffic_algorithmic": B * N * (EULER // R * 4 + 2 * 3 * 8 + 2 * 8),
                "kernel": "wc_sde_kernel (one launch = %d Euler steps of %d sims)" % (EULER, B),
                "algorithmic_flops_per_node_step": fl,
                "note": "bound from PMC: VALU issue (pmc.valu_issue_busy_frac); the coupling runs on the fp16 "
                        "MFMA (issued_mfma) beside it. frac = algorithmic flops / fp32 vector peak"}
        # SURVEY.md 8(d)'s state-streaming price (24 B per node-step) for the north star's "HBM roofline"
        # wording: a register-resident integrator moves none of it, so the ratio is not a roofline fraction
        gbps = per_launch_ns * 24 / t_launch / 1e9
        roof["state_streaming_equiv"] = {"bytes_per_node_step": 24, "GBps": gbps, "x_hbm_peak": gbps / PEAK_HBM_GBPS}
    else:
        # C5 (persist_kernel, wc_sde_large.hip): one launch integrates the whole chunk with the state in
        # registers; each Euler step is a 1024 x 2560 x 1024 fp16x3 GEMM whose operands stream from
        # L2 / Infinity Cache (the E image handed over between the node-block workgroups every step).
        # Priced against the fp16 MFMA that runs the contraction (the work actually issued, padding
        # included); the operand stream that binds it is reported beside
        ifl = issued_mfma_flops_per_node_step(N)
        achieved = per_launch_ns * ifl / t_launch / 1e12
        Np, Bp = -(-N // 128) * 128, -(-B // 80) * 80
        res_k = min(Np // 32, 8) * 32  # K columns of each connectome tile kept in LDS (kPRes chunks of 32)
        # operand bytes per step: the streamed part of the A rows + the E image, per workgroup
        stream = (Np // 128) * (Bp // 80) * (128 * (Np - res_k) + 80 * Np) * 4
        gbps = stream * EULER / t_launch / 1e9
        opnd = {"bytes_per_step": stream, "GBps": gbps, "ic_gather_peak_GBps": PEAK_IC_GATHER_GBPS,
                "x_ic_gather_peak": gbps / PEAK_IC_GATHER_GBPS,
                "peak_note": "MI355X_MICROARCH.md 'Indexed rows: gather into LDS': rows from the Infinity Cache "
                             "8.6 TB/s chip-wide, L2-resident rows 16.8-18.8 TB/s"}
        tcc = stamped(os.path.join(ROOT, "profiles", "pmc_c5_tcc.json"))
        if tcc.get("l2_hit_rate") is not None and tcc.get("kernel") == pmc_d.get("kernel"):
            # the requests the L2 serves at the L2-resident rate, the rest at the Infinity-Cache rate
            h = tcc["l2_hit_rate"]
            ceil = 1.0 / (h / PEAK_L2_GATHER_GBPS + (1 - h) / PEAK_IC_GATHER_GBPS)
            opnd.update({"l2_hit_rate": h, "split_peak_GBps": ceil, "frac": gbps / ceil,
                         "model": "ceiling = 1 / (h / 18.8 TB/s + (1 - h) / 8.6 TB/s), h = PMC L2 hit rate "
                                  "(profiles/pmc_c5_tcc.json, stamped on this library)"})
        roof = {"bound": "mfma", "achieved": achieved, "peak": PEAK_F16_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / PEAK_F16_TFLOPS, "traffic": traffic,
                "traffic_algorithmic": per_launch_ns * 24,
                "kernel": "persist_kernel (wc_sde_large.hip; one launch = %d Euler steps of %d sims, state in "
                          "registers)" % (EULER, B),
                "algorithmic_flops_per_node_step": fl,
                "issued_f16_flops_per_node_step": ifl,
                "algorithmic_tflops_fp32_equiv": per_launch_ns * fl / t_launch / 1e12,
                "operand_stream": opnd,
                "note": "frac = the issued fp16x3 coupling flops (padding included) over the dense fp16 MFMA peak. "
                        "operand_stream prices the per-step operand bytes (streamed connectome rows + E image) "
                        "against the L2-hit / Infinity-Cache-miss split of the gather rates; neither ceiling is "
                        "reached: the step is latency-bound (DESIGN.md 3.1b). traffic = PMC FETCH+WRITE per "
                        "launch; traffic_algorithmic = 24 B per node-step of state streaming, which this kernel "
                        "does not move"}
    roof["kernel_ms_per_launch"] = kern["sde"]
    roof["pmc"] = util or None
    roof["pmc_lib_sha256"] = stamp if pmc_d else None
    if pmc_refused:  # counters of another build are not attached (they would describe other code)
        roof["pmc_refused"] = pmc_refused
    roof["issued_mfma"] = issued if N <= 96 else None
    out = {
        "metric": "node-timesteps/sec (90-node WC, (G,sigma)x50-seed sweep) at 1/2/4/8 GPUs"
                  + ("" if args.config == "c3" else " [config 5: 1000-node synthetic connectome]"),
        "value": value,
        "unit": "node-timesteps/sec",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f32 (fp16x3 22-bit coupling)" if args.precision == "f32" else "f64",
        "dtype_detail": ("E, I, sigmoids fp32; CM.E on the fp16 MFMA as three cross terms of two-part fp16 "
                         "(22-bit) operands with fp32 accumulation; a_ie a compensated fp32 pair"
                         if args.precision == "f32" else "fp64 throughout (fp64 MFMA coupling)"),
        "data": "synthetic noise (Philox), " + ("real 90-node SC_opti_25julio connectome" if args.config == "c3"
                                                else "synthetic 1000-node connectome (datasets.synthetic_sc)"),
        "config": {"workload": ("C3: full homogeneous (G,sigma) sweep x 50 seeds (whole_sweep_both.py) per GPU; "
                                if args.config == "c3" else
                                "C5: 1000-node synthetic connectome, 2,500 sims of the (G,sigma) grid per GPU; ")
                               + "one step = 2000 recorded samples (40,000 Euler steps, tau_ip=2) of every simulation"
                               + ("" if args.sde_only else
                                  " + streamed BOLD/band-pass of the 2000 samples + one Welch segment"),
                   "sims_per_gpu": B, "sims_total": B_all, "nodes": N, "euler_steps_per_step": EULER * CHUNKS,
                   "record_every": R, "parallelism": f"sims sharded x{world} ({args.scaling} scaling)"},
        "roofline": roof,
        "kernel_ms": kern,
        "weak_scaling": weak,
    }
    if rank == 0 and world == 1 and cpu_seconds:
        out["cpu_baseline"] = cpu_baseline(sc, seconds=cpu_seconds, numpy_leg=cpu_numpy)
    else:
        out["cpu_baseline"] = None
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", default="f32", choices=("f32", "f64"))
    ap.add_argument("--config", default="c3", choices=("c3", "c5"),
                    help="c3: 20,000 sims x 90 nodes per GPU (the metric's config); c5: the 1000-node "
                         "synthetic connectome, 2,500 sims per GPU (20,000 over 8 GPUs)")
    ap.add_argument("--sde-only", action="store_true",
                    help="time the integrator alone (no streamed BOLD / Welch consumers)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="nccl (RCCL, one GPU per rank); gloo only to rehearse several ranks on one GPU")
    ap.add_argument("--cpu-seconds", type=float, default=8.0)
    ap.add_argument("--scaling", default=None, choices=("weak", "strong"),
                    help="strong (the c3 default): the one c3 sweep (20,000 sims) or c5 sweep (20,000 sims over 8 "
                         "GPUs = 2,500 x 8) split round-robin over the ranks; weak (the c5 default): 20,000 (c3) / "
                         "2,500 (c5) sims per rank")
    ap.add_argument("--secondary-steps", type=int, default=2,
                    help="the default c3 f32 line also times the C5 (1000-node) and the fp64 (reference precision) "
                         "workloads for this many steps each, reported under `secondary` (0: skip)")
    ap.add_argument("--weak-steps", type=int, default=2,
                    help="c3, strong, N > 1: also time this many steps of the weak-scaling job (every rank its "
                         "own 20,000-sim sweep) and report its aggregate as weak_scaling (0: skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dist_backend == "gloo":  # rehearsal: ranks may share a device
        local %= torch.cuda.device_count()
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")

    out = measure(args, world, rank, local, dist, None if args.no_cpu_baseline else args.cpu_seconds)
    if args.config == "c3" and args.precision == "f32" and not args.sde_only and args.secondary_steps > 0:
        # north_star asks for the 1000-node throughput and the reference-precision line beside the
        # headline: both timed in the same run, each with its own roofline, kernel times and CPU baseline
        sec = {}
        for name, cfg, prec in (("c5", "c5", "f32"), ("f64", "c3", "f64")):
            a2 = argparse.Namespace(**vars(args))
            a2.config, a2.precision, a2.scaling, a2.weak_steps = cfg, prec, None, 0
            a2.steps, a2.warmup = args.secondary_steps, 1
            torch.cuda.empty_cache()
            r = measure(a2, world, rank, local, dist,
                        None if args.no_cpu_baseline else args.cpu_seconds / 2, cpu_numpy=(cfg == "c5"))
            sec[name] = {k: r[k] for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "scaling",
                                           "dtype", "dtype_detail", "data", "config", "roofline", "kernel_ms",
                                           "cpu_baseline")}
        out["secondary"] = sec
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
