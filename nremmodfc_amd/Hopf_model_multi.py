"""Drop-in for the reference's Hopf_model_multi.py (the SC optimiser's network model).

Same module surface (Hopf_model_multi.py:21-187): the globals a, w, beta, dt,
teq, tmax, downsamp, nnodes, ones_vector, M, norm, G, seed; Sim(verbose) ->
(results [Nmax][nnodes][2], time_vector); ParamsNode / ParamsNet / ParamsSim.
Callers mutate the globals and call Sim(), as optimize_SC_Hopf.py:18-39 does.

The Euler-Maruyama loop (Hopf_model :46-59, Noise :63-69, Sim :79-156) runs in
libwcsde.so (wc_hopf_integrate, csrc/wc_hopf.hip), fp64, batched:
sim_batch(seeds) integrates one simulation per seed in one launch, which is what
the optimiser (nremmodfc_amd.optimize_sc) uses.  Hopf_model and Noise, fused into
that kernel, are also callable on their own (one drift / one noise evaluation, as
device tensor operations; the noise from torch's device generator seeded by set_seed).

Deliberate deviations:
  * noise: the build's Philox stream keyed by the seed (numba's per-thread RNG
    cannot be reproduced outside numba);
  * initial conditions: np.random.RandomState(seed).uniform(0.01, 1, (N, 2)), what
    :121 draws when set_seed() has seeded NumPy's generator (in the jitted
    reference set_seed only seeds numba's generator, so :121 is unseeded);
  * the default M (:34) is a Watts-Strogatz graph built with numpy, seeded with 0
    (the reference calls networkx unseeded; every caller replaces M anyway).
"""
import numpy as np
import torch

from . import _lib

# Model parameters (Hopf_model_multi.py:21-25)
a = 0.0
w = 0.05 * 2 * np.pi
beta = 0.032

# Simulation parameters (:27-31)
dt = 1e-1
teq = 60
tmax = 1200
downsamp = 1


def watts_strogatz(n, k, p, seed=0):
    """Ring lattice of n nodes joined to their k nearest neighbours, every edge
    rewired with probability p (networkx.watts_strogatz_graph's algorithm), as a
    dense 0/1 matrix."""
    rng = np.random.default_rng(seed)
    adj = np.zeros((n, n))
    for j in range(1, k // 2 + 1):
        for u in range(n):
            v = (u + j) % n
            adj[u, v] = adj[v, u] = 1
    for j in range(1, k // 2 + 1):
        for u in range(n):
            v = (u + j) % n
            if rng.random() < p and adj[u, v]:
                cand = [x for x in range(n) if x != u and not adj[u, x]]
                if cand:
                    nv = cand[rng.integers(len(cand))]
                    adj[u, v] = adj[v, u] = 0
                    adj[u, nv] = adj[nv, u] = 1
    return adj


# Network parameters (:33-39)
nnodes = 90
ones_vector = np.ones(nnodes).reshape((1, nnodes))
M = watts_strogatz(nnodes, 8, 0.075)
norm = np.mean(np.sum(M, 0))
G = 0.25
seed = 0


def _col(v, device):
    return torch.as_tensor(np.asarray(v, dtype=np.float64).reshape(nnodes, 1), device=device)


def Hopf_model(x, y, t, device="cuda"):
    """Hopf_model_multi.py:46-59: the drift of one Euler step at the column states x, y (nnodes, 1)
    -> hstack((x_dot, y_dot)) (nnodes, 2).  IsynX_i = G / norm sum_j M_ij (x_j - x_i) (:50-54), the
    same sums wc_hopf_integrate forms per step."""
    X, Y = _col(x, device), _col(y, device)
    gm = torch.as_tensor(_check_m(), device=device) * (G / norm)
    isx = gm @ X - gm.sum(1, keepdim=True) * X
    isy = gm @ Y - gm.sum(1, keepdim=True) * Y
    r2 = X * X + Y * Y
    xd = (a - r2) * X - w * Y + isx
    yd = (a - r2) * Y + w * X + isy
    return torch.cat((xd, yd), dim=1).cpu().numpy()


_noise_gen = {}


def Noise(x, y, t, device="cuda"):
    """Hopf_model_multi.py:63-69: beta * N(0, 1) for x and y of every node -> (nnodes, 2), drawn
    from torch's generator on the device, seeded by set_seed (Sim() itself uses the kernel's
    Philox stream keyed by the seed)."""
    gen = _noise_gen.get(str(device))
    if gen is None:
        gen = _noise_gen[str(device)] = torch.Generator(device=device)
        gen.manual_seed(int(seed))
    z = torch.randn((nnodes, 2), generator=gen, dtype=torch.float64, device=device)
    return (z * beta).cpu().numpy()


def set_seed(s):
    """Hopf_model_multi.py:73-76: the seed of the next Sim() (and of Noise's generator)."""
    global seed
    seed = s
    _noise_gen.clear()
    return s


def initial_conditions(s, n):
    """(x, y) initial state of seed s: uniform(0.01, 1) per node and variable (:121)."""
    ic = np.random.RandomState(s).uniform(0.01, 1, (n, 2))
    return ic[:, 0].copy(), ic[:, 1].copy()


def _params():
    return _lib.WCHopfParamsC(float(a), float(w), float(beta), float(dt), float(G), float(norm))


def _check_m():
    m = np.asarray(M)
    if m.ndim != 2 or m.shape[0] != m.shape[1] or m.shape[0] != nnodes:
        raise ValueError("check M dimensions (", m.shape, ") and number of nodes (", nnodes, ")")
    return np.ascontiguousarray(m, dtype=np.float64)


_seed_cache = {}


def sim_batch(seeds, want_y=False, device="cuda"):
    """One Sim() per seed in a single launch.

    Returns x (and y) of the kept samples, time-major [Nmax][B][nnodes] fp64 device
    tensors: row k is the state after (Neq + k) * downsamp Euler steps, i.e.
    Sim()'s results[k, :, 0 / 1] (Hopf_model_multi.py:116-149).
    """
    L = _lib.lib()
    m = torch.from_numpy(_check_m()).to(device)
    n = m.shape[0]
    seeds = [int(s) for s in seeds]
    B = len(seeds)
    neq = int(teq / dt / downsamp)
    nmax = int(tmax / dt / downsamp)
    # initial states and Philox keys depend only on the seeds: uploaded once per seed list (the
    # optimiser reuses the same seeds every iteration; each small host->device copy costs ~1 ms)
    ck = (tuple(seeds), n, str(device))
    if ck not in _seed_cache:
        ics = [initial_conditions(s, n) for s in seeds]
        xy0 = torch.from_numpy(np.concatenate([np.stack([c[0] for c in ics]).ravel(),
                                               np.stack([c[1] for c in ics]).ravel()])).to(device)
        _seed_cache.clear()
        _seed_cache[ck] = (xy0, torch.tensor(seeds, dtype=torch.int64, device=device))
    xy0, keys = _seed_cache[ck]
    x = xy0[:B * n].view(B, n).clone()  # integrated in place
    y = xy0[B * n:].view(B, n).clone()
    ws = torch.empty(L.wc_hopf_workspace_size(B, n) // 8 + 1, dtype=torch.float64, device=device)
    rx = torch.empty((nmax, B, n), dtype=torch.float64, device=device)
    ry = torch.empty_like(rx) if want_y else None
    hp = _params()
    st = _lib.stream_handle()
    ds = int(downsamp)
    # transient: Neq records' worth of steps, nothing kept (results[Neq:], :152)
    rc = L.wc_hopf_integrate(hp, B, n, _lib.ptr(m), _lib.ptr(keys), _lib.ptr(x), _lib.ptr(y), 0, neq * ds, 0,
                             None, None, _lib.ptr(ws), ws.numel() * 8, st)
    _lib.check(rc, "wc_hopf_integrate (transient)")
    rc = L.wc_hopf_integrate(hp, B, n, _lib.ptr(m), _lib.ptr(keys), _lib.ptr(x), _lib.ptr(y), neq * ds, nmax * ds,
                             ds, _lib.ptr(rx), _lib.ptr(ry), _lib.ptr(ws), ws.numel() * 8, st)
    _lib.check(rc, "wc_hopf_integrate")
    return (rx, ry) if want_y else rx


def Sim(verbose=True):
    """Hopf_model_multi.py:79-156 -> (results [Nmax][nnodes][2], time_vector)."""
    rx, ry = sim_batch([seed], want_y=True)
    if verbose:
        print(f"Elapsed time: {int(tmax + teq)} seconds")
    results = torch.stack((rx[:, 0, :], ry[:, 0, :]), dim=-1).cpu().numpy()
    nmax = int(tmax / dt / downsamp)
    return results, np.linspace(0, tmax, nmax)


def ParamsNode():
    return {"a": a, "beta": beta, "w": w}


def ParamsNet():
    return {"nnodes": nnodes, "G": G, "norm": norm}


def ParamsSim():
    return {"tmax": tmax, "teq": teq, "dt": dt, "downsamp": downsamp, "seed": seed}
