"""Drop-in for netwWilsonCowanPlastic.py: same module globals, run(), simBOLD().

Callers keep the reference's style (whole_sweep_both.py:39-78):

    from nremmodfc_amd import netwWilsonCowanPlastic as wc
    wc.P = 0.4; wc.rhoE = 0.18; wc.CM = struct
    wc.tTrans1 = 1; wc.tTrans2 = 400; ...; wc.timeSim = np.arange(0, tstop, wc.dtSim)
    wc.G = 0.16; wc.sigmaE = 7.68; wc.sid = seed
    wc.run.recompile()            # accepted, no-op (globals are read at call time)
    tray = wc.run()               # (len(time), 3, N) float64, like the reference
    BOLD = wc.simBOLD(tray[:, 0, :], nnodes=90)

Globals are read when run() is called (numba froze them at compile time,
hence the reference's recompile() calls; here that step is unnecessary but
harmless).  Differences, by design:
  * the noise stream is the build's Philox stream keyed by `sid` (the
    reference's numba RNG ignores sid and is seeded from os.urandom);
  * `precision` ("f32" default, "f64" parity mode) selects the kernel path.
All integration and filtering run in libwcsde.so; there is no CPU path.
"""
import numpy as np
import torch

from . import sigchain
from .model import Batch, WCParams, sim_keys

# ---- MODEL PARAMETERS (wc:20-38) ----
a_ee = 3.5; a_ie_0 = 2.5
a_ei = 3.75; a_ii = 0
tauE = 0.010; tauI = 0.020
P = 0.4
Q = 0
rhoE = 0.14
tau_ip = 2
rE, rI = 0.5, 0.5
mu = 1
sigmaE = 4
sigmaI = 4

# ---- time grids (wc:41-52) ----
tTrans1 = 600
tTrans2 = 600
tstop = 600
dt = 0.002
dtSim = 0.0001
downsamp = int(dt / dtSim)
timeTrans1 = np.arange(0, tTrans1, dtSim)
timeTrans2 = np.arange(0, tTrans2, dtSim)
timeSim = np.arange(0, tstop, dtSim)
time = np.arange(0, tstop, dt)

# ---- noise (wc:55-59) ----
D = 0.002
sqdtD = D / np.sqrt(dtSim)
sid = 12

# ---- network (wc:61-68): the reference draws a random CM after np.random.seed(12) ----
G = 0.7
CM = np.random.RandomState(12).uniform(size=(90, 90))  # = np.random.seed(12); np.random.uniform(size=(90, 90))
nnodes = len(CM)
N = len(CM)

precision = "f32"
device = "cuda"


def S(x, sigma, mu):
    """Logistic sigmoid (wc:72-74): 1/(1+exp(-(x-mu)*sigma)).  Elementwise numpy
    helper for callers; the integrator evaluates it inside the HIP kernel."""
    return 1 / (1 + np.exp(-(np.asarray(x) - mu) * sigma))


class _Recompilable:
    """Callable with the no-op .recompile() of a numba dispatcher."""

    def __init__(self, fn):
        self._fn = fn
        self.__doc__ = fn.__doc__
        self.__name__ = fn.__name__

    def __call__(self, *a, **k):
        return self._fn(*a, **k)

    def recompile(self):
        return None


def _params():
    g = globals()
    if float(g["D"]) / np.sqrt(float(g["dtSim"])) != float(g["sqdtD"]):
        raise ValueError("set wc.sqdtD = wc.D / sqrt(wc.dtSim) after changing D or dtSim (wc:57)")
    return WCParams(a_ee=a_ee, a_ie_0=a_ie_0, a_ei=a_ei, a_ii=a_ii, tauE=tauE, tauI=tauI, P=P, rhoE=rhoE, rE=rE,
                    rI=rI, mu=mu, sigmaI=sigmaI, D=D, dtSim=dtSim, dt=dt)


RHS_STREAM = 0xFFFFFFFF  # Philox stream of wilsonCowan()'s noise: not run()'s (0) nor a sweep cell's
_rhs_steps = {}  # sid -> Philox step of that sid's next wilsonCowan() call: each call draws fresh noise (wc:80)


def _wilsonCowan(t, X, sigmaE, mu, tau_ip, G):
    """wilsonCowan(t, X, sigmaE, mu, tau_ip, G) of wc:77-83 -> (3, N) float64 derivatives
    (dE/dt, dI/dt, da_ie/dt), evaluated on the device (wc_rhs).  Like the reference it draws
    new noise on every call: the normals of Philox step 0, 1, 2, ... of key (sid, RHS_STREAM),
    counted per sid, so they are independent of the normals run() draws for the same sid
    (stream 0).  `t` is unused, as in the reference."""
    from . import _lib
    X = np.ascontiguousarray(X, dtype=np.float64)
    cm = np.asarray(CM, dtype=np.float64)
    n = cm.shape[0]
    if X.shape != (3, n):
        raise ValueError(f"X must be (3, N) = (3, {n}) rows (E, I, a_ie)")
    p = _params()
    p.mu = float(mu)
    dev = torch.device(device)
    tens = lambda a: torch.as_tensor(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
    g = tens(np.broadcast_to(np.asarray(G, dtype=np.float64), (n,)))
    s = tens(np.broadcast_to(np.asarray(sigmaE, dtype=np.float64), (n,)))
    keys = torch.from_numpy(sim_keys([sid], [RHS_STREAM]).view(np.int64).copy()).to(dev)
    step = _rhs_steps.get(int(sid), 0)
    x = tens(X)
    out = torch.empty_like(x)
    rc = _lib.lib().wc_rhs(p.to_c(), 1, n, _lib.ptr(tens(cm)), _lib.ptr(g), _lib.ptr(s), _lib.ptr(keys),
                           step, float(tau_ip), _lib.ptr(x), _lib.ptr(out), _lib.stream_handle())
    _lib.check(rc, "wc_rhs")
    _rhs_steps[int(sid)] = step + 1
    return out.cpu().numpy()


wilsonCowan = _Recompilable(_wilsonCowan)


def _run(verbose=False):
    """run() of wc:86-137 on the GPU: returns Y_t (len(time), 3, N) float64 with the
    state (E, I, a_ie) before every downsamp-th step of the recorded phase."""
    cm = np.asarray(CM, dtype=np.float64)
    n = cm.shape[0]
    if int(N) != n:
        raise ValueError(f"wc.N ({N}) must equal len(wc.CM) ({n}) -- the reference sizes its noise with N (wc:68)")
    p = _params()
    ds = int(dt / dtSim)
    n1, n2, n3 = len(timeTrans1), len(timeTrans2), len(timeSim)
    bt = Batch(cm, np.broadcast_to(np.asarray(G, dtype=np.float64), (n,)),
               np.broadcast_to(np.asarray(sigmaE, dtype=np.float64), (n,)), sim_keys([sid], [0]), p, precision,
               device)
    chunk = 1_000_000
    for nsteps, tau in ((n1, 0.05), (n2, 1.0)):
        done = 0
        while done < nsteps:
            k = min(chunk, nsteps - done)
            bt.integrate(k, tau)
            done += k
        if verbose:
            print(f"transient phase done ({nsteps} steps)")
    n_rec = -(-n3 // ds)
    rec = [torch.empty((n_rec, 1, n), dtype=bt.rec_dtype, device=bt.device) for _ in range(3)]
    done, r0 = 0, 0
    chunk_r = (chunk // ds) * ds
    while done < n3:
        k = min(chunk_r, n3 - done)
        bt.integrate(k, 2, ds, rec[0][r0:], rec[1][r0:], rec[2][r0:])
        done += k
        r0 += -(-k // ds)
    bt.check()
    Y_t = np.zeros((len(time), 3, n))
    m = min(len(time), n_rec)
    for j in range(3):
        Y_t[:m, j, :] = rec[j][:m, 0, :].double().cpu().numpy()
    return Y_t


run = _Recompilable(_run)


def simBOLD(E_t, nnodes=90, BOLD_downsamp=1000):
    """simBOLD (wc:140-158): Balloon-Windkessel BOLD of E_t [T][nnodes] at step
    dt*downsamp, drop 2000 samples, Bessel band-pass filtfilt, [::BOLD_downsamp]."""
    E = torch.as_tensor(np.ascontiguousarray(E_t, dtype=np.float64)).to(device)
    if E.ndim != 2 or E.shape[1] != nnodes:
        raise ValueError("E_t must be (time, nnodes)")
    return sigchain.sim_bold(E, bold_downsamp=BOLD_downsamp, bold_dt=dt * downsamp).cpu().numpy()
