"""CPU ORACLE -- test infrastructure, never the product path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  It restates the reference algorithm on the CPU in fp64:

  * liborc.so (wc_oracle.c): the Euler-Maruyama loop of netwWilsonCowanPlastic.py
    (S wc:72-74, wilsonCowan wc:77-83, run wc:86-137) with the build's Philox
    noise stream, and the Balloon-Windkessel BOLD stage (assumed form of the
    missing BOLDModel.BD.Sim, called at wc:144);
  * sigchain.py (numpy): simBOLD's band-pass/filtfilt/decimation (wc:140-158),
    corrcoef FC, utils.get_all_metrics / kuramoto (utils.py:24-50), the Welch
    peak frequency of the drivers (whole_sweep_both.py:90-95).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liborc.so")


class OrcParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in (
        "a_ee", "a_ei", "a_ii", "tauE", "tauI", "P", "rhoE", "rE", "rI", "mu", "sigmaI",
        "sqdtD", "dtSim")]


class OrcHopfParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_double) for n in ("a", "w", "beta", "dt", "G", "norm")]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = ctypes.CDLL(LIB)
        dp = ctypes.POINTER(ctypes.c_double)
        l.orc_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
        l.orc_step_normals.argtypes = [ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, dp]
        l.orc_wc_integrate.restype = ctypes.c_int
        l.orc_wc_integrate.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int, dp, dp, dp,
                                       ctypes.c_uint64, dp, dp, dp, ctypes.c_int64, ctypes.c_int64,
                                       ctypes.c_double, ctypes.c_int64, dp, dp, dp]
        l.orc_wc_integrate_batch.restype = ctypes.c_int
        l.orc_wc_integrate_batch.argtypes = [ctypes.POINTER(OrcParams), ctypes.c_int, ctypes.c_int,
                                             dp, dp, dp, ctypes.POINTER(ctypes.c_uint64), dp, dp, dp,
                                             ctypes.c_int64, ctypes.c_int64, ctypes.c_double,
                                             ctypes.c_int64, dp, ctypes.c_int]
        l.orc_bold.argtypes = [dp, ctypes.c_int64, ctypes.c_int, ctypes.c_double, dp]
        l.orc_hopf_integrate_batch.restype = ctypes.c_int
        l.orc_hopf_integrate_batch.argtypes = [ctypes.POINTER(OrcHopfParams), ctypes.c_int, ctypes.c_int, dp,
                                               ctypes.POINTER(ctypes.c_uint64), dp, dp, ctypes.c_int64,
                                               ctypes.c_int64, ctypes.c_int64, dp]
        _lib = l
    return _lib


def _dp(a):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


def params_c(p):
    """OrcParams from a nremmodfc_amd.model.WCParams-like object."""
    return OrcParams(p.a_ee, p.a_ei, p.a_ii, p.tauE, p.tauI, p.P, p.rhoE, p.rE, p.rI, p.mu,
                     p.sigmaI, p.sqdtD, p.dtSim)


def philox(ctr, key):
    c = (ctypes.c_uint32 * 4)(*ctr)
    k = (ctypes.c_uint32 * 2)(*key)
    o = (ctypes.c_uint32 * 4)()
    lib().orc_philox4x32_10(c, k, o)
    return list(o)


def step_normals(key, step, N):
    z = np.empty(N, dtype=np.float64)
    lib().orc_step_normals(ctypes.c_uint64(int(key)), step, N, _dp(z))
    return z


class OracleBatch:
    """CPU mirror of nremmodfc_amd.model.Batch (fp64, same semantics)."""

    def __init__(self, sc, G, sigmaE, keys, params):
        self.p = params
        self.sc = np.ascontiguousarray(sc, dtype=np.float64)
        self.N = N = self.sc.shape[0]
        self.keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint64).reshape(-1))
        self.B = B = self.keys.shape[0]
        self.G = np.ascontiguousarray(np.broadcast_to(_bcast(G, B, N), (B, N)), dtype=np.float64)
        self.sigmaE = np.ascontiguousarray(np.broadcast_to(_bcast(sigmaE, B, N), (B, N)), dtype=np.float64)
        self.E = np.full((B, N), params.E0)
        self.I = np.full((B, N), params.I0)
        self.A = np.full((B, N), params.a_ie_0)
        self.step = 0
        self._pc = params_c(params)

    def integrate(self, nsteps, tau_ip, rec_every=0, nthreads=0):
        """Returns recE [B][n_rec][N] when rec_every > 0."""
        n_rec = -(-nsteps // rec_every) if rec_every else 0
        rec = np.empty((self.B, n_rec, self.N)) if rec_every else None
        rc = lib().orc_wc_integrate_batch(
            ctypes.byref(self._pc), self.B, self.N, _dp(self.sc), _dp(self.G), _dp(self.sigmaE),
            self.keys.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), _dp(self.E), _dp(self.I),
            _dp(self.A), self.step, nsteps, float(tau_ip), rec_every, _dp(rec), nthreads)
        assert rc == 0
        self.step += nsteps
        return rec


def _bcast(x, B, N):
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1 and x.shape[0] == B and B != N:
        return x[:, None]
    return x


def bold(E_t, dt):
    """Balloon-Windkessel BOLD of E_t [T][N] (assumed BD.Sim, see wc_oracle.c)."""
    E_t = np.ascontiguousarray(E_t, dtype=np.float64)
    T, N = E_t.shape
    out = np.empty_like(E_t)
    lib().orc_bold(_dp(E_t), T, N, float(dt), _dp(out))
    return out


def hopf_integrate(params, M, keys, x, y, step0, nsteps, rec_every=0):
    """Batched Hopf network (orc_hopf_integrate_batch).  params: dict a, w, beta, dt, G,
    norm; M [N][N]; x, y [B][N] updated in place.  Returns rec [B][n_rec][N] or None."""
    B, N = x.shape
    M = np.ascontiguousarray(M, dtype=np.float64)
    k = np.ascontiguousarray(keys, dtype=np.uint64)
    n_rec = -(-nsteps // rec_every) if rec_every else 0
    rec = np.empty((B, n_rec, N)) if rec_every else None
    hp = OrcHopfParams(*(float(params[n]) for n in ("a", "w", "beta", "dt", "G", "norm")))
    rc = lib().orc_hopf_integrate_batch(ctypes.byref(hp), B, N, _dp(M),
                                        k.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), _dp(x), _dp(y),
                                        int(step0), int(nsteps), int(rec_every), _dp(rec))
    assert rc == 0
    return rec
