"""Wilson-Cowan plastic network: parameters, schedule and the batched GPU integrator.

Reference: netwWilsonCowanPlastic.py (constants wc:20-57, S wc:72-74,
wilsonCowan wc:77-83, run wc:86-137) and the driver overrides of
whole_sweep_both.py:39-52.  Integration runs in libwcsde.so (HIP, gfx950); this
module only owns parameters and device buffers.
"""
from __future__ import annotations

import ctypes
import dataclasses
import math
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib

F32, F64 = "f32", "f64"
_PREC = {F32: _lib.WC_F32, F64: _lib.WC_F64}


@dataclasses.dataclass
class WCParams:
    """Node constants of netwWilsonCowanPlastic.py:20-57 (module defaults)."""
    a_ee: float = 3.5
    a_ie_0: float = 2.5      # initial a_ie (wc:23, used as Var init wc:99)
    a_ei: float = 3.75
    a_ii: float = 0.0
    tauE: float = 0.010
    tauI: float = 0.020
    P: float = 0.4
    rhoE: float = 0.14
    rE: float = 0.5
    rI: float = 0.5
    mu: float = 1.0
    sigmaI: float = 4.0
    D: float = 0.002
    dtSim: float = 0.0001
    dt: float = 0.002        # storage interval (wc:44)
    E0: float = 0.1          # wc:91
    I0: float = 0.1          # wc:92

    @property
    def sqdtD(self) -> float:
        return self.D / math.sqrt(self.dtSim)  # wc:57

    @property
    def downsamp(self) -> int:
        return int(self.dt / self.dtSim)  # wc:46

    def to_c(self) -> _lib.WCParamsC:
        return _lib.WCParamsC(self.a_ee, self.a_ei, self.a_ii, self.tauE, self.tauI, self.P,
                              self.rhoE, self.rE, self.rI, self.mu, self.sigmaI, self.sqdtD,
                              self.dtSim)


def driver_params(**kw) -> WCParams:
    """Parameters as every sweep driver sets them (whole_sweep_both.py:39-40)."""
    p = WCParams(P=0.4, rhoE=0.18)
    return dataclasses.replace(p, **kw)


@dataclasses.dataclass
class Schedule:
    """Step counts of the three Euler phases (wc:101-135) and the recording rate.

    Drivers: tTrans1=1 s, tTrans2=400 s, tstop=600 s at dtSim=1e-4
    (whole_sweep_both.py:43-50) -> 10,000 / 4,000,000 / 6,000,000 steps.
    """
    n_trans1: int = 10_000
    n_trans2: int = 4_000_000
    n_sim: int = 6_000_000
    tau_ip: tuple = (0.05, 1.0, 2.0)   # wc:95, wc:110, wc:118
    rec_every: int = 20                # downsamp = dt/dtSim (wc:121)

    @property
    def n_total(self) -> int:
        return self.n_trans1 + self.n_trans2 + self.n_sim

    @property
    def n_rec(self) -> int:
        return -(-self.n_sim // self.rec_every)

    @classmethod
    def from_seconds(cls, tTrans1=1.0, tTrans2=400.0, tstop=600.0, dtSim=1e-4, dt=0.002):
        # lengths exactly as the reference builds them: len(np.arange(0, T, dtSim))
        return cls(len(np.arange(0, tTrans1, dtSim)), len(np.arange(0, tTrans2, dtSim)),
                   len(np.arange(0, tstop, dtSim)), rec_every=int(dt / dtSim))


def sim_keys(seeds: Sequence[int], streams: Sequence[int]) -> np.ndarray:
    """64-bit Philox keys: low word = seed, high word = stream (cell) id.

    The reference never applies its seed (SURVEY.md 8c gotcha 2); the build
    defines seed -> noise stream deterministically and independently of how
    simulations are sharded over ranks.
    """
    s = np.asarray(seeds, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    c = np.asarray(streams, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    return (c << np.uint64(32)) | s


class Batch:
    """Device state of B simulations of an N-node network (all fp64, [B][N])."""

    def __init__(self, sc, G, sigmaE, keys, params: Optional[WCParams] = None,
                 precision: str = F32, device="cuda"):
        self.params = params or driver_params()
        self.precision = precision
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is not None and \
                self.device.index != torch.cuda.current_device():
            # libwcsde launches on torch's current stream of the CURRENT device: a batch on
            # another GPU would get kernels on the wrong device's stream (fail, do not guess)
            raise ValueError(f"Batch on {self.device} but the current device is cuda:{torch.cuda.current_device()}: "
                             f"call torch.cuda.set_device({self.device.index}) first")
        sc = torch.as_tensor(np.asarray(sc, dtype=np.float64)).to(self.device).contiguous()
        if sc.ndim != 2 or sc.shape[0] != sc.shape[1]:
            raise ValueError("sc must be N x N")
        self.N = N = sc.shape[0]
        keys = np.asarray(keys, dtype=np.uint64).reshape(-1)
        self.B = B = keys.shape[0]

        def per_node(x):
            x = torch.from_numpy(np.array(x, dtype=np.float64))
            if x.ndim == 0:
                x = x.expand(B, N)
            elif x.ndim == 1 and x.shape[0] == B:
                x = x[:, None].expand(B, N)
            elif x.ndim == 1 and x.shape[0] == N:
                x = x[None, :].expand(B, N)
            if tuple(x.shape) != (B, N):
                raise ValueError(f"parameter shape {tuple(x.shape)} is not broadcastable to {(B, N)}")
            return x.contiguous().to(self.device)

        self.sc = sc
        self.G = per_node(G)
        self.sigmaE = per_node(sigmaE)
        self.keys = torch.from_numpy(keys.view(np.int64).copy()).to(self.device)
        p = self.params
        self.E = torch.full((B, N), p.E0, dtype=torch.float64, device=self.device)
        self.I = torch.full((B, N), p.I0, dtype=torch.float64, device=self.device)
        self.A = torch.full((B, N), p.a_ie_0, dtype=torch.float64, device=self.device)
        nbytes = _lib.lib().wc_workspace_size(B, N, _PREC[precision])
        self.ws = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=self.device)
        self.step = 0  # global step counter (Philox counter of the next step)
        self._pc = p.to_c()

    @property
    def rec_dtype(self):
        return torch.float32 if self.precision == F32 else torch.float64

    def integrate(self, nsteps: int, tau_ip: float, rec_every: int = 0, recE=None, recI=None,
                  recA=None, stream=None, rec_ld: int = 0):
        """Advance every simulation by nsteps (one wc_integrate call).

        rec_ld = 0: records land time-major [n_rec][B][N]; rec_ld > 0: node-major,
        record k of column c = b*N + n at flat index c*rec_ld + k of the buffer
        (the buffer may be a view starting at a ring slot).
        """
        L = _lib.lib()
        if rec_every:
            n_rec = -(-nsteps // rec_every)
            need = n_rec * self.B * self.N if rec_ld == 0 else (self.B * self.N - 1) * rec_ld + n_rec
            for r in (recE, recI, recA):
                if r is not None and (r.dtype != self.rec_dtype or r.numel() < need):
                    raise ValueError("record buffer has the wrong dtype or is too small")
        rc = L.wc_integrate(ctypes.byref(self._pc), _PREC[self.precision], self.B, self.N,
                            _lib.ptr(self.sc), _lib.ptr(self.G), _lib.ptr(self.sigmaE),
                            _lib.ptr(self.keys), _lib.ptr(self.E), _lib.ptr(self.I), _lib.ptr(self.A),
                            self.step, nsteps, float(tau_ip), rec_every, rec_ld, _lib.ptr(recE),
                            _lib.ptr(recI), _lib.ptr(recA), _lib.ptr(self.ws), self.ws.numel(),
                            _lib.stream_handle(stream))
        _lib.check(rc, "wc_integrate")
        self.step += nsteps

    def check(self, stream=None):
        """Wait for the batch's work and raise if an integrator call failed on the device.

        wc_integrate_status (the one synchronising call of the integrator ABI) reports a timed-out
        inter-workgroup wait of the last N > 96 call; such a call poisons E, I, a_ie with NaN, which
        every later call carries, so a NaN state also flags an earlier one.  Called once per batch.
        """
        L = _lib.lib()
        rc = L.wc_integrate_status(_lib.ptr(self.ws), self.B, self.N, _PREC[self.precision],
                                   _lib.stream_handle(stream))
        _lib.check(rc, "wc_integrate")
        if self.N > 96 and self.precision == F32 and bool(torch.isnan(self.E).any()):
            # (only the persistent N > 96 path poisons the state; a NaN here can also come from
            # non-finite inputs)
            why = "an earlier persistent call's wait timed out, or non-finite inputs (G, sigmaE, initial state)"
            raise _lib.WCSDEError(f"wc_integrate: NaN state ({why})")

    def state(self):
        return self.E, self.I, self.A


def run_batch(sc, G, sigmaE, keys, schedule: Schedule = None, params: WCParams = None,
              precision: str = F32, record=("E",), chunk: int = 2_000_000, device="cuda"):
    """Full three-phase run() for a batch (wc:86-137) on the GPU.

    Returns a dict of recorded trajectories, each a device tensor
    [n_rec][B][N] (time-major) holding the state before every rec_every-th
    step of the final phase -- the batched form of Y_t[:, k, :].
    """
    sch = schedule or Schedule()
    bt = Batch(sc, G, sigmaE, keys, params, precision, device)
    for n, tau in ((sch.n_trans1, sch.tau_ip[0]), (sch.n_trans2, sch.tau_ip[1])):
        done = 0
        while done < n:
            k = min(chunk, n - done)
            bt.integrate(k, tau)
            done += k
    rec = {name: torch.empty((sch.n_rec, bt.B, bt.N), dtype=bt.rec_dtype, device=bt.device)
           for name in record}
    R = sch.rec_every
    chunk_r = max(R, (chunk // R) * R)
    done = 0
    while done < sch.n_sim:
        k = min(chunk_r, sch.n_sim - done)
        r0 = done // R
        sl = {n: rec[n][r0:] for n in rec}
        bt.integrate(k, sch.tau_ip[2], R, sl.get("E"), sl.get("I"), sl.get("A"))
        done += k
    bt.check()
    return rec, bt
