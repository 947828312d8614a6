"""The whole per-simulation flow of the sweep drivers, streamed on one GPU.

For a batch of simulations this reproduces, per simulation, what
whole_sweep_both.py:65-95 (and _maps.py:100-128, run_many_seeds.py:106-133)
do one simulation at a time:

  tray = wc.run()                  three Euler phases (wc:101-135)    -> wc_integrate
  BOLD = wc.simBOLD(E_t, 90)       (wc:140-158)                       -> wc_bold_*
  sFC  = np.corrcoef(BOLD.T)                                          -> wc_fc_metrics
  utils.get_all_metrics(sFC, empFC_s) for W, N1, N2, N3               -> wc_fc_metrics
  welch(E_t.T, fs=500, nperseg=4000) peak                             -> wc_welch_*
  utils.kuramoto(BOLD), np.mean(sFC)                                  -> wc_hilbert_phase + wc_fc_metrics

The recorded phase runs in chunks of `chunk_samples` samples (20 Euler steps
each; 2000 by default).  The integrator writes each chunk time-major ([chunk][C]
fp32, 14.4 GB at 20,000 x 90: full-line stores); the BOLD stream consumes it
right away and in the same pass writes it node-major into one slot of a 6000-sample
ring ([C][6000] fp32, 43.2 GB), from which the completed 4000-sample Welch
segments are transformed two at a time (one launch reads their shared half once
from HBM) -- the 648 MB/simulation trajectory of the reference never exists.
(2000-sample slots start 8000 B apart, a multiple of 64 B; with 1000-sample slots
every other slot sits 32 B off a line and its node-major rows cost the BOLD pass
~0.55 ms more per 1000 samples at C3, profiles/r04_ab/ring_align.log.)
"""
from __future__ import annotations

import dataclasses
import time
from typing import Dict, Optional

import numpy as np
import torch

from .model import F32, Batch, Schedule, WCParams, driver_params
from .sigchain import NEQ, WELCH_HOP, WELCH_NPERSEG, BoldStream, WelchAccumulator, fc_metrics

STATES = ("W", "N1", "N2", "N3")


@dataclasses.dataclass
class SweepResult:
    """Per-simulation outputs (host numpy)."""
    metrics: np.ndarray          # [B][K][4] corr, euc, ssim, new_metric (K = len(states))
    mean: np.ndarray             # [B]   np.mean(sFC)
    sync: np.ndarray             # [B]
    meta: np.ndarray             # [B]
    peakfreq: np.ndarray         # [B]   Hz
    states: tuple
    fc: Optional[np.ndarray] = None     # [B][N][N] when requested
    bold: Optional[np.ndarray] = None   # [M][B][N] when requested
    timings: Optional[dict] = None

    def columns(self):
        """The 16 metric columns of the reference's TSV rows (whole_sweep_both.py:115-116)."""
        out = {}
        for k, st in enumerate(self.states):
            out[f"ssim{st}"] = self.metrics[:, k, 2]
        for k, st in enumerate(self.states):
            out[f"corr{st}"] = self.metrics[:, k, 0]
        for k, st in enumerate(self.states):
            out[f"e{st}"] = self.metrics[:, k, 1]
        out["sync"], out["meta"], out["mean"], out["peakfreq"] = self.sync, self.meta, self.mean, self.peakfreq
        return out


def check_supported(N, schedule: Schedule = None, chunk_samples: int = 2000):
    """Raise before any device work if the pipeline cannot produce every output for
    an N-node connectome on this schedule (the epilogue's limits included)."""
    sch = schedule or Schedule()
    if N < 7:
        raise ValueError("the SSIM of get_all_metrics needs N >= 7 (7x7 window, utils.py:48)")
    if WELCH_HOP % chunk_samples or (sch.n_sim % sch.rec_every):
        raise ValueError("chunk_samples must divide 2000 and n_sim must be a multiple of rec_every")
    if sch.n_sim // sch.rec_every < NEQ + 16:
        raise ValueError(f"simBOLD needs at least {NEQ + 16} recorded samples (Neq + filtfilt padlen)")


def run_sweep(sc, G, sigmaE, keys, empfcs: Dict[str, np.ndarray] = None, schedule: Schedule = None,
              params: WCParams = None, precision: str = F32, chunk_samples: int = 2000,
              bold_downsamp: int = 1000, max_launch_steps: int = 500_000, want_fc=False, want_bold=False,
              device="cuda", progress=None, init_state: Optional[Dict[str, np.ndarray]] = None) -> SweepResult:
    """Run B simulations end to end and return the reference's per-simulation outputs.

    init_state: optional {"E", "I", "A"} -> [B][N] initial state instead of run()'s
    (0.1, 0.1, a_ie_0) (wc:90-99), e.g. to measure how a perturbation propagates."""
    sch = schedule or Schedule()
    p = params or driver_params()
    R = sch.rec_every
    check_supported(np.asarray(sc).shape[0], sch, chunk_samples)
    T = sch.n_sim // R  # recorded samples = len(wc.time)
    t_start = time.perf_counter()
    bt = Batch(sc, G, sigmaE, keys, p, precision, device)
    B, N = bt.B, bt.N
    for name, x in (init_state or {}).items():
        getattr(bt, name).copy_(torch.as_tensor(np.asarray(x, dtype=np.float64).reshape(B, N)))
    C = B * N
    # ---- transients (no recording) ----
    for n, tau in ((sch.n_trans1, sch.tau_ip[0]), (sch.n_trans2, sch.tau_ip[1])):
        done = 0
        while done < n:
            k = min(max_launch_steps, n - done)
            bt.integrate(k, tau)
            done += k
            if progress:
                progress("transient", bt.step, sch.n_total)
    # ---- recorded phase, streamed ----
    # a 6000-sample ring: Welch takes its segments two at a time (one launch reads their shared
    # half once from HBM), the last one alone if the count is odd
    nslots = (WELCH_NPERSEG + WELCH_HOP) // chunk_samples
    ld = nslots * chunk_samples
    ring = torch.empty(C * ld, dtype=bt.rec_dtype, device=bt.device)
    # fp32: the integrator writes each chunk time-major (full-line stores) and the BOLD
    # pass transposes it into the node-major Welch ring; fp64: straight into the ring
    tmaj = torch.empty(chunk_samples * C, dtype=bt.rec_dtype, device=bt.device) if precision == F32 else None
    bold = BoldStream(C, T, NEQ, bold_downsamp, p.dt * p.downsamp, bt.device)  # BOLD_dt = dt*downsamp (wc:144)
    welch = WelchAccumulator(B, N, bt.device) if T >= WELCH_NPERSEG else None
    next_seg, t_done, k = 0, 0, 0
    while t_done < T:
        n_samp = min(chunk_samples, T - t_done)
        slot = k % nslots
        if tmaj is not None:
            bt.integrate(n_samp * R, sch.tau_ip[2], R, tmaj)
            bold.feed(tmaj, n_samp, e_ld=0, copy=ring, copy_ld=ld, copy_offset=slot * chunk_samples)
        else:
            bt.integrate(n_samp * R, sch.tau_ip[2], R, ring[slot * chunk_samples:], rec_ld=ld)
            bold.feed(ring, n_samp, e_ld=ld, offset=slot * chunk_samples)
        t_done += n_samp
        k += 1
        while welch is not None and next_seg * WELCH_HOP + WELCH_NPERSEG + WELCH_HOP <= t_done:
            welch.accumulate(ring, ld, chunk_samples, nslots, next_seg * WELCH_HOP, nseg=2)
            next_seg += 2
        if progress:
            progress("recorded", bt.step, sch.n_total)
    if welch is not None and next_seg * WELCH_HOP + WELCH_NPERSEG <= T:  # an odd last segment (still in the ring)
        welch.accumulate(ring, ld, chunk_samples, nslots, next_seg * WELCH_HOP)
        next_seg += 1
    bt.check()  # waits for the stream (the phase timings below are of finished work) and raises on a device failure
    t_sde = time.perf_counter()
    # ---- epilogue ----
    states = tuple(empfcs.keys()) if empfcs else ()
    emp = np.stack([empfcs[s] for s in states]) if states else None
    bold_out = bold.finish()  # [M][C]
    fc, met, extra = fc_metrics(bold_out, B, N, emp, kuramoto=True, want_fc=want_fc)
    peak = welch.peak()[0] if welch is not None else torch.full((B,), float("nan"), device=bt.device)
    torch.cuda.synchronize(bt.device)
    t_end = time.perf_counter()
    extra_h = extra.cpu().numpy()
    return SweepResult(metrics=met.cpu().numpy(), mean=extra_h[:, 0], sync=extra_h[:, 1], meta=extra_h[:, 2],
                       peakfreq=peak.cpu().numpy(), states=states,
                       fc=fc.cpu().numpy() if want_fc else None,
                       bold=bold_out.reshape(-1, B, N).cpu().numpy() if want_bold else None,
                       timings={"integrate_and_stream_s": t_sde - t_start, "epilogue_s": t_end - t_sde,
                                "node_steps": B * N * sch.n_total})
