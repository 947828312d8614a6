"""Device-side signal chain: BOLD + band-pass filtfilt + decimation, FC and
goodness of fit, Kuramoto, Welch peak -- thin wrappers over libwcsde.so.

References: simBOLD netwWilsonCowanPlastic.py:140-158; np.corrcoef
whole_sweep_both.py:81; utils.get_all_metrics / kuramoto utils.py:34-50; Welch
peak whole_sweep_both.py:90-95.  Every array stays on the device; columns are
c = b*N + n.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from .filters import bold_band, lfilter_zi

NEQ = 2000          # wc:145
WELCH_NPERSEG = 4000  # whole_sweep_both.py:90
WELCH_HOP = WELCH_NPERSEG // 2


def _ptr_at(t, offset_elems=0):
    """Device pointer to element `offset_elems` of a contiguous tensor."""
    if not t.is_cuda or not t.is_contiguous():
        raise _lib.WCSDEError("libwcsde takes contiguous device tensors only")
    return ctypes.c_void_p(t.data_ptr() + offset_elems * t.element_size())


class BoldStream:
    """simBOLD for C columns fed in consecutive sample chunks (any chunking).

    n_total = number of E samples per column (len(wc.time)); output after
    finish(): [M][C] fp64 = filtfilt(b, a, BOLD[neq:], axis=0)[::dec].
    """

    def __init__(self, C, n_total, neq=NEQ, dec=1000, bold_dt=0.04, device="cuda"):
        b, a = bold_band(bold_dt)
        zi = lfilter_zi(b, a)
        self.cfg = _lib.WCBoldCfgC(bold_dt, neq, n_total, dec, (ctypes.c_double * 5)(*b),
                                   (ctypes.c_double * 5)(*a), (ctypes.c_double * 4)(*zi))
        L = _lib.lib()
        self.C, self.n_total, self.device = int(C), int(n_total), torch.device(device)
        if n_total - neq < 16:
            raise ValueError("simBOLD needs at least neq + 16 samples (filtfilt padlen 15)")
        self.M = int(L.wc_bold_blocks(ctypes.byref(self.cfg)))
        nd = L.wc_bold_state_doubles(ctypes.byref(self.cfg), self.C)
        self.state = torch.empty(nd, dtype=torch.float64, device=self.device)
        _lib.check(L.wc_bold_init(ctypes.byref(self.cfg), self.C, _lib.ptr(self.state), _lib.stream_handle()),
                   "wc_bold_init")
        self.t = 0

    def feed(self, E, Tc=None, e_ld=0, offset=0, copy=None, copy_ld=0, copy_offset=0):
        """Feed the next Tc samples.  E time-major [Tc][C] (e_ld=0), or a node-major
        buffer with sample tt of column c at flat index offset + c*e_ld + tt.
        copy (fp32 time-major E only): also write the chunk node-major into
        copy at flat index copy_offset + c*copy_ld + tt (the Welch ring)."""
        if Tc is None:
            Tc = E.shape[0]
        f64 = E.dtype == torch.float64
        if not f64 and E.dtype != torch.float32:
            raise TypeError("E must be float32 or float64")
        cp = _ptr_at(copy, copy_offset) if copy is not None else None
        rc = _lib.lib().wc_bold_chunk(ctypes.byref(self.cfg), self.C, _ptr_at(E, offset), int(f64), e_ld, self.t,
                                      Tc, _lib.ptr(self.state), cp, copy_ld, _lib.stream_handle())
        _lib.check(rc, "wc_bold_chunk")
        self.t += Tc

    def finish(self):
        if self.t != self.n_total:
            raise RuntimeError(f"BoldStream fed {self.t} of {self.n_total} samples")
        out = torch.empty((self.M, self.C), dtype=torch.float64, device=self.device)
        _lib.check(_lib.lib().wc_bold_finish(ctypes.byref(self.cfg), self.C, _lib.ptr(self.state), _lib.ptr(out),
                                             _lib.stream_handle()), "wc_bold_finish")
        return out


def hilbert_phase(x):
    """Unit phasors of hilbert(x, axis=0) for x [M][C] fp64 -> [M][C][2]."""
    M, C = x.shape
    ph = torch.empty((M, C, 2), dtype=torch.float64, device=x.device)
    ws = torch.empty(M, dtype=torch.float64, device=x.device)
    _lib.check(_lib.lib().wc_hilbert_phase(C, M, _lib.ptr(x.contiguous()), _lib.ptr(ph), _lib.ptr(ws),
                                           ws.numel() * 8, _lib.stream_handle()), "wc_hilbert_phase")
    return ph


def fc_metrics(bold=None, B=None, N=None, empfc=None, fc_in=None, kuramoto=True, want_fc=False, data_range=1.0):
    """Per simulation: FC (np.corrcoef(BOLD.T)), get_all_metrics vs each empfc,
    mean(FC), Kuramoto sync/meta.

    bold [M][B*N] or [M][B][N] fp64, or fc_in [B][N][N] instead.  empfc: [K][N][N]
    tensor/array or None.  Returns (fc [B][N][N] | None, metrics [B][K][4], extra [B][3]).
    """
    L = _lib.lib()
    if bold is not None:
        M = bold.shape[0]
        bold = bold.reshape(M, B * N).contiguous()
        dev = bold.device
    else:
        fc_in = fc_in.contiguous()
        B, N = fc_in.shape[0], fc_in.shape[1]
        M, dev = 2, fc_in.device
        kuramoto = False
    K = 0 if empfc is None else int(empfc.shape[0])
    emp = None if empfc is None else torch.as_tensor(np.asarray(empfc, dtype=np.float64)).to(dev).contiguous()
    metrics = torch.empty((B, max(K, 1), 4), dtype=torch.float64, device=dev)
    extra = torch.empty((B, 3), dtype=torch.float64, device=dev)
    fc = torch.empty((B, N, N), dtype=torch.float64, device=dev) if want_fc else None
    ph = hilbert_phase(bold) if kuramoto else None
    nws = L.wc_fc_metrics_workspace_size(B, N, M, K, int(want_fc))  # 0 for N <= 96
    ws = torch.empty(nws // 8 + 1, dtype=torch.float64, device=dev) if nws else None
    rc = L.wc_fc_metrics(B, N, M, _lib.ptr(bold) if bold is not None else None, _lib.ptr(fc_in), _lib.ptr(emp), K,
                         float(data_range), _lib.ptr(ph), _lib.ptr(fc), _lib.ptr(metrics), _lib.ptr(extra),
                         _lib.ptr(ws), nws, _lib.stream_handle())
    _lib.check(rc, "wc_fc_metrics")
    return fc, metrics[:, :K], extra


def kuramoto(x, B=1, N=None):
    """utils.kuramoto of x [M][B*N] (or [M][N]) fp64 on the device -> [B][2] (sync, meta)."""
    M = x.shape[0]
    x = x.reshape(M, -1).contiguous()
    N = x.shape[1] // B if N is None else N
    ph = hilbert_phase(x)
    out = torch.empty((B, 2), dtype=torch.float64, device=x.device)
    _lib.check(_lib.lib().wc_kuramoto(B, N, M, _lib.ptr(ph), _lib.ptr(out), _lib.stream_handle()), "wc_kuramoto")
    return out


def hma(fc, want_clus_num=False):
    """HMA integration / segregation of B FC matrices on the device (HMA.py:30-203
    as run_many_seeds.py:130-133 uses it).

    fc [B][N][N] (or [N][N]) fp64 device tensor, clipped in place (FC < 0 -> 0,
    as HMA.py:55).  Returns a dict of device tensors: hin [B], hse [B],
    hin_node [B][N], hse_node [B][N], sv [B][N] (+ clus_num [B][N-1] int32).
    """
    L = _lib.lib()
    if fc.dim() == 2:
        fc = fc.unsqueeze(0)
    if fc.dtype != torch.float64 or not fc.is_contiguous():
        raise _lib.WCSDEError("hma: fc must be a contiguous fp64 device tensor (it is clipped in place)")
    B, N = fc.shape[0], fc.shape[1]
    dev = fc.device
    out = {k: torch.empty(s, dtype=torch.float64, device=dev)
           for k, s in (("hin", (B,)), ("hse", (B,)), ("hin_node", (B, N)), ("hse_node", (B, N)), ("sv", (B, N)))}
    cn = torch.empty((B, N - 1), dtype=torch.int32, device=dev) if want_clus_num else None
    if N <= HMA_JACOBI_MAX_N:
        rc = L.wc_hma(B, N, _lib.ptr(fc), _lib.ptr(out["hin"]), _lib.ptr(out["hse"]), _lib.ptr(out["hin_node"]),
                      _lib.ptr(out["hse_node"]), _lib.ptr(cn), _lib.ptr(out["sv"]), _lib.stream_handle())
        _lib.check(rc, "wc_hma")
        return _with_cn(out, cn)
    if N > HMA_MODES_MAX_N:  # fail before the eigensolver, not in wc_hma_modes
        raise _lib.WCSDEError(f"hma: N = {N} > {HMA_MODES_MAX_N} (wc_hma_modes keeps 40 B of labels per node in LDS)")
    # N > 96: F and V no longer fit one workgroup's LDS.  The eigensystem of the symmetrised
    # positive part comes from the batched device eigensolver (rocSOLVER through torch.linalg.eigh),
    # everything after it -- ranks, module levels, Balance, nodal measures -- from wc_hma_modes.
    fc.clamp_(min=0.0)  # HMA.py:55: the caller's FC is clipped in place
    for b0 in range(0, B, HMA_EIGH_BATCH):
        b1 = min(B, b0 + HMA_EIGH_BATCH)
        f = fc[b0:b1]
        lam, V = torch.linalg.eigh((f + f.transpose(1, 2)) / 2)
        vt = V.transpose(1, 2).contiguous()  # row j = eigenvector j (coalesced rows per level)
        sl = {k: v[b0:b1] for k, v in out.items()}
        rc = L.wc_hma_modes(b1 - b0, N, _lib.ptr(lam.contiguous()), _lib.ptr(vt), _lib.ptr(sl["hin"]),
                            _lib.ptr(sl["hse"]), _lib.ptr(sl["hin_node"]), _lib.ptr(sl["hse_node"]),
                            _lib.ptr(cn[b0:b1] if cn is not None else None), _lib.ptr(sl["sv"]),
                            _lib.stream_handle())
        _lib.check(rc, "wc_hma_modes")
        del lam, V, vt
    return _with_cn(out, cn)


HMA_JACOBI_MAX_N = 96   # wc_hma: F and V (2 N^2 fp64) in one workgroup's LDS
HMA_MODES_MAX_N = 4096  # wc_hma_modes: 2 N fp64 + 6 N int32 label arrays (40 N B) in 160 KB of LDS
HMA_EIGH_BATCH = 64     # N > 96: matrices per eigensolver call (bounds the V buffers)


def _with_cn(out, cn):
    if cn is not None:
        out["clus_num"] = cn
    return out


class WelchAccumulator:
    """Running node-summed |FFT|^2 of 4000-sample Hann segments (welch, nperseg=4000)."""

    def __init__(self, B, N, device="cuda"):
        L = _lib.lib()
        self.B, self.N, self.device = B, N, torch.device(device)
        self.bins = L.wc_welch_bins()
        self.ws = torch.empty(L.wc_welch_workspace_size() // 8, dtype=torch.float64, device=self.device)
        _lib.check(L.wc_welch_prepare(_lib.ptr(self.ws), self.ws.numel() * 8, _lib.stream_handle()),
                   "wc_welch_prepare")
        self.acc = torch.zeros((B, self.bins), dtype=torch.float64, device=self.device)
        self.nseg = 0

    def accumulate(self, E, ld, slot, nslots, seg0, nseg=1):
        """Add segments [seg0 + 2000 k, seg0 + 2000 k + 4000), k < nseg (1, 2 or 4), of every column of
        the node-major ring E (segments in one launch read their shared halves once from HBM)."""
        f64 = E.dtype == torch.float64
        rc = _lib.lib().wc_welch_accumulate(self.B, self.N, _ptr_at(E), int(f64), ld, slot, nslots, seg0, nseg,
                                            _lib.ptr(self.ws), _lib.ptr(self.acc), _lib.stream_handle())
        _lib.check(rc, "wc_welch_accumulate")
        self.nseg += nseg

    def peak(self, fs=500.0, want_psd=False):
        peak = torch.empty(self.B, dtype=torch.float64, device=self.device)
        psd = torch.empty((self.B, self.bins), dtype=torch.float64, device=self.device) if want_psd else None
        _lib.check(_lib.lib().wc_welch_peak(self.B, self.N, self.nseg, fs, _lib.ptr(self.acc), _lib.ptr(peak),
                                            _lib.ptr(psd), _lib.stream_handle()), "wc_welch_peak")
        return peak, psd


def welch_peak(E_t, fs=500.0, want_psd=False):
    """whole_sweep_both.py:90-95 for E [T][B][N] (time-major): peak frequency per
    simulation (and the node-mean PSD)."""
    T, B, N = E_t.shape
    nodemajor = E_t.reshape(T, B * N).t().contiguous()  # [C][T]
    wa = WelchAccumulator(B, N, E_t.device)
    nseg = (T - WELCH_NPERSEG) // WELCH_HOP + 1
    for s in range(nseg):
        wa.accumulate(nodemajor, T, T, 1, s * WELCH_HOP)
    return wa.peak(fs, want_psd)


def sim_bold(E_t, bold_downsamp=1000, neq=NEQ, bold_dt=0.04):
    """simBOLD (wc:140-158) of E [T][C] (time-major, any C) -> [M][C] fp64."""
    T = E_t.shape[0]
    C = int(np.prod(E_t.shape[1:]))
    bs = BoldStream(C, T, neq, bold_downsamp, bold_dt, E_t.device)
    bs.feed(E_t.reshape(T, C).contiguous())
    return bs.finish()


def corrcoef(x, B, N):
    """np.corrcoef(x[:, b, :].T) for every b of a time-major [M][B][N] fp64 device series
    (wc_corrcoef: split over time blocks, for long series and small batches) -> [B][N][N]."""
    L = _lib.lib()
    x = x.contiguous()
    M = x.shape[0]
    fc = torch.empty((B, N, N), dtype=torch.float64, device=x.device)
    ws = torch.empty(L.wc_corrcoef_workspace_size(B, N, M) // 8 + 1, dtype=torch.float64, device=x.device)
    _lib.check(L.wc_corrcoef(B, N, M, _lib.ptr(x), _lib.ptr(fc), _lib.ptr(ws), ws.numel() * 8,
                             _lib.stream_handle()), "wc_corrcoef")
    return fc
