"""CPU ORACLE for the per-simulation signal chain -- test infrastructure only.

Restates, in numpy/fp64, what the reference does after run():

  simBOLD           netwWilsonCowanPlastic.py:140-158  (BD.Sim -> [2000:] -> bessel
                    band-pass -> filtfilt(axis=0) -> [::BOLD_downsamp])
  sFC               whole_sweep_both.py:81             np.corrcoef(BOLD.T)
  get_all_metrics   utils.py:42-50 (+ new_metric utils.py:28-31)
  kuramoto          utils.py:34-40
  Welch peak        whole_sweep_both.py:90-95

Third-party algorithms on that path (not vendored in /root/reference, versions
unpinned by it; restated from their published definitions and pinned by golden
vectors generated in this container, tests/golden/make_golden.py):
  scipy.signal.bessel / lfilter_zi / lfilter / filtfilt / welch / hilbert
      (SciPy 1.15.3, system Python; 1.7.1 in /opt/conda)
  skimage.metrics.structural_similarity (scikit-image 0.18.3, /opt/conda)
"""
import ctypes
import math

import numpy as np

from . import _dp, bold, lib

NEQ = 2000  # wc:145


# ---------------- filter design: scipy.signal.bessel(N, Wn, 'bandpass') ----------------
def _bessel_poles_phase(order):
    """besselap(N, norm='phase'): roots of the reverse Bessel polynomial theta_N,
    scaled by a_last^(-1/N) (a_last = (2N)!/(N! 2^N))."""
    # theta_N(s) = sum_k (2N-k)! / (2^(N-k) k! (N-k)!) s^k
    coeffs = [math.factorial(2 * order - k) // (2 ** (order - k) * math.factorial(k) * math.factorial(order - k))
              for k in range(order + 1)]
    p = np.roots(coeffs[::-1]).astype(complex)
    a_last = math.factorial(2 * order) // math.factorial(order) // 2 ** order
    return p * 10 ** (-math.log10(a_last) / order)


def bessel_bandpass(order, wn):
    """(b, a) of scipy.signal.bessel(order, wn, btype='bandpass') (digital, fs=2)."""
    wn = np.asarray(wn, dtype=float)
    fs = 2.0
    warped = 2 * fs * np.tan(np.pi * wn / fs)
    bw = warped[1] - warped[0]
    wo = np.sqrt(warped[0] * warped[1])
    p = _bessel_poles_phase(order)
    k = 1.0
    # lp2bp_zpk
    p_lp = p * bw / 2
    p_bp = np.concatenate((p_lp + np.sqrt(p_lp ** 2 - wo ** 2), p_lp - np.sqrt(p_lp ** 2 - wo ** 2)))
    z_bp = np.zeros(order, dtype=complex)
    k_bp = k * bw ** order
    # bilinear_zpk (fs=2)
    fs2 = 2.0 * fs
    z_z = (fs2 + z_bp) / (fs2 - z_bp)
    p_z = (fs2 + p_bp) / (fs2 - p_bp)
    z_z = np.append(z_z, -np.ones(order))
    k_z = k_bp * np.real(np.prod(fs2 - z_bp) / np.prod(fs2 - p_bp))
    b = np.real(k_z * np.poly(z_z))
    a = np.real(np.poly(p_z))
    return b, a


def lfilter_zi(b, a):
    """scipy.signal.lfilter_zi: steady-state initial conditions for a unit step."""
    b = np.asarray(b, float) / a[0]
    a = np.asarray(a, float) / a[0]
    n = max(len(a), len(b))
    comp = np.zeros((n - 1, n - 1))
    comp[0, :] = -a[1:]
    comp[1:, :-1] += np.eye(n - 2)
    IminusA = np.eye(n - 1) - comp.T
    B = b[1:] - a[1:] * b[0]
    return np.linalg.solve(IminusA, B)


def lfilter(b, a, x, zi):
    """DF2T IIR along axis 0 of x [n][m] (C, fp64); returns (y, zf)."""
    x = np.ascontiguousarray(x, dtype=np.float64)
    if x.ndim == 1:
        y, zf = lfilter(b, a, x[:, None], np.asarray(zi, float).reshape(-1, 1))
        return y[:, 0], zf[:, 0]
    n, m = x.shape
    order = len(a) - 1
    b = np.ascontiguousarray(b, float)
    a = np.ascontiguousarray(a, float)
    z = np.ascontiguousarray(np.broadcast_to(np.asarray(zi, float).reshape(order, -1), (order, m)))
    y = np.empty_like(x)
    lib().orc_lfilter(_dp(b), _dp(a), order, _dp(x), n, m, _dp(z), _dp(y))
    return y, z


lib().orc_lfilter.argtypes = [ctypes.POINTER(ctypes.c_double)] * 2 + [ctypes.c_int, ctypes.POINTER(ctypes.c_double),
                                                                     ctypes.c_int64, ctypes.c_int] + \
    [ctypes.POINTER(ctypes.c_double)] * 2


def filtfilt(b, a, x):
    """scipy.signal.filtfilt(b, a, x, axis=0) with padtype='odd', padlen=3*max(len(a),len(b))."""
    x = np.asarray(x, dtype=np.float64)
    padlen = 3 * max(len(a), len(b))
    ext = np.concatenate((2 * x[0] - x[padlen:0:-1], x, 2 * x[-1] - x[-2:-padlen - 2:-1]), axis=0)
    zi = lfilter_zi(b, a)
    zi_m = zi[:, None] * ext[0][None, :] if x.ndim == 2 else zi * ext[0]
    y, _ = lfilter(b, a, ext, zi_m)
    y0 = y[-1]
    zi_m = zi[:, None] * y0[None, :] if x.ndim == 2 else zi * y0
    y, _ = lfilter(b, a, y[::-1], zi_m)
    return y[::-1][padlen:-padlen]


def bold_filter_coeffs(bold_dt=0.04):
    """wc:152 -- a, b = signal.bessel(2, [2*0.01*BOLD_dt, 2*0.1*BOLD_dt], btype='bandpass')."""
    return bessel_bandpass(2, [2 * 0.01 * bold_dt, 2 * 0.1 * bold_dt])


def sim_bold(E_t, bold_downsamp=1000, dt=0.002, downsamp=20):
    """simBOLD (wc:140-158) with the Balloon-Windkessel BD.Sim of wc_oracle.c."""
    bold_dt = dt * downsamp
    B = bold(E_t, bold_dt)[NEQ:]
    b, a = bold_filter_coeffs(bold_dt)
    return filtfilt(b, a, B)[::bold_downsamp]


# ---------------- FC and goodness of fit (utils.py) ----------------
def flat_fc(fc):
    """utils.py:24-26 / :44-45 -- strict upper triangle, row-major."""
    n = len(fc)
    return np.concatenate([fc[i, i + 1:] for i in range(n)])


def uniform_filter(img, size=7):
    """scipy.ndimage.uniform_filter (mode='reflect'), separable: axis 0 then axis 1."""
    r = size // 2
    out = img.astype(np.float64)
    for ax in (0, 1):
        pad = [(0, 0), (0, 0)]
        pad[ax] = (r, r)
        p = np.pad(out, pad, mode="symmetric")  # ndimage 'reflect' == numpy 'symmetric'
        acc = np.zeros_like(out)
        for k in range(size):
            sl = [slice(None), slice(None)]
            sl[ax] = slice(k, k + out.shape[ax])
            acc += p[tuple(sl)]
        out = acc / size
    return out


def ssim(im1, im2, data_range=1.0, win_size=7, K1=0.01, K2=0.03):
    """skimage.metrics.structural_similarity(im1, im2, data_range=...) defaults:
    uniform 7x7 window, sample covariance (NP/(NP-1)), mean over the image cropped
    by (win_size-1)//2 on every side."""
    NP = win_size ** 2
    cov_norm = NP / (NP - 1)
    ux, uy = uniform_filter(im1, win_size), uniform_filter(im2, win_size)
    uxx, uyy, uxy = uniform_filter(im1 * im1, win_size), uniform_filter(im2 * im2, win_size), \
        uniform_filter(im1 * im2, win_size)
    vx = cov_norm * (uxx - ux * ux)
    vy = cov_norm * (uyy - uy * uy)
    vxy = cov_norm * (uxy - ux * uy)
    C1, C2 = (K1 * data_range) ** 2, (K2 * data_range) ** 2
    A1, A2 = 2 * ux * uy + C1, 2 * vxy + C2
    B1, B2 = ux ** 2 + uy ** 2 + C1, vx + vy + C2
    S = (A1 * A2) / (B1 * B2)
    pad = (win_size - 1) // 2
    return S[pad:-pad, pad:-pad].mean()


def get_all_metrics(sFC, empFC, data_range=1):
    """utils.py:42-50 -> (corr, euc, ssim, new_metric)."""
    fs, fe = flat_fc(sFC), flat_fc(empFC)
    corr = np.corrcoef(fs, fe)[0, 1]
    euc = np.linalg.norm(fe - fs)
    s = ssim(sFC, empFC, data_range=data_range)
    newm = 1 - np.corrcoef(fs, fe)[0, 1] + (fs.mean() - fe.mean()) ** 2
    return corr, euc, s, newm


def hilbert(x):
    """scipy.signal.hilbert(x, axis=0): analytic signal via FFT."""
    N = x.shape[0]
    Xf = np.fft.fft(x, N, axis=0)
    h = np.zeros(N)
    if N % 2 == 0:
        h[0] = h[N // 2] = 1
        h[1:N // 2] = 2
    else:
        h[0] = 1
        h[1:(N + 1) // 2] = 2
    return np.fft.ifft(Xf * h.reshape((N,) + (1,) * (x.ndim - 1)), axis=0)


def kuramoto(sign):
    """utils.py:34-40 -> (sync, meta)."""
    analytic = hilbert(sign)
    R = np.abs(np.mean(np.exp(1j * np.angle(analytic)), axis=1))
    return R.mean(), R.std()


def welch_psd(x, fs, nperseg):
    """scipy.signal.welch(x, fs, nperseg) along the last axis: periodic Hann,
    noverlap = nperseg//2, constant detrend, density scaling, one-sided, mean."""
    n = np.arange(nperseg)
    win = 0.5 - 0.5 * np.cos(2 * np.pi * n / nperseg)
    step = nperseg - nperseg // 2
    nseg = (x.shape[-1] - nperseg) // step + 1
    scale = 1.0 / (fs * (win * win).sum())
    acc = 0.0
    for s in range(nseg):
        seg = x[..., s * step:s * step + nperseg]
        seg = seg - seg.mean(axis=-1, keepdims=True)
        X = np.fft.rfft(win * seg, axis=-1)
        P = (X.conj() * X).real * scale
        if nperseg % 2 == 0:
            P[..., 1:-1] *= 2
        else:
            P[..., 1:] *= 2
        acc = acc + P
    return np.fft.rfftfreq(nperseg, 1.0 / fs), acc / nseg


def welch_peak(E_t, fs=500.0, nperseg=4000):
    """whole_sweep_both.py:90-95: first argmax of the node-mean Welch PSD of E_t (T x N)."""
    freqs, P = welch_psd(np.asarray(E_t, float).T, fs, nperseg)
    meanpow = P.mean(axis=0)
    return freqs[np.where(meanpow == meanpow.max())[0][0]]


def sim_metrics(E_t, empFCs, bold_downsamp=1000):
    """The per-simulation epilogue of whole_sweep_both.py:79-95 on one E_t (T x N)."""
    BOLD = sim_bold(E_t, bold_downsamp)
    sFC = np.corrcoef(BOLD.T)
    out = {}
    for st, emp in empFCs.items():
        c, e, s, _ = get_all_metrics(sFC, emp, 1)
        out[f"corr{st}"], out[f"e{st}"], out[f"ssim{st}"] = c, e, s
    out["sync"], out["meta"] = kuramoto(BOLD)
    out["mean"] = np.mean(sFC)
    out["peakfreq"] = welch_peak(E_t)
    return out, BOLD, sFC
