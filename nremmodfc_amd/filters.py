"""Host-side filter design for simBOLD's band-pass (netwWilsonCowanPlastic.py:152).

Tiny fp64 numpy design math (no trajectory touches the host): the digital
Bessel band-pass of scipy.signal.bessel(2, [2*0.01*dt, 2*0.1*dt], 'bandpass')
(analog prototype besselap(N, norm='phase') -> lp2bp -> bilinear at fs=2,
the published SciPy algorithm) and lfilter_zi's steady-state initial
conditions.  The filtering itself runs in libwcsde.so (wc_bold_*).
"""
import math

import numpy as np


def bessel_poles_phase(order):
    """Poles of besselap(order, norm='phase'): roots of the reverse Bessel
    polynomial theta_N scaled by a_last^(-1/N), a_last = (2N)!/(N! 2^N)."""
    coeffs = [math.factorial(2 * order - k) // (2 ** (order - k) * math.factorial(k) * math.factorial(order - k))
              for k in range(order + 1)]
    p = np.roots(coeffs[::-1]).astype(complex)
    a_last = math.factorial(2 * order) // math.factorial(order) // 2 ** order
    return p * 10 ** (-math.log10(a_last) / order)


def bessel_bandpass(order, wn):
    """(b, a) of scipy.signal.bessel(order, wn, btype='bandpass'), digital."""
    wn = np.asarray(wn, dtype=float)
    if wn.shape != (2,) or not (0 < wn[0] < wn[1] < 1):
        raise ValueError("wn must be two normalised frequencies 0 < w0 < w1 < 1")
    fs = 2.0
    warped = 2 * fs * np.tan(np.pi * wn / fs)
    bw = warped[1] - warped[0]
    wo = np.sqrt(warped[0] * warped[1])
    p_lp = bessel_poles_phase(order) * bw / 2
    p_bp = np.concatenate((p_lp + np.sqrt(p_lp ** 2 - wo ** 2), p_lp - np.sqrt(p_lp ** 2 - wo ** 2)))
    z_bp = np.zeros(order, dtype=complex)
    k_bp = bw ** order
    fs2 = 2.0 * fs
    z_z = np.append((fs2 + z_bp) / (fs2 - z_bp), -np.ones(order))
    p_z = (fs2 + p_bp) / (fs2 - p_bp)
    k_z = k_bp * np.real(np.prod(fs2 - z_bp) / np.prod(fs2 - p_bp))
    return np.real(k_z * np.poly(z_z)), np.real(np.poly(p_z))


def lfilter_zi(b, a):
    """Initial state of a DF2T filter for a unit step (scipy.signal.lfilter_zi)."""
    b = np.asarray(b, float) / a[0]
    a = np.asarray(a, float) / a[0]
    n = max(len(a), len(b))
    comp = np.zeros((n - 1, n - 1))
    comp[0, :] = -a[1:]
    comp[1:, :-1] += np.eye(n - 2)
    return np.linalg.solve(np.eye(n - 1) - comp.T, b[1:] - a[1:] * b[0])


def bold_band(bold_dt=0.04):
    """wc:152: a, b = signal.bessel(2, [2*0.01*BOLD_dt, 2*0.1*BOLD_dt], btype='bandpass')
    (the reference's (a, b) are (numerator, denominator))."""
    return bessel_bandpass(2, [2 * 0.01 * bold_dt, 2 * 0.1 * bold_dt])
