"""Drop-in for the FC/observable part of utils.py (utils.py:18-50).

get_all_metrics and kuramoto run in libwcsde.so (wc_fc_metrics,
wc_hilbert_phase + wc_kuramoto); the small array helpers the reference defines
next to them (flat_FC, new_metric, cohen_d) are kept as host numpy one-liners
for callers that import them.  Plotting/analysis helpers of utils.py
(sub_weight, cortex_mat, RSN_profile_FC, find_extreme, xy2plotcor,
fill_missing, scale_mat, envelope) are not on the sweep path
and are not mirrored.
"""
import numpy as np
import torch

from . import sigchain

device = "cuda"


def cohen_d(x, y):
    """utils.py:18-22 -- effect size between two samples."""
    nx, ny = len(x), len(y)
    dof = nx + ny - 2
    return (np.mean(x) - np.mean(y)) / np.sqrt(((nx - 1) * np.std(x, ddof=1) ** 2 + (ny - 1) * np.std(y, ddof=1) ** 2)
                                               / dof)


def flat_FC(FC):
    """utils.py:24-26 -- strict upper triangle, row-major."""
    n = len(FC)
    return np.concatenate([FC[i, i + 1:] for i in range(n)])


def new_metric(flat1, flat2):
    """utils.py:28-31."""
    return 1 - np.corrcoef(flat1, flat2)[0, 1] + (flat1.mean() - flat2.mean()) ** 2


def kuramoto(sign):
    """utils.py:34-40: (sync, meta) of the Kuramoto order parameter of sign (T x N)
    from the phases of its analytic signal (hilbert along axis 0)."""
    x = torch.as_tensor(np.ascontiguousarray(sign, dtype=np.float64)).to(device)
    if x.ndim != 2:
        raise ValueError("sign must be (time, nodes)")
    out = sigchain.kuramoto(x, B=1, N=x.shape[1]).cpu().numpy()[0]
    return out[0], out[1]


def get_all_metrics(sFC, empFC, data_range=1):
    """utils.py:42-50 -> (corr, euc, ssim, new_metric) of sFC against empFC:
    Pearson and Euclidean distance of the strict upper triangles, skimage SSIM
    (7x7 uniform window, sample covariance), and new_metric."""
    s = np.asarray(sFC, dtype=np.float64)
    e = np.asarray(empFC, dtype=np.float64)
    if s.shape != e.shape or s.ndim != 2 or s.shape[0] != s.shape[1]:
        raise ValueError("sFC and empFC must be square matrices of the same shape")
    fc = torch.as_tensor(np.ascontiguousarray(s)).to(device)[None]
    _, met, _ = sigchain.fc_metrics(fc_in=fc, empfc=e[None], data_range=data_range)
    corr, euc, ssim, newm = met[0, 0].cpu().numpy()
    return corr, euc, ssim, newm
