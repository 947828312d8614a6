"""The three graph_utils helpers the SC optimiser uses (graph_utils.py:92-164).

Same call surface and results as the reference's get_uptri, matrix_recon and
thresholding (the rest of its 2,600-line toolbox is analysis outside the sweep
path).  Host numpy on N x N matrices: O(N^2) bookkeeping
once per optimiser iteration.
"""
import numpy as np


def get_uptri(x):
    """Strict upper triangle, row-major (graph_utils.py:92-105)."""
    x = np.asarray(x)
    return x[np.triu_indices(x.shape[0], 1)].astype(np.float64)


def matrix_recon(x):
    """Symmetric matrix with zero diagonal from its strict upper triangle (graph_utils.py:107-119)."""
    x = np.asarray(x, dtype=np.float64)
    n = int((1 + np.sqrt(1 + 8 * len(x))) // 2)
    m = np.zeros((n, n))
    m[np.triu_indices(n, 1)] = x
    return m + m.T


def thresholding(x, threshold=0.20, zero_diag=True, direct="undirected"):
    """Keep the strongest `threshold` fraction of links (graph_utils.py:135-164).

    Like the reference, zero_diag fills the caller's diagonal with 0 in place, and
    the kept set is np.argsort(...)[::-1][:k] (ties resolved as numpy resolves them).
    """
    n = x.shape[0]
    if zero_diag:
        np.fill_diagonal(x, 0)
    if direct == "directed":
        xv = x.reshape((1, n * n))
        k = int((n * n - n) * threshold)
        keep = np.argsort(xv)[0, ::-1][:k]
        out = np.zeros(n * n)
        out[keep] = xv[0, keep]
        return out.reshape((n, n))
    if direct == "undirected":
        xv = get_uptri(x)
        k = int(((n * n - n) // 2) * threshold)
        keep = np.argsort(xv)[::-1][:k]
        out = np.zeros_like(xv)
        out[keep] = xv[keep]
        return matrix_recon(out)
    raise ValueError("Invalid type of matrix -> direct options: undirected or directed")
