"""Hierarchical module analysis of FC (integration / segregation), drop-in for HMA.py.

Same algorithm and call surface as the reference's HMA.py:30-203 (Wang et al.
2019, 2021; adapted by C. Coronel): eigenmode-based hierarchical modules of the
positive part of FC -> Clus_num / Clus_size per level -> integration Hin and
segregation Hse, global and nodal.  The reference builds the module tree with
exec/eval of generated variable names; here the tree is plain lists, with the
same ordering (level k+1 lists, for every module of level k in order, its
negative part then its positive part; empty modules dropped).

The per-matrix functions run on the host (numpy SVD), with the reference's call
surface.  The sweep path uses integration_segregation_batch: the same quantities
for a whole batch on the device (wc_hma / wc_hma_modes, nremmodfc_amd/csrc/wc_hma.hip;
SURVEY.md 8f rank 3), at any N.  Like the reference, every function clips the caller's FC
in place (FC[FC < 0] = 0, HMA.py:55) -- run_many_seeds saves that clipped sFC.
"""
import numpy as np


def _positive_sym(FC):
    FC[FC < 0] = 0          # in place, as the reference (HMA.py:55, :123, :178)
    return (FC + FC.T) / 2


def Functional_HP(FC):
    """Hierarchical modules (HMA.py:30-103) -> [Clus_num, Clus_size, H_all]."""
    N = FC.shape[0]
    F = _positive_sym(FC)
    u, s, v = np.linalg.svd(F)
    H1 = [np.argwhere(u[:, 1] < 0)[:, 0], np.argwhere(u[:, 1] >= 0)[:, 0]]
    H_all = [H1]
    Clus_num = [1]
    Clus_size = [[N]]
    prev_named = H1  # level-k modules in index order (neg, pos per parent)
    for mode in range(1, N - 1):
        x = np.argwhere(u[:, mode + 1] >= 0)[:, 0]
        y = np.argwhere(u[:, mode + 1] < 0)[:, 0]
        H = prev_named[:2 * Clus_num[mode - 1]]
        idx = np.array([len(h) for h in H])
        H = [H[f] for f in range(len(idx)) if idx[f] != 0]
        idx = [idx[f] for f in range(len(idx)) if idx[f] != 0]
        Clus_size.append(idx)
        Clus_num.append(len(H))
        level, named = [], []
        for h in H:
            pos = np.intersect1d(h, x)
            neg = np.intersect1d(h, y)
            level += [pos, neg]   # the reference appends H_{j+2} (pos) then H_{j+1} (neg)
            named += [neg, pos]   # ... and the next level reads them by index: neg first
        H_all.append(level)
        prev_named = named
    return [Clus_num, Clus_size, H_all]


def _hf(FC, Clus_num, Clus_size):
    N = FC.shape[0]
    F = _positive_sym(FC)
    u, s, v = np.linalg.svd(F)
    s[s < 0] = 0
    s = s ** 2
    p = np.zeros(N - 1)
    for i in range(0, len(Clus_num) - 1):
        p[i] = np.sum(np.abs(np.array(Clus_size[i]) - N / Clus_num[i])) / N
    HF = s[0:(N - 1)] * np.array(Clus_num) * (1 - p)
    return HF, u, N


def Balance(FC, Clus_num, Clus_size):
    """Integration and segregation components (HMA.py:107-151) -> [Hin, Hse]."""
    HF, _, N = _hf(FC, Clus_num, Clus_size)
    return [np.sum(HF[0]) / N ** 2, np.sum(HF[1:(N - 1)]) / N ** 2]


def nodal_measures(FC, Clus_num, Clus_size):
    """Nodal integration / segregation (HMA.py:155-203) -> [Hin_nodal, Hse_nodal]."""
    HF, u, N = _hf(FC, Clus_num, Clus_size)
    Hin_nodal = HF[0] / N * u[:, 0] ** 2
    Hse_nodal = np.zeros(N)
    for i in range(1, N - 1):
        Hse_nodal += HF[i] / N * u[:, i] ** 2
    return [Hin_nodal, Hse_nodal]


def integration_segregation(sFC):
    """run_many_seeds.py:130-136 for one simulation: the dict it pickles."""
    cn, cs, _ = Functional_HP(sFC)
    hin, hse = Balance(sFC, cn, cs)
    hin_n, hse_n = nodal_measures(sFC, cn, cs)
    return {"Hin_sim": hin, "Hse_sim": hse, "Hin_node_sim": hin_n, "Hse_node_sim": hse_n, "sFC": sFC}


def integration_segregation_batch(sfcs, device="cuda"):
    """integration_segregation for a batch [B][N][N] on the device: one wc_hma launch
    (Jacobi in LDS) for N <= 96; for N > 96 the batched device eigensolver and one
    wc_hma_modes launch (sigchain.hma).

    Returns one dict per matrix with the keys run_many_seeds.py:134-136 pickles;
    sFC is the clipped matrix (as the reference saves it).
    """
    import torch

    from . import sigchain
    fc = torch.as_tensor(np.ascontiguousarray(np.asarray(sfcs, dtype=np.float64))).to(device)
    r = sigchain.hma(fc)
    clipped = fc.cpu().numpy()
    hin, hse = r["hin"].cpu().numpy(), r["hse"].cpu().numpy()
    hin_n, hse_n = r["hin_node"].cpu().numpy(), r["hse_node"].cpu().numpy()
    return [{"Hin_sim": np.float64(hin[b]), "Hse_sim": np.float64(hse[b]), "Hin_node_sim": hin_n[b],
             "Hse_node_sim": hse_n[b], "sFC": clipped[b]} for b in range(fc.shape[0])]
