"""Input data of the reference, shipped as exact .npy copies (nremmodfc_amd/data/).

SC_opti_25julio.txt (structural connectome, loaded at whole_sweep_both.py:34),
empirical/mean_mat_{W,N1,N2,N3}_8dic24.txt (empirical FC, whole_sweep_both.py:36-37)
empirical/maps/*.npy (NA/ACh proxy maps, whole_sweep_both_maps.py:44-65) and
empirical/structural_Deco_AAL.txt (the SC optimiser's starting connectome,
optimize_SC_Hopf.py:28).
The SHUFFLED_*_LABELS_*.npy files of the reference are pickled object arrays and
are not shipped (nothing on the hot path reads them).
"""
import os

import numpy as np

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
STATES = ("W", "N1", "N2", "N3")

# whole_sweep_both_maps.py:35-41 / run_many_seeds.py:66-72
MAPNAMES_ACH = ["HOMO", "DIST_VAChT_feobv_hc18_aghourian", "SHUFFLED_SYMM_DIST_VAChT_feobv_hc18_aghourian"]
MAPNAMES_NA = ["HOMO", "DIST_LC_proj", "SHUFFLED_SYMM_DIST_LC_proj"]


def load_sc():
    return np.load(os.path.join(DATA, "SC_opti_25julio.npy"))


def load_deco_sc():
    """empirical/structural_Deco_AAL.txt (optimize_SC_Hopf.py:28)."""
    return np.load(os.path.join(DATA, "structural_Deco_AAL.npy"))


def load_empfc(state):
    return np.load(os.path.join(DATA, f"mean_mat_{state}_8dic24.npy"))


def load_map(name, n=90):
    """Map normalised to mean 1 (whole_sweep_both_maps.py:47-57); HOMO = ones.
    The division happens in the file's dtype (float32 for the VAChT maps), as
    the reference does, and only then is widened to float64.  For n != 90 (the
    synthetic connectome) the maps are synthetic_map()s: ACh seed 1001, NA seed
    1002, the SHUFFLED_* names a fixed permutation of them."""
    if name != "HOMO" and n != 90:
        m = synthetic_map(n, 1001 if "VAChT" in name else 1002)
        return m[np.random.default_rng(7).permutation(n)] if name.startswith("SHUFFLED") else m
    m = np.ones(n) if name == "HOMO" else np.load(os.path.join(DATA, name + ".npy"))
    return (m / m.mean()).astype(np.float64)


def synthetic_sc(n=1000, seed=1000, density=0.395, mean_rowsum=2.51):
    """Synthetic connectome for the N=1000 configuration: symmetric,
    uniform weights on a random support of the given density, zero diagonal,
    scaled so the mean row sum matches SC_opti_25julio (2.51)."""
    rng = np.random.default_rng(seed)
    w = rng.uniform(size=(n, n))
    mask = rng.uniform(size=(n, n)) < density
    m = np.triu(w * mask, 1)
    m = m + m.T
    return m * (mean_rowsum / m.sum(axis=1).mean())


def synthetic_map(n=1000, seed=1001):
    """Seeded log-normal heterogeneity map with mean 1 (N=1000 maps mode)."""
    m = np.random.default_rng(seed).lognormal(0.0, 0.3, n)
    return m / m.mean()
