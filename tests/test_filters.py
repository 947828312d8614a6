"""Host-side filter design of the product (nremmodfc_amd/filters.py) vs SciPy goldens (no GPU)."""
import os

import numpy as np

from nremmodfc_amd import filters

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_scipy.npz")


def test_bold_band_matches_scipy():
    g = np.load(G)
    b, a = filters.bold_band(0.04)
    np.testing.assert_allclose(b, g["b"], rtol=1e-12, atol=1e-18)
    np.testing.assert_allclose(a, g["a"], rtol=1e-13)
    np.testing.assert_allclose(filters.lfilter_zi(b, a), g["zi"], rtol=1e-10)


def test_bessel_rejects_bad_band():
    import pytest
    with pytest.raises(ValueError):
        filters.bessel_bandpass(2, [0.5, 0.1])
