"""The oracle's signal chain pinned to golden vectors (no GPU).

golden_scipy.npz: SciPy; golden_utils.npz: the reference's utils.py under
scikit-image 0.18.3; golden_hma.npz: the reference's HMA.py -- see
tests/golden/make_golden.py.
"""
import os

import numpy as np
import pytest

import oracle.sigchain as osg
from nremmodfc_amd import datasets
from tests.golden.make_golden import inputs

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def inp():
    return inputs()


@pytest.fixture(scope="module")
def gs():
    return np.load(os.path.join(G, "golden_scipy.npz"))


@pytest.fixture(scope="module")
def gu():
    return np.load(os.path.join(G, "golden_utils.npz"))


def test_bessel_and_zi(gs):
    b, a = osg.bold_filter_coeffs(0.04)
    np.testing.assert_allclose(b, gs["b"], rtol=1e-12, atol=1e-18)
    np.testing.assert_allclose(a, gs["a"], rtol=1e-13)
    np.testing.assert_allclose(osg.lfilter_zi(gs["b"], gs["a"]), gs["zi"], rtol=1e-10)


def test_filtfilt_full_length(inp, gs):
    y = osg.filtfilt(gs["b"], gs["a"], inp["bold"])
    np.testing.assert_array_equal(y[::1000], gs["filtfilt_dec"])  # same association order as scipy
    np.testing.assert_array_equal(y[:3000], gs["filtfilt_head"])
    np.testing.assert_array_equal(y[-3000:], gs["filtfilt_tail"])


def test_welch(inp, gs):
    f, P = osg.welch_psd(inp["e_t"].T, 500.0, 4000)
    np.testing.assert_allclose(f, gs["welch_f"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(P, gs["welch_P"], rtol=1e-9, atol=1e-18)
    meanpow = gs["welch_P"].mean(axis=0)
    assert osg.welch_peak(inp["e_t"]) == gs["welch_f"][np.argmax(meanpow)]


def test_hilbert(inp, gs):
    np.testing.assert_allclose(osg.hilbert(inp["hil"]), gs["hilbert"], rtol=1e-12, atol=1e-12)


def test_get_all_metrics_vs_reference_utils(inp, gu):
    emps = [datasets.load_empfc(s) for s in ("W", "N1", "N2", "N3")]
    fcs = inp["fcs"] + [emps[0], emps[3]]
    for i, fc in enumerate(fcs):
        for k, e in enumerate(emps):
            got = osg.get_all_metrics(fc, e, 1)
            np.testing.assert_allclose(got, gu["metrics"][i, k], rtol=1e-10, atol=1e-12)


def test_kuramoto_vs_reference_utils(inp, gu):
    for i, k in enumerate(inp["kur"]):
        np.testing.assert_allclose(osg.kuramoto(k), gu["kuramoto"][i], rtol=1e-11)
