"""The fp64 parity path's straight-line elementary functions (nremmodfc_amd/csrc/wc_device.h, f64m)
against extended-precision references, over the inputs the integrator gives them.

They replace ocml's exp / log / sincospi and the IEEE division in the fp64 integrator
(netwWilsonCowanPlastic.py:72-83 in fp64: the sigmoid S() of wc:72-74 and the Box-Muller normals
standing in for np.random.normal of wc:80).  End-to-end parity of the fp64 path (1e-14 against the
oracle, 6e-15 against the reference's own run() under noise replay) is in test_sde_gpu.py; this file
pins each function alone with an explicit ulp bound:

* log_u24 and sincospi_v23 over ALL 2^23 odd v < 2^24 (every uniform the noise stream can give);
* exp2 over the clamp range and densely over |t| <= 80; rcp and sqrt_pos over positive normals;
* the fp64 sigmoid 1 / (1 + 2^t), t = (mu - x) s log2(e): its relative error grows with |t|, because t
  is rounded before the exponential (about 2.08 |t| units of 2^-53 from the three roundings of t; at
  |t| = 40 that is ~80 units, tens of ulp) -- the bound below states exactly that.

The kernels are evaluated through libwcsde_diag.so's wc_diag_f64m (csrc/wcsde_diag.h, the diagnostic
build __graft_entry__.build() makes beside the product library).  The references use numpy's 80-bit
long double with exact argument reductions (log1p near 1, quarter turns by integer arithmetic).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

PI_L = np.longdouble("3.14159265358979323846264338327950288")
LN2_L = np.longdouble("0.693147180559945309417232121458176568")


@pytest.fixture(scope="module")
def diag(cuda):
    from nremmodfc_amd import _build
    assert os.path.exists(_build.DIAG_LIB), "libwcsde_diag.so missing: __graft_entry__.build() makes it"
    lib = ctypes.CDLL(_build.DIAG_LIB)
    lib.wc_diag_f64m.restype = ctypes.c_int
    lib.wc_diag_f64m.argtypes = [ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    return lib


def _run(lib, fn, x, nout):
    xin = torch.as_tensor(x).cuda()
    n = len(x) if fn != 4 else len(x) // 2
    out = torch.empty(nout, dtype=torch.float64, device="cuda")
    rc = lib.wc_diag_f64m(fn, n, ctypes.c_void_p(xin.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                          ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    return out.cpu().numpy()


def _ulps(got, ref):
    """|got - ref| in units of the spacing of the float64 nearest ref."""
    r64 = ref.astype(np.float64)
    return (np.abs(got.astype(np.longdouble) - ref) / np.spacing(np.abs(r64)).astype(np.longdouble)).astype(np.float64)


def test_log_u24_all_odd_v(diag):
    v = np.arange(1, 1 << 24, 2, dtype=np.uint32)
    got = _run(diag, 2, v, len(v))
    vl = v.astype(np.longdouble)
    ref = np.where(v >= (1 << 23), np.log1p((vl - (1 << 24)) / (1 << 24)), np.log(vl / (1 << 24)))
    u = _ulps(got, ref)
    print(f"TOL log_u24: max {u.max():.3f} ulp (bound 2) over {len(v)} odd v")
    assert u.max() <= 2.0


def test_sincospi_v23_all_odd_v(diag):
    v = np.arange(1, 1 << 24, 2, dtype=np.uint32)
    got = _run(diag, 3, v, 2 * len(v)).reshape(-1, 2)
    m = (v.astype(np.int64) + (1 << 21)) >> 22                      # nearest quarter turn of pi v 2^-23
    r = (v.astype(np.int64) - (m << 22)).astype(np.longdouble) / (1 << 23)  # exact, |r| <= 1/4
    s, c = np.sin(PI_L * r), np.cos(PI_L * r)
    q = m & 3
    sin_ref = np.select([q == 0, q == 1, q == 2, q == 3], [s, c, -s, -c])
    cos_ref = np.select([q == 0, q == 1, q == 2, q == 3], [c, -s, -c, s])
    us, uc = _ulps(got[:, 0], sin_ref), _ulps(got[:, 1], cos_ref)
    print(f"TOL sincospi_v23: sin max {us.max():.3f} ulp, cos max {uc.max():.3f} ulp (bound 2)")
    assert us.max() <= 2.0 and uc.max() <= 2.0


def test_exp2_and_rcp(diag):
    rng = np.random.default_rng(7)
    t = np.concatenate([np.linspace(-80, 80, 1 << 20), rng.uniform(-1000, 1000, 1 << 18), [-1000.0, 1000.0, 0.0]])
    got = _run(diag, 0, t, len(t))
    u = _ulps(got, np.exp2(t.astype(np.longdouble)))
    print(f"TOL exp2: max {u.max():.3f} ulp (bound 2) over |t| <= 1000")
    assert u.max() <= 2.0
    d = np.concatenate([1.0 + rng.random(1 << 19), np.exp(rng.uniform(-300, 300, 1 << 19))])
    got = _run(diag, 1, d, len(d))
    u = _ulps(got, 1 / d.astype(np.longdouble))
    print(f"TOL rcp: max {u.max():.3f} ulp (bound 1)")
    assert u.max() <= 1.0


def test_sqrt_pos(diag):
    """The Box-Muller radius sqrt(-2 ln u) without the library's scaling: over the whole range of
    -2 ln u for 24-bit uniforms, [2^-23, 33.3], and beyond."""
    rng = np.random.default_rng(5)
    x = np.concatenate([np.exp(rng.uniform(np.log(2.0 ** -24), np.log(40.0), 1 << 20)), [2.0 ** -23, 33.27]])
    got = _run(diag, 5, x, len(x))
    u = _ulps(got, np.sqrt(x.astype(np.longdouble)))
    print(f"TOL sqrt_pos: max {u.max():.3f} ulp (bound 1)")
    assert u.max() <= 1.0


def test_f64_sigmoid_error_grows_with_t(diag):
    """S(x) of wc:72-74 as the fp64 integrator evaluates it: relative error <= (2.5 |t| + 8) 2^-53."""
    rng = np.random.default_rng(11)
    x = rng.uniform(-6.0, 8.0, 1 << 20)
    s = rng.uniform(3.5, 8.5, 1 << 20)
    xs = np.stack([x, s], 1).reshape(-1)
    got = _run(diag, 4, xs, len(x))
    xl, sl = x.astype(np.longdouble), s.astype(np.longdouble)
    ref = 1 / (1 + np.exp(-(xl - 1) * sl))
    rel = (np.abs(got.astype(np.longdouble) - ref) / ref).astype(np.float64) * 2.0 ** 53
    t = np.abs((1 - x) * s * 1.4426950408889634)
    excess = rel - 2.5 * t
    print(f"TOL f64 sigmoid: max rel {rel.max():.1f} x 2^-53 at |t| <= {t.max():.1f}; "
          f"max (rel - 2.5|t|) {excess.max():.2f} (bound 8); at |t| < 1: {rel[t < 1].max():.2f}")
    assert excess.max() <= 8.0


def test_table_coefficients_equal_literals(diag):
    """WC_F64_TAB = 1 reads the coefficients from the kCoefDev table instead of folding literals in;
    both come from one list (wc_device.h), so each function gives the same bits either way."""
    v = np.arange(1, 1 << 24, 2 * 97, dtype=np.uint32)
    np.testing.assert_array_equal(_run(diag, 18, v, len(v)), _run(diag, 2, v, len(v)))
    np.testing.assert_array_equal(_run(diag, 19, v, 2 * len(v)), _run(diag, 3, v, 2 * len(v)))
    t = np.linspace(-1000, 1000, 1 << 18)
    np.testing.assert_array_equal(_run(diag, 16, t, len(t)), _run(diag, 0, t, len(t)))
