"""libwcsde.so builds, loads and exports every symbol include/wcsde.h declares (no GPU)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "wcsde.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", src)) - {"if", "sizeof", "defined"})


def test_header_parses():
    fns = header_functions()
    assert "wc_integrate" in fns and "wc_last_error" in fns


def test_library_exports_header_symbols():
    from nremmodfc_amd import _build, _lib
    _build.build()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_functions():
        assert hasattr(lib, name), name


def test_product_library_has_no_diagnostic_entry_points():
    """The ablation entry point ships only in libwcsde_diag.so (csrc/wcsde_diag.h)."""
    from nremmodfc_amd import _build
    _build.build()
    lib = ctypes.CDLL(_build.LIB)
    assert not hasattr(lib, "wc_diag_integrate")
    assert not hasattr(lib, "wc_large_diag")


def test_abi_version_and_workspace():
    from nremmodfc_amd import _lib
    L = _lib.lib()
    assert L.wcsde_abi_version() == 7
    # N <= 96: sized for the 3-part 16-bit image and a 256-B slot behind it (the fp16x2 image and its
    # two scale floats fit inside; the three-part fp16 A/B variant's scales go in the slot)
    assert L.wc_workspace_size(20000, 90, _lib.WC_F32) == 6 * 3 * 3 * 64 * 16 + 256
    assert L.wc_workspace_size(20000, 90, _lib.WC_F64) == 6 * 6 * 64 * 4 * 8
    assert L.wc_workspace_size(1, 16, _lib.WC_F32) == 2 * 1 * 3 * 64 * 16 + 256
    # N > 96 (wc_sde_large.hip): fp16x2 A image + 2 scale floats (one 256-B slot) + 6 fp32 state arrays
    # (E, I, a_ie pair, G, slope) + 2 fp16x2 E operand images
    Bp, Np = 2560, 1024
    # + per-simulation (G, slope) pairs and the uniformity flag (one 256-B slot)
    # + the status word of the last call (one 256-B slot after both layouts)
    want = (Np // 16) * (Np // 32) * 2 * 64 * 16 + 256 + Bp * Np * (6 * 4 + 2 * 4) + Bp * 8 + 256 + 256
    assert L.wc_workspace_size(2500, 1000, _lib.WC_F32) == want
    assert L.wc_workspace_size(2500, 1000, _lib.WC_F64) == (Np // 16) * (Np // 4) * 64 * 8 + Bp * Np * 6 * 8 + 256


def test_invalid_arguments_fail_loudly():
    """Argument validation happens before any device work (runs without a GPU)."""
    from nremmodfc_amd import _lib
    L = _lib.lib()
    p = _lib.WCParamsC()
    rc = L.wc_integrate(ctypes.byref(p), 0, 0, 90, *([None] * 7), 0, 1, 1.0, 0, 0, None, None, None,
                        None, 0, None)
    assert rc == -1
    assert b"invalid" in L.wc_last_error()
    rc = L.wc_integrate(ctypes.byref(p), 0, 4, 300_000, *([ctypes.c_void_p(16)] * 7), 0, 1, 1.0, 0, 0,
                        None, None, None, ctypes.c_void_p(16), 1 << 20, None)
    assert rc == -2
    rc = L.wc_integrate(ctypes.byref(p), 0, 2500, 1000, *([ctypes.c_void_p(16)] * 7), 0, 1, 1.0, 0, 0,
                        None, None, None, ctypes.c_void_p(16), 1 << 20, None)
    assert rc == -3  # the N > 96 path needs its state image
    # the signal-chain entry points validate before touching the device too
    cfg = _lib.WCBoldCfgC()
    cfg.dec, cfg.neq, cfg.n_total = 1000, 2000, 2010  # fewer than neq + 16 samples
    assert L.wc_bold_init(ctypes.byref(cfg), 10, ctypes.c_void_p(16), None) == -1
    assert L.wc_fc_metrics(1, 200, 298, None, None, None, 0, 1.0, None, None, None, None, None, 0, None) == -1
    vp = ctypes.c_void_p(16)
    assert L.wc_fc_metrics_workspace_size(4, 90, 298, 4, 0) == 0           # N <= 96: LDS only
    need = L.wc_fc_metrics_workspace_size(4, 1000, 298, 0, 0)             # N > 96: the FC tiles in global memory
    assert need >= 4 * 1000 * 1000 * 8
    assert L.wc_fc_metrics_workspace_size(4, 1000, 298, 0, 1) < need - 4 * 1000 * 1000 * 8 + 1
    assert L.wc_fc_metrics(4, 1000, 298, vp, None, None, 0, 1.0, None, None, None, vp, vp, need - 8, None) == -3
    assert L.wc_fc_metrics(4, 6, 298, vp, None, None, 0, 1.0, None, None, None, vp, None, 0, None) == -1
    assert L.wc_kuramoto(0, 90, 298, None, None, None) == -1
    assert L.wc_welch_bins() == 2001


def test_hma_validates_without_device_work():
    from nremmodfc_amd import _lib
    L = _lib.lib()
    vp = ctypes.c_void_p(16)
    assert L.wc_hma(4, 90, None, vp, vp, vp, vp, None, None, None) == -1
    assert L.wc_hma(4, 97, vp, vp, vp, vp, vp, None, None, None) == -2
    assert b"96" in L.wc_last_error()
    # N > 96 goes through wc_hma_modes (caller's eigensystem): it validates before launching too
    assert L.wc_hma_modes(4, 1000, None, vp, vp, vp, vp, vp, None, None, None) == -1
    assert L.wc_hma_modes(4, 2, vp, vp, vp, vp, vp, vp, None, None, None) == -1
    assert L.wc_hma_modes(1, 20000, vp, vp, vp, vp, vp, vp, None, None, None) == -2


def test_rhs_validates_without_device_work():
    from nremmodfc_amd import _lib
    L = _lib.lib()
    p = _lib.WCParamsC()
    vp = ctypes.c_void_p(16)
    assert L.wc_rhs(ctypes.byref(p), 0, 90, vp, vp, vp, vp, 0, 1.0, vp, vp, None) == -1
    assert L.wc_rhs(ctypes.byref(p), 1, 90, vp, vp, vp, vp, 1 << 48, 1.0, vp, vp, None) == -2


def test_corrcoef_validates_without_device_work():
    from nremmodfc_amd import _lib
    L = _lib.lib()
    vp = ctypes.c_void_p(16)
    assert L.wc_corrcoef_workspace_size(10, 90, 6000) > 10 * 90 * 90 * 8
    assert L.wc_corrcoef_workspace_size(0, 90, 6000) == 0
    assert L.wc_corrcoef_workspace_size(10, 1000, 6000) == 2 * 10 * 1000 * 8  # N > 96: means and sds
    assert L.wc_corrcoef(10, 1000, 6000, vp, vp, vp, 64, None) == -3        # N > 96 workspace
    assert L.wc_corrcoef(10, 1, 6000, vp, vp, vp, 1 << 30, None) == -1       # N < 2
    assert L.wc_corrcoef(10, 90, 1, vp, vp, vp, 1 << 30, None) == -1     # M < 2
    assert L.wc_corrcoef(10, 90, 6000, vp, vp, vp, 64, None) == -3       # workspace
    assert b"workspace" in L.wc_last_error()
