"""ctypes binding of libwcsde.so (the C ABI of include/wcsde.h).

There is no CPU fallback: if the library is missing or a call fails, an
exception is raised.  PyTorch supplies device memory and streams only; torch is
imported first so that the library binds to the same HIP runtime instance.
"""
import ctypes
import os

import torch  # noqa: F401  (loads the process' HIP runtime before libwcsde.so)

from ._build import LIB_LOAD as LIB_PATH

WC_F32, WC_F64 = 0, 1

_ERRORS = {-1: "EINVAL", -2: "EUNSUPPORTED", -3: "EWORKSPACE", -4: "EHIP"}


class WCParamsC(ctypes.Structure):
    """Mirror of ``wc_params`` (include/wcsde.h)."""
    _fields_ = [(n, ctypes.c_double) for n in (
        "a_ee", "a_ei", "a_ii", "tauE", "tauI", "P", "rhoE", "rE", "rI", "mu", "sigmaI",
        "sqdtD", "dtSim")]


class WCBoldCfgC(ctypes.Structure):
    """Mirror of ``wc_bold_cfg`` (include/wcsde.h)."""
    _fields_ = [("dt", ctypes.c_double), ("neq", ctypes.c_int64), ("n_total", ctypes.c_int64),
                ("dec", ctypes.c_int64), ("b", ctypes.c_double * 5), ("a", ctypes.c_double * 5),
                ("zi", ctypes.c_double * 4)]


class WCHopfParamsC(ctypes.Structure):
    """Mirror of ``wc_hopf_params`` (include/wcsde.h)."""
    _fields_ = [(n, ctypes.c_double) for n in ("a", "w", "beta", "dt", "G", "norm")]


class WCSDEError(RuntimeError):
    pass


_lib = None

c_int, c_i64, c_sz, c_dbl, c_vp = ctypes.c_int, ctypes.c_int64, ctypes.c_size_t, ctypes.c_double, ctypes.c_void_p

_SIGNATURES = {
    "wcsde_abi_version": (c_int, []),
    "wc_last_error": (ctypes.c_char_p, []),
    "wc_workspace_size": (c_sz, [c_int, c_int, c_int]),
    "wc_integrate": (c_int, [ctypes.POINTER(WCParamsC), c_int, c_int, c_int,
                             c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp,
                             c_i64, c_i64, c_dbl, c_i64, c_i64, c_vp, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "wc_integrate_status": (c_int, [c_vp, c_int, c_int, c_int, c_vp]),
    "wc_noise": (c_int, [c_int, c_int, c_int, c_vp, c_i64, c_vp, c_vp]),
    "wc_bold_blocks": (c_i64, [ctypes.POINTER(WCBoldCfgC)]),
    "wc_bold_state_doubles": (c_sz, [ctypes.POINTER(WCBoldCfgC), c_i64]),
    "wc_bold_init": (c_int, [ctypes.POINTER(WCBoldCfgC), c_i64, c_vp, c_vp]),
    "wc_bold_chunk": (c_int, [ctypes.POINTER(WCBoldCfgC), c_i64, c_vp, c_int, c_i64, c_i64, c_i64, c_vp, c_vp, c_i64,
                              c_vp]),
    "wc_bold_finish": (c_int, [ctypes.POINTER(WCBoldCfgC), c_i64, c_vp, c_vp, c_vp]),
    "wc_hilbert_phase": (c_int, [c_i64, c_int, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "wc_fc_metrics_workspace_size": (c_sz, [c_int, c_int, c_int, c_int, c_int]),
    "wc_fc_metrics": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_int, c_dbl, c_vp, c_vp, c_vp, c_vp, c_vp, c_sz,
                              c_vp]),
    "wc_kuramoto": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp]),
    "wc_corrcoef_workspace_size": (c_sz, [c_int, c_int, c_int]),
    "wc_corrcoef": (c_int, [c_int, c_int, c_int, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "wc_hma": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wc_hma_modes": (c_int, [c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp, c_vp]),
    "wc_rhs": (c_int, [ctypes.POINTER(WCParamsC), c_int, c_int, c_vp, c_vp, c_vp, c_vp, c_i64, c_dbl, c_vp, c_vp,
                       c_vp]),
    "wc_hopf_workspace_size": (c_sz, [c_int, c_int]),
    "wc_hopf_integrate": (c_int, [ctypes.POINTER(WCHopfParamsC), c_int, c_int, c_vp, c_vp, c_vp, c_vp,
                                  c_i64, c_i64, c_i64, c_vp, c_vp, c_vp, c_sz, c_vp]),
    "wc_filtfilt": (c_int, [c_int, ctypes.POINTER(c_dbl), ctypes.POINTER(c_dbl), ctypes.POINTER(c_dbl),
                            c_i64, c_i64, c_vp, c_vp, c_vp]),
    "wc_welch_workspace_size": (c_sz, []),
    "wc_welch_bins": (c_int, []),
    "wc_welch_prepare": (c_int, [c_vp, c_sz, c_vp]),
    "wc_welch_accumulate": (c_int, [c_int, c_int, c_vp, c_int, c_i64, c_i64, c_i64, c_i64, c_int, c_vp, c_vp, c_vp]),
    "wc_welch_peak": (c_int, [c_int, c_int, c_int, c_dbl, c_vp, c_vp, c_vp, c_vp]),
}


def lib():
    """Load libwcsde.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise WCSDEError(f"{LIB_PATH} not found: build it with `python -m nremmodfc_amd._build` "
                             "(or __graft_entry__.build()); there is no CPU fallback")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(l, name)
            fn.restype = res
            fn.argtypes = args
        _lib = l
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().wc_last_error().decode(errors="replace")
        raise WCSDEError(f"{what} failed: {_ERRORS.get(rc, rc)}: {msg}")


def ptr(t):
    """Device pointer of a tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise WCSDEError("libwcsde takes device tensors only")
    if not t.is_contiguous():
        raise WCSDEError("libwcsde takes contiguous tensors only")
    return ctypes.c_void_p(t.data_ptr())


def stream_handle(stream=None):
    s = torch.cuda.current_stream() if stream is None else stream
    return ctypes.c_void_p(s.cuda_stream)
