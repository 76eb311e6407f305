"""ctypes wrapper of oracle/edt_cpu.c — the C2 CPU baseline (TEST / BENCH
INFRASTRUCTURE, never imported by the engine): WG-SDF-1 distances and SDF
bytes of an atlas coverage by an exact Felzenszwalb–Huttenlocher EDT on
`threads` OpenMP threads."""
import ctypes
import os

import numpy as np

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libedt_cpu.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make oracle`")
        _lib = ctypes.CDLL(path)
        _lib.edt_cpu_sdf.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        _lib.edt_cpu_sdf.restype = ctypes.c_int
    return _lib


def edt_sdf(cov: np.ndarray, spread: int, threads: int = 1):
    """(d2in u16, d2out u16, sdf u8) of coverage cov [H, W] (same as font_oracle.edt_sdf)."""
    cov = np.ascontiguousarray(cov, np.uint8)
    H, W = cov.shape
    d2in = np.empty((H, W), np.uint16)
    d2out = np.empty((H, W), np.uint16)
    sdf = np.empty((H, W), np.uint8)
    lib().edt_cpu_sdf(cov.ctypes.data, W, H, spread, threads, d2in.ctypes.data, d2out.ctypes.data, sdf.ctypes.data)
    return d2in, d2out, sdf
