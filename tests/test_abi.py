"""CPU: the C-ABI library loads and exports every entry point include/wgraph.h
declares; host-side tables the engine derives are exact."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "wgraph.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(wg_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_declares_entry_points():
    names = declared_functions()
    assert "wg_layout_build" in names and "wg_emit_vertices" in names and "wg_row_geometry" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol():
    import wgraph
    lib = ctypes.CDLL(wgraph.LIB_PATH)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing
    assert set(wgraph.EXPORTED_SYMBOLS) <= set(declared_functions())
    assert lib.wg_abi_version() == 2


def test_engine_refuses_without_gpu_instead_of_falling_back():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import wgraph
    with pytest.raises(RuntimeError):
        wgraph.Engine()


def _height_of_gap(d):
    """compute_row_heights (:486-507) for one gap, via the C oracle's rules."""
    log_max = math.log(1.0 + 2592000.0 / 7200.0)
    clamped = min(float(d), 2592000.0)
    ratio = math.log(1.0 + clamped / 7200.0) / log_max
    h = np.float32(np.float32(28.0) + np.float32(np.float32(28.0) * np.float32(ratio)))
    return math.floor(float(h) + 0.5)


def test_height_thresholds_are_exact():
    """The engine's 28 gap thresholds reproduce compute_row_heights for every gap."""
    import wgraph
    lib = ctypes.CDLL(wgraph.LIB_PATH)
    th = np.zeros(28, np.uint32)
    lib.wg_debug_height_thresholds(th.ctypes.data_as(ctypes.c_void_p))
    gaps = np.arange(0, 2592002, dtype=np.int64)
    # vectorised restatement of the f64 -> f32 chain
    log_max = math.log(1.0 + 2592000.0 / 7200.0)
    ratio = np.log1p(np.minimum(gaps, 2592000).astype(np.float64) / 7200.0)
    # np.log1p differs from log(1+x) in the last ulp; use the exact formula
    ratio = np.log(1.0 + np.minimum(gaps, 2592000).astype(np.float64) / 7200.0) / log_max
    h = np.float32(28.0) + np.float32(28.0) * ratio.astype(np.float32)
    expect = np.floor(h.astype(np.float64) + 0.5)  # heights are positive: round half up == half away
    got = 28 + (gaps[:, None] >= th[None, :].astype(np.int64)).sum(1)
    bad = np.nonzero(expect != got)[0]
    assert bad.size == 0, (bad[:10], expect[bad[:10]], got[bad[:10]])
    # spot-check the scalar path too
    for d in (0, 1, 59, 7199, 7200, 86400, 2591999, 2592000, 10 ** 9):
        assert _height_of_gap(d) == 28 + int((min(d, 2592001) >= th.astype(np.int64)).sum())
