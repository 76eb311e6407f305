"""ctypes binding of the multi-threaded CPU baseline (oracle/libcpu_mt.so).

BASELINE / TEST INFRASTRUCTURE ONLY: bench.py's `cpu_baseline_threads` leg
and tests/test_cpu_mt.py use it; the product never does.  `MtLayout` mirrors
oracle_c.OracleLayout (build + row_geometry_with_bands + graph_cell emission,
commit_graph.rs:265-399, 803-908) on `threads` OpenMP threads, bit-exact with
the single-thread oracle.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .oracle_c import _HERE, _Geom, _Layout, _arr, _geom_to_dict, abi

_lib = None


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(_HERE, "libcpu_mt.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make oracle`")
        L = ctypes.CDLL(path)
        L.wgm_layout_build.argtypes = [ctypes.POINTER(abi.Commits), ctypes.c_int, ctypes.POINTER(_Layout)]
        L.wgm_row_geometry.argtypes = [ctypes.POINTER(_Layout), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                       ctypes.POINTER(_Geom)]
        L.wgm_layout_free.argtypes = [ctypes.POINTER(_Layout)]
        L.wgm_geometry_free.argtypes = [ctypes.POINTER(_Geom)]
        L.wgm_emit_vertices.argtypes = [ctypes.POINTER(_Layout), ctypes.POINTER(_Geom), ctypes.c_uint64,
                                        ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_void_p),
                                        ctypes.POINTER(ctypes.c_uint64)]
        L.wgm_emit_vertices_into.argtypes = [ctypes.POINTER(_Layout), ctypes.POINTER(_Geom), ctypes.c_uint64,
                                             ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int,
                                             ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                             ctypes.POINTER(ctypes.c_uint64)]
        L.wgm_free.argtypes = [ctypes.c_void_p]
        L.wgm_phase_ms.argtypes = [ctypes.c_void_p]
        L.wgm_max_threads.restype = ctypes.c_int
        _lib = L
    return _lib


def max_threads() -> int:
    """omp_get_max_threads(): OMP_NUM_THREADS when set, else the CPUs OpenMP sees."""
    return int(lib().wgm_max_threads())


PHASES = ("id_table", "lane_walk", "edges", "heights_row_top", "build_geometry", "banded_geometry", "emission")


def phase_ms() -> dict:
    out = np.zeros(8, np.float64)
    lib().wgm_phase_ms(out.ctypes.data)
    return {k: float(out[i]) for i, k in enumerate(PHASES)}


class MtLayout:
    """OracleLayout on `threads` threads (0: omp_get_max_threads())."""

    def __init__(self, dag, threads=0):
        self.dag = dag
        self.threads = threads
        self._c = abi.commits_struct(dag)
        self._L = _Layout()
        self._g = None
        if lib().wgm_layout_build(ctypes.byref(self._c), threads, ctypes.byref(self._L)) != 0:
            raise MemoryError("wgm_layout_build failed")
        L = self._L
        self.n, self.max_lane, self.n_slots, self.graph_width = L.n, L.max_lane, L.n_slots, L.graph_width
        self.lane = _arr(L.lane, np.uint32, L.n)
        self.color = _arr(L.color, np.uint8, L.n)
        self.edges = _arr(L.edges, np.uint32, L.n_edges * 5).reshape(-1, 5)
        self.build_geometry = _geom_to_dict(L.geom)

    def row_geometry(self, band=None) -> dict:
        if self._g is not None:
            lib().wgm_geometry_free(ctypes.byref(self._g))
        self._g = _Geom()
        self._band = None if band is None else np.ascontiguousarray(band, np.float32)
        self._time = np.ascontiguousarray(self.dag.time, np.int64)
        rc = lib().wgm_row_geometry(ctypes.byref(self._L), self._time.ctypes.data,
                                    None if self._band is None else self._band.ctypes.data, self.threads,
                                    ctypes.byref(self._g))
        if rc != 0:
            raise MemoryError("wgm_row_geometry failed")
        return _geom_to_dict(self._g)

    def emit_vertices(self, row_begin, row_end, selected=-1, palette=None, copy=True):
        """Vertices of rows [row_begin, row_end); copy=False returns only the
        count and the offsets (the buffer is freed without a copy: timing)."""
        pal = np.ascontiguousarray(abi.DEFAULT_PALETTE if palette is None else palette, np.float32)
        g = self._L.geom if self._g is None else self._g
        pv, po, pn = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_uint64()
        rc = lib().wgm_emit_vertices(ctypes.byref(self._L), ctypes.byref(g), row_begin, row_end, selected,
                                     pal.ctypes.data, self.threads, ctypes.byref(pv), ctypes.byref(po),
                                     ctypes.byref(pn))
        if rc != 0:
            raise ValueError("wgm_emit_vertices failed")
        n = pn.value
        v = (_arr(pv.value, abi.VERTEX_DTYPE, n) if n else np.zeros(0, abi.VERTEX_DTYPE)) if copy else n
        off = _arr(po.value, np.uint64, row_end - row_begin + 1)
        lib().wgm_free(pv.value)
        lib().wgm_free(po.value)
        return v, off

    def emit_vertices_into(self, row_begin, row_end, dst, off, selected=-1, palette=None) -> int:
        """Emit into caller-owned buffers (dst: VERTEX_DTYPE array, off: uint64
        [rows + 1]), reused frame after frame; returns the vertex count, or
        raises when dst is too small."""
        pal = np.ascontiguousarray(abi.DEFAULT_PALETTE if palette is None else palette, np.float32)
        g = self._L.geom if self._g is None else self._g
        assert off.dtype == np.uint64 and len(off) >= row_end - row_begin + 1 and off.flags.c_contiguous
        assert dst.dtype == abi.VERTEX_DTYPE and dst.flags.c_contiguous
        pn = ctypes.c_uint64()
        rc = lib().wgm_emit_vertices_into(ctypes.byref(self._L), ctypes.byref(g), row_begin, row_end, selected,
                                          pal.ctypes.data, self.threads, dst.ctypes.data, len(dst), off.ctypes.data,
                                          ctypes.byref(pn))
        if rc != 0:
            raise ValueError(f"wgm_emit_vertices_into failed ({rc}: {pn.value} vertices for {len(dst)})")
        return pn.value

    def close(self):
        if self._g is not None:
            lib().wgm_geometry_free(ctypes.byref(self._g))
            self._g = None
        if self._L is not None:
            lib().wgm_layout_free(ctypes.byref(self._L))
            self._L = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
