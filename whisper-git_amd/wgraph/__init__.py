"""wgraph — MI355X commit-graph render-prep engine (host side).

Python mirror of the reference's `GraphLayout` interface
(/root/reference/src/commit_graph.rs:240-507) over the engine's C ABI
(include/wgraph.h, libwgraph.so).  Every computation runs in the HIP engine;
there is no CPU fallback: if the shared library or a gfx950 device is
missing, constructing an Engine raises.

    layout = GraphLayout()                      # GraphLayout::new   (:261)
    layout.build(commits)                       # GraphLayout::build (:265)
    layout.get(oid)                             # GraphLayout::get   (:357)
    layout.max_lane, layout.edges, layout.row_geometry, layout.graph_width
    layout.row_geometry_with_bands(commits, bands)     # (:367)
    compute_row_heights(commits)                # (:486)
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

from . import abi

_HERE = os.path.dirname(os.path.abspath(__file__))
# WGRAPH_LIB selects an alternative in-tree build of the same engine (kernel variants)
LIB_PATH = os.environ.get("WGRAPH_LIB") or os.path.join(_HERE, "libwgraph.so")
_lib = None


class WgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{abi.ERRORS.get(code, code)}: {msg}")
        self.code = code


def lib():
    """Load libwgraph.so (fails loudly; there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: build it with `make engine` or __graft_entry__.build()")
        # One HIP runtime per process.  torch ships its own libamdhip64
        # (SONAME libamdhip64.so.7) and loads it by the name libamdhip64.so,
        # which does not match an /opt/rocm copy loaded earlier: loading the
        # engine first leaves two runtimes in a process that later uses
        # torch.cuda ("No HIP GPUs are available").  With torch imported first
        # the engine binds to torch's runtime.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, u64, i64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32
        sig = {
            "wg_create": ([ctypes.c_int], vp), "wg_destroy": ([vp], None),
            "wg_last_error": ([vp], ctypes.c_char_p), "wg_abi_version": ([], ctypes.c_int),
            "wg_set_stream": ([vp, vp], ctypes.c_int), "wg_synchronize": ([vp], ctypes.c_int),
            "wg_set_option": ([vp, ctypes.c_int, i64], ctypes.c_int),
            "wg_layout_build": ([vp, ctypes.POINTER(abi.Commits)], ctypes.c_int),
            "wg_layout_summary_get": ([vp, ctypes.POINTER(abi.LayoutSummary)], ctypes.c_int),
            "wg_copy_lanes": ([vp, vp, vp], ctypes.c_int),
            "wg_copy_edges": ([vp, vp], ctypes.c_int),
            "wg_copy_row_heights": ([vp, vp], ctypes.c_int),
            "wg_compute_row_heights": ([vp, vp, u64, i32, vp], ctypes.c_int),
            "wg_row_geometry": ([vp, vp, i32], ctypes.c_int),
            "wg_row_geometry_list": ([vp, ctypes.POINTER(abi.Commits), vp, i32], ctypes.c_int),
            "wg_layout_build_frame": ([vp, ctypes.POINTER(abi.Commits), vp, i32], ctypes.c_int),
            "wg_geometry_summary_get": ([vp, ctypes.POINTER(abi.GeometrySummary)], ctypes.c_int),
            "wg_copy_geometry": ([vp, ctypes.POINTER(abi.GeometryHost)], ctypes.c_int),
            "wg_emit_vertices": ([vp, u64, u64, i64, vp], ctypes.c_int),
            "wg_vertex_summary_get": ([vp, ctypes.POINTER(abi.VertexSummary)], ctypes.c_int),
            "wg_vertex_placement_get": ([vp, vp, vp, vp], ctypes.c_int),
            "wg_copy_vertices": ([vp, u64, u64, vp], ctypes.c_int),
            "wg_copy_vertex_offsets": ([vp, vp], ctypes.c_int),
            "wg_device_views_get": ([vp, ctypes.POINTER(abi.DeviceViews)], ctypes.c_int),
            "wg_enable_timing": ([vp, ctypes.c_int], ctypes.c_int),
            "wg_debug_counters": ([vp, vp, ctypes.c_int], ctypes.c_int),
            "wg_stage_timings": ([vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p),
                                  ctypes.POINTER(ctypes.c_float)], ctypes.c_int),
            "wg_font_atlas_build": ([vp, ctypes.c_int, vp, u64, ctypes.POINTER(abi.AtlasParams)], ctypes.c_int),
            "wg_font_atlas_info": ([vp, ctypes.c_int, ctypes.POINTER(abi.AtlasInfo)], ctypes.c_int),
            "wg_copy_font_atlas": ([vp, ctypes.c_int, vp, vp, vp, vp, vp], ctypes.c_int),
            "wg_emit_glyphs": ([vp, u64, u64, vp, vp, i32, ctypes.POINTER(abi.TextParams)], ctypes.c_int),
            "wg_glyph_summary_get": ([vp, ctypes.POINTER(abi.GlyphSummary)], ctypes.c_int),
            "wg_copy_glyph_vertices": ([vp, u64, u64, vp], ctypes.c_int),
            "wg_copy_glyph_offsets": ([vp, vp], ctypes.c_int),
            "wg_shard_build_begin": ([vp, ctypes.POINTER(abi.Commits), ctypes.c_int, ctypes.c_int, u64, u64,
                                      ctypes.POINTER(abi.ShardMsg)], ctypes.c_int),
            "wg_shard_geometry_begin": ([vp, vp, i32, ctypes.POINTER(abi.ShardMsg)], ctypes.c_int),
            "wg_shard_build_frame_begin": ([vp, ctypes.POINTER(abi.Commits), ctypes.c_int, ctypes.c_int, u64, u64, vp, i32,
                                            ctypes.POINTER(abi.ShardMsg)], ctypes.c_int),
            "wg_shard_copy_msg": ([vp, vp], ctypes.c_int),
            "wg_shard_pack_slot": ([vp, vp, u64], ctypes.c_int),
            "wg_shard_slot_heads": ([vp, vp, u64, ctypes.c_int, vp], ctypes.c_int),
            "wg_shard_msg_bytes": ([vp, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "wg_match_rows": ([vp, vp, u64, u64, u64, ctypes.POINTER(abi.RowText), ctypes.POINTER(ctypes.c_uint64)],
                              ctypes.c_int),
            "wg_copy_match_flags": ([vp, vp], ctypes.c_int),
            "wg_order_rows": ([vp, vp, u64, vp, u64, vp, u64, i32, vp, i32], ctypes.c_int),
            "wg_render": ([vp, ctypes.POINTER(abi.RenderParams), vp, i32], ctypes.c_int),
            "wg_write_png": ([ctypes.c_char_p, vp, ctypes.c_uint32, ctypes.c_uint32], ctypes.c_int),
            "wg_lower_utf8": ([vp, u64, vp, u64, ctypes.POINTER(ctypes.c_uint64)], ctypes.c_int),
            "wg_shard_exchange": ([vp, vp, u64, ctypes.POINTER(ctypes.c_uint64), vp, ctypes.POINTER(abi.ShardMsg)],
                                  ctypes.c_int),
        }
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
        _lib = L
    return _lib


EXPORTED_SYMBOLS = (
    "wg_abi_version", "wg_create", "wg_destroy", "wg_last_error", "wg_set_stream", "wg_synchronize", "wg_set_option",
    "wg_layout_build", "wg_layout_summary_get", "wg_copy_lanes", "wg_copy_edges", "wg_copy_row_heights",
    "wg_compute_row_heights", "wg_row_geometry", "wg_row_geometry_list", "wg_layout_build_frame", "wg_geometry_summary_get", "wg_copy_geometry", "wg_emit_vertices",
    "wg_vertex_summary_get", "wg_vertex_placement_get", "wg_copy_vertices", "wg_copy_vertex_offsets", "wg_device_views_get",
    "wg_enable_timing", "wg_stage_timings", "wg_debug_counters", "wg_shard_build_begin", "wg_shard_build_frame_begin", "wg_shard_geometry_begin",
    "wg_shard_copy_msg", "wg_shard_msg_bytes", "wg_shard_pack_slot", "wg_shard_slot_heads", "wg_shard_exchange", "wg_font_atlas_build", "wg_font_atlas_info", "wg_copy_font_atlas",
    "wg_emit_glyphs", "wg_glyph_summary_get", "wg_copy_glyph_vertices", "wg_copy_glyph_offsets",
    "wg_match_rows", "wg_copy_match_flags", "wg_lower_utf8", "wg_order_rows", "wg_render", "wg_write_png")


def to_lowercase(b: bytes) -> bytes:
    """Rust str::to_lowercase of UTF-8 bytes with the engine's own tables (host)."""
    b = bytes(b)
    src = np.frombuffer(b, np.uint8) if b else np.zeros(1, np.uint8)
    n = ctypes.c_uint64()
    rc = lib().wg_lower_utf8(src.ctypes.data, len(b), None, 0, ctypes.byref(n))
    if rc != abi.WG_OK:
        raise WgError(rc, "wg_lower_utf8")
    out = np.empty(max(1, n.value), np.uint8)
    lib().wg_lower_utf8(src.ctypes.data, len(b), out.ctypes.data, n.value, ctypes.byref(n))
    return out[:n.value].tobytes()


def write_png(path: str, rgba: np.ndarray) -> None:
    """RGBA8 [H, W, 4] -> PNG file (the engine's writer, host code)."""
    a = np.ascontiguousarray(rgba, np.uint8)
    h, w = a.shape[:2]
    rc = lib().wg_write_png(os.fsencode(path), a.ctypes.data, w, h)
    if rc != abi.WG_OK:
        raise WgError(rc, f"wg_write_png({path})")


FONT_DIR = os.path.join(os.path.dirname(_HERE), "fonts")
FONTS = {0: os.path.join(FONT_DIR, "Roboto-Regular.ttf"), 1: os.path.join(FONT_DIR, "Roboto-Bold.ttf")}


class Engine:
    """One wg_ctx (one per thread), bound to one GPU."""

    def __init__(self, device: int = -1):
        L = lib()
        self._ctx = L.wg_create(device)
        if not self._ctx:
            raise RuntimeError("wg_create failed: no gfx950 (MI355X) device visible to HIP")
        self._keep = []

    # -- plumbing --------------------------------------------------------------
    def _check(self, rc: int):
        if rc != abi.WG_OK:
            raise WgError(rc, lib().wg_last_error(self._ctx).decode(errors="replace"))

    def close(self):
        if getattr(self, "_ctx", None):
            lib().wg_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, hip_stream_ptr: int | None):
        self._check(lib().wg_set_stream(self._ctx, hip_stream_ptr))
        self._stream_ptr = hip_stream_ptr or None

    def synchronize(self):
        self._check(lib().wg_synchronize(self._ctx))

    def set_lane_path(self, general: bool):
        """Force the general lane walk (True) or auto-select (False)."""
        self._check(lib().wg_set_option(self._ctx, 1, 1 if general else 0))

    def set_defer_validation(self, on: bool):
        """WG_OPT_DEFER_VALIDATION: a speculative build is validated with the
        next emission's vertex-total read instead of before build() returns
        (results identical; a build that does not hold is redone there)."""
        self._check(lib().wg_set_option(self._ctx, 5, 1 if on else 0))

    def set_replay_mode(self, mode: int):
        """WG_OPT_REPLAY_MODE: 0 auto, 1 the chunked fixed-point replay, 2 the
        single-wave serial replay, 3 the compacted fixed point (leaked slots
        struck out; speed only, results identical)."""
        self._check(lib().wg_set_option(self._ctx, 8, int(mode)))

    def set_dc_warmup(self, events: int):
        """WG_OPT_DC_WARMUP: the compacted replay's first-iteration warm-up
        (events, a multiple of 64; 0 = auto)."""
        self._check(lib().wg_set_option(self._ctx, 10, int(events)))

    def set_join_fused(self, on: bool):
        """WG_OPT_JOIN_FUSED: the id table's place pass inside the window probe,
        or (default) the table built on the side stream beside it."""
        self._check(lib().wg_set_option(self._ctx, 11, int(bool(on))))

    def set_vtx_tile(self, verts: int):
        """WG_OPT_VTX_TILE: vertices per emission tile (1024, 2048; 0 = auto)."""
        self._check(lib().wg_set_option(self._ctx, 12, int(verts)))

    def set_match_threads(self, threads: int):
        """WG_OPT_MATCH_THREADS: threads per 256-row workgroup of the search
        kernel: 512 (default, 0) or 256.  Speed only."""
        self._check(lib().wg_set_option(self._ctx, 14, int(threads)))

    def set_fused_read(self, on: bool):
        """WG_OPT_FUSED_READ: the emission's host read written by the kernel
        that computes the vertex total (default) or by a read kernel."""
        self._check(lib().wg_set_option(self._ctx, 13, int(bool(on))))

    def set_slice_lists(self, mode: int):
        """WG_OPT_SLICE_LISTS: a deferred-validation build leaves its geometry
        lists to the next whole-list emission, which builds them in two row
        slices, the second beside the first slice's tiles (speed only).
        0 off (default), 1 lists of >= 2^18 rows, 2 any list past 256 rows."""
        self._check(lib().wg_set_option(self._ctx, 9, int(mode)))

    def set_shard_spec_replay(self, on: bool):
        """WG_OPT_SHARD_SPEC_REPLAY: the sharded build's X3 step replays the
        global lane events without a host read, the replay checked with the
        local geometry pass's validation words (default on; a replay that
        misses is redone there, no extra exchange)."""
        self._check(lib().wg_set_option(self._ctx, 7, 1 if on else 0))

    # -- layout ----------------------------------------------------------------------
    def build(self, dag=None, commits: abi.Commits | None = None):
        """GraphLayout::build on a wgraph.synth.Dag (host) or a prepared wg_commits."""
        if commits is None:
            commits = abi.commits_struct(dag)
            self._keep = [dag]
        self._commits = commits
        self._check(lib().wg_layout_build(self._ctx, ctypes.byref(commits)))

    def build_frame(self, dag=None, commits: abi.Commits | None = None, band=None, device_ptr: int | None = None):
        """build() then row_geometry(band) in one call (wg_layout_build_frame):
        the frame's banded row_top runs on the side stream beside the build."""
        if commits is None:
            commits = abi.commits_struct(dag)
            self._keep = [dag]
        self._commits = commits
        if device_ptr is not None:
            self._check(lib().wg_layout_build_frame(self._ctx, ctypes.byref(commits), device_ptr, abi.WG_DEVICE))
        else:
            b = np.ascontiguousarray(band, np.float32)
            self._band = b
            self._check(lib().wg_layout_build_frame(self._ctx, ctypes.byref(commits), b.ctypes.data, abi.WG_HOST))

    # -- row-sharded build (one rank per GPU; see wgraph.shard.ShardComm) ------------------
    def shard_build(self, commits: abi.Commits, world: int, rank: int, row_begin: int, row_end: int, comm):
        """GraphLayout::build of rows [row_begin, row_end) of a device-resident
        list every rank holds; `comm` all-gathers the engine's messages."""
        self._commits = commits
        msg = abi.ShardMsg()
        self._check(lib().wg_shard_build_begin(self._ctx, ctypes.byref(commits), world, rank, row_begin, row_end,
                                               ctypes.byref(msg)))
        self._shard_loop(msg, comm)

    def shard_build_frame(self, commits: abi.Commits, world: int, rank: int, row_begin: int, row_end: int, comm,
                          band=None, device_ptr: int | None = None):
        """shard_build then shard_geometry(band) in one sharded call
        (wg_shard_build_frame_begin): one exchange and one geometry pass fewer."""
        self._commits = commits
        msg = abi.ShardMsg()
        if device_ptr is not None:
            ptr, res = device_ptr, abi.WG_DEVICE
        else:
            b = np.ascontiguousarray(band, np.float32)
            self._band = b
            ptr, res = b.ctypes.data, abi.WG_HOST
        self._check(lib().wg_shard_build_frame_begin(self._ctx, ctypes.byref(commits), world, rank, row_begin, row_end,
                                                     ptr, res, ctypes.byref(msg)))
        self._shard_loop(msg, comm)

    def shard_geometry(self, comm, band=None, device_ptr: int | None = None):
        """row_geometry_with_bands of this rank's shard (band = the whole list's)."""
        msg = abi.ShardMsg()
        if device_ptr is not None:
            self._check(lib().wg_shard_geometry_begin(self._ctx, device_ptr, abi.WG_DEVICE, ctypes.byref(msg)))
        elif band is None:
            self._check(lib().wg_shard_geometry_begin(self._ctx, None, abi.WG_HOST, ctypes.byref(msg)))
        else:
            b = np.ascontiguousarray(band, np.float32)
            self._band = b
            self._check(lib().wg_shard_geometry_begin(self._ctx, b.ctypes.data, abi.WG_HOST, ctypes.byref(msg)))
        self._shard_loop(msg, comm)

    def _shard_loop(self, msg, comm):
        # wg_shard_exchange may leave reads of the gathered buffer queued on the
        # engine's stream: each buffer is kept until the next wg_shard_copy_msg
        # (which synchronises that stream) has returned.  When the engine runs
        # on the transport's stream, slots are packed in stream order instead
        # (wg_shard_pack_slot, no host synchronisation before the collective).
        pack = read_heads = None
        if getattr(comm, "on_device", False) and getattr(self, "_stream_ptr", None):
            import torch
            if torch.cuda.current_stream(comm.device).cuda_stream == self._stream_ptr:
                def pack(slot, cap):
                    self._check(lib().wg_shard_pack_slot(self._ctx, slot, cap))

                if 3 * comm.world <= 64:
                    def read_heads(ptr, stride):   # polled device read in stream order (no stream sync)
                        h = np.empty(3 * comm.world, np.uint64)
                        self._check(lib().wg_shard_slot_heads(self._ctx, ptr, stride, comm.world, h.ctypes.data))
                        return h.reshape(comm.world, 3)
        while not msg.done:
            nbytes = int(msg.bytes)
            if nbytes == abi.WG_SHARD_BYTES_ON_DEVICE:
                if pack is not None:
                    nbytes = 0   # the slot is written on the device, length included
                else:            # a host transport writes the slot header itself: it needs the length
                    n = ctypes.c_uint64(0)
                    self._check(lib().wg_shard_msg_bytes(self._ctx, ctypes.byref(n)))
                    nbytes = int(n.value)
            gathered, off, stride, sizes = comm.allgather(
                nbytes, lambda dst: self._check(lib().wg_shard_copy_msg(self._ctx, dst)), step=int(msg.step),
                pack=pack, read_heads=read_heads)
            self._gathered = gathered
            sz = (ctypes.c_uint64 * len(sizes))(*sizes)
            heads = getattr(comm, "heads", None)   # host copy of each message's 16-byte header, if the comm has it
            hp = heads.ctypes.data if heads is not None else None
            self._check(lib().wg_shard_exchange(self._ctx, gathered.data_ptr() + off, stride, sz, hp, ctypes.byref(msg)))
            del gathered

    def layout_summary(self) -> abi.LayoutSummary:
        s = abi.LayoutSummary()
        self._check(lib().wg_layout_summary_get(self._ctx, ctypes.byref(s)))
        return s

    def lanes(self):
        s = self.layout_summary()
        lane = np.empty(s.n_rows, np.uint32)
        color = np.empty(s.n_rows, np.uint8)
        self._check(lib().wg_copy_lanes(self._ctx, lane.ctypes.data, color.ctypes.data))
        return lane, color

    def edges(self) -> np.ndarray:
        s = self.layout_summary()
        e = np.empty(s.n_edges, abi.EDGE_DTYPE)
        if s.n_edges:
            self._check(lib().wg_copy_edges(self._ctx, e.ctypes.data))
        return e

    def row_heights(self) -> np.ndarray:
        s = self.layout_summary()
        h = np.empty(s.n_rows, np.float32)
        self._check(lib().wg_copy_row_heights(self._ctx, h.ctypes.data))
        return h

    # -- geometry ---------------------------------------------------------------------
    def row_geometry(self, band=None, device_ptr: int | None = None):
        """row_geometry_with_bands; band None -> build()'s default geometry."""
        if device_ptr is not None:
            self._check(lib().wg_row_geometry(self._ctx, device_ptr, abi.WG_DEVICE))
        elif band is None:
            self._check(lib().wg_row_geometry(self._ctx, None, abi.WG_HOST))
        else:
            b = np.ascontiguousarray(band, np.float32)
            self._band = b
            self._check(lib().wg_row_geometry(self._ctx, b.ctypes.data, abi.WG_HOST))

    def row_geometry_list(self, dag=None, band=None, commits: abi.Commits | None = None):
        """row_geometry_with_bands(commits, band_heights) with its commits
        argument (wg_row_geometry_list): heights from dag's times (or a
        prepared wg_commits, e.g. device-resident), geometry from the built
        edges; the list must have the built list's length."""
        c = abi.commits_struct(dag) if commits is None else commits
        self._keep_list = [dag, c]
        b = None
        if band is not None:
            b = np.ascontiguousarray(band, np.float32)
            self._band = b
        self._check(lib().wg_row_geometry_list(self._ctx, ctypes.byref(c), b.ctypes.data if b is not None else None,
                                                abi.WG_HOST))

    def geometry_summary(self) -> abi.GeometrySummary:
        s = abi.GeometrySummary()
        self._check(lib().wg_geometry_summary_get(self._ctx, ctypes.byref(s)))
        return s

    def geometry(self) -> dict:
        s = self.geometry_summary()
        n = s.n_rows
        g = dict(height=np.empty(n, np.float32), node_y=np.empty(n, np.float32),
                 row_top=np.empty(n + 1, np.float32), vert_off=np.empty(n + 1, np.uint32),
                 vert=np.empty(s.n_vert, np.uint32), curve_off=np.empty(n + 1, np.uint32),
                 curve=np.empty((s.n_curve, 8), np.float32), curve_color=np.empty(s.n_curve, np.uint8))
        d = abi.GeometryHost()
        for k, a in g.items():
            setattr(d, k, a.ctypes.data if a.size else None)
        self._check(lib().wg_copy_geometry(self._ctx, ctypes.byref(d)))
        return g

    # -- vertices ------------------------------------------------------------------------
    def emit_vertices(self, row_begin=0, row_end=None, selected=-1, palette=None):
        if row_end is None:
            ls = self.layout_summary()
            row_end = ls.row_begin + ls.n_rows
        pal = np.ascontiguousarray(abi.DEFAULT_PALETTE if palette is None else palette, np.float32)
        self._check(lib().wg_emit_vertices(self._ctx, row_begin, row_end, selected, pal.ctypes.data))

    def vertex_summary(self) -> abi.VertexSummary:
        s = abi.VertexSummary()
        self._check(lib().wg_vertex_summary_get(self._ctx, ctypes.byref(s)))
        return s

    def vertices(self, first=0, count=None) -> np.ndarray:
        s = self.vertex_summary()
        if count is None:
            count = s.n_vertices - first
        v = np.empty(count, abi.VERTEX_DTYPE)
        self._check(lib().wg_copy_vertices(self._ctx, first, count, v.ctypes.data if count else None))
        return v

    def vertex_offsets(self) -> np.ndarray:
        s = self.vertex_summary()
        o = np.empty(s.row_end - s.row_begin + 1, np.uint64)
        self._check(lib().wg_copy_vertex_offsets(self._ctx, o.ctypes.data))
        return o

    def device_views(self) -> abi.DeviceViews:
        v = abi.DeviceViews()
        self._check(lib().wg_device_views_get(self._ctx, ctypes.byref(v)))
        return v

    # -- SDF font atlas (WG-SDF-1) ----------------------------------------------------------
    def build_font_atlas(self, slot: int, ttf=None, width=1024, height=1024, em_px=96.0, spread=8, first=32, last=126):
        """Rasterise + EDT a TrueType font into atlas slot (0 regular, 1 bold)."""
        if ttf is None:
            ttf = FONTS[slot]
        if isinstance(ttf, str):   # a font file: read once per path and modification time
            key = (ttf, os.stat(ttf).st_mtime_ns)
            cache = self.__dict__.setdefault("_font_files", {})
            if key not in cache:
                data = open(ttf, "rb").read()
                cache[key] = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
            buf = cache[key]
        else:
            data = bytes(ttf)
            buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
        p = abi.AtlasParams(width, height, em_px, spread, first, last)
        self._check(lib().wg_font_atlas_build(self._ctx, slot, buf, len(buf), ctypes.byref(p)))

    def atlas_info(self, slot: int) -> abi.AtlasInfo:
        i = abi.AtlasInfo()
        self._check(lib().wg_font_atlas_info(self._ctx, slot, ctypes.byref(i)))
        return i

    def atlas(self, slot: int) -> dict:
        i = self.atlas_info(slot)
        shape = (i.height, i.width)
        out = dict(sdf=np.empty(shape, np.uint8), cov=np.empty(shape, np.uint8), d2in=np.empty(shape, np.uint16),
                   d2out=np.empty(shape, np.uint16), glyphs=np.empty(i.n_glyphs, abi.GLYPH_DTYPE))
        self._check(lib().wg_copy_font_atlas(self._ctx, slot, out["sdf"].ctypes.data, out["cov"].ctypes.data,
                                             out["d2in"].ctypes.data, out["d2out"].ctypes.data,
                                             out["glyphs"].ctypes.data))
        return out

    # -- glyph quads (WG-TEXT-1) --------------------------------------------------------------
    def emit_glyphs(self, row_begin=0, row_end=None, summaries=None, device=None, **params):
        """Text quads of rows [row_begin, row_end).  summaries: (bytes uint8
        array, offsets uint64 [N+1]) host arrays, or device=(ptr, off_ptr)."""
        if row_end is None:
            ls = self.layout_summary()
            row_end = ls.row_begin + ls.n_rows
        p = abi.text_params(**params)
        if device is not None:
            self._check(lib().wg_emit_glyphs(self._ctx, row_begin, row_end, device[0], device[1], abi.WG_DEVICE,
                                             ctypes.byref(p)))
        elif summaries is None:
            self._check(lib().wg_emit_glyphs(self._ctx, row_begin, row_end, None, None, abi.WG_HOST, ctypes.byref(p)))
        else:
            b = np.ascontiguousarray(summaries[0], np.uint8)
            o = np.ascontiguousarray(summaries[1], np.uint64)
            self._text_keep = (b, o)
            self._check(lib().wg_emit_glyphs(self._ctx, row_begin, row_end, b.ctypes.data if b.size else o.ctypes.data,
                                             o.ctypes.data, abi.WG_HOST, ctypes.byref(p)))

    # -- consumer adapter (screenshot_mode.rs:101-141; WG-RAST-1) ---------------------------
    def render(self, width, height, top_row=None, scale=1.0, graph_x=0.0, origin_y=0.0, clear=(0.09, 0.1, 0.12, 1.0),
               graph=True, text=True, device_ptr: int | None = None):
        """Rasterise the last emissions into RGBA8 [height, width, 4] (host),
        or into device memory at device_ptr (returns None)."""
        p = abi.RenderParams()
        p.width, p.height, p.scale, p.graph_x, p.origin_y = width, height, scale, graph_x, origin_y
        p.top_row = self.layout_summary().row_begin if top_row is None else top_row
        p.clear[:] = [float(x) for x in (list(clear) + [1.0])[:4]]
        p.layers = (abi.WG_RENDER_GRAPH if graph else 0) | (abi.WG_RENDER_TEXT if text else 0)
        if device_ptr is not None:
            self._check(lib().wg_render(self._ctx, ctypes.byref(p), device_ptr, abi.WG_DEVICE))
            return None
        img = np.empty((height, width, 4), np.uint8)
        self._check(lib().wg_render(self._ctx, ctypes.byref(p), img.ctypes.data, abi.WG_HOST))
        return img

    # -- row order (commit_graph_with_orphans git/mod.rs:761-775, insert_synthetics_sorted :234-242) ----
    def order_rows(self, walk_time, orphan_time=None, syn_time=None, device=None, out_device_ptr=None):
        """perm[final row] = source row (walk, then orphans, then synthetics).
        Host int64 arrays, or device=((walk_ptr, n), (orphan_ptr, n), (syn_ptr, n));
        out_device_ptr: write the permutation to device memory instead (returns None)."""
        if device is not None:
            (pw, nw), (po, no), (ps, ns) = device
            res = abi.WG_DEVICE
        else:
            arrs = [np.ascontiguousarray(np.zeros(0) if a is None else a, np.int64)
                    for a in (walk_time, orphan_time, syn_time)]
            self._order_keep = arrs
            (pw, po, ps), (nw, no, ns) = [a.ctypes.data if a.size else None for a in arrs], [a.size for a in arrs]
            res = abi.WG_HOST
        if out_device_ptr is not None:
            self._check(lib().wg_order_rows(self._ctx, pw, nw, po, no, ps, ns, res, out_device_ptr, abi.WG_DEVICE))
            return None
        perm = np.empty(max(1, nw + no + ns), np.uint32)
        self._check(lib().wg_order_rows(self._ctx, pw, nw, po, no, ps, ns, res, perm.ctypes.data, abi.WG_HOST))
        return perm[:nw + no + ns]

    # -- search-match flags (commit_matches_query, commit_graph.rs:1509-1523) -------------
    def match_rows(self, query, row_begin=0, row_end=None, summaries=None, authors=None, device=None) -> int:
        """history_view's match flags (:1320-1332) for rows [row_begin, row_end)
        of the built list; returns the match count.  summaries / authors:
        (bytes uint8, offsets uint64 [N+1]) host arrays, or device=((sum_ptr,
        sum_off_ptr), (auth_ptr, auth_off_ptr)) device pointers (None: empty).
        Later emissions dim the rows that do not match (empty query: none)."""
        if row_end is None:
            row_end = self._n_list()
        q = query.encode() if isinstance(query, str) else bytes(query)
        t = abi.RowText()
        keep = []
        if device is not None:
            t.residency = abi.WG_DEVICE
            (t.summary, t.summary_off), (t.author, t.author_off) = [(None, None) if f is None else f for f in device]
        else:
            t.residency = abi.WG_HOST
            for f, (bn, on) in ((summaries, ("summary", "summary_off")), (authors, ("author", "author_off"))):
                if f is None:
                    continue
                b = np.ascontiguousarray(f[0], np.uint8)
                o = np.ascontiguousarray(f[1], np.uint64)
                keep += [b, o]
                setattr(t, bn, b.ctypes.data if b.size else o.ctypes.data)
                setattr(t, on, o.ctypes.data)
        self._match_keep = keep
        qa = np.frombuffer(q, np.uint8) if q else np.zeros(1, np.uint8)
        cnt = ctypes.c_uint64()
        self._check(lib().wg_match_rows(self._ctx, qa.ctypes.data, len(q), row_begin, row_end, ctypes.byref(t),
                                        ctypes.byref(cnt)))
        self._match_rows = row_end - row_begin
        return int(cnt.value)

    def match_flags(self) -> np.ndarray:
        out = np.empty(getattr(self, "_match_rows", 0), np.uint8)
        self._check(lib().wg_copy_match_flags(self._ctx, out.ctypes.data if out.size else None))
        return out

    def _n_list(self) -> int:
        c = getattr(self, "_commits", None)
        return int(c.n_commits) if c is not None else self.layout_summary().n_rows

    def glyph_summary(self) -> abi.GlyphSummary:
        s = abi.GlyphSummary()
        self._check(lib().wg_glyph_summary_get(self._ctx, ctypes.byref(s)))
        return s

    def glyph_vertices(self, first=0, count=None) -> np.ndarray:
        s = self.glyph_summary()
        if count is None:
            count = s.n_vertices - first
        v = np.empty(count, abi.TEXT_VERTEX_DTYPE)
        self._check(lib().wg_copy_glyph_vertices(self._ctx, first, count, v.ctypes.data if count else None))
        return v

    def glyph_offsets(self) -> np.ndarray:
        s = self.glyph_summary()
        o = np.empty(s.row_end - s.row_begin + 1, np.uint64)
        self._check(lib().wg_copy_glyph_offsets(self._ctx, o.ctypes.data))
        return o

    # -- timing ----------------------------------------------------------------------------
    def debug_counters(self) -> np.ndarray:
        """wg_debug_counters: [3] replay iterations, [4] events, [5] shard mode,
        [6..8] speculative builds / lanes redone / geometry redone, [9] sharded
        blind replays, [10] serial pass, [11] sliced emissions, [12] the
        replay's form (100 + words chunked, 200 + words serial, 300 + words
        compacted), [13] leaked slots struck out, [14] its warm-up."""
        out = np.zeros(16, np.uint32)
        self._check(lib().wg_debug_counters(self._ctx, out.ctypes.data, 16))
        return out

    def enable_timing(self, on=True, reserve: int = 0):
        """Start (or stop) the per-stage HIP-event log; `reserve` pre-creates
        that many stage slots so none is created inside a timed region."""
        self._check(lib().wg_enable_timing(self._ctx, max(int(reserve), 1) if on else 0))

    def timings(self) -> list[tuple[str, float]]:
        n = ctypes.c_int()
        names = (ctypes.c_char_p * abi.WG_STAGE_MAX)()
        ms = (ctypes.c_float * abi.WG_STAGE_MAX)()
        self._check(lib().wg_stage_timings(self._ctx, ctypes.byref(n), names, ms))
        return [(names[i].decode(), float(ms[i])) for i in range(n.value)]


# ---------------------------------------------------------------------------
# Reference-shaped API (commit_graph.rs:162-507)
# ---------------------------------------------------------------------------
@dataclass
class CommitLayout:            # :162-166
    lane: int
    color: int                 # palette index (LANE_COLORS[lane % 6] or ORPHAN)


@dataclass
class GraphEdge:               # :173-180
    child_row: int
    child_lane: int
    parent_row: int
    parent_lane: int
    color: int


@dataclass
class CurveSegment:            # :186-193
    p0: tuple
    p1: tuple
    p2: tuple
    p3: tuple
    color: int


@dataclass
class RowGeometry:             # :208-233
    height: float
    full_verticals: list
    top_half_verticals: list
    bottom_half_verticals: list
    curves: list
    node_y: float


def commits_to_soa(commits):
    """[CommitInfo-like dicts: id(bytes20), time, parents(list[bytes20]), orphan] -> Dag."""
    from .synth import Dag
    n = len(commits)
    oid = np.zeros((n, 20), np.uint8)
    time = np.zeros(n, np.int64)
    poff = np.zeros(n + 1, np.uint32)
    flags = np.zeros(n, np.uint8)
    pl = []
    for i, c in enumerate(commits):
        oid[i] = np.frombuffer(bytes(c["id"]), np.uint8)
        time[i] = int(c["time"])
        flags[i] = (1 if c.get("orphan") else 0) | (2 if c.get("synthetic") else 0)
        pl.extend(bytes(p) for p in c["parents"])
        poff[i + 1] = len(pl)
    poid = np.frombuffer(b"".join(pl), np.uint8).reshape(-1, 20).copy() if pl else np.zeros((0, 20), np.uint8)
    return Dag(oid, time, poff, poid, flags, np.zeros(n, np.float32))


def geometry_rows(g: dict) -> list:
    """CSR geometry (wgraph.h layout) -> list[RowGeometry]."""
    rows = []
    n = len(g["height"])
    for r in range(n):
        full, top, bottom = [], [], []
        for v in g["vert"][g["vert_off"][r]:g["vert_off"][r + 1]]:
            v = int(v)
            entry = (v & 0xFFFFFF, (v >> 28) & 0xF)
            (full, top, bottom)[(v >> 24) & 3].append(entry)
        curves = []
        for k in range(int(g["curve_off"][r]), int(g["curve_off"][r + 1])):
            p = g["curve"][k]
            curves.append(CurveSegment((p[0], p[1]), (p[2], p[3]), (p[4], p[5]), (p[6], p[7]), int(g["curve_color"][k])))
        rows.append(RowGeometry(float(g["height"][r]), full, top, bottom, curves, float(g["node_y"][r])))
    return rows


class GraphLayout:
    """Drop-in for whisper-git's GraphLayout, backed by the HIP engine."""

    def __init__(self, engine: Engine | None = None):
        self.engine = engine or Engine()
        self._ids = {}
        self.max_lane = 0
        self.edges: list[GraphEdge] = []
        self.row_geometry: list[RowGeometry] = []
        self.graph_width = 0.0

    @classmethod
    def new(cls):
        return cls()

    def build(self, commits):
        dag = commits if hasattr(commits, "parent_off") else commits_to_soa(commits)
        self.engine.build(dag)
        s = self.engine.layout_summary()
        self.max_lane = int(s.max_lane)
        self.graph_width = float(s.graph_width)
        lane, color = self.engine.lanes()
        self._ids = {bytes(dag.oid[i]): CommitLayout(int(lane[i]), int(color[i])) for i in range(dag.n)}
        self.edges = [GraphEdge(*map(int, e)) for e in self.engine.edges()]
        self.row_geometry = geometry_rows(self.engine.geometry())

    def get(self, oid: bytes):
        return self._ids.get(bytes(oid))

    def row_geometry_with_bands(self, commits, band_heights):
        """Heights from `commits` (compute_row_heights(commits), :372), edges
        from the built layout; commits must have the built list's length."""
        dag = commits if hasattr(commits, "parent_off") else commits_to_soa(commits)
        band = np.zeros(dag.n, np.float32)
        m = min(dag.n, len(band_heights))
        band[:m] = np.asarray(band_heights[:m], np.float32)
        self.engine.row_geometry_list(dag, band)
        return geometry_rows(self.engine.geometry())


def compute_row_heights(commits) -> np.ndarray:
    """compute_row_heights (:486-507) on the engine."""
    dag = commits if hasattr(commits, "parent_off") else commits_to_soa(commits)
    t = np.ascontiguousarray(dag.time, np.int64)
    h = np.empty(len(t), np.float32)
    e = Engine()
    try:
        e._check(lib().wg_compute_row_heights(e._ctx, t.ctypes.data, len(t), abi.WG_HOST, h.ctypes.data))
        return h
    finally:
        e.close()
