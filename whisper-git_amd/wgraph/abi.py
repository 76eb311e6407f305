"""ctypes mirror of include/wgraph.h (types and constants only)."""
from __future__ import annotations

import ctypes

import numpy as np

WG_OK, WG_E_INVALID, WG_E_HIP, WG_E_NOMEM, WG_E_STATE, WG_E_UNSUPPORTED, WG_E_NODEVICE = 0, -1, -2, -3, -4, -5, -6
WG_HOST, WG_DEVICE = 0, 1
WG_FLAG_ORPHAN, WG_FLAG_SYNTHETIC = 0x1, 0x2
WG_VERT_FULL, WG_VERT_TOP, WG_VERT_BOTTOM = 0, 1, 2
WG_COLOR_ORPHAN, WG_COLOR_FOREGROUND, WG_PALETTE_SIZE = 6, 7, 8
WG_STAGE_MAX = 1024
VTX_PER_VERTICAL, VTX_PER_CURVE, VTX_PER_NODE, VTX_PER_RING = 6, 96, 72, 144

ERRORS = {WG_E_INVALID: "WG_E_INVALID", WG_E_HIP: "WG_E_HIP", WG_E_NOMEM: "WG_E_NOMEM",
          WG_E_STATE: "WG_E_STATE", WG_E_UNSUPPORTED: "WG_E_UNSUPPORTED", WG_E_NODEVICE: "WG_E_NODEVICE"}


class Commits(ctypes.Structure):
    _fields_ = [("n_commits", ctypes.c_uint64), ("n_parents", ctypes.c_uint64),
                ("oid", ctypes.c_void_p), ("time", ctypes.c_void_p),
                ("parent_off", ctypes.c_void_p), ("parent_oid", ctypes.c_void_p),
                ("flags", ctypes.c_void_p), ("residency", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class Edge(ctypes.Structure):
    _fields_ = [("child_row", ctypes.c_uint32), ("child_lane", ctypes.c_uint32),
                ("parent_row", ctypes.c_uint32), ("parent_lane", ctypes.c_uint32),
                ("color", ctypes.c_uint32)]


class LayoutSummary(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_uint64), ("n_edges", ctypes.c_uint64),
                ("max_lane", ctypes.c_uint32), ("n_slots", ctypes.c_uint32),
                ("graph_width", ctypes.c_float), ("lane_path", ctypes.c_uint32),
                ("row_begin", ctypes.c_uint64)]


class AtlasParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("em_px", ctypes.c_float),
                ("spread", ctypes.c_uint32), ("first_char", ctypes.c_uint32), ("last_char", ctypes.c_uint32)]


class AtlasInfo(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("spread", ctypes.c_uint32),
                ("n_glyphs", ctypes.c_uint32), ("n_edges", ctypes.c_uint32), ("far_d2", ctypes.c_uint32),
                ("em_px", ctypes.c_float), ("ascent", ctypes.c_float), ("descent", ctypes.c_float),
                ("line_gap", ctypes.c_float), ("first_char", ctypes.c_uint32)]


GLYPH_DTYPE = np.dtype([("codepoint", "<u4"), ("advance", "<f4"), ("bearing_x", "<i4"), ("bearing_top", "<i4"),
                        ("w", "<u4"), ("h", "<u4"), ("atlas_x", "<u4"), ("atlas_y", "<u4")])
# WG-SDF-1 defaults: Roboto at 96 px/em (48 px text at 2x oversampling), 8 px spread, ASCII 32..126
ATLAS_DEFAULTS = dict(width=1024, height=1024, em_px=96.0, spread=8, first=32, last=126)


class TextParams(ctypes.Structure):
    _fields_ = [("slot", ctypes.c_int32), ("text_px", ctypes.c_float), ("sha_x", ctypes.c_float),
                ("summary_x", ctypes.c_float), ("summary_max_x", ctypes.c_float), ("time_right_x", ctypes.c_float),
                ("baseline_dy", ctypes.c_float), ("now", ctypes.c_int64), ("color_sha", ctypes.c_float * 4),
                ("color_summary", ctypes.c_float * 4), ("color_time", ctypes.c_float * 4)]


class GlyphSummary(ctypes.Structure):
    _fields_ = [("row_begin", ctypes.c_uint64), ("row_end", ctypes.c_uint64), ("n_quads", ctypes.c_uint64),
                ("n_vertices", ctypes.c_uint64), ("checksum", ctypes.c_uint64)]


TEXT_VERTEX_DTYPE = np.dtype([(k, "<f4") for k in ("x", "y", "u", "v", "r", "g", "b", "a")])
# WG-TEXT-1 default columns (pixels, row-local; the graph column is 6 lanes x 24 px wide)
TEXT_DEFAULTS = dict(slot=0, text_px=13.0, sha_x=152.0, summary_x=214.0, summary_max_x=900.0, time_right_x=980.0,
                     baseline_dy=4.5, now=1_704_067_200,   # 2024-01-01T00:00:00Z, where synthetic histories start
                     color_sha=(0.55, 0.58, 0.62, 1.0), color_summary=(0.9, 0.91, 0.93, 1.0),
                     color_time=(0.55, 0.58, 0.62, 1.0))


def text_params(**kw) -> TextParams:
    d = dict(TEXT_DEFAULTS, **kw)
    p = TextParams()
    for k, v in d.items():
        if k.startswith("color_"):
            getattr(p, k)[:] = [float(x) for x in v]
        else:
            setattr(p, k, v)
    return p


class RowText(ctypes.Structure):
    _fields_ = [("summary", ctypes.c_void_p), ("summary_off", ctypes.c_void_p), ("author", ctypes.c_void_p),
                ("author_off", ctypes.c_void_p), ("residency", ctypes.c_int32), ("reserved", ctypes.c_int32)]


WG_DIM_ALPHA = 0.3
WG_RENDER_GRAPH, WG_RENDER_TEXT = 1, 2


class RenderParams(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("scale", ctypes.c_float),
                ("graph_x", ctypes.c_float), ("origin_y", ctypes.c_float), ("top_row", ctypes.c_uint64),
                ("clear", ctypes.c_float * 4), ("layers", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


WG_SHARD_BYTES_ON_DEVICE = 2 ** 64 - 1   # wg_shard_msg.bytes: the length is written by the engine's kernels


class ShardMsg(ctypes.Structure):
    _fields_ = [("send", ctypes.c_void_p), ("bytes", ctypes.c_uint64), ("done", ctypes.c_int32),
                ("step", ctypes.c_int32)]


class GeometrySummary(ctypes.Structure):
    _fields_ = [("n_rows", ctypes.c_uint64), ("n_vert", ctypes.c_uint64),
                ("n_curve", ctypes.c_uint64), ("total_height", ctypes.c_float),
                ("scan_path", ctypes.c_uint32)]


class GeometryHost(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("height", "node_y", "row_top", "vert_off", "vert", "curve_off", "curve", "curve_color")]


class VertexSummary(ctypes.Structure):
    _fields_ = [("row_begin", ctypes.c_uint64), ("row_end", ctypes.c_uint64),
                ("n_vertices", ctypes.c_uint64), ("checksum", ctypes.c_uint64)]


class DeviceViews(ctypes.Structure):
    _fields_ = [(k, ctypes.c_void_p) for k in
                ("lane", "color", "edges", "height", "node_y", "row_top", "vert_off", "vert",
                 "curve_off", "curve", "curve_color", "vtx_off", "vertices")]


EDGE_DTYPE = np.dtype([("child_row", "<u4"), ("child_lane", "<u4"), ("parent_row", "<u4"),
                       ("parent_lane", "<u4"), ("color", "<u4")])
VERTEX_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("r", "<f4"), ("g", "<f4"), ("b", "<f4"), ("a", "<f4")])

# Default palette (RGBA): stands in for the aetna theme tokens the reference
# resolves at paint time (commit_graph.rs:59-70; tokens are theme-dependent).
DEFAULT_PALETTE = np.array([
    [0.231, 0.510, 0.965, 1.0],   # PRIMARY
    [0.133, 0.773, 0.369, 1.0],   # SUCCESS
    [0.961, 0.620, 0.043, 1.0],   # WARNING
    [0.024, 0.714, 0.831, 1.0],   # INFO
    [0.937, 0.267, 0.267, 1.0],   # DESTRUCTIVE
    [0.898, 0.906, 0.922, 1.0],   # FOREGROUND (lane 5)
    [0.612, 0.639, 0.686, 1.0],   # MUTED_FOREGROUND (orphan)
    [0.898, 0.906, 0.922, 1.0],   # FOREGROUND (selected ring)
], dtype=np.float32)


def commits_struct(dag, residency=WG_HOST) -> Commits:
    """Host Dag (wgraph.synth.Dag) -> wg_commits; arrays must stay alive."""
    c = Commits()
    c.n_commits = dag.n
    c.n_parents = dag.e
    c.oid = dag.oid.ctypes.data
    c.time = dag.time.ctypes.data
    c.parent_off = dag.parent_off.ctypes.data
    c.parent_oid = dag.parent_oid.ctypes.data if dag.e else dag.oid.ctypes.data
    c.flags = dag.flags.ctypes.data
    c.residency = residency
    return c
