"""Second, independent CPU restatement of the commit-graph path (TEST ONLY).

TEST INFRASTRUCTURE: imported only by tests/ as a cross-check of the C
oracle (oracle/wg_oracle.c).  It transliterates
/root/reference/src/commit_graph.rs with Python containers that mirror the
Rust ones (dict for HashMap<Oid, _>, a list of Optional[bytes] for
`active_lanes: Vec<Option<Oid>>`) and numpy.float32 scalars for every f32
operation, so each rounding happens where Rust's does.  Pure-Python loops:
small inputs only (<= a few thousand rows).

Parity is "unpinned by reference fixtures" for lanes/edges/paths (the
reference has no tests for them); the two restatements must
agree bit for bit on every golden DAG (tests/test_oracle_crosscheck.py).
"""
from __future__ import annotations

import math
import struct

import numpy as np

F = np.float32

ROW_HEIGHT = F(28.0)          # commit_graph.rs:30
LANE_W = F(24.0)              # :33
LANE_COUNT_VISUAL = 6         # :37
NODE_Y = ROW_HEIGHT / F(2.0)  # :43
MAX_EXTRA_HEIGHT = ROW_HEIGHT  # :47
TIME_BASE_SECONDS = 7200.0    # :51
TIME_MAX_DELTA_SECONDS = 30.0 * 24.0 * 3600.0  # :54
LINE_WIDTH = F(2.0)           # :775
NODE_RADIUS = F(5.0)          # :778
SELECTED_RING_WIDTH = F(2.5)  # :780
ORPHAN = 6
FOREGROUND = 7


def rs_round(x: np.float32) -> np.float32:
    """Rust f32::round: half away from zero (numpy rounds half to even)."""
    x = F(x)
    if not np.isfinite(x):
        return x
    fl = F(math.floor(float(x)))
    diff = F(x - fl)  # exact for |x| < 2**23
    if abs(float(x)) >= 2.0 ** 23:
        return x
    if diff > F(0.5):
        return F(fl + F(1.0))
    if diff < F(0.5):
        return fl
    return F(fl + F(1.0)) if x > 0 else fl


def rs_clamp(x, lo, hi):
    x = F(x)
    if x < lo:
        x = F(lo)
    if x > hi:
        x = F(hi)
    return x


class Cubic:
    """Cubic (commit_graph.rs:614-695)."""

    def __init__(self, p0, p1, p2, p3):
        self.p = [(F(p0[0]), F(p0[1])), (F(p1[0]), F(p1[1])),
                  (F(p2[0]), F(p2[1])), (F(p3[0]), F(p3[1]))]

    def y_at(self, t):  # :623-629, left-to-right
        t = F(t)
        s = F(F(1.0) - t)
        a = F(F(F(s * s) * s) * self.p[0][1])
        b = F(F(F(F(F(3.0) * s) * s) * t) * self.p[1][1])
        c = F(F(F(F(F(3.0) * s) * t) * t) * self.p[2][1])
        d = F(F(F(t * t) * t) * self.p[3][1])
        return F(F(F(a + b) + c) + d)

    def t_at_y(self, target):  # :635-654
        target = F(target)
        if target <= self.p[0][1]:
            return F(0.0)
        if target >= self.p[3][1]:
            return F(1.0)
        lo, hi = F(0.0), F(1.0)
        for _ in range(40):
            mid = F(F(lo + hi) * F(0.5))
            if self.y_at(mid) < target:
                lo = mid
            else:
                hi = mid
        return F(F(lo + hi) * F(0.5))

    def split(self, t):  # :656-678
        t = F(t)

        def lerp(a, b):
            return (F(a[0] + F(F(b[0] - a[0]) * t)), F(a[1] + F(F(b[1] - a[1]) * t)))

        p0, p1, p2, p3 = self.p
        q01, q12, q23 = lerp(p0, p1), lerp(p1, p2), lerp(p2, p3)
        r012, r123 = lerp(q01, q12), lerp(q12, q23)
        s = lerp(r012, r123)
        return Cubic(p0, q01, r012, s), Cubic(s, r123, q23, p3)

    def subcurve(self, a, b):  # :683-694
        a, b = F(a), F(b)
        if a <= F(0.0) and b >= F(1.0):
            return self
        _, right = self.split(rs_clamp(a, 0.0, 1.0))
        if b >= F(1.0):
            return right
        new_t = rs_clamp(F(F(b - a) / F(F(1.0) - a)), 0.0, 1.0)
        left, _ = right.split(new_t)
        return left


def compute_row_heights(times):  # :486-507
    n = len(times)
    if n == 0:
        return []
    log_max = math.log(1.0 + TIME_MAX_DELTA_SECONDS / TIME_BASE_SECONDS)
    out = []
    for i in range(n):
        if i + 1 < n:
            delta = float(abs(int(times[i]) - int(times[i + 1])))
            clamped = min(delta, TIME_MAX_DELTA_SECONDS)
            ratio = math.log(1.0 + clamped / TIME_BASE_SECONDS) / log_max
            h = F(ROW_HEIGHT + F(MAX_EXTRA_HEIGHT * F(ratio)))
        else:
            h = ROW_HEIGHT
        out.append(rs_round(h))
    return out


class RowGeometry:  # :208-233
    def __init__(self, height=ROW_HEIGHT, node_y=NODE_Y):
        self.height = F(height)
        self.node_y = F(node_y)
        self.full, self.top, self.bottom, self.curves = [], [], [], []


def decompose_edge_into_rows(edge, row_top_y, rows):  # :525-608
    c, cl, p, pl, color = edge
    if c >= p:
        return
    if cl == pl:
        rows[c].bottom.append((cl, color))
        for r in range(c + 1, p):
            rows[r].full.append((cl, color))
        rows[p].top.append((cl, color))
        return
    child_y = F(row_top_y[c] + rows[c].node_y)
    parent_y = F(row_top_y[p] + rows[p].node_y)
    dy = F(parent_y - child_y)
    curve = Cubic((F(cl), child_y), (F(cl), F(child_y + F(dy * F(0.4)))),
                  (F(pl), F(parent_y - F(dy * F(0.4)))), (F(pl), parent_y))
    for row in range(c, p + 1):
        row_top = row_top_y[row]
        row_bot = row_top_y[row + 1]
        strip_top = child_y if row == c else row_top
        strip_bot = parent_y if row == p else row_bot
        if F(strip_bot - strip_top) < F(1e-4):
            continue
        t_a = F(0.0) if row == c else curve.t_at_y(strip_top)
        t_b = F(1.0) if row == p else curve.t_at_y(strip_bot)
        sub = curve.subcurve(t_a, t_b)
        seg = []
        for (x, y) in sub.p:
            seg += [F(x), F(y - row_top)]
        rows[row].curves.append((seg, color))


class GraphLayout:
    """GraphLayout (commit_graph.rs:240-472). commits: list of dicts with
    keys id (bytes), time (int), parents (list of bytes), orphan (bool)."""

    def __init__(self):
        self.layouts = {}
        self.active_lanes = []
        self.max_lane = 0
        self.edges = []
        self.row_geometry = []
        self.graph_width = F(0.0)

    def build(self, commits):  # :265-355
        self.layouts = {}
        self.active_lanes = []
        self.max_lane = 0
        self.edges = []
        commit_set = {c["id"]: None for c in commits}
        row_by_oid = {}
        for i, c in enumerate(commits):
            row_by_oid[c["id"]] = i
        for c in commits:
            lane = self._find_or_assign_lane(c["id"])
            color = ORPHAN if c.get("orphan") else lane % 6
            self.layouts[c["id"]] = (lane, color)
            for i in range(len(self.active_lanes)):
                if i != lane and self.active_lanes[i] == c["id"]:
                    self.active_lanes[i] = None
            self._update_lanes_for_parents(c, lane, commit_set)
            self._update_peak()
        for child_row, c in enumerate(commits):
            cl = self.layouts.get(c["id"])
            if cl is None:
                continue
            for pid in c["parents"]:
                if pid not in row_by_oid or pid not in self.layouts:
                    continue
                self.edges.append((child_row, cl[0], row_by_oid[pid], self.layouts[pid][0], cl[1]))
        heights = compute_row_heights([c["time"] for c in commits])
        row_top_y = []
        acc = F(0.0)
        for h in heights:
            row_top_y.append(acc)
            acc = F(acc + h)
        row_top_y.append(acc)
        self.row_geometry = [RowGeometry(height=h) for h in heights]
        for e in self.edges:
            decompose_edge_into_rows(e, row_top_y, self.row_geometry)
        self.row_top_y = row_top_y
        visible = min(self.max_lane + 1, LANE_COUNT_VISUAL)
        self.graph_width = max(F(F(visible) * LANE_W), LANE_W)

    def get(self, oid):
        return self.layouts.get(oid)

    def row_geometry_with_bands(self, commits, band_heights):  # :367-399
        heights = compute_row_heights([c["time"] for c in commits])
        row_top_y = []
        acc = F(0.0)
        for i, h in enumerate(heights):
            band = F(band_heights[i]) if i < len(band_heights) else F(0.0)
            row_top_y.append(acc)
            acc = F(acc + F(h + band))
        row_top_y.append(acc)
        geom = []
        for i, h in enumerate(heights):
            band = F(band_heights[i]) if i < len(band_heights) else F(0.0)
            geom.append(RowGeometry(height=rs_round(F(h + band)), node_y=rs_round(F(band + NODE_Y))))
        for e in self.edges:
            decompose_edge_into_rows(e, row_top_y, geom)
        return geom, row_top_y

    def _find_or_assign_lane(self, oid):  # :401-412
        for lane, occ in enumerate(self.active_lanes):
            if occ == oid:
                return lane
        lane = self._lowest_free_lane()
        while len(self.active_lanes) <= lane:
            self.active_lanes.append(None)
        return lane

    def _lowest_free_lane(self):  # :414-423
        for lane, occ in enumerate(self.active_lanes):
            if occ is None:
                return lane
        self.active_lanes.append(None)
        return len(self.active_lanes) - 1

    def _update_lanes_for_parents(self, c, commit_lane, commit_set):  # :425-460
        while len(self.active_lanes) <= commit_lane:
            self.active_lanes.append(None)
        parents = c["parents"]
        if not parents:
            self.active_lanes[commit_lane] = None
            return
        fp = parents[0]
        self.active_lanes[commit_lane] = fp if fp in commit_set else None
        for pid in parents[1:]:
            if pid not in commit_set:
                continue
            if pid in self.active_lanes:
                continue
            lane = self._lowest_free_lane()
            while len(self.active_lanes) <= lane:
                self.active_lanes.append(None)
            self.active_lanes[lane] = pid

    def _update_peak(self):  # :462-471
        for i in range(len(self.active_lanes) - 1, -1, -1):
            if self.active_lanes[i] is not None:
                if i > self.max_lane:
                    self.max_lane = i
                return


def flatten_geometry(geom, row_top_y):
    """RowGeometry list -> the CSR layout of include/wgraph.h."""
    n = len(geom)
    height = np.array([g.height for g in geom], dtype=np.float32)
    node_y = np.array([g.node_y for g in geom], dtype=np.float32)
    vert_off, vert, curve_off, curve, curve_color = [0], [], [0], [], []
    for g in geom:
        for kind, lst in ((0, g.full), (1, g.top), (2, g.bottom)):
            for lane, color in lst:
                vert.append(lane | (kind << 24) | (color << 28))
        vert_off.append(len(vert))
        for seg, color in g.curves:
            curve.append(seg)
            curve_color.append(color)
        curve_off.append(len(curve))
    return dict(
        height=height, node_y=node_y,
        row_top=np.array(row_top_y, dtype=np.float32).reshape(n + 1),
        vert_off=np.array(vert_off, dtype=np.uint32), vert=np.array(vert, dtype=np.uint32),
        curve_off=np.array(curve_off, dtype=np.uint32),
        curve=np.array(curve, dtype=np.float32).reshape(-1, 8),
        curve_color=np.array(curve_color, dtype=np.uint8))


def commits_from_soa(oid, time, parent_off, parent_oid, flags):
    """wg_commits SoA -> list of commit dicts."""
    n = len(time)
    out = []
    for i in range(n):
        ps = [bytes(parent_oid[k]) for k in range(parent_off[i], parent_off[i + 1])]
        out.append(dict(id=bytes(oid[i]), time=int(time[i]), parents=ps,
                        orphan=bool(flags[i] & 1) if flags is not None else False))
    return out


# --- WG-TESS-1, independent of wg_oracle.c --------------------
def _hexf(s):
    return F(float.fromhex(s))


_C15, _C30, _C45, _S15 = (_hexf("0x1.ee8dd4p-1"), _hexf("0x1.bb67aep-1"),
                         _hexf("0x1.6a09e6p-1"), _hexf("0x1.0907dcp-2"))
_H = F(0.5)
UC_COS = [F(1), _C15, _C30, _C45, _H, _S15, F(0), -_S15, -_H, -_C45, -_C30, -_C15, F(-1),
          -_C15, -_C30, -_C45, -_H, -_S15, F(0), _S15, _H, _C45, _C30, _C15, F(1)]
UC_SIN = [F(0), _S15, _H, _C45, _C30, _C15, F(1), _C15, _C30, _C45, _H, _S15, F(0),
          -_S15, -_H, -_C45, -_C30, -_C15, F(-1), -_C15, -_C30, -_C45, -_H, -_S15, F(0)]


def _visible_lanes(gw):
    q = rs_round(F(F(gw) / LANE_W))
    return max(int(q), 1)


def lane_center_x(lane, gw):  # :786-790
    vis = _visible_lanes(gw)
    return F(F(F(min(lane, vis - 1)) * LANE_W) + F(LANE_W * F(0.5)))


def emit_row_vertices(geom_row, node_lane, node_color, selected, gw, palette):
    """graph_cell (:803-908) tessellated per WG-TESS-1 -> list of 6-float tuples."""
    out = []
    hw = F(LINE_WIDTH * F(0.5))
    pal = [tuple(F(v) for v in palette[k]) for k in range(8)]
    h, ny = geom_row.height, geom_row.node_y

    def vert(x, y0, y1, col):
        xl, xr = F(x - hw), F(x + hw)
        for (a, b) in ((xl, y0), (xr, y0), (xl, y1), (xr, y0), (xr, y1), (xl, y1)):
            out.append((a, b) + pal[col])

    for kind, lst in ((0, geom_row.full), (1, geom_row.top), (2, geom_row.bottom)):
        for lane, col in lst:
            x = lane_center_x(lane, gw)
            if kind == 0:
                vert(x, F(0.0), h, col)
            elif kind == 1:
                vert(x, F(0.0), ny, col)
            else:
                vert(x, ny, h, col)
    vis = _visible_lanes(gw)
    for seg, col in geom_row.curves:
        X = [F(F(rs_clamp(seg[2 * q], 0.0, F(vis - 1)) * LANE_W) + F(LANE_W * F(0.5))) for q in range(4)]
        Y = [F(seg[2 * q + 1]) for q in range(4)]
        L, R = [], []
        for j in range(17):
            t = F(F(j) * F(0.0625))
            s = F(F(1.0) - t)
            w0 = F(F(s * s) * s)
            w1 = F(F(F(F(3.0) * s) * s) * t)
            w2 = F(F(F(F(3.0) * s) * t) * t)
            w3 = F(F(t * t) * t)
            px = F(F(F(F(w0 * X[0]) + F(w1 * X[1])) + F(w2 * X[2])) + F(w3 * X[3]))
            py = F(F(F(F(w0 * Y[0]) + F(w1 * Y[1])) + F(w2 * Y[2])) + F(w3 * Y[3]))
            d0 = F(F(F(3.0) * s) * s)
            d1 = F(F(F(6.0) * s) * t)
            d2 = F(F(F(3.0) * t) * t)
            dx = F(F(F(d0 * F(X[1] - X[0])) + F(d1 * F(X[2] - X[1]))) + F(d2 * F(X[3] - X[2])))
            dy = F(F(F(d0 * F(Y[1] - Y[0])) + F(d1 * F(Y[2] - Y[1]))) + F(d2 * F(Y[3] - Y[2])))
            ln = F(np.sqrt(F(F(dx * dx) + F(dy * dy))))
            if ln > F(0.0):
                nx, nyy = F(-dy / ln), F(dx / ln)
            else:
                nx, nyy = F(1.0), F(0.0)
            L.append((F(px + F(hw * nx)), F(py + F(hw * nyy))))
            R.append((F(px - F(hw * nx)), F(py - F(hw * nyy))))
        for j in range(16):
            for p in (L[j], R[j], L[j + 1], R[j], R[j + 1], L[j + 1]):
                out.append(p + pal[col])
    cx = lane_center_x(node_lane, gw)
    r = NODE_RADIUS
    for j in range(24):
        out.append((cx, ny) + pal[node_color])
        out.append((F(cx + F(r * UC_COS[j])), F(ny + F(r * UC_SIN[j]))) + pal[node_color])
        out.append((F(cx + F(r * UC_COS[j + 1])), F(ny + F(r * UC_SIN[j + 1]))) + pal[node_color])
    if selected:
        ri = F(NODE_RADIUS - F(SELECTED_RING_WIDTH * F(0.5)))
        ro = F(NODE_RADIUS + F(SELECTED_RING_WIDTH * F(0.5)))
        for j in range(24):
            o0 = (F(cx + F(ro * UC_COS[j])), F(ny + F(ro * UC_SIN[j])))
            i0 = (F(cx + F(ri * UC_COS[j])), F(ny + F(ri * UC_SIN[j])))
            o1 = (F(cx + F(ro * UC_COS[j + 1])), F(ny + F(ro * UC_SIN[j + 1])))
            i1 = (F(cx + F(ri * UC_COS[j + 1])), F(ny + F(ri * UC_SIN[j + 1])))
            for p in (o0, i0, o1, i0, i1, o1):
                out.append(p + pal[FOREGROUND])
    return out


def f32_bits(x):
    return struct.unpack("<I", struct.pack("<f", float(x)))[0]
