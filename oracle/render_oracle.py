"""CPU oracle for the consumer adapter's rasteriser (WG-RAST-1) — TEST
INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's CPU baseline may import
this module; the engine never calls it.

The reference renders through aetna-vulkano (absent third-party code;
screenshot_mode.rs:101-141 only drives it), so WG-RAST-1 is a frozen spec
(whisper-git_amd/csrc/wg_render.hip header) and this is its
restatement in numpy float32, triangle by triangle in painter's order over
the pixels of each triangle's bounding box: parity unpinned against the
reference, pinned against this restatement (and, for the PNG container,
against PIL's decoder).
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def _edge(ax, ay, bx, by, px, py):
    return (bx - ax) * (py - ay) - (by - ay) * (px - ax)


def _owns(ax, ay, bx, by):
    return by < ay or (by == ay and bx > ax)


def render(width, height, row_top, top_row, scale=1.0, graph_x=0.0, origin_y=0.0, clear=(0.0, 0.0, 0.0),
           graph=None, text=None, sdf=None, k=0.0):
    """graph = (vertices f32 [n, 6] or VERTEX_DTYPE, per-row vertex offsets, row_begin);
    text = (vertices f32 [n, 8], per-row QUAD offsets, row_begin); row_top indexed by
    global row; sdf = the glyph atlas (u8 [H, W]); k = 2 * spread * text_px / em_px * scale.
    Returns RGBA8 [height, width, 4]."""
    scale, graph_x, origin_y, k = F32(scale), F32(graph_x), F32(origin_y), F32(k)
    img = np.empty((height, width, 3), F32)
    img[:] = np.array(clear[:3], F32)
    layers = []
    if graph is not None:
        v, off, rb = graph
        v = np.ascontiguousarray(v).view(F32).reshape(-1, 6)
        layers.append((0, v, np.asarray(off, np.int64), rb))
    if text is not None:
        v, off, rb = text
        v = np.ascontiguousarray(v).view(F32).reshape(-1, 8)
        layers.append((1, v, np.asarray(off, np.int64) * 6, rb))
    if not layers:
        return _quantize(img)
    lo = min(rb for _, _, _, rb in layers)
    hi = max(rb + len(off) - 1 for _, _, off, rb in layers)
    rt = np.asarray(row_top, F32)
    inv = F32(1.0) / F32(255.0)
    if sdf is not None:
        sdf_f = sdf.astype(F32) * inv
        ah, aw = sdf.shape
    for r in range(lo, hi):
        yr = F32(F32(rt[r] - rt[top_row]) + origin_y)
        for kind, v, off, rb in layers:
            if not rb <= r < rb + len(off) - 1:
                continue
            for t in range(int(off[r - rb]) // 3, int(off[r - rb + 1]) // 3):
                tv = v[3 * t:3 * t + 3]
                dx = graph_x if kind == 0 else F32(0.0)
                X = [F32(F32(tv[i, 0] + dx) * scale) for i in range(3)]
                Y = [F32(F32(tv[i, 1] + yr) * scale) for i in range(3)]
                U = [tv[i, 2] for i in range(3)] if kind == 1 else [F32(0)] * 3
                V = [tv[i, 3] for i in range(3)] if kind == 1 else [F32(0)] * 3
                col = tv[0, 2:6] if kind == 0 else tv[0, 4:8]
                area = F32(_edge(X[0], Y[0], X[1], Y[1], X[2], Y[2]))
                if area < 0:
                    X[1], X[2] = X[2], X[1]
                    Y[1], Y[2] = Y[2], Y[1]
                    U[1], U[2] = U[2], U[1]
                    V[1], V[2] = V[2], V[1]
                    area = F32(-area)
                if not area > 0:
                    continue
                minx, maxx, miny, maxy = min(X), max(X), min(Y), max(Y)
                x0 = max(0, int(np.floor(minx)) - 1)
                x1 = min(width, int(np.ceil(maxx)) + 1)
                y0 = max(0, int(np.floor(miny)) - 1)
                y1 = min(height, int(np.ceil(maxy)) + 1)
                if x0 >= x1 or y0 >= y1:
                    continue
                cx = np.arange(x0, x1).astype(F32) + F32(0.5)
                cy = np.arange(y0, y1).astype(F32) + F32(0.5)
                cx, cy = np.meshgrid(cx, cy)
                m = (cx >= minx) & (cx <= maxx) & (cy >= miny) & (cy <= maxy)
                w0 = _edge(X[1], Y[1], X[2], Y[2], cx, cy)
                w1 = _edge(X[2], Y[2], X[0], Y[0], cx, cy)
                w2 = _edge(X[0], Y[0], X[1], Y[1], cx, cy)
                m &= (w0 > 0) | ((w0 == 0) & _owns(X[1], Y[1], X[2], Y[2]))
                m &= (w1 > 0) | ((w1 == 0) & _owns(X[2], Y[2], X[0], Y[0]))
                m &= (w2 > 0) | ((w2 == 0) & _owns(X[0], Y[0], X[1], Y[1]))
                if not m.any():
                    continue
                sa = np.full(m.shape, col[3], F32)
                if kind == 1:
                    u = ((w0 * U[0] + w1 * U[1]) + w2 * U[2]) / area
                    vv = ((w0 * V[0] + w1 * V[1]) + w2 * V[2]) / area
                    fx = u * F32(aw) - F32(0.5)
                    fy = vv * F32(ah) - F32(0.5)
                    fx0, fy0 = np.floor(fx), np.floor(fy)
                    ax_, ay_ = fx - fx0, fy - fy0
                    ix = np.where(np.isfinite(fx0), fx0, 0).astype(np.int64)
                    iy = np.where(np.isfinite(fy0), fy0, 0).astype(np.int64)
                    xa, xb = np.clip(ix, 0, aw - 1), np.clip(ix + 1, 0, aw - 1)
                    ya, yb = np.clip(iy, 0, ah - 1), np.clip(iy + 1, 0, ah - 1)
                    s00, s10, s01, s11 = sdf_f[ya, xa], sdf_f[ya, xb], sdf_f[yb, xa], sdf_f[yb, xb]
                    top = s00 + (s10 - s00) * ax_
                    bot = s01 + (s11 - s01) * ax_
                    d = top + (bot - top) * ay_
                    al = np.clip((d - F32(0.5)) * k + F32(0.5), F32(0), F32(1))
                    sa = sa * al
                ia = F32(1.0) - sa
                blk = img[y0:y1, x0:x1]
                for ch in range(3):
                    blk[..., ch] = np.where(m, col[ch] * sa + blk[..., ch] * ia, blk[..., ch])
    return _quantize(img)


def _quantize(img):
    q = np.floor(np.clip(img, F32(0), F32(1)) * F32(255.0) + F32(0.5)).astype(np.uint8)
    out = np.full(img.shape[:2] + (4,), 255, np.uint8)
    out[..., :3] = q
    return out
