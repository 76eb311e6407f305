"""CPU restatement of the SDF font atlas, frozen spec WG-SDF-1.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline, never by the product path.

The reference's legacy atlas builder (fontdue + "custom EDT",
docs/render_engine.md:105-112) is absent from the snapshot and fontdue is
not vendored, so parity with it is UNPINNED.  This restatement pins what can
be pinned:
  * the outline parse is independent of the engine's (fontTools instead of
    wg_font.hip's TrueType reader), so the two cross-check each other;
  * the distance transform is checked against scipy.ndimage's exact EDT
    (tests/test_font_oracle.py; min(d^2, far) agreement on every pixel);
  * the coverage is sanity-checked against FreeType (PIL) rendering of the
    same glyphs (tolerance, different rasterisers).
Every f32 operation follows wg_font.hip in order (numpy float32 ops are
IEEE, no fused multiply-add), so the engine must match byte for byte.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32
QUAD_STEPS = 8
OFFS = np.array([0.125, 0.375, 0.625, 0.875], F32)


def _flatten(pts, on, scale):
    """One closed TrueType contour -> list of (x0, y0, x1, y1) f32 lines, y up."""
    n = len(pts)
    if n < 2:
        return []
    pts = [(F32(x), F32(y)) for x, y in pts]
    s = next((i for i in range(n) if on[i]), n)
    if s == n:
        start = (F32((pts[0][0] + pts[1][0]) * F32(0.5)), F32((pts[0][1] + pts[1][1]) * F32(0.5)))
        order = [(1 + m) % n for m in range(n)]
    else:
        start = pts[s]
        order = [(s + 1 + m) % n for m in range(n - 1)]
    out = [start]
    cur, ctrl = start, None

    def quad(p0, c, p1):
        for k in range(1, QUAD_STEPS + 1):
            t = F32(k) * F32(1.0 / QUAD_STEPS)
            mt = F32(1.0) - t
            a, b, d = mt * mt, F32(2.0) * mt * t, t * t
            out.append((a * p0[0] + b * c[0] + d * p1[0], a * p0[1] + b * c[1] + d * p1[1]))

    for i in order:
        p = pts[i]
        if on[i]:
            if ctrl is not None:
                quad(cur, ctrl, p)
                ctrl = None
            else:
                out.append(p)
            cur = p
        else:
            if ctrl is not None:
                mid = (F32((ctrl[0] + p[0]) * F32(0.5)), F32((ctrl[1] + p[1]) * F32(0.5)))
                quad(cur, ctrl, mid)
                cur = mid
            ctrl = p
    if ctrl is not None:
        quad(cur, ctrl, start)
    else:
        out.append(start)
    lines = []
    for (xa, ya), (xb, yb) in zip(out[:-1], out[1:]):
        x0, y0, x1, y1 = xa * scale, ya * scale, xb * scale, yb * scale
        if y0 != y1:
            lines.append((x0, y0, x1, y1))
    return lines


def glyph_lines(font, glyph_name, scale):
    glyf = font["glyf"]
    g = glyf[glyph_name]
    if g.numberOfContours == 0:
        return []
    coords, ends, flags = g.getCoordinates(glyf)
    lines, a = [], 0
    for e in ends:
        pts = [tuple(int(v) for v in coords[i]) for i in range(a, e + 1)]
        on = [bool(flags[i] & 1) for i in range(a, e + 1)]
        lines += _flatten(pts, on, scale)
        a = e + 1
    return lines


def coverage(lines, bx0, by1, cw, ch, spread):
    """4x4-sample non-zero-winding coverage (0..16) of a glyph cell."""
    ci = np.arange(cw, dtype=np.int32) - spread
    cj = np.arange(ch, dtype=np.int32) - spread
    px = (bx0 + ci).astype(F32)                      # pixel left edge
    py = (by1 - cj).astype(F32)                      # pixel top edge (y up)
    X = (px[None, :, None] + OFFS[None, None, :]).astype(F32)            # (1, cw, 4)
    Y = (py[:, None] - OFFS[None, :]).astype(F32)                         # (ch, 4)
    wind = np.zeros((ch, 4, cw, 4), np.int32)
    for (x0, y0, x1, y1) in lines:
        up = y0 < y1
        ylo, yhi = (y0, y1) if up else (y1, y0)
        m = (ylo <= Y) & (Y < yhi)                                        # (ch, 4)
        rows = np.nonzero(m.any(axis=1))[0]
        if rows.size == 0:
            continue
        Yr, mr = Y[rows], m[rows]
        t = ((Yr - y0) / (y1 - y0)).astype(F32)
        xi = (x0 + t * (x1 - x0)).astype(F32)                             # (r, 4)
        hit = (xi[:, :, None, None] > X.reshape(1, 1, cw, 4)) & mr[:, :, None, None]
        wind[rows] += np.where(hit, 1 if up else -1, 0).astype(np.int32)
    return (wind != 0).sum(axis=(1, 3)).astype(np.uint8)


def build_atlas(ttf_path, width=1024, height=1024, em_px=80.0, spread=8, first=32, last=126):
    """WG-SDF-1 atlas: dict(cov, sdf, d2in, d2out, glyphs, far_d2, ...)."""
    from fontTools.ttLib import TTFont
    font = TTFont(ttf_path)
    upem = font["head"].unitsPerEm
    scale = F32(F32(em_px) / F32(upem))
    cmap, hmtx, glyf = font.getBestCmap(), font["hmtx"], font["glyf"]
    cov = np.zeros((height, width), np.uint8)
    glyphs = []
    cx = cy = row_h = 0
    for ch in range(first, last + 1):
        name = cmap.get(ch, ".notdef")
        adv = F32(F32(hmtx[name][0]) * scale)
        g = glyf[name]
        rec = dict(codepoint=ch, advance=adv, bearing_x=0, bearing_top=0, w=0, h=0, atlas_x=0, atlas_y=0)
        if g.numberOfContours != 0:
            bx0 = int(np.floor(F32(g.xMin) * scale)); bx1 = int(np.ceil(F32(g.xMax) * scale))
            by0 = int(np.floor(F32(g.yMin) * scale)); by1 = int(np.ceil(F32(g.yMax) * scale))
            w, h = bx1 - bx0, by1 - by0
            cw, chh = w + 2 * spread, h + 2 * spread
            if cx + cw > width:
                cx, cy, row_h = 0, cy + row_h, 0
            if cw > width or cy + chh > height:
                raise ValueError("atlas too small")
            c = coverage(glyph_lines(font, name, scale), bx0, by1, cw, chh, spread)
            cov[cy:cy + chh, cx:cx + cw] = c
            rec.update(bearing_x=bx0, bearing_top=by1, w=w, h=h, atlas_x=cx, atlas_y=cy)
            cx += cw
            row_h = max(row_h, chh)
        glyphs.append(rec)
    d2in, d2out, sdf, far = edt_sdf(cov, spread)
    return dict(cov=cov, sdf=sdf, d2in=d2in, d2out=d2out, glyphs=glyphs, far_d2=far, ascent=F32(font["hhea"].ascent) * scale,
                descent=F32(font["hhea"].descent) * scale)


def _col_dist(mask, far):
    """Per pixel: rows to the nearest True pixel in its column (capped at far)."""
    H, W = mask.shape
    down = np.empty((H, W), np.int32)
    d = np.full(W, far, np.int32)
    for y in range(H):
        d = np.where(mask[y], 0, np.minimum(d + 1, far))
        down[y] = d
    d = np.full(W, far, np.int32)
    for y in range(H - 1, -1, -1):
        d = np.where(mask[y], 0, np.minimum(d + 1, far))
        down[y] = np.minimum(down[y], d)
    return down


def edt_sdf(cov, spread):
    """Two-pass bounded EDT (R = 4 * spread) + SDF bytes, as wg_font.hip."""
    R = 4 * spread
    far = R + 1
    inside = cov >= 8
    gin = _col_dist(~inside, far).astype(np.int64) ** 2     # inside pixels: to the nearest outside pixel
    gout = _col_dist(inside, far).astype(np.int64) ** 2
    cap = far * far
    H, W = cov.shape

    def rows(g):
        best = g.copy()
        for o in range(1, R + 1):
            left = np.full_like(g, np.iinfo(np.int64).max)
            right = np.full_like(g, np.iinfo(np.int64).max)
            left[:, o:] = g[:, :-o] + o * o
            right[:, :-o] = g[:, o:] + o * o
            best = np.minimum(best, np.minimum(left, right))
        return np.minimum(best, cap)

    a, b = rows(gin), rows(gout)
    signed = np.sqrt(b.astype(F32)) - np.sqrt(a.astype(F32))
    k = F32(F32(127.5) / F32(spread))
    v = (F32(127.5) - signed.astype(F32) * k).astype(F32)
    v = np.clip(v, F32(0.0), F32(255.0))
    sdf = np.floor(v + F32(0.5)).astype(np.uint8)
    return a.astype(np.uint16), b.astype(np.uint16), sdf, cap
