"""CPU restatement of the glyph quads, frozen spec WG-TEXT-1.

TEST INFRASTRUCTURE ONLY (tests/, smoke, bench cpu_baseline).

Follows the reference's row text: short SHA = first 7 hex digits of the id
(git/mod.rs:300), summary or "(no summary)" (commit_graph.rs:1003-1007),
format_relative_time (git/mod.rs:34-49) with `now` as an input.  The legacy
quad layout (TextRenderer::layout_text, docs/render_engine.md:113-131) is
absent from the snapshot: parity with it is UNPINNED; the relative-time
strings are pinned by the reference's thresholds (tests/test_text_oracle.py).
f32 operations in wg_text.hip's order.
"""
from __future__ import annotations

import numpy as np

F32 = np.float32


def relative_time(now: int, t: int) -> bytes:
    """git/mod.rs:34-49 (format_relative_time), `now` explicit."""
    d = max(now - t, 0)
    if d < 60:
        return b"just now"
    if d < 3600:
        return b"%dm" % (d // 60)
    if d < 86400:
        return b"%dh" % (d // 3600)
    if d < 604800:
        return b"%dd" % (d // 86400)
    if d < 2592000:
        return b"%dw" % (d // 604800)
    if d < 31536000:
        return b"%dmo" % (d // 2592000)
    return b"%dy" % (d // 31536000)


def short_id(oid_row: np.ndarray) -> bytes:
    return bytes(oid_row[:4]).hex()[:7].encode()


def emit_glyphs(dag, node_y, glyphs, atlas_w, atlas_h, spread, em_px, rb, re, summaries=None, match=None, match_rb=0,
                **params):
    """-> (TextVertex f32 array (6 per quad, 8 floats each), per-row quad offsets).
    match: search-match flags of rows [match_rb, ...): rows flagged 0 at
    opacity 0.3 (commit_graph.rs:1467, 1482; alpha * 0.3f)."""
    from wgraph import abi
    p = dict(abi.TEXT_DEFAULTS, **params)
    first = int(glyphs[0]["codepoint"])
    scale = F32(F32(p["text_px"]) / F32(em_px))
    adv = [F32(g["advance"]) for g in glyphs]
    col = [np.array(p[k], F32) for k in ("color_sha", "color_summary", "color_time")]
    inv_w, inv_h = F32(F32(1.0) / F32(atlas_w)), F32(F32(1.0) / F32(atlas_h))
    sp = F32(spread)

    def gid(b):
        g = b - first
        return g if 0 <= g < len(glyphs) else ord("?") - first

    quads, offs = [], [0]
    for r in range(rb, re):
        base = F32(F32(node_y[r]) + F32(p["baseline_dy"]))
        sha = b"" if (dag.flags[r] & abi.WG_FLAG_SYNTHETIC) else short_id(dag.oid[r])
        s = b""
        if summaries is not None:
            s = bytes(summaries[0][int(summaries[1][r]):int(summaries[1][r + 1])])
        if not s:
            s = b"(no summary)"
        tm = relative_time(int(p["now"]), int(dag.time[r]))
        w = F32(0.0)
        for b in tm:
            w = F32(w + adv[gid(b)] * scale)
        runs = ((sha, F32(p["sha_x"]), F32(3.0e38), 0), (s, F32(p["summary_x"]), F32(p["summary_max_x"]), 1),
                (tm, F32(F32(p["time_right_x"]) - w), F32(3.0e38), 2))
        for text, x, max_x, rid in runs:
            pen = x
            for b in text:
                g = gid(b)
                nxt = F32(pen + adv[g] * scale)
                if nxt > max_x:
                    break
                if glyphs[g]["w"]:
                    quads.append((pen, base, g, rid))
                pen = nxt
        offs.append(len(quads))
    out = np.zeros((len(quads) * 6, 8), F32)
    for i, (pen, base, g, rid) in enumerate(quads):
        gl = glyphs[g]
        cw, ch = F32(int(gl["w"]) + 2 * spread), F32(int(gl["h"]) + 2 * spread)
        x0 = F32(pen + (F32(gl["bearing_x"]) - sp) * scale)
        y0 = F32(base - (F32(gl["bearing_top"]) + sp) * scale)
        x1, y1 = F32(x0 + cw * scale), F32(y0 + ch * scale)
        u0, v0 = F32(F32(gl["atlas_x"]) * inv_w), F32(F32(gl["atlas_y"]) * inv_h)
        u1, v1 = F32((F32(gl["atlas_x"]) + cw) * inv_w), F32((F32(gl["atlas_y"]) + ch) * inv_h)
        for k, (x, y, u, v) in enumerate(((x0, y0, u0, v0), (x1, y0, u1, v0), (x0, y1, u0, v1),
                                          (x1, y0, u1, v0), (x1, y1, u1, v1), (x0, y1, u0, v1))):
            out[i * 6 + k, :4] = (x, y, u, v)
            out[i * 6 + k, 4:] = col[rid]
    offs = np.array(offs, np.uint64)
    if match is not None:
        from oracle.oracle_c import dim_rows
        dim_rows(out, offs * 6, rb, match, match_rb, None)
    return out, offs
