"""Headless screenshot of the history view's graph + text columns (the
engine-side counterpart of screenshot_mode.rs:101-141): build a commit list,
lay it out, emit one viewport's vertex and glyph buffers, rasterise them on
the GPU (WG-RAST-1) and save a PNG.

    python -m wgraph.screenshot out.png [--kind random13] [--rows 100000]
        [--top 0] [--width 1280] [--height 800] [--scale 1.0] [--query fix]
"""
from __future__ import annotations

import argparse
import sys

import numpy as np

from . import Engine, abi, synth, write_png


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m wgraph.screenshot")
    ap.add_argument("out")
    ap.add_argument("--kind", default="random13", choices=sorted(synth.PRESETS))
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--top", type=int, default=0, help="first row of the viewport")
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--query", default="", help="search query: non-matching rows are dimmed")
    ap.add_argument("--selected", type=int, default=None)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)

    d = synth.generate(a.kind, a.rows)
    summ, auth = synth.text_fields(d.n)
    eng = Engine(a.device)
    try:
        eng.build(d)
        eng.row_geometry(d.band)
        g = eng.geometry()
        # rows that can appear in the viewport (row_top is non-decreasing for these bands)
        rt = g["row_top"]
        top = min(a.top, d.n - 1)
        bottom = top + a.height / a.scale
        end = int(np.searchsorted(rt, rt[top] + bottom, side="right")) + 1
        end = min(max(end, top + 1), d.n)
        if a.query:
            eng.match_rows(a.query, top, end, summaries=summ, authors=auth)
        eng.emit_vertices(top, end, selected=top + 3 if a.selected is None else a.selected)
        eng.build_font_atlas(0)
        eng.emit_glyphs(top, end, summaries=summ, now=int(d.time.max()) + 86400)
        img = eng.render(a.width, a.height, top_row=top, scale=a.scale, graph_x=8.0, origin_y=4.0)
        write_png(a.out, img)
        print(f"{a.out}: rows {top}..{end} of {d.n}, {a.width}x{a.height} at scale {a.scale}", file=sys.stderr)
    finally:
        eng.close()


if __name__ == "__main__":
    main()
