"""GPU consumer adapter (WG-RAST-1, wg_render) against the numpy restatement,
byte for byte: graph + glyph layers, banded rows, the selected ring, search
dimming, HiDPI scale, viewports that start mid-list and clip rows at both
edges, negative bands (non-monotonic row_top), and the PNG writer."""
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from oracle import oracle_c, render_oracle as ro, search_oracle as so, text_oracle
from wgraph import abi, synth

pytestmark = pytest.mark.gpu


def _scene(engine, d, og, o, rb, re_, sel, summ=None, match=None):
    engine.emit_vertices(rb, re_, selected=sel)
    gv, goff = o.emit_vertices(rb, re_, selected=sel, **({} if match is None else match))
    assert engine.vertices().tobytes() == gv.tobytes()
    return gv, goff


@pytest.mark.parametrize("scale,origin_y,top", [(1.0, 0.0, 200), (1.5, 7.25, 203), (2.0, -40.0, 210)])
def test_render_graph_and_text_equal_oracle(engine, scale, origin_y, top):
    d = synth.generate("random13", 2000, seed=17)
    summ, auth = synth.text_fields(d.n, seed=1)
    engine.build(d)
    engine.row_geometry(d.band)
    o = oracle_c.OracleLayout(d)
    og = o.row_geometry(d.band)
    rb, re_ = 195, 260
    gv, goff = _scene(engine, d, og, o, rb, re_, 207)
    z = np.load(os.path.join(GOLDEN_DIR, "font_regular.npz"), allow_pickle=False)
    p = abi.ATLAS_DEFAULTS
    engine.build_font_atlas(0)
    kw = dict(now=int(d.time.max()) + 86400)
    engine.emit_glyphs(rb, re_, summaries=summ, **kw)
    tv, toff = text_oracle.emit_glyphs(d, og["node_y"], z["glyphs"], p["width"], p["height"], p["spread"], p["em_px"],
                                       rb, re_, summaries=summ, **kw)
    W, H = 720, 560
    got = engine.render(W, H, top_row=top, scale=scale, graph_x=4.0, origin_y=origin_y)
    k = np.float32(np.float32(np.float32(2.0) * np.float32(p["spread"])) *
                   np.float32(np.float32(abi.TEXT_DEFAULTS["text_px"]) / np.float32(p["em_px"]))) * np.float32(scale)
    want = ro.render(W, H, og["row_top"], top, scale=scale, graph_x=4.0, origin_y=origin_y,
                     clear=(0.09, 0.1, 0.12), graph=(gv, goff, rb), text=(tv, toff, rb), sdf=z["sdf"], k=k)
    diff = np.argwhere((got != want).any(-1))
    assert diff.size == 0, (len(diff), diff[:5])
    assert (got[..., :3] != np.array([23, 26, 31], np.uint8)).any(-1).mean() > 0.05   # something was drawn
    o.close()


def test_render_dimmed_rows_and_negative_bands(engine, tmp_path):
    d = synth.generate("linux", 800, seed=3)
    band = d.band.copy()
    band[310] = -45.0          # row 310's strip has negative height: row_top not monotonic
    band[330] = 12.5
    summ, auth = synth.text_fields(d.n, seed=4)
    engine.build(d)
    engine.row_geometry(band)
    o = oracle_c.OracleLayout(d)
    og = o.row_geometry(band)
    try:
        engine.match_rows("fix", 280, 360, summaries=summ, authors=auth)
        flags = engine.match_flags()
        want_f, _ = so.match_rows(d, b"fix", summ, auth, 280, 360)
        assert (flags == want_f).all()
        gv, goff = _scene(engine, d, og, o, 290, 350, 300, match=dict(match=flags, match_rb=280))
        got = engine.render(400, 900, top_row=290, graph=True, text=False)
        want = ro.render(400, 900, og["row_top"], 290, clear=(0.09, 0.1, 0.12), graph=(gv, goff, 290))
        assert (got == want).all()
        import wgraph
        from PIL import Image
        path = str(tmp_path / "shot.png")
        wgraph.write_png(path, got)
        assert (np.asarray(Image.open(path)) == got).all()
    finally:
        engine.match_rows("")
        o.close()
