"""GPU glyph quads (WG-TEXT-1) against the oracle, bit for bit: every
TextVertex of every row, per-row quad offsets and the checksum, with the
committed Roboto atlas glyph table, banded geometry, synthetic rows,
non-ASCII bytes, empty summaries and clipped long summaries."""
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from oracle import text_oracle as to
from wgraph import abi, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def atlas_glyphs():
    z = np.load(os.path.join(GOLDEN_DIR, "font_regular.npz"), allow_pickle=False)
    return z["glyphs"]


@pytest.mark.parametrize("kind,n,rng_", [("random13", 4000, (0, 4000)), ("anomaly", 600, (100, 500)),
                                         ("linear", 300, (0, 300))])
def test_glyph_quads_match_oracle(engine, atlas_glyphs, kind, n, rng_):
    from oracle import oracle_c
    p = abi.ATLAS_DEFAULTS
    engine.build_font_atlas(0)
    d = synth.generate(kind, n, seed=41)
    s = synth.summaries(n, seed=3)
    engine.build(d)
    engine.row_geometry(d.band)
    o = oracle_c.OracleLayout(d)
    og = o.row_geometry(d.band)
    rb, re_ = rng_
    kw = dict(now=int(d.time.max()) + 3 * 86400, summary_max_x=520.0)   # clips the longer summaries
    engine.emit_glyphs(rb, re_, summaries=s, **kw)
    want, woff = to.emit_glyphs(d, og["node_y"], atlas_glyphs, p["width"], p["height"], p["spread"], p["em_px"], rb, re_,
                                summaries=s, **kw)
    got = engine.glyph_vertices().view(np.float32).reshape(-1, 8)
    assert got.shape == want.shape
    assert got.tobytes() == want.tobytes()
    assert (engine.glyph_offsets() == woff).all()
    assert engine.glyph_summary().checksum == oracle_c.vertex_checksum(want.reshape(-1, 6))
    o.close()


def test_glyphs_without_summaries(engine, atlas_glyphs):
    p = abi.ATLAS_DEFAULTS
    engine.build_font_atlas(0)
    d = synth.generate("wide16", 200, seed=2)
    engine.build(d)
    engine.emit_glyphs(0, 200)
    g = engine.geometry()
    want, _ = to.emit_glyphs(d, g["node_y"], atlas_glyphs, p["width"], p["height"], p["spread"], p["em_px"], 0, 200)
    assert engine.glyph_vertices().view(np.float32).reshape(-1, 8).tobytes() == want.tobytes()
