"""GPU SDF font atlas (WG-SDF-1) against the oracle goldens, byte for byte:
coverage, SDF, both squared-distance maps (digests) and the glyph table, for
Roboto Regular and Bold at the default 1024x1024 / 96 px/em / spread 8."""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("slot,name", [(0, "regular"), (1, "bold")])
def test_atlas_matches_golden(engine, slot, name):
    z = np.load(os.path.join(GOLDEN_DIR, f"font_{name}.npz"), allow_pickle=False)
    w, h, em, sp, first, last = z["params"]
    engine.build_font_atlas(slot, width=int(w), height=int(h), em_px=float(em), spread=int(sp), first=int(first),
                            last=int(last))
    a = engine.atlas(slot)
    info = engine.atlas_info(slot)
    assert info.n_glyphs == int(last - first + 1) and info.far_d2 == (4 * int(sp) + 1) ** 2
    np.testing.assert_array_equal(a["cov"], z["cov"])
    np.testing.assert_array_equal(a["sdf"], z["sdf"])
    assert hashlib.sha256(a["d2in"].tobytes()).hexdigest() == str(z["d2in_sha"])
    assert hashlib.sha256(a["d2out"].tobytes()).hexdigest() == str(z["d2out_sha"])
    assert a["glyphs"].tobytes() == z["glyphs"].tobytes()


def test_small_atlas_and_errors(engine):
    from wgraph import WgError
    from oracle import font_oracle as fo
    from wgraph import FONTS
    engine.build_font_atlas(0, width=256, height=256, em_px=20.0, spread=3, first=48, last=57)   # digits
    a = engine.atlas(0)
    o = fo.build_atlas(FONTS[0], 256, 256, 20.0, 3, 48, 57)
    np.testing.assert_array_equal(a["sdf"], o["sdf"])
    np.testing.assert_array_equal(a["cov"], o["cov"])
    with pytest.raises(WgError):
        engine.build_font_atlas(0, width=64, height=64, em_px=96.0)     # does not fit
    with pytest.raises(WgError):
        engine.build_font_atlas(1, ttf=b"not a font")


def test_rebuilds_reuse_the_parse_and_follow_changes(engine):
    """A rebuild of the same font at the same parameters skips the TrueType
    parse and the uploads (the slot keeps the font's length, hash and
    parameters) and still gives the golden bytes; a different font or
    parameter in the same slot is parsed again, and a failed build in between
    leaves nothing to reuse."""
    from wgraph import FONTS, WgError
    z = [np.load(os.path.join(GOLDEN_DIR, f"font_{n}.npz"), allow_pickle=False) for n in ("regular", "bold")]
    w, h, em, sp, first, last = z[0]["params"]
    kw = dict(width=int(w), height=int(h), em_px=float(em), spread=int(sp), first=int(first), last=int(last))
    bold = open(FONTS[1], "rb").read()
    for ttf, want in ((None, 0), (None, 0), (bold, 1), (bold, 1), (None, 0)):
        engine.build_font_atlas(0, ttf=ttf, **kw)
        a = engine.atlas(0)
        np.testing.assert_array_equal(a["sdf"], z[want]["sdf"])
        assert a["glyphs"].tobytes() == z[want]["glyphs"].tobytes()
    with pytest.raises(WgError):
        engine.build_font_atlas(0, width=64, height=64, em_px=96.0)      # does not fit: the slot's key is dropped
    engine.build_font_atlas(0, **kw)
    np.testing.assert_array_equal(engine.atlas(0)["sdf"], z[0]["sdf"])
