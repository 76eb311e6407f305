"""WG-SDF-1 oracle (oracle/font_oracle.py) against its pins, on the CPU.

* distance transform: scipy.ndimage.distance_transform_edt on every pixel
  (exact squared distances up to 4*spread, "far" beyond);
* coverage: FreeType rendering of the same font size through PIL (different
  rasteriser and hinting -> overlap tolerance, per glyph and on average);
* the committed goldens reproduce.
Parity with the reference's fontdue path is unpinned (absent from the
snapshot).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import ROOT, GOLDEN_DIR
from oracle import font_oracle as fo
from wgraph import abi

FONT = os.path.join(ROOT, "whisper-git_amd", "fonts", "Roboto-Regular.ttf")


@pytest.fixture(scope="module")
def atlas():
    p = abi.ATLAS_DEFAULTS
    return fo.build_atlas(FONT, p["width"], p["height"], p["em_px"], p["spread"], p["first"], p["last"])


def test_edt_matches_scipy(atlas):
    from scipy import ndimage
    R = 4 * abi.ATLAS_DEFAULTS["spread"]
    inside = atlas["cov"] >= 8
    for ours, ref in ((atlas["d2in"], ndimage.distance_transform_edt(inside)),
                      (atlas["d2out"], ndimage.distance_transform_edt(~inside))):
        r2 = np.rint(ref ** 2).astype(np.int64)
        near = r2 <= R * R
        assert near.sum() > 100_000
        np.testing.assert_array_equal(ours.astype(np.int64)[near], r2[near])
        assert (ours.astype(np.int64)[~near] > R * R).all()


def test_edt_small_cases_against_scipy():
    from scipy import ndimage
    rng = np.random.default_rng(3)
    for trial in range(6):
        cov = np.where(rng.random((61, 77)) < [0.02, 0.2, 0.5, 0.9, 0.98, 0.999][trial], 16, 0).astype(np.uint8)
        a, b, sdf, far = fo.edt_sdf(cov, 2)
        inside = cov >= 8
        for ours, m in ((a, inside), (b, ~inside)):
            if m.all() or not m.any():
                continue
            r2 = np.rint(ndimage.distance_transform_edt(m) ** 2).astype(np.int64)
            near = r2 <= 64
            np.testing.assert_array_equal(ours.astype(np.int64)[near], r2[near])
            assert (ours.astype(np.int64)[~near] > 64).all()
        assert ((sdf > 127) == inside).all()


def test_coverage_close_to_freetype(atlas):
    from PIL import Image, ImageDraw, ImageFont
    sp = abi.ATLAS_DEFAULTS["spread"]
    font = ImageFont.truetype(FONT, int(abi.ATLAS_DEFAULTS["em_px"]))
    ious = []
    for g in atlas["glyphs"]:
        if g["w"] == 0:
            continue
        img = Image.new("L", (300, 300), 0)
        ImageDraw.Draw(img).text((100, 200), chr(g["codepoint"]), font=font, fill=255, anchor="ls")
        pil = np.array(img) >= 128
        ours = np.zeros_like(pil)
        c = atlas["cov"][g["atlas_y"]:g["atlas_y"] + g["h"] + 2 * sp, g["atlas_x"]:g["atlas_x"] + g["w"] + 2 * sp] >= 8
        y0, x0 = 200 - g["bearing_top"] - sp, 100 + g["bearing_x"] - sp
        ours[y0:y0 + c.shape[0], x0:x0 + c.shape[1]] = c
        ious.append((ours & pil).sum() / (ours | pil).sum())
    assert len(ious) == 94            # ASCII 33..126 (space is blank)
    assert min(ious) > 0.75 and np.mean(ious) > 0.94


@pytest.mark.parametrize("name,path", [("regular", "Roboto-Regular.ttf"), ("bold", "Roboto-Bold.ttf")])
def test_golden_reproduces(name, path):
    z = np.load(os.path.join(GOLDEN_DIR, f"font_{name}.npz"), allow_pickle=False)
    w, h, em, sp, first, last = z["params"]
    a = fo.build_atlas(os.path.join(ROOT, "whisper-git_amd", "fonts", path), int(w), int(h), float(em), int(sp),
                       int(first), int(last))
    np.testing.assert_array_equal(a["sdf"], z["sdf"])
    np.testing.assert_array_equal(a["cov"], z["cov"])
    assert hashlib.sha256(a["d2in"].tobytes()).hexdigest() == str(z["d2in_sha"])
    assert hashlib.sha256(a["d2out"].tobytes()).hexdigest() == str(z["d2out_sha"])
