"""Golden SDF atlases (WG-SDF-1) from the CPU oracle, pinned against scipy.

Run from the repo root:  python tests/golden/make_font_golden.py
Writes tests/golden/font_<regular|bold>.npz: sdf and coverage atlases, the
glyph table, and SHA-256 digests of the two squared-distance maps.  Before
writing, the oracle's distances are checked against
scipy.ndimage.distance_transform_edt on every pixel (exact below the
4*spread bound, "far" beyond), so the committed atlases carry that pin.
"""
import hashlib
import os
import sys

import numpy as np
from scipy import ndimage

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))
from oracle import font_oracle as fo  # noqa: E402
from wgraph import abi  # noqa: E402


def pin_against_scipy(a, spread):
    R = 4 * spread
    inside = a["cov"] >= 8
    for ours, ref in ((a["d2in"], ndimage.distance_transform_edt(inside)),
                      (a["d2out"], ndimage.distance_transform_edt(~inside))):
        r2 = np.rint(ref.astype(np.float64) ** 2).astype(np.int64)
        near = r2 <= R * R
        assert (ours.astype(np.int64)[near] == r2[near]).all()
        assert (ours.astype(np.int64)[~near] > R * R).all()


def main():
    p = abi.ATLAS_DEFAULTS
    for slot, name in ((0, "regular"), (1, "bold")):
        path = os.path.join(ROOT, "whisper-git_amd", "fonts", ["Roboto-Regular.ttf", "Roboto-Bold.ttf"][slot])
        a = fo.build_atlas(path, p["width"], p["height"], p["em_px"], p["spread"], p["first"], p["last"])
        pin_against_scipy(a, p["spread"])
        g = np.array([tuple(x[k] for k in abi.GLYPH_DTYPE.names) for x in a["glyphs"]], abi.GLYPH_DTYPE)
        np.savez_compressed(os.path.join(ROOT, "tests", "golden", f"font_{name}.npz"), sdf=a["sdf"], cov=a["cov"],
                            glyphs=g, d2in_sha=hashlib.sha256(a["d2in"].tobytes()).hexdigest(),
                            d2out_sha=hashlib.sha256(a["d2out"].tobytes()).hexdigest(),
                            params=np.array([p["width"], p["height"], p["em_px"], p["spread"], p["first"], p["last"]],
                                            np.float64))
        print(name, "ok")


if __name__ == "__main__":
    main()
