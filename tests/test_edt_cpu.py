"""C2's CPU leg (oracle/edt_cpu.c: exact Felzenszwalb–Huttenlocher EDT, the
BASELINE.md §2 plan) must produce the WG-SDF-1 atlas the engine and the numpy
restatement produce: an exact EDT capped at (4*spread+1)^2 equals the
window-bounded EDT, and the SDF bytes follow from the same f32 formula."""
import os

import numpy as np
import pytest

from oracle import edt_cpu, font_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("threads", [1, 4])
@pytest.mark.parametrize("seed,shape,spread", [(0, (64, 96), 3), (1, (128, 40), 8), (2, (7, 5), 1)])
def test_fh_edt_equals_bounded_edt(seed, shape, spread, threads):
    rng = np.random.default_rng(seed)
    cov = np.zeros(shape, np.uint8)
    for _ in range(6):   # blobs of coverage 0..16
        cy, cx, r = rng.integers(0, shape[0]), rng.integers(0, shape[1]), rng.integers(1, 12)
        yy, xx = np.ogrid[:shape[0], :shape[1]]
        cov = np.maximum(cov, np.where((yy - cy) ** 2 + (xx - cx) ** 2 <= r * r, rng.integers(6, 17), 0).astype(np.uint8))
    want = font_oracle.edt_sdf(cov, spread)
    got = edt_cpu.edt_sdf(cov, spread, threads)
    for k, (g, w) in enumerate(zip(got, want[:3])):
        assert g.dtype == w.dtype and (g == w).all(), k


def test_fh_edt_on_the_regular_atlas_golden():
    z = np.load(os.path.join(ROOT, "tests", "golden", "font_regular.npz"), allow_pickle=False)
    d2in, d2out, sdf = edt_cpu.edt_sdf(z["cov"], 8, 2)
    assert (sdf == z["sdf"]).all()
