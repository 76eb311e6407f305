"""CPU: the WG-RAST-1 restatement on hand-checked scenes, and the engine's
PNG writer (host code of the C-ABI library) decoded by PIL."""
import numpy as np

from oracle import render_oracle as ro


def _quad(x0, y0, x1, y1, rgba):
    # two triangles sharing the diagonal, SplineVertex layout {x, y, r, g, b, a}
    pts = [(x0, y0), (x1, y0), (x0, y1), (x1, y0), (x1, y1), (x0, y1)]
    return np.array([[x, y, *rgba] for x, y in pts], np.float32)


def test_axis_aligned_quad_covers_pixel_centres_inside():
    v = _quad(2.0, 1.0, 6.0, 4.0, (1, 0, 0, 1))
    img = ro.render(10, 6, np.array([0, 28], np.float32), 0, graph=(v, [0, 6], 0))
    red = (img[..., 0] == 255) & (img[..., 1] == 0)
    want = np.zeros((6, 10), bool)
    want[1:4, 2:6] = True          # centres x+0.5 in [2, 6], y+0.5 in [1, 4]
    assert (red == want).all()


def test_shared_diagonal_is_blended_once():
    # half-transparent white over black: every covered pixel exactly once -> 128
    v = _quad(0.0, 0.0, 8.0, 8.0, (1, 1, 1, 0.5))
    img = ro.render(8, 8, np.array([0, 28], np.float32), 0, graph=(v, [0, 6], 0))
    assert (img[..., 0] == 128).all()


def test_row_offsets_and_scale():
    v = _quad(0.0, 0.0, 2.0, 2.0, (0, 1, 0, 1))
    rt = np.array([0, 10, 20], np.float32)
    img = ro.render(8, 40, rt, 0, scale=2.0, origin_y=1.0, graph=(np.concatenate([v, v]), [0, 6, 12], 0))
    g = img[..., 1] == 255
    assert g[2:6, 0:4].all() and g[22:26, 0:4].all() and g.sum() == 32


def test_png_writer_round_trip(tmp_path):
    from PIL import Image
    import wgraph
    a = (np.random.default_rng(0).random((37, 301, 4)) * 255).astype(np.uint8)
    p = str(tmp_path / "x.png")
    wgraph.write_png(p, a)
    assert (np.asarray(Image.open(p)) == a).all()
    big = np.zeros((300, 300, 4), np.uint8)       # > 64 KiB of scanlines: several stored blocks
    big[..., 1] = np.arange(300, dtype=np.uint8)[None, :]
    wgraph.write_png(p, big)
    assert (np.asarray(Image.open(p)) == big).all()
