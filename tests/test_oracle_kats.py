"""The reference's own known-answer tests (commit_graph.rs:1593-1742), ported.

They pin the oracles (C and numpy restatements) to the only behaviour the
reference's test suite fixes for this path, with the reference's tolerances.
"""
import numpy as np
import pytest

from oracle import oracle_c, oracle_py as P
from wgraph import commits_to_soa

ROW_HEIGHT = 28.0
NODE_Y = 14.0
MAX_EXTRA_HEIGHT = 28.0
C = np.array([0.0, 0.0, 0.0, 0.4, 3.0, 0.6, 3.0, 1.0], np.float32)  # (:1595-1600)


def uniform_offsets(n):  # (:1627-1629)
    return [np.float32(i * ROW_HEIGHT) for i in range(n + 1)]


@pytest.mark.parametrize("impl", ["c", "py"])
def test_cubic_t_at_y_recovers_endpoints(impl):  # :1593-1605
    if impl == "c":
        t_at_y = lambda y: oracle_c.cubic_t_at_y(C, y)  # noqa: E731
        y_at = lambda t: oracle_c.cubic_y_at(C, t)  # noqa: E731
    else:
        cu = P.Cubic(C[0:2], C[2:4], C[4:6], C[6:8])
        t_at_y, y_at = cu.t_at_y, cu.y_at
    assert abs(t_at_y(0.0) - 0.0) < 1e-3
    assert abs(t_at_y(1.0) - 1.0) < 1e-3
    assert abs(y_at(t_at_y(0.5)) - 0.5) < 1e-3


@pytest.mark.parametrize("impl", ["c", "py"])
def test_cubic_subcurve_endpoints_match_y_at(impl):  # :1607-1622
    if impl == "c":
        sub = oracle_c.cubic_subcurve(C, 0.25, 0.75)
        ya, yb = oracle_c.cubic_y_at(C, 0.25), oracle_c.cubic_y_at(C, 0.75)
        s0, s3 = sub[1], sub[7]
    else:
        cu = P.Cubic(C[0:2], C[2:4], C[4:6], C[6:8])
        s = cu.subcurve(0.25, 0.75)
        ya, yb = cu.y_at(0.25), cu.y_at(0.75)
        s0, s3 = s.p[0][1], s.p[3][1]
    assert abs(s0 - ya) < 1e-3
    assert abs(s3 - yb) < 1e-3


def _decompose_py(edge, n):
    rows = [P.RowGeometry() for _ in range(n)]
    P.decompose_edge_into_rows(edge, uniform_offsets(n), rows)
    return [dict(full=len(r.full), top=len(r.top), bottom=len(r.bottom),
                 curves=[np.asarray(c[0], np.float32) for c in r.curves]) for r in rows]


def _decompose_c(edge, n):
    """The C oracle's decompose_edge_into_rows — the restatement the GPU
    parity tests compare with — over the same default rows and offsets."""
    from wgraph import abi
    g = oracle_c.decompose_edges([edge], uniform_offsets(n))
    out = []
    for r in range(n):
        v = (g["vert"][g["vert_off"][r]:g["vert_off"][r + 1]] >> 24) & 3
        out.append(dict(full=int((v == abi.WG_VERT_FULL).sum()), top=int((v == abi.WG_VERT_TOP).sum()),
                        bottom=int((v == abi.WG_VERT_BOTTOM).sum()),
                        curves=list(g["curve"][g["curve_off"][r]:g["curve_off"][r + 1]])))
    return out


def _decompose(impl, edge, n):
    return _decompose_c(edge, n) if impl == "c" else _decompose_py(edge, n)


@pytest.mark.parametrize("impl", ["c", "py"])
def test_decompose_same_lane_emits_top_full_bottom_verticals(impl):  # :1631-1651
    rows = _decompose(impl, (0, 1, 3, 1, 0), 4)
    assert rows[0]["bottom"] == 1 and rows[0]["full"] == 0 and rows[0]["top"] == 0
    assert rows[1]["full"] == 1 and rows[2]["full"] == 1
    assert rows[3]["top"] == 1


@pytest.mark.parametrize("impl", ["c", "py"])
def test_decompose_cross_lane_emits_one_curve_per_spanned_row(impl):  # :1653-1674
    rows = _decompose(impl, (0, 0, 3, 2, 0), 4)
    assert [len(r["curves"]) for r in rows] == [1, 1, 1, 1]
    for r in rows:
        assert not r["full"] and not r["top"] and not r["bottom"]


@pytest.mark.parametrize("impl", ["c", "py"])
def test_decompose_cross_lane_segment_y_spans_row_strip(impl):  # :1676-1702
    rows = _decompose(impl, (0, 0, 2, 1, 0), 3)
    c0, c1, c2 = rows[0]["curves"][0], rows[1]["curves"][0], rows[2]["curves"][0]
    assert abs(c0[1] - NODE_Y) < 0.5 and abs(c0[7] - ROW_HEIGHT) < 0.5
    assert abs(c1[1] - 0.0) < 0.5 and abs(c1[7] - ROW_HEIGHT) < 0.5
    assert abs(c2[1] - 0.0) < 0.5 and abs(c2[7] - NODE_Y) < 0.5


def test_decompose_c_and_py_agree_bitwise():
    """Both restatements give the same curve bits on the KAT edges."""
    for edge, n in (((0, 0, 3, 2, 0), 4), ((0, 0, 2, 1, 0), 3), ((1, 3, 5, 0, 2), 7)):
        a, b = _decompose_c(edge, n), _decompose_py(edge, n)
        for ra, rb in zip(a, b):
            assert (ra["full"], ra["top"], ra["bottom"]) == (rb["full"], rb["top"], rb["bottom"])
            assert len(ra["curves"]) == len(rb["curves"])
            for ca, cb in zip(ra["curves"], rb["curves"]):
                assert np.asarray(ca, np.float32).tobytes() == np.asarray(cb, np.float32).tobytes(), edge


def _heights_c(times):
    d = commits_to_soa([dict(id=bytes([i]) * 20, time=t, parents=[]) for i, t in enumerate(times)])
    o = oracle_c.OracleLayout(d)
    return o.heights


@pytest.mark.parametrize("impl", ["c", "py"])
def test_compute_row_heights_clamps_to_min_for_dense_commits(impl):  # :1704-1723
    times = [1_000_000, 1_000_000 - 60]
    h = _heights_c(times) if impl == "c" else P.compute_row_heights(times)
    assert len(h) == 2
    assert abs(h[0] - ROW_HEIGHT) < 1.0
    assert abs(h[1] - ROW_HEIGHT) < 1.0


@pytest.mark.parametrize("impl", ["c", "py"])
def test_compute_row_heights_saturates_at_max_for_long_gaps(impl):  # :1725-1742
    times = [1_000_000_000, 1_000_000_000 - 60 * 24 * 3600]
    h = _heights_c(times) if impl == "c" else P.compute_row_heights(times)
    expected = round(ROW_HEIGHT + MAX_EXTRA_HEIGHT)
    assert abs(h[0] - expected) < 1.0
