"""The multi-threaded CPU baseline (oracle/cpu_mt.c, bench.py's
cpu_baseline_threads) computes exactly what the single-thread oracle computes:
lanes, colours, slot counts, edges, the build's and the banded geometry, and
every vertex, bit for bit, on every preset and at several thread counts
(commit_graph.rs:265-399, 803-908)."""
import numpy as np
import pytest

from oracle import cpu_mt, oracle_c

from wgraph import synth


def _same_geometry(a, b):
    for k in ("height", "node_y", "row_top", "vert_off", "vert", "curve_off", "curve", "curve_color"):
        x, y = a[k], b[k]
        assert x.shape == y.shape, k
        assert x.tobytes() == y.tobytes(), k


@pytest.mark.parametrize("threads", [1, 3, 8])
@pytest.mark.parametrize("kind,n", [("random13", 3000), ("linux", 4000), ("wide16", 3000), ("anomaly", 2000),
                                    ("skew", 3000), ("linuxwide", 3000), ("linear", 500)])
def test_mt_equals_oracle(kind, n, threads):
    d = synth.generate(kind, n)
    o = oracle_c.OracleLayout(d)
    m = cpu_mt.MtLayout(d, threads)
    assert (m.max_lane, m.n_slots) == (o.max_lane, o.n_slots)
    assert np.float32(m.graph_width) == o.graph_width
    assert (m.lane == o.lane).all() and (m.color == o.color).all()
    assert m.edges.tobytes() == o.edges.tobytes()
    _same_geometry(m.build_geometry, o.geometry)
    _same_geometry(m.row_geometry(d.band), o.row_geometry(d.band))
    sel = n // 3
    for r0, r1 in ((0, n), (n // 5, n // 2), (n - 1, n), (7, 7)):
        mv, moff = m.emit_vertices(r0, r1, selected=sel)
        ov, ooff = o.emit_vertices(r0, r1, selected=sel)
        assert (moff == ooff).all()
        assert mv.tobytes() == ov.tobytes()
        dst = np.zeros(len(ov) + 5, ov.dtype)
        off = np.zeros(r1 - r0 + 1, np.uint64)
        assert m.emit_vertices_into(r0, r1, dst, off, selected=sel) == len(ov)
        assert dst[:len(ov)].tobytes() == ov.tobytes() and (off == ooff).all()
    with pytest.raises(ValueError):
        m.emit_vertices_into(0, n, np.zeros(3, ov.dtype), np.zeros(n + 1, np.uint64))
    m.close()
    o.close()


def test_mt_empty_and_single():
    for n in (0, 1):
        d = synth.generate("random13", max(n, 1)).slice_rows(n)
        o = oracle_c.OracleLayout(d)
        m = cpu_mt.MtLayout(d, 4)
        assert (m.max_lane, m.n_slots, len(m.edges)) == (o.max_lane, o.n_slots, len(o.edges))
        mv, _ = m.emit_vertices(0, n)
        ov, _ = o.emit_vertices(0, n)
        assert mv.tobytes() == ov.tobytes()


def test_mt_duplicate_ids_keep_the_last_row():
    # anomaly lists hold duplicate ids (:272-274 last write wins); the
    # concurrent table must resolve every duplicate to its last row whatever
    # order the threads insert in
    d = synth.generate("anomaly", 6000, p_dup_oid=0.05)
    o = oracle_c.OracleLayout(d)
    for t in (2, 8):
        m = cpu_mt.MtLayout(d, t)
        assert (m.lane == o.lane).all() and m.edges.tobytes() == o.edges.tobytes()
        m.close()


def test_phase_timings_are_reported():
    d = synth.generate("random13", 1000)
    m = cpu_mt.MtLayout(d, 2)
    m.row_geometry(d.band)
    m.emit_vertices(0, d.n)
    ph = cpu_mt.phase_ms()
    assert set(ph) == set(cpu_mt.PHASES) and all(v >= 0 for v in ph.values())
