"""GPU parity: the HIP engine through the C ABI against the oracle.

Bar: bit-exact for lanes, colours, max_lane, edges, heights, per-row list
contents and order, row_top_y, and every f32 of the curve records and the
vertex buffers (the north star allows 1 ulp on fp32 vertex positions; the
engine is held to 0 ulp and the test reports the ulp distance if it ever
differs).  Small cases compare against the committed goldens; larger ones
against the C oracle run in-process; the full-size configuration through
size-independent checks (checksums, monotone row_top, count identities).
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden
from wgraph import abi, synth

pytestmark = pytest.mark.gpu


def ulp_diff(a, b):
    ai = a.view(np.int32).astype(np.int64)
    bi = b.view(np.int32).astype(np.int64)
    ai = np.where(ai < 0, -(ai & 0x7FFFFFFF), ai)
    bi = np.where(bi < 0, -(bi & 0x7FFFFFFF), bi)
    return np.abs(ai - bi)


def assert_bits(name, got, want):
    got = np.ascontiguousarray(got)
    want = np.ascontiguousarray(want)
    assert got.shape == want.shape, (name, got.shape, want.shape)
    if got.tobytes() != want.tobytes():
        if got.dtype == np.float32:
            d = ulp_diff(got.reshape(-1), want.reshape(-1))
            idx = np.nonzero(d)[0]
            raise AssertionError(f"{name}: {idx.size} f32 mismatches, max {d.max()} ulp, first at {idx[:5]}: "
                                 f"{got.reshape(-1)[idx[:5]]} vs {want.reshape(-1)[idx[:5]]}")
        idx = np.nonzero(got.reshape(-1) != want.reshape(-1))[0]
        raise AssertionError(f"{name}: {idx.size} mismatches, first at {idx[:5]}: "
                             f"{got.reshape(-1)[idx[:5]]} vs {want.reshape(-1)[idx[:5]]}")


def check_layout(engine, g):
    s = engine.layout_summary()
    assert s.max_lane == int(g["max_lane"])
    assert np.float32(s.graph_width) == np.float32(g["graph_width"])
    lane, color = engine.lanes()
    assert_bits("lane", lane, g["lane"])
    assert_bits("color", color, g["color"])
    e = engine.edges()
    assert_bits("edges", e.view(np.uint32).reshape(-1, 5) if len(e) else np.zeros((0, 5), np.uint32), g["edges"])
    assert_bits("heights", engine.row_heights(), g["heights"])


def check_geometry(engine, g, prefix):
    got = engine.geometry()
    for k in ("height", "node_y", "row_top", "vert_off", "vert", "curve_off", "curve", "curve_color"):
        assert_bits(prefix + k, got[k], g[prefix + k])


@pytest.mark.parametrize("name", golden_names())
def test_golden_full_pipeline(engine, name):
    d, g = load_golden(name)
    engine.build(d)
    check_layout(engine, g)
    check_geometry(engine, g, "build_")          # GraphLayout::build's row_geometry
    engine.row_geometry(g["band"])               # row_geometry_with_bands
    check_geometry(engine, g, "band_")
    engine.emit_vertices(0, d.n, selected=int(g["selected"]))
    s = engine.vertex_summary()
    assert s.n_vertices == int(g["vtx_off"][-1])
    assert_bits("vtx_off", engine.vertex_offsets(), g["vtx_off"])
    head = int(g["vertices_head_rows"])
    nh = int(g["vtx_off"][head])
    v = engine.vertices(0, nh).view(np.float32).reshape(-1, 6)
    assert_bits("vertices", v, g["vertices"])
    assert s.checksum == int(g["vertex_checksum"])


def ids_distinct(d) -> bool:
    return len({bytes(r) for r in d.oid}) == d.n


@pytest.mark.parametrize("name", golden_names())
def test_golden_lanes_both_paths(engine, name):
    """The event-compressed fast path and the general walk give identical layouts;
    only duplicate ids take the general walk (parents at earlier rows and self
    parents are leaky events of the fast path)."""
    d, g = load_golden(name)
    try:
        for general in (True, False):
            engine.set_lane_path(general)
            engine.build(d)
            check_layout(engine, g)
            s = engine.layout_summary()
            if d.n:
                expect_path = 1 if (general or not ids_distinct(d)) else 0
                assert s.lane_path == expect_path, (name, general, s.lane_path)
                assert s.n_slots == int(g["n_slots"])
    finally:
        engine.set_lane_path(False)


@pytest.mark.parametrize("kind,n", [("random13", 200000), ("linux", 300000), ("wide16", 300000)])
def test_fast_lanes_match_oracle_large(engine, kind, n):
    from oracle import oracle_c
    d = synth.generate(kind, n, seed=99)
    o = oracle_c.OracleLayout(d)
    engine.build(d)
    s = engine.layout_summary()
    assert s.lane_path == 0
    assert s.max_lane == o.max_lane and s.n_slots == o.n_slots
    lane, color = engine.lanes()
    assert_bits("lane", lane, o.lane)
    assert_bits("color", color, o.color)


@pytest.mark.parametrize("kind,n", [("random13", 20000), ("linux", 30000), ("wide16", 50000), ("anomaly", 5000),
                                    ("linear", 10000)])
def test_against_oracle_midsize(engine, kind, n):
    from oracle import oracle_c
    d = synth.generate(kind, n, seed=1234 + n)
    o = oracle_c.OracleLayout(d)
    engine.build(d)
    s = engine.layout_summary()
    assert s.max_lane == o.max_lane
    lane, color = engine.lanes()
    assert_bits("lane", lane, o.lane)
    assert_bits("color", color, o.color)
    assert_bits("edges", engine.edges(), o.edges)
    got = engine.geometry()
    for k, v in o.geometry.items():
        assert_bits("build_" + k, got[k], v)
    engine.row_geometry(d.band)
    og = o.row_geometry(d.band)
    got = engine.geometry()
    for k, v in og.items():
        assert_bits("band_" + k, got[k], v)
    sel = n // 3
    engine.emit_vertices(0, n, selected=sel)
    ov, ooff = o.emit_vertices(0, n, selected=sel)
    assert_bits("vtx_off", engine.vertex_offsets(), ooff)
    sv = engine.vertex_summary()
    assert sv.checksum == __import__("oracle").oracle_c.vertex_checksum(ov)
    # a window of rows bit-for-bit
    a, b = int(ooff[sel - 5]), int(ooff[sel + 5])
    assert_bits("vertices", engine.vertices(a, b - a).view(np.float32), ov[a:b].view(np.float32))


@pytest.mark.parametrize("name", golden_names())
def test_golden_geometry_lds_sweep(engine, name):
    """Every chunk through the LDS sweep (register capacity 0): same lists."""
    from wgraph import lib
    d, g = load_golden(name)
    engine._check(lib().wg_set_option(engine._ctx, 3, 0))
    try:
        engine.build(d)
        check_geometry(engine, g, "build_")
    finally:
        engine._check(lib().wg_set_option(engine._ctx, 3, 512))


def test_partial_row_range(engine):
    from oracle import oracle_c
    d = synth.generate("random13", 5000, seed=77)
    o = oracle_c.OracleLayout(d)
    engine.build(d)
    engine.row_geometry(d.band)
    o.row_geometry(d.band)
    for rb, re_, sel in ((100, 700, 400), (4999, 5000, 4999), (0, 1, -1), (2500, 2500, -1)):
        engine.emit_vertices(rb, re_, selected=sel)
        ov, ooff = o.emit_vertices(rb, re_, selected=sel)
        assert_bits("vtx_off", engine.vertex_offsets(), ooff)
        if len(ov):
            assert_bits("vertices", engine.vertices().view(np.float32), ov.view(np.float32))


def test_row_top_exact_beyond_2_24(engine):
    """1.3M rows: row_top crosses 2^24 and 2^25 px; the transducer scan must
    reproduce the sequential f32 accumulation bit for bit (:329-335)."""
    from oracle import oracle_c
    d = synth.generate("linux", 1_300_000)
    o = oracle_c.OracleLayout(d)
    engine.build(d)
    got = engine.geometry()
    assert got["row_top"][-1] > 2 ** 25
    assert_bits("row_top", got["row_top"], o.geometry["row_top"])
    assert_bits("vert_off", got["vert_off"], o.geometry["vert_off"])
    assert_bits("curve", got["curve"], o.geometry["curve"])
    assert engine.geometry_summary().scan_path == 0


@pytest.mark.parametrize("kind,n", [("random13", 100_000), ("linux", 1_300_000)], ids=["C3", "C4"])
def test_baseline_configs_vertex_checksum(engine, kind, n):
    """BASELINE configs C3 (100k DAG, 1.3 parents per commit) and C4 (the
    Linux-kernel-shaped 1.3M-commit DAG) on one GPU, full path (build + banded
    geometry + emission): the whole vertex buffer checksummed against the CPU
    oracle's (emitted and checksummed in pieces of 100k rows, each at its
    offset)."""
    from oracle import oracle_c
    d = synth.generate(kind, n)
    o = oracle_c.OracleLayout(d)
    try:
        engine.build(d)
        engine.row_geometry(d.band)
        sel = n // 2 + 1
        engine.emit_vertices(0, d.n, selected=sel)
        vs = engine.vertex_summary()
        o.row_geometry(d.band)
        total, first = 0, 0
        for a in range(0, d.n, 100_000):
            b = min(d.n, a + 100_000)
            ov, _ = o.emit_vertices(a, b, selected=sel)
            total = (total + oracle_c.vertex_checksum(ov, first)) & 0xFFFFFFFFFFFFFFFF
            first += len(ov)
            del ov
        assert vs.n_vertices == first
        assert vs.checksum == total
    finally:
        o.close()


@pytest.mark.parametrize("tile", [1024, 2048, 4096])
@pytest.mark.parametrize("kind,n", [("wide16", 50_000), ("linuxwide", 20_000), ("random13", 30_000), ("anomaly", 5000)])
def test_emission_tile_sizes(kind, n, tile):
    """WG_OPT_VTX_TILE: the emission's workgroup tile (1024 or 2048 vertices,
    auto picks 2048 for lists past 4e8 vertices) changes nothing: the whole
    vertex buffer, its row offsets and a partial row range with a selected row
    bit-exact against the oracle (WG-TESS-1), twice on one context (the
    second emission launched on the buffers in place)."""
    import wgraph
    from oracle import oracle_c
    d = synth.generate(kind, n, seed=29)
    o = oracle_c.OracleLayout(d)
    eng = wgraph.Engine(0)
    try:
        eng.set_vtx_tile(tile)
        eng.build(d)
        eng.row_geometry(d.band)
        o.row_geometry(d.band)
        for rb, re_, sel in ((0, n, n // 3), (n // 5, n // 5 + 777, n // 5 + 10)):
            for _ in range(2):
                eng.emit_vertices(rb, re_, selected=sel)
                ov, ooff = o.emit_vertices(rb, re_, selected=sel)
                assert eng.vertex_offsets().tobytes() == ooff.tobytes(), (kind, tile, rb)
                vs = eng.vertex_summary()
                assert vs.n_vertices == len(ov) and vs.checksum == oracle_c.vertex_checksum(ov), (kind, tile, rb)
    finally:
        eng.close()
        o.close()


def test_bands_with_fractional_and_negative_values(engine):
    """Non-integer bands keep the transducer path exact; a negative band forces
    the serial path, which must also be exact."""
    from oracle import oracle_c
    d = synth.generate("wide16", 40000, seed=5)
    o = oracle_c.OracleLayout(d)
    engine.build(d)
    rng = np.random.default_rng(0)
    for band in (rng.uniform(0, 40, d.n).astype(np.float32),
                 np.where(rng.random(d.n) < 0.01, -3.0, 30.0).astype(np.float32)):
        engine.row_geometry(band)
        og = o.row_geometry(band)
        got = engine.geometry()
        for k in ("row_top", "height", "node_y", "vert", "curve"):
            assert_bits(k, got[k], og[k])


def test_banded_passes_reuse_the_swept_lists(engine):
    """Geometry passes on the same layout reuse the swept lists: the curve
    superset is re-filtered only when a row's strip flags change (bands that
    zero a row's height or put its node at the row's bottom).  Every pass must
    equal the oracle's."""
    from oracle import oracle_c
    d = synth.generate("wide16", 30000, seed=9)
    o = oracle_c.OracleLayout(d)
    engine.build(d)
    h = engine.row_heights()
    rng = np.random.default_rng(3)
    plain = rng.uniform(0, 20, d.n).astype(np.float32)
    odd = plain.copy()
    pick = rng.random(d.n) < 0.02
    odd[pick] = -h[pick]                                  # zero-height rows
    lift = (rng.random(d.n) < 0.02) & ~pick
    odd[lift] = (6.0 - h[lift]).astype(np.float32)        # node below the row's bottom
    engine.enable_timing(True, reserve=256)
    for band in (plain, plain, odd, odd, plain, None):
        engine.row_geometry(band)
        og = o.row_geometry(band)
        got = engine.geometry()
        for k in ("row_top", "height", "node_y", "vert_off", "vert", "curve_off", "curve", "curve_color"):
            assert_bits(k, got[k], og[k])
    names = [n for n, _ in engine.timings()]
    engine.enable_timing(False)
    # the repeated plain / odd frames are bitwise-equal to the geometry in place
    # and skip the pass entirely (per-frame reuse); the other four re-filter
    assert names.count("geom_reuse") == 4 and names.count("geom_lists") == 0


def test_empty_and_single(engine):
    d = synth.generate("linear", 1)
    engine.build(d)
    assert engine.layout_summary().max_lane == 0
    engine.emit_vertices(0, 1, selected=0)
    assert engine.vertex_summary().n_vertices == abi.VTX_PER_NODE + abi.VTX_PER_RING


def test_full_size_properties(engine):
    """BASELINE config size (1M rows): size-independent identities."""
    d = synth.generate("wide16", 1_000_000)
    engine.build(d)
    engine.row_geometry(d.band)
    g = engine.geometry()
    assert np.all(np.diff(g["row_top"]) >= 28.0)
    nv = np.diff(g["vert_off"].astype(np.int64))
    nc = np.diff(g["curve_off"].astype(np.int64))
    engine.emit_vertices(0, d.n, selected=7)
    off = engine.vertex_offsets()
    want = 6 * nv + 96 * nc + 72
    want[7] += 144
    assert (np.diff(off.astype(np.int64)) == want).all()
