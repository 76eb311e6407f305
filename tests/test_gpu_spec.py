"""Speculative builds (wg_layout_build with one host read):
once an exact build has sized a context's buffers, later builds launch
everything on upper bounds and capacities and validate once at the end;
what did not hold is redone by the exact stages.  One fresh engine walks a
sequence of lists through every branch — same list again (no redo), larger
lists (geometry past its capacity), a list that is not well formed (lanes
redone by the exact walk), a list whose replay needs more iterations than the
blind count — and every build is bit-exact against the oracle."""
import numpy as np
import pytest

from test_gpu_parity import assert_bits
from wgraph import synth

pytestmark = pytest.mark.gpu


def full_check(eng, d, o, tag):
    s = eng.layout_summary()
    assert s.max_lane == o.max_lane, tag
    assert np.float32(s.graph_width) == np.float32(o.graph_width), tag
    lane, color = eng.lanes()
    assert_bits(tag + " lane", lane, o.lane)
    assert_bits(tag + " color", color, o.color)
    assert_bits(tag + " edges", eng.edges(), o.edges)
    got = eng.geometry()
    for k, v in o.geometry.items():
        assert_bits(f"{tag} build_{k}", got[k], v)
    gs = eng.geometry_summary()
    assert gs.n_vert == len(o.geometry["vert"]) and gs.n_curve == len(o.geometry["curve"]), tag
    eng.row_geometry(d.band)
    og = o.row_geometry(d.band)
    got = eng.geometry()
    for k, v in og.items():
        assert_bits(f"{tag} band_{k}", got[k], v)
    gs = eng.geometry_summary()   # the frame pass's summary is read lazily
    assert np.float32(gs.total_height) == og["row_top"][-1] and gs.n_curve == len(og["curve"]), tag
    sel = d.n // 2
    eng.emit_vertices(0, d.n, selected=sel)
    ov, _ = o.emit_vertices(0, d.n, selected=sel)
    from oracle import oracle_c
    assert eng.vertex_summary().checksum == oracle_c.vertex_checksum(ov), tag


def test_speculative_build_sequence():
    import wgraph
    from oracle import oracle_c
    eng = wgraph.Engine(0)
    try:
        seq = [("wide16", 3000, 1), ("wide16", 3000, 1), ("wide16", 3000, 2), ("wide16", 40000, 3),
               ("anomaly", 2000, 4), ("random13", 20000, 5), ("linux", 60000, 6), ("linux", 60000, 6),
               ("linear", 500, 7), ("wide16", 40000, 3)]
        redo = []
        for i, (kind, n, seed) in enumerate(seq):
            d = synth.generate(kind, n, seed=seed)
            o = oracle_c.OracleLayout(d)
            eng.build(d)
            c = eng.debug_counters()
            redo.append((int(c[6]), int(c[7]), int(c[8])))
            full_check(eng, d, o, f"#{i} {kind}/{n}")
            o.close()
        builds, redo_lanes, redo_geom = redo[-1]
        assert builds == len(seq) - 1                 # every build after the first speculated
        assert redo[1] == (1, 0, 0)                   # the same list again: nothing redone
        assert redo[3][2] > redo[2][2]                # 40k rows after 3k: lists past their capacity
        assert redo[4][1] > redo[3][1]                # duplicate ids / skewed parents: the exact walk
        assert redo[9][2] == redo[8][2]               # 40k rows again: the buffers fit, the geometry stands
        assert redo[7][1:] == redo[6][1:]             # the Linux-shaped list again: blind count adapted, no redo
    finally:
        eng.close()


def test_deferred_validation_sequence():
    """WG_OPT_DEFER_VALIDATION: each build is validated by the emission's
    vertex-total read (build -> banded frame pass -> emission with no host
    read between them); a build that does not hold is redone there together
    with the frame pass and the emission.  The same branch-walking sequence,
    every step bit-exact against the oracle; every other build also goes
    through the settle path of a host query right after the build."""
    import wgraph
    from oracle import oracle_c
    eng = wgraph.Engine(0)
    try:
        eng.set_defer_validation(True)
        seq = [("wide16", 3000, 1), ("wide16", 3000, 1), ("wide16", 40000, 3), ("anomaly", 2000, 4),
               ("random13", 20000, 5), ("linux", 60000, 6), ("linux", 60000, 6), ("skew", 30000, 8),
               ("linear", 500, 7), ("wide16", 40000, 3), ("linuxwide", 20000, 9)]
        last = None
        for i, (kind, n, seed) in enumerate(seq):
            d = synth.generate(kind, n, seed=seed)
            o = oracle_c.OracleLayout(d)
            tag = f"#{i} {kind}/{n}"
            eng.build(d)
            if i % 2:   # a host query settles the build first
                s = eng.layout_summary()
                assert s.max_lane == o.max_lane, tag
                got = eng.geometry()
                for k, v in o.geometry.items():
                    assert_bits(f"{tag} build_{k}", got[k], v)
            eng.row_geometry(d.band)
            sel = d.n // 3
            eng.emit_vertices(0, d.n, selected=sel)   # validates a deferred build
            og = o.row_geometry(d.band)
            ov, _ = o.emit_vertices(0, d.n, selected=sel)
            assert eng.vertex_summary().checksum == oracle_c.vertex_checksum(ov), tag
            assert eng.vertex_summary().n_vertices == len(ov), tag
            got = eng.geometry()
            for k, v in og.items():
                assert_bits(f"{tag} band_{k}", got[k], v)
            lane, color = eng.lanes()
            assert_bits(tag + " lane", lane, o.lane)
            assert_bits(tag + " color", color, o.color)
            assert_bits(tag + " edges", eng.edges(), o.edges)
            assert eng.layout_summary().max_lane == o.max_lane, tag
            o.close()
            last = eng.debug_counters()
        assert int(last[6]) == len(seq) - 1   # every build after the first speculated
        assert int(last[8]) >= 2              # and some were redone (capacity, well-formedness)
    finally:
        eng.close()


@pytest.mark.gpu
@pytest.mark.parametrize("defer", [False, True])
def test_build_frame_sequence(defer):
    """wg_layout_build_frame = wg_layout_build + wg_row_geometry(band), the
    frame's row_top computed beside the build: bit-exact against the oracle's
    build + row_geometry_with_bands over a sequence of lists (host and device
    bands, repeats, a redone speculative build), with plain builds and
    frame passes interleaved; an empty list too."""
    import torch
    import wgraph
    from oracle import oracle_c
    eng = wgraph.Engine(0)
    try:
        eng.set_defer_validation(defer)
        seq = [("wide16", 3000, 1), ("wide16", 3000, 1), ("wide16", 40000, 3), ("anomaly", 2000, 4),
               ("random13", 20000, 5), ("linux", 60000, 6), ("linear", 500, 7), ("skew", 30000, 8),
               ("linuxwide", 20000, 9)]
        for i, (kind, n, seed) in enumerate(seq):
            d = synth.generate(kind, n, seed=seed)
            o = oracle_c.OracleLayout(d)
            tag = f"#{i} {kind}/{n} defer={defer}"
            keep = None
            if i % 3 == 0:
                eng.build_frame(d, band=d.band)
            elif i % 3 == 1:
                keep = torch.from_numpy(d.band).to("cuda:0")
                torch.cuda.synchronize()
                eng.build_frame(d, device_ptr=keep.data_ptr())
            else:
                eng.build(d)
                eng.row_geometry(d.band)
            b2 = d.band.copy()
            b2[d.n // 2:] += 7.0
            fb = d.band
            if i % 4 == 3:   # another frame before anything reads the build
                eng.row_geometry(b2)
                fb = b2
            elif i % 4 == 1:   # the same bands again: nothing to do
                eng.row_geometry(d.band)
            sel = d.n // 3
            eng.emit_vertices(0, d.n, selected=sel)
            og = o.row_geometry(fb)
            ov, _ = o.emit_vertices(0, d.n, selected=sel)
            assert eng.vertex_summary().checksum == oracle_c.vertex_checksum(ov), tag
            got = eng.geometry()
            for k, v in og.items():
                assert_bits(f"{tag} band_{k}", got[k], v)
            lane, color = eng.lanes()
            assert_bits(tag + " lane", lane, o.lane)
            assert_bits(tag + " color", color, o.color)
            # the next frame with other bands goes through the normal frame pass
            eng.row_geometry(b2 if fb is d.band else d.band)
            og2 = o.row_geometry(b2 if fb is d.band else d.band)
            got = eng.geometry()
            for k, v in og2.items():
                assert_bits(f"{tag} reband_{k}", got[k], v)
            o.close()
            del keep
        e = synth.generate("linear", 0, seed=1)
        eng.build_frame(e, band=e.band)
        assert eng.geometry_summary().n_rows == 0
    finally:
        eng.close()


@pytest.mark.parametrize("kind,n", [("wide16", 120000), ("linuxwide", 40000), ("skew", 60000), ("random13", 100000)])
def test_sliced_lists_emission(kind, n):
    """WG_OPT_SLICE_LISTS: a deferred-validation build_frame leaves its
    geometry lists to the whole-list emission, which builds rows [0, h) and
    emits their tiles while rows [h, N) are built beside them.  Three steps
    (the exact first build, then speculative ones: the split's first guess,
    then the last frame's split tile) and the same steps with slicing off:
    every vertex buffer and the frame's geometry bit-exact against the
    oracle."""
    import wgraph
    from oracle import oracle_c
    d = synth.generate(kind, n, seed=11)
    o = oracle_c.OracleLayout(d)
    og = o.row_geometry(d.band)
    sel = n // 5
    ov, _ = o.emit_vertices(0, n, selected=sel)
    want = oracle_c.vertex_checksum(ov)
    try:
        for sliced in (2, 0):
            eng = wgraph.Engine(0)
            try:
                eng.set_defer_validation(True)
                eng.set_slice_lists(sliced)
                for step in range(3):
                    tag = f"{kind}/{n} sliced={sliced} step {step}"
                    eng.build_frame(d, band=d.band)
                    eng.emit_vertices(0, n, selected=sel)
                    vs = eng.vertex_summary()
                    assert vs.n_vertices == len(ov) and vs.checksum == want, tag
                got = eng.geometry()
                for k, v in og.items():
                    assert_bits(f"{kind} sliced={sliced} {k}", got[k], v)
                dc = eng.debug_counters()
                assert int(dc[6]) == 2   # the later builds speculated
                assert int(dc[11]) == (2 if sliced else 0)   # and their emissions sliced the lists
            finally:
                eng.close()
    finally:
        o.close()


def test_duplicate_ids_window_row_differs_from_table_row():
    """Round 4's illegal memory access: with duplicate ids the
    window probe's row for an id (the next 64 rows' ids, wg_hash.hip) and the
    table's (the last occurrence wins, commit_graph.rs:273-274) differ, and
    the lane-chain kernels queued before the host knows the list is not well
    formed wrote past a child list.  The list that faulted (anomaly, 5000
    rows, seed 77) on a fresh context (the exact build) and on a context whose
    earlier build lets it speculate, twice; every build bit-exact against the
    oracle through the general walk (lane_path 1), geometry and vertices too."""
    import wgraph
    from oracle import oracle_c
    d = synth.generate("anomaly", 5000, seed=77)
    o = oracle_c.OracleLayout(d)
    try:
        eng = wgraph.Engine(0)
        try:
            eng.build(d)
            assert eng.layout_summary().lane_path == 1
            full_check(eng, d, o, "fresh")
        finally:
            eng.close()
        eng = wgraph.Engine(0)
        try:
            w = synth.generate("wide16", 6000, seed=3)
            eng.build(w)
            for k in range(2):
                eng.build(d)
                full_check(eng, d, o, f"speculating #{k}")
                assert eng.layout_summary().lane_path == 1
            assert int(eng.debug_counters()[7]) >= 1   # the speculative lanes were redone by the exact walk
        finally:
            eng.close()
    finally:
        o.close()


@pytest.mark.parametrize("fused", [True, False])
def test_fused_join_with_deferred_clear_cycle(fused):
    """with deferred validation, a list of at least slice_min_rows
    rows leaves the next build's id table to be emptied by the emission, on
    the side stream beside its tiles.  The next build fills that table — on
    the main stream when the join is fused — so it must wait for the clear.
    Build / frame / emit cycles alternating two such lists (different ids in
    the same table slots), every step bit-exact against the oracle."""
    import wgraph
    from oracle import oracle_c
    lists = [synth.generate("wide16", 300_000, seed=31), synth.generate("random13", 300_000, seed=32)]
    want = []
    for d in lists:
        o = oracle_c.OracleLayout(d)
        o.row_geometry(d.band)
        ov, _ = o.emit_vertices(0, d.n, selected=d.n // 2)
        want.append((o.lane.copy(), o.max_lane, oracle_c.vertex_checksum(ov), len(ov)))
        o.close()
    eng = wgraph.Engine(0)
    try:
        eng.set_defer_validation(True)
        eng.set_join_fused(fused)
        for step in range(6):
            k = step % 2
            d = lists[k]
            eng.build_frame(d, band=d.band)
            eng.emit_vertices(0, d.n, selected=d.n // 2)
            vs = eng.vertex_summary()
            tag = f"fused={fused} step {step}"
            assert vs.n_vertices == want[k][3] and vs.checksum == want[k][2], tag
            lane, _ = eng.lanes()
            assert_bits(tag + " lane", lane, want[k][0])
            assert eng.layout_summary().max_lane == want[k][1], tag
    finally:
        eng.close()


@pytest.mark.parametrize("defer", [False, True])
def test_lds_sweep_skipped_then_needed(defer):
    """r06: a speculative geometry pass skips the LDS sweep's launch when the
    context's last exact pass had no chunk past the register sweep; a chunk
    that then needs it raises the capacity word and the pass is redone exactly
    (here the register sweep's capacity is cut to 64 edges per chunk after two
    builds, so every chunk of the next list is wide).  Every build bit-exact,
    and the next speculative pass launches the LDS sweep again."""
    import wgraph
    from oracle import oracle_c
    from wgraph import lib
    eng = wgraph.Engine(0)
    try:
        eng.set_defer_validation(defer)
        seq = [("wide16", 3000, 1, 512), ("wide16", 3000, 1, 512), ("wide16", 3000, 2, 64),
               ("wide16", 3000, 2, 64), ("random13", 5000, 3, 512)]
        redo = []
        for i, (kind, n, seed, cap) in enumerate(seq):
            eng._check(lib().wg_set_option(eng._ctx, 3, cap))   # WG_OPT_SWEEP_REG
            d = synth.generate(kind, n, seed=seed)
            o = oracle_c.OracleLayout(d)
            eng.build(d)
            full_check(eng, d, o, f"#{i} {kind}/{n} cap {cap}")
            redo.append(int(eng.debug_counters()[8]))
            o.close()
        assert redo[1] == redo[0]          # no wide chunk: the skipped LDS sweep costs nothing
        assert redo[2] > redo[1]           # every chunk wide: the skipped sweep is redone exactly
        assert redo[3] == redo[2]          # the next pass launches the LDS sweep: no redo
    finally:
        eng.close()
