"""Hand-worked lane pins (VERDICT r02 "next round" #4).

The reference's own tests pin no lane index, max_lane or edge (SURVEY §4:
its 7 KATs cover Cubic, decomposition and heights only) and the reference
cannot be built here (no Rust toolchain).  Each case below was worked out BY
HAND from commit_graph.rs — the commit loop (:276-295), find_or_assign_lane
(:401-412), lowest_free_lane (:414-423), the duplicate-waiter free
(:287-291), update_lanes_for_parents (:425-460), update_peak (:462-471), the
colour rule (:278-283) and the edge loop (:301-320) — stepping
`active_lanes` row by row (the trace is in each case's comment).  The
expected arrays are literals, independent of both CPU restatements
(oracle/wg_oracle.c, oracle/oracle_py.py) and of the engine, which all three
must reproduce.

Edges are (child_row, child_lane, parent_row, parent_lane, colour index).
"""
import numpy as np
import pytest

from wgraph.synth import Dag

# name: (rows [(id, [parent ids], orphan?)], lanes, max_lane, n_slots, edges, colours)
# ids not listed as a row ("X", "Y") are parents outside the list.
CASES = {
    # A:[B] B:[C] C:[D] D:[] — slot0 B, C, D, None.
    "linear": (
        [("A", ["B"], 0), ("B", ["C"], 0), ("C", ["D"], 0), ("D", [], 0)],
        [0, 0, 0, 0], 0, 1,
        [(0, 0, 1, 0, 0), (1, 0, 2, 0, 0), (2, 0, 3, 0, 0)], [0, 0, 0, 0]),
    # A -> [C]; B: no free slot, push 1, [C,C] (max 1); C takes slot 0 and
    # frees slot 1 (:287-291), [D,_]; D slot 0.
    "duplicate_first_parent_waiters": (
        [("A", ["C"], 0), ("B", ["C"], 0), ("C", ["D"], 0), ("D", [], 0)],
        [0, 1, 0, 0], 1, 2,
        [(0, 0, 2, 0, 0), (1, 1, 2, 0, 1), (2, 0, 3, 0, 0)], [0, 1, 0, 0]),
    # M: slot0 A, secondary B not present -> push 1, [A,B]; B at 1 -> [A,A];
    # A at 0 frees 1, no parents -> [_,_].
    "merge_allocates_secondary": (
        [("M", ["A", "B"], 0), ("B", ["A"], 0), ("A", [], 0)],
        [0, 1, 0], 1, 2,
        [(0, 0, 2, 0, 0), (0, 0, 1, 1, 0), (1, 1, 2, 0, 1)], [0, 1, 0]),
    # P: [B]; M: push 1, slot1 A, secondary B already waited for (slot 0):
    # no allocation (:451), [B,A]; A -> [B,C]; B -> [C,C]; C frees 1.
    "secondary_parent_deduplicated": (
        [("P", ["B"], 0), ("M", ["A", "B"], 0), ("A", ["C"], 0), ("B", ["C"], 0), ("C", [], 0)],
        [0, 1, 1, 0, 0], 1, 2,
        [(0, 0, 3, 0, 0), (1, 1, 2, 1, 1), (1, 1, 3, 0, 1), (2, 1, 4, 0, 1), (3, 0, 4, 0, 0)],
        [0, 1, 1, 0, 0]),
    # T: [U]; M: push 1; first parent X outside the list -> slot1 None, the
    # secondary B takes the lowest free slot = M's own slot 1 (:441-458),
    # [U,B]; U frees 0 -> [_,B]; B frees 1.
    "secondary_reuses_own_slot": (
        [("T", ["U"], 0), ("M", ["X", "B"], 0), ("U", [], 0), ("B", [], 0)],
        [0, 1, 0, 1], 1, 2,
        [(0, 0, 2, 0, 0), (1, 1, 3, 1, 1)], [0, 1, 0, 1]),
    # A: slot0 B, secondaries C, D pushed to 1, 2: the peak counts the slots
    # update_lanes_for_parents set (:462-471), max_lane 2 at row 0.
    "octopus_peak_after_update": (
        [("A", ["B", "C", "D"], 0), ("B", ["E"], 0), ("C", ["E"], 0), ("D", ["E"], 0), ("E", [], 0)],
        [0, 0, 1, 2, 0], 2, 3,
        [(0, 0, 1, 0, 0), (0, 0, 2, 1, 0), (0, 0, 3, 2, 0), (1, 0, 4, 0, 0), (2, 1, 4, 0, 1), (3, 2, 4, 0, 2)],
        [0, 0, 1, 2, 0]),
    # C's first parent P is at an EARLIER row (clock skew re-sorted by time,
    # git/mod.rs:767-772): push 1, slot1 = P and nothing ever frees it; R
    # reuses slot 0.  The edge is still listed (:301-320).
    "parent_at_earlier_row_leaks": (
        [("P", ["Q"], 0), ("C", ["P"], 0), ("Q", [], 0), ("R", [], 0)],
        [0, 1, 0, 0], 1, 2,
        [(0, 0, 2, 0, 0), (1, 1, 0, 0, 1)], [0, 1, 0, 0]),
    # P: [_]; A: lane 0, slot0 Z, secondary P (earlier row) not present ->
    # push 1, leaked [Z,P]; B: push 2, slot2 Z, secondary P already held
    # (slot 1) -> no allocation, [Z,P,Z] max 2; Z frees 2, [_,P,_].
    "leaky_secondary_deduplicated": (
        [("P", [], 0), ("A", ["Z", "P"], 0), ("B", ["Z", "P"], 0), ("Z", [], 0)],
        [0, 0, 2, 0], 2, 3,
        [(1, 0, 3, 0, 0), (1, 0, 0, 0, 0), (2, 2, 3, 0, 2), (2, 2, 0, 0, 2)], [0, 0, 2, 0]),
    # S lists itself: slot0 = S after its own row, leaked; T pushes 1.
    "self_parent": (
        [("S", ["S"], 0), ("T", [], 0)],
        [0, 1], 0, 2,
        [(0, 0, 0, 0, 0)], [0, 1]),
    # seven tips waiting for R: lanes 0..6 (colour 6 % 6 = 0, :278-283), R
    # takes slot 0 and frees the other six.
    "seven_tips": (
        [(f"T{i}", ["R"], 0) for i in range(7)] + [("R", [], 0)],
        [0, 1, 2, 3, 4, 5, 6, 0], 6, 7,
        [(i, i, 7, 0, i % 6) for i in range(7)], [0, 1, 2, 3, 4, 5, 0, 0]),
    # A repeats B (the secondary is present: no allocation) — two edges; B's
    # parent X is outside the list -> slot None, no edge; C (orphan) takes
    # slot 0 and gets ORPHAN_COLOR (6).
    "repeated_and_outside_parents_orphan": (
        [("A", ["B", "B"], 0), ("B", ["X"], 0), ("C", [], 1)],
        [0, 0, 0], 0, 1,
        [(0, 0, 1, 0, 0), (0, 0, 1, 0, 0)], [0, 0, 6]),
    # A:[C] B:[C] -> [C,C]; C frees 1 -> [E,_]; D: lowest free is slot 1
    # (not a push) -> [E,E]; E frees 1.
    "freed_slot_reused": (
        [("A", ["C"], 0), ("B", ["C"], 0), ("C", ["E"], 0), ("D", ["E"], 0), ("E", [], 0)],
        [0, 1, 0, 1, 0], 1, 2,
        [(0, 0, 2, 0, 0), (1, 1, 2, 0, 1), (2, 0, 4, 0, 0), (3, 1, 4, 0, 1)], [0, 1, 0, 1, 0]),
}


def oid_of(name: str) -> bytes:
    b = name.encode()
    return (b + b"\x00" * 20)[:19] + bytes([len(b)])


def case_dag(rows) -> Dag:
    n = len(rows)
    oid = np.array([list(oid_of(r[0])) for r in rows], np.uint8).reshape(n, 20)
    time = (1_700_000_000 - 3600 * np.arange(n)).astype(np.int64)
    poff = np.zeros(n + 1, np.uint32)
    pids = []
    for i, r in enumerate(rows):
        pids += [oid_of(p) for p in r[1]]
        poff[i + 1] = len(pids)
    poid = np.array([list(p) for p in pids], np.uint8).reshape(-1, 20) if pids else np.zeros((0, 20), np.uint8)
    flags = np.array([r[2] for r in rows], np.uint8)
    return Dag(oid, time, poff, poid, flags, np.zeros(n, np.float32))


def expected(name):
    rows, lanes, max_lane, n_slots, edges, colors = CASES[name]
    return (np.array(lanes, np.uint32), max_lane, n_slots,
            np.array(edges, np.uint32).reshape(-1, 5), np.array(colors, np.uint8))


def test_at_least_eight_cases_cover_the_rules():
    assert len(CASES) >= 8


@pytest.mark.parametrize("name", sorted(CASES))
def test_c_oracle_matches_hand_worked(name):
    from oracle import oracle_c
    d = case_dag(CASES[name][0])
    lanes, max_lane, n_slots, edges, colors = expected(name)
    o = oracle_c.OracleLayout(d)
    assert o.lane.tolist() == lanes.tolist()
    assert (o.max_lane, o.n_slots) == (max_lane, n_slots)
    assert o.edges.view(np.uint32).reshape(-1, 5).tolist() == edges.tolist()
    assert o.color.tolist() == colors.tolist()


@pytest.mark.parametrize("name", sorted(CASES))
def test_py_oracle_matches_hand_worked(name):
    from oracle import oracle_py as P
    d = case_dag(CASES[name][0])
    lanes, max_lane, n_slots, edges, colors = expected(name)
    commits = P.commits_from_soa(d.oid, d.time, d.parent_off, d.parent_oid, d.flags)
    g = P.GraphLayout()
    g.build(commits)
    assert [g.get(c["id"])[0] for c in commits] == lanes.tolist()
    assert [g.get(c["id"])[1] for c in commits] == colors.tolist()
    assert (g.max_lane, len(g.active_lanes)) == (max_lane, n_slots)
    assert [list(e) for e in g.edges] == edges.tolist()


def test_seven_tips_clamps_x_to_the_visible_lanes():
    """lane_center_x (:786-790): lane 6 draws at min(6, 5) * 24 + 12 = 132.
    Row 6's node fan centre is (132, 14); nothing of the row lies right of the
    clamped node's edge (132 + NODE_RADIUS)."""
    from oracle import oracle_c
    d = case_dag(CASES["seven_tips"][0])
    o = oracle_c.OracleLayout(d)
    o.row_geometry(None)
    v, off = o.emit_vertices(6, 7)
    xy = np.stack([v["x"], v["y"]], 1)
    assert ((xy[:, 0] == 132.0) & (xy[:, 1] == 14.0)).any()
    assert xy[:, 0].max() <= 137.0
    assert o.graph_width == np.float32(144.0)   # min(max_lane + 1, 6) * 24 (:353-354)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_matches_hand_worked(engine, name):
    d = case_dag(CASES[name][0])
    lanes, max_lane, n_slots, edges, colors = expected(name)
    try:
        for general in (True, False):
            engine.set_lane_path(general)
            engine.build(d)
            s = engine.layout_summary()
            assert s.lane_path == (1 if general else 0)
            lane, color = engine.lanes()
            assert lane.tolist() == lanes.tolist()
            assert color.tolist() == colors.tolist()
            assert (s.max_lane, s.n_slots) == (max_lane, n_slots)
            e = engine.edges()
            got = e.view(np.uint32).reshape(-1, 5) if len(e) else np.zeros((0, 5), np.uint32)
            assert got.tolist() == edges.tolist()
    finally:
        engine.set_lane_path(False)
