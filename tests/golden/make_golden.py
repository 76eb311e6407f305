"""Generate the committed golden fixtures under tests/golden/.

The reference (Rust + libgit2 + Vulkan) cannot be built or run in this
container, so no reference-produced vectors exist.
Fixtures are produced by the C oracle (oracle/wg_oracle.c) and accepted only
if the independent numpy restatement (oracle/oracle_py.py) reproduces every
output bit for bit.  Inputs are hand-built DAGs covering the edge cases the
reference tolerates (merges, octopus merges, duplicate first parents,
orphans whose parent sits at an earlier row, a secondary parent reusing the
committing row's own slot, > 6 lanes, duplicate ids, self parents) plus
seeded synthetic DAGs.

Run:  python tests/golden/make_golden.py      (rewrites tests/golden/*.npz)
"""
from __future__ import annotations

import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))
sys.path.insert(0, ROOT)

from wgraph import abi, synth  # noqa: E402
from wgraph import commits_to_soa  # noqa: E402
from oracle import oracle_c, oracle_py as P  # noqa: E402


def oid(name: str) -> bytes:
    return hashlib.sha1(name.encode()).digest()


def dag_from_spec(spec, t0=1_700_000_000):
    """spec: list of (name, [parent names], dt_seconds, orphan)."""
    commits = []
    t = t0
    for name, parents, dt, orphan in spec:
        t -= dt
        commits.append(dict(id=oid(name), time=t, parents=[oid(p) for p in parents], orphan=orphan))
    d = commits_to_soa(commits)
    return d


HAND = {
    # 0: merge commit, 1/2: both sides, 3: base
    "merge_basic": [("M", ["B", "C"], 0, False), ("B", ["D"], 600, False), ("C", ["D"], 4000, False),
                    ("D", [], 90000, False)],
    "octopus": [("O", ["A", "B", "C", "D"], 0, False), ("A", ["E"], 60, False), ("B", ["E"], 60, False),
                ("C", ["E"], 60, False), ("D", ["E"], 60, False), ("E", [], 7200, False)],
    # two children share a first parent (duplicate waiters freed, :287-291)
    "dup_first_parent": [("X", ["P"], 0, False), ("Y", ["P"], 30, False), ("P", ["Q"], 86400, False),
                         ("Q", [], 100, False)],
    # orphan re-sorted by time lands below its parent (git/mod.rs:767-772):
    # its lane waits forever and its edge is skipped (:526-528)
    "orphan_skew": [("A", ["B"], 0, False), ("B", ["C"], 500, False), ("O", ["A"], 10, True),
                    ("C", [], 3600, False)],
    # first parent outside the list frees the row's own slot before the
    # secondary is placed, so the secondary reuses it (:441-445, :454)
    "secondary_reuses_slot": [("T", ["Q"], 0, False), ("M", ["Z_outside", "B"], 100, False),
                              ("B", ["C"], 200, False), ("Q", ["C"], 300, False), ("C", [], 400, False)],
    # ten tips converge: lanes beyond LANE_COUNT_VISUAL clamp to the right (:786-790, :846-850)
    "wide_lanes": [(f"t{k}", ["base"], 1000 * k, False) for k in range(10)] + [("base", [], 5000000, False)],
    # a duplicated id: last occurrence wins in row_by_oid / layouts (:273-274, :283)
    "dup_ids": [("A", ["B"], 0, False), ("B", ["C"], 10, False), ("A", ["C"], 20, False), ("C", [], 30, False)],
    "self_parent": [("S", ["S", "R"], 0, False), ("R", [], 50, False)],
    "empty": [],
    "single": [("only", [], 0, False)],
    "repeated_parent": [("M", ["A", "B", "B", "A"], 0, False), ("A", ["C"], 10, False), ("B", ["C"], 10, False),
                        ("C", [], 10, False)],
}


def outputs(d, band, selected):
    o = oracle_c.OracleLayout(d)
    out = dict(max_lane=np.uint32(o.max_lane), n_slots=np.uint32(o.n_slots),
               graph_width=np.float32(o.graph_width), lane=o.lane, color=o.color,
               edges=o.edges.view(np.uint32).reshape(-1, 5) if len(o.edges) else np.zeros((0, 5), np.uint32),
               heights=o.heights)
    for k, v in o.geometry.items():
        out["build_" + k] = v
    gb = o.row_geometry(band)
    for k, v in gb.items():
        out["band_" + k] = v
    v, off = o.emit_vertices(0, d.n, selected=selected)
    out["vertices"] = v.view(np.float32).reshape(-1, 6) if len(v) else np.zeros((0, 6), np.float32)
    out["vtx_off"] = off
    out["selected"] = np.int64(selected)
    o.close()
    return out


def crosscheck(d, band, selected, out):
    """Independent numpy restatement must agree bit for bit."""
    commits = P.commits_from_soa(d.oid, d.time, d.parent_off, d.parent_oid, d.flags)
    g = P.GraphLayout()
    g.build(commits)
    lanes = np.array([g.get(c["id"])[0] for c in commits], np.uint32)
    cols = np.array([g.get(c["id"])[1] for c in commits], np.uint8)
    assert (lanes == out["lane"]).all() and (cols == out["color"]).all()
    assert g.max_lane == int(out["max_lane"])
    assert np.float32(g.graph_width) == out["graph_width"] or d.n == 0
    pe = np.array(g.edges, dtype=np.uint32).reshape(-1, 5)
    assert (pe == out["edges"]).all()
    fb = P.flatten_geometry(g.row_geometry, g.row_top_y)
    for k, v in fb.items():
        assert v.tobytes() == out["build_" + k].tobytes(), k
    geom, rt = g.row_geometry_with_bands(commits, list(band))
    fg = P.flatten_geometry(geom, rt)
    for k, v in fg.items():
        assert v.tobytes() == out["band_" + k].tobytes(), k
    verts = []
    for r in range(d.n):
        lc = g.get(commits[r]["id"])
        verts += P.emit_row_vertices(geom[r], lc[0], lc[1], r == selected, g.graph_width, abi.DEFAULT_PALETTE)
    pv = np.array(verts, np.float32).reshape(-1, 6)
    assert pv.tobytes() == out["vertices"].tobytes()


HEAD_ROWS = 40


def save_case(name, d, band, selected):
    out = outputs(d, band, selected)
    if d.n <= 3000:
        crosscheck(d, band, selected, out)
    # keep fixtures small: full vertex buffers only for hand-built DAGs;
    # larger cases keep rows [0, HEAD_ROWS) plus a checksum of all vertices
    v = out["vertices"]
    out["vertex_checksum"] = np.uint64(oracle_c.vertex_checksum(v.view(abi.VERTEX_DTYPE).reshape(-1)))
    if d.n > 100:
        out["vertices"] = v[: int(out["vtx_off"][HEAD_ROWS])]
        out["vertices_head_rows"] = np.int64(HEAD_ROWS)
    else:
        out["vertices_head_rows"] = np.int64(d.n)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), oid=d.oid, time=d.time, parent_off=d.parent_off,
                        parent_oid=d.parent_oid, flags=d.flags, band=band, **out)
    print(f"{name}: n={d.n} edges={len(out['edges'])} max_lane={int(out['max_lane'])} "
          f"vert={len(out['band_vert'])} curves={len(out['band_curve'])} vertices={len(out['vertices'])}")


def main():
    for name, spec in HAND.items():
        d = dag_from_spec(spec)
        band = np.zeros(d.n, np.float32)
        band[::3] = 30.0   # PILLS_BAND_HEIGHT on every third row (:106)
        save_case(name, d, band, selected=min(1, d.n - 1) if d.n else -1)
    for kind, n in (("anomaly", 64), ("anomaly", 600), ("random13", 1000), ("linux", 1000), ("wide16", 1000),
                    ("linear", 300)):
        d = synth.generate(kind, n)
        save_case(f"{kind}_{n}", d, d.band, selected=n // 2)


if __name__ == "__main__":
    main()
