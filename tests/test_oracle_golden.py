"""CPU: the oracle against the committed golden fixtures, and the two
independent restatements against each other on fresh synthetic DAGs.

The fixtures were produced by the C oracle and accepted only after the numpy
restatement matched them bit for bit (tests/golden/make_golden.py).  Parity
with the reference itself is unpinned beyond the ported KATs
(test_oracle_kats.py): the reference cannot run here.
"""
import numpy as np
import pytest

from conftest import golden_names, load_golden
from oracle import oracle_c, oracle_py as P
from wgraph import abi, synth


@pytest.mark.parametrize("name", golden_names())
def test_c_oracle_reproduces_golden(name):
    d, g = load_golden(name)
    o = oracle_c.OracleLayout(d)
    assert o.max_lane == int(g["max_lane"])
    assert (o.lane == g["lane"]).all() and (o.color == g["color"]).all()
    e = o.edges.view(np.uint32).reshape(-1, 5) if len(o.edges) else np.zeros((0, 5), np.uint32)
    assert (e == g["edges"]).all()
    assert o.heights.tobytes() == g["heights"].tobytes()
    for k, v in o.geometry.items():
        assert v.tobytes() == g["build_" + k].tobytes(), k
    gb = o.row_geometry(g["band"])
    for k, v in gb.items():
        assert v.tobytes() == g["band_" + k].tobytes(), k
    v, off = o.emit_vertices(0, d.n, selected=int(g["selected"]))
    assert (off == g["vtx_off"]).all()
    head = int(g["vertices_head_rows"])
    vf = v.view(np.float32).reshape(-1, 6)[: int(off[head])] if d.n else np.zeros((0, 6), np.float32)
    assert vf.tobytes() == g["vertices"].tobytes()
    assert oracle_c.vertex_checksum(v) == int(g["vertex_checksum"])


@pytest.mark.parametrize("kind,n,seed", [("anomaly", 300, 7), ("random13", 300, 11), ("linux", 300, 3),
                                         ("wide16", 300, 5), ("anomaly", 150, 99)])
def test_restatements_agree(kind, n, seed):
    d = synth.generate(kind, n, seed=seed)
    o = oracle_c.OracleLayout(d)
    commits = P.commits_from_soa(d.oid, d.time, d.parent_off, d.parent_oid, d.flags)
    g = P.GraphLayout()
    g.build(commits)
    assert g.max_lane == o.max_lane
    assert (np.array([g.get(c["id"])[0] for c in commits], np.uint32) == o.lane).all()
    pe = np.array(g.edges, np.uint32).reshape(-1, 5)
    assert (pe == o.edges.view(np.uint32).reshape(-1, 5)).all()
    geom, rt = g.row_geometry_with_bands(commits, list(d.band))
    fg = P.flatten_geometry(geom, rt)
    og = o.row_geometry(d.band)
    for k, v in fg.items():
        assert v.tobytes() == og[k].tobytes(), k
    v, off = o.emit_vertices(0, 60, selected=5)
    pv = []
    for r in range(60):
        lc = g.get(commits[r]["id"])
        pv += P.emit_row_vertices(geom[r], lc[0], lc[1], r == 5, g.graph_width, abi.DEFAULT_PALETTE)
    assert np.array(pv, np.float32).tobytes() == v.view(np.float32).tobytes()


def test_rs_round_is_half_away_from_zero():
    assert P.rs_round(np.float32(0.5)) == 1.0
    assert P.rs_round(np.float32(1.5)) == 2.0
    assert P.rs_round(np.float32(2.5)) == 3.0
    assert P.rs_round(np.float32(-0.5)) == -1.0
    assert P.rs_round(np.float32(44.49999)) == 44.0
