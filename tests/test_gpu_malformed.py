"""Randomised malformed lists through the speculative build, the deferred
validation and the frame call (kernels are queued before
the host knows whether a list is well formed).  Each list mixes what the
reference accepts without complaint (commit_graph.rs:272-320, 401-471):
duplicate ids (the last row wins, :273-274), parents at earlier rows and at
the row itself, parents not in the list (:306-311), a parent named twice,
rows without parents, long and short edges, synthetic rows.  One context
walks them all, alternating the validation modes, and every build is
bit-exact against the oracle: lanes, colours, edges, both geometries and the
vertex buffer's checksum."""
import numpy as np
import pytest

from test_gpu_spec import full_check
from wgraph import synth

pytestmark = pytest.mark.gpu


def _malformed(rng, n):
    base = synth.generate("random13", n, seed=int(rng.integers(1 << 30)))
    oid = base.oid.copy()
    k = int(rng.integers(1, max(2, n // 40)))
    oid[rng.integers(0, n, k)] = oid[rng.integers(0, n, k)]          # duplicate ids
    counts = rng.integers(1, 3, n).astype(np.int64)
    counts[rng.random(n) < 0.05] = 0
    po = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint32)
    e = int(po[-1])
    rows = np.repeat(np.arange(n), counts)
    far = rng.random(e) < 0.02
    later = np.minimum(rows + np.where(far, rng.integers(64, 5000, e), rng.integers(1, 64, e)), n - 1)
    earlier = (rows - rng.integers(0, 300, e)).clip(0, n - 1)        # includes the row itself
    pick = rng.random(e)
    target = np.where((pick < 0.99) | (pick > 0.996), later, earlier)
    parents = oid[target].copy()
    missing = pick > 0.996                                           # ids not in the list
    parents[missing] = rng.integers(0, 256, (int(missing.sum()), 20), dtype=np.uint8)
    rep = np.flatnonzero((pick > 0.97) & (pick <= 0.99))              # a parent named twice in its row
    for j in rep:
        if j > 0 and rows[j - 1] == rows[j]:
            parents[j] = parents[j - 1]
    flags = base.flags.copy()
    flags[rng.random(n) < 0.02] |= 2                                 # synthetic rows (WG_FLAG_SYNTHETIC)
    return synth.Dag(oid, base.time.copy(), po, parents, flags, base.band.copy())


def test_random_malformed_lists():
    import wgraph
    from oracle import oracle_c
    rng = np.random.default_rng(2024)
    eng = wgraph.Engine(0)
    try:
        sizes = [500, 3000, 3000, 6000, 1200, 6000, 4000, 300] + [int(x) for x in rng.integers(200, 6000, 8)]
        for i, n in enumerate(sizes):
            d = _malformed(rng, n)
            o = oracle_c.OracleLayout(d)
            eng.set_defer_validation(i % 2 == 1)
            if i % 3 == 2:   # the frame call: the build's geometry pass takes the bands
                eng.build_frame(d, band=d.band)
                og = o.row_geometry(d.band)
                got = eng.geometry()
                for key, v in og.items():
                    assert (got[key].tobytes() == v.tobytes()), f"#{i} frame {key}"
            eng.build(d)
            full_check(eng, d, o, f"#{i} malformed/{n}")
            o.close()
        c = eng.debug_counters()
        assert int(c[6]) >= len(sizes) - 1   # every build after the first speculated
    finally:
        eng.close()


@pytest.mark.parametrize("world,n,seed", [(2, 3000, 1), (3, 5000, 2), (4, 2500, 3)])
def test_random_malformed_lists_sharded(world, n, seed):
    """The same lists on row shards in lockstep (whatever mode the engines
    settle on: sharded, or the whole list where it must be), every rank
    bit-exact against the oracle."""
    from test_gpu_shard import _lockstep_build_check
    rng = np.random.default_rng(4242 + seed)
    _lockstep_build_check(_malformed(rng, n), world, None)
