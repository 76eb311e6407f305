"""GPU row order (wg_order_rows) against the oracle, index for index:
commit_graph_with_orphans' stable time re-sort (git/mod.rs:761-775) and
insert_synthetics_sorted (git/mod.rs:234-242), host and device inputs."""
import numpy as np
import pytest

from oracle.order_oracle import order_rows
from wgraph import synth

pytestmark = pytest.mark.gpu


def _cases():
    rng = np.random.default_rng(3)
    d = synth.generate("linux", 20000, seed=4)
    t = d.time
    yield "walk only", t, [], []
    yield "linux + orphans", t, np.sort(rng.choice(t, 100))[::-1], []
    yield "orphans + synthetics", t, np.sort(rng.choice(t, 50))[::-1], np.concatenate(
        [rng.choice(t, 6), [t.max() + 5, t.min() - 5, t[100], t[100]]])
    yield "ties everywhere", rng.integers(0, 5, 5000), rng.integers(0, 5, 40), rng.integers(-1, 6, 64)
    yield "int64 extremes", np.array([2**62, -2**62, 0, 2**63 - 1, -2**63, 5]), np.array([2**63 - 1, -2**63]), \
        np.array([-2**63, 2**63 - 1, 0])
    yield "synthetics only", [], [], [3, 1, 2, 2, 9]
    yield "empty", [], [], []
    yield "one orphan", [7], [9], []


@pytest.mark.parametrize("case", list(_cases()), ids=lambda c: c[0])
def test_order_rows_equal_oracle(engine, case):
    _, w, o, s = case
    want = order_rows(w, o, s)
    got = engine.order_rows(w, o, s)
    assert got.tolist() == want.tolist()


def test_order_rows_device_resident(engine):
    import torch
    rng = np.random.default_rng(8)
    w = rng.integers(1_600_000_000, 1_700_000_000, 300_000)
    o = np.sort(rng.integers(1_600_000_000, 1_700_000_000, 100))[::-1].copy()
    s = rng.integers(1_600_000_000, 1_700_000_000, 5)
    tw, to, ts = (torch.from_numpy(a).cuda() for a in (w, o, s))
    out = torch.empty(w.size + o.size + s.size, dtype=torch.int32, device="cuda")
    engine.order_rows(None, device=((tw.data_ptr(), w.size), (to.data_ptr(), o.size), (ts.data_ptr(), s.size)),
                      out_device_ptr=out.data_ptr())
    torch.cuda.synchronize()
    want = np.argsort(-np.concatenate([w, o]), kind="stable")   # the same stable sort, numpy's own
    got = out.cpu().numpy().view(np.uint32)
    assert got.tolist() == order_rows(w, o, s).tolist()
    assert np.array_equal(np.delete(got, np.flatnonzero(got >= w.size + o.size)), want)
