"""BASELINE config C5 at its full size: the 8M-commit wide synthetic DAG
(<= 16 lanes) sharded 8 ways, every rank checked against the CPU oracle.

Eight engine contexts on one GPU run the row-sharded protocol in lockstep
(tests/test_gpu_shard.py::_lockstep: slots packed by wg_shard_pack_slot in
stream order and gathered side by side — the device-transport path bench.py
takes over RCCL, without the collective itself).  Each rank's lanes, colours,
row_top at its end row, vertex count and whole vertex-buffer checksum must
equal tests/golden/c5_shards.json, which the C oracle produced by emitting
that rank's rows in 100k-row pieces (tests/golden/make_c5_golden.py).
"""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c5_eight_shards_full_size():
    import torch
    import wgraph
    from wgraph import abi, lib, synth
    from test_gpu_shard import _lockstep

    with open(os.path.join(ROOT, "tests", "golden", "c5_shards.json")) as f:
        gold = json.load(f)
    n, world = gold["rows"], gold["world"]
    d = synth.generate(gold["preset"], n, seed=gold["seed"])
    dev = torch.device("cuda", 0)
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1), d.flags, d.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    # a non-default stream shared by the engines and torch (the default
    # stream's handle 0 would give each engine a stream of its own, unordered
    # with torch's reads of the packed slots)
    ts = torch.cuda.Stream(dev)
    ts.wait_stream(torch.cuda.current_stream(dev))
    stream_ctx = torch.cuda.stream(ts)
    stream_ctx.__enter__()
    engines = [wgraph.Engine(0) for _ in range(world)]
    try:
        for e in engines:
            e.set_stream(ts.cuda_stream)
        rng = [(g["row_begin"], g["row_end"]) for g in gold["ranks"]]
        _lockstep(engines, lambda e, r, m: lib().wg_shard_build_begin(e._ctx, ctypes.byref(c), world, r,
                                                                       rng[r][0], rng[r][1], m))
        _lockstep(engines, lambda e, r, m: lib().wg_shard_geometry_begin(e._ctx, keep[5].data_ptr(), abi.WG_DEVICE, m))
        for r, e in enumerate(engines):
            g = gold["ranks"][r]
            s, t = rng[r]
            assert int(e.debug_counters()[5]) == 1, f"rank {r}: the sharded path was not taken"
            assert e.layout_summary().max_lane == gold["max_lane"]
            lane, color = e.lanes()
            assert hashlib.sha256(lane.astype(np.uint32).tobytes()).hexdigest() == g["lane_sha256"], f"rank {r} lanes"
            assert hashlib.sha256(color.tobytes()).hexdigest() == g["color_sha256"], f"rank {r} colours"
            rt = e.geometry()["row_top"]
            assert int(rt[-1:].view(np.uint32)[0]) == g["row_top_end_bits"], f"rank {r} row_top_y[{t}]"
            e.emit_vertices(s, t, selected=gold["selected"])
            vs = e.vertex_summary()
            assert vs.n_vertices == g["n_vertices"], f"rank {r} vertex count"
            assert f"{vs.checksum:#018x}" == g["checksum"], f"rank {r} vertex checksum"
    finally:
        for e in engines:
            e.close()
        stream_ctx.__exit__(None, None, None)
        del keep
        torch.cuda.empty_cache()
