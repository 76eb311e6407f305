"""Is k_vtx_tile slower when other large buffers live on the device?

The shard emulation (emulate_shards.py) measures the emission stage at
~1.17 ms on every emulated rank against ~1.0 ms for the single-GPU step in
the same process, with equal vertex counts.  This probe times the single-GPU
step's emission stage (HIP events, emission-only) on one engine, then again
after other engines holding the same buffers exist, then on a new engine
created after them.

usage: python3 profiles/emit_probe.py [--rows 1000000] [--others 2] [--steps 5]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--others", type=int, default=2)
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    import torch
    import wgraph
    from wgraph import abi, synth
    dev = torch.device("cuda", 0)
    d = synth.generate("wide16", args.rows)
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1), d.flags, d.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)

    def step(e):
        e.build(commits=c)
        e.row_geometry(device_ptr=keep[5].data_ptr())
        e.emit_vertices(0, d.n, selected=7, palette=pal)

    def emit_ms(e):
        step(e)
        e.synchronize()
        wgraph.lib().wg_set_option(e._ctx, 4, 1)
        e.enable_timing(True, reserve=64 * args.steps)
        for _ in range(args.steps):
            step(e)
        e.synchronize()
        t = {}
        for name, ms in e.timings():
            t[name] = t.get(name, 0.0) + ms / args.steps
        e.enable_timing(False)
        return round(t.get("vtx_emit", float("nan")), 4)

    res = {}
    first = wgraph.Engine(0)
    res["first_alone"] = emit_ms(first)
    others = [wgraph.Engine(0) for _ in range(args.others)]
    res["others"] = [emit_ms(o) for o in others]
    res["first_again"] = emit_ms(first)
    last = wgraph.Engine(0)
    res["new_after_others"] = emit_ms(last)
    res["gpu_mem_used_GB"] = round(torch.cuda.mem_get_info()[1] / 1e9 - torch.cuda.mem_get_info()[0] / 1e9, 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
