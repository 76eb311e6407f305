"""Host time of a step's calls (enqueue cost, no synchronisation inside
except the emission's vertex-total read) against the step's wall time.

usage: python3 profiles/host_cost.py [--kind random13 --rows 100000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000)
    ap.add_argument("--kind", default="random13")
    ap.add_argument("--steps", type=int, default=30)
    args = ap.parse_args()
    import torch
    import wgraph
    from wgraph import abi, synth
    dev = torch.device("cuda", 0)
    d = synth.generate(args.kind, args.rows)
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1), d.flags, d.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    s = torch.cuda.Stream(dev)
    torch.cuda.set_stream(s)
    eng = wgraph.Engine(0)
    eng.set_stream(s.cuda_stream)
    eng.set_defer_validation(True)
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)
    for _ in range(5):
        eng.build_frame(commits=c, device_ptr=keep[5].data_ptr())
        eng.emit_vertices(0, d.n, selected=7, palette=pal)
    torch.cuda.synchronize()
    tb, te, tw = [], [], []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        eng.build_frame(commits=c, device_ptr=keep[5].data_ptr())
        t1 = time.perf_counter()
        eng.emit_vertices(0, d.n, selected=7, palette=pal)
        t2 = time.perf_counter()
        tb.append(t1 - t0)
        te.append(t2 - t1)
    torch.cuda.synchronize()
    # steps back to back (the bench's loop) for the wall time per step
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.build_frame(commits=c, device_ptr=keep[5].data_ptr())
        eng.emit_vertices(0, d.n, selected=7, palette=pal)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / args.steps
    # the bare ctypes + engine entry cost: a call that launches nothing
    t0 = time.perf_counter()
    for _ in range(1000):
        eng.layout_summary()
    q = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"kind": args.kind, "rows": args.rows, "build_frame_call_ms": round(1e3 * float(np.median(tb)), 4),
                      "emit_call_ms": round(1e3 * float(np.median(te)), 4), "step_wall_ms": round(wall, 4),
                      "summary_call_us": round(q, 3)}))


if __name__ == "__main__":
    main()
