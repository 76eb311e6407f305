"""A/B of one engine option on the full step (build_frame + emission, inputs
in HBM) of small and mid-size lists, alternated in one process so the box's
drift cancels: python3 profiles/small_step_ab.py [option] [steps] [pairs]

option: join_fused (the id table's place pass inside the window probe, settle
on the main stream; default off) — prints one JSON line per (list, setting)
with the median ms/step over the pairs."""
import json
import os
import statistics
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.environ.get("WG_PKG_DIR") or os.path.join(HERE, "..", "whisper-git_amd"))

LISTS = [("linear", 10_000), ("random13", 100_000), ("random13", 250_000), ("wide16", 250_000),
         ("wide16", 500_000), ("wide16", 1_000_000)]


def main():
    import torch
    import wgraph
    from wgraph import abi, synth
    opt = sys.argv[1] if len(sys.argv) > 1 else "join_fused"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    pairs = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    dev = torch.device("cuda", 0)
    for kind, n in LISTS:
        d = synth.generate(kind, n)
        keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                       d.parent_oid.reshape(-1), d.flags, d.band)]
        c = abi.Commits()
        c.n_commits, c.n_parents = d.n, d.e
        c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
        c.residency = abi.WG_DEVICE
        engs = {}
        for on in (False, True):
            e = wgraph.Engine(0)
            e.set_stream(torch.cuda.current_stream(dev).cuda_stream)
            getattr(e, "set_" + opt)(on)
            engs[on] = e
        ms = {False: [], True: []}
        for _ in range(pairs):
            for on in (False, True):
                e = engs[on]
                for _ in range(5):
                    e.build_frame(commits=c, device_ptr=keep[5].data_ptr())
                    e.emit_vertices(0, d.n, selected=7)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    e.build_frame(commits=c, device_ptr=keep[5].data_ptr())
                    e.emit_vertices(0, d.n, selected=7)
                torch.cuda.synchronize()
                ms[on].append((time.perf_counter() - t0) * 1e3 / steps)
        for on in (False, True):
            print(json.dumps({"list": kind, "rows": n, opt: on, "ms_per_step": round(statistics.median(ms[on]), 4),
                              "runs": [round(x, 4) for x in ms[on]],
                              "n_vertices": int(engs[on].vertex_summary().n_vertices)}), flush=True)
        for e in engs.values():
            e.close()
        del keep


if __name__ == "__main__":
    main()
