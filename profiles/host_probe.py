"""Host time per step (API calls + syncs inside the engine) against the GPU
step time: python3 profiles/host_probe.py"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    import torch
    import wgraph
    from wgraph import abi, synth
    dev = torch.device("cuda", 0)
    d = synth.generate("wide16", 1_000_000)
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1), d.flags, d.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    eng = wgraph.Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)
    tb, tg, te = [], [], []
    for it in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.build(commits=c)
        t1 = time.perf_counter()
        eng.row_geometry(device_ptr=keep[5].data_ptr())
        t2 = time.perf_counter()
        eng.emit_vertices(0, d.n, selected=7, palette=pal)
        t3 = time.perf_counter()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if it >= 5:
            tb.append(t1 - t0); tg.append(t2 - t1); te.append(t3 - t2)
            print(f"build {1e3*(t1-t0):.3f} geom {1e3*(t2-t1):.3f} emit-call {1e3*(t3-t2):.3f} "
                  f"tail-wait {1e3*(t4-t3):.3f} total {1e3*(t4-t0):.3f} ms", flush=True)
    print(f"median host ms: build {1e3*np.median(tb):.3f} geom {1e3*np.median(tg):.3f} emit {1e3*np.median(te):.3f}")


if __name__ == "__main__":
    main()
