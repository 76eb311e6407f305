"""One BASELINE config's full step (build + banded geometry + emission) a few
times, for profiling: python3 profiles/config_step.py <kind> <rows> [steps]"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    import torch
    import wgraph
    from wgraph import abi, synth
    kind, n = sys.argv[1], int(sys.argv[2])
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda", 0)
    d = synth.generate(kind, n)
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1), d.flags, d.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    eng = wgraph.Engine(0)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    eng.enable_timing(True, reserve=64 * (steps + 1))
    for _ in range(steps):
        eng.build(commits=c)
        eng.row_geometry(device_ptr=keep[5].data_ptr())
        eng.emit_vertices(0, d.n, selected=7)
    torch.cuda.synchronize()
    st = {}
    for name, ms in eng.timings():
        st[name] = st.get(name, 0.0) + ms / steps
    g = eng.geometry_summary()
    print({k: round(v, 4) for k, v in st.items()}, "n_vert", g.n_vert, "n_curve", g.n_curve,
          "debug", [int(x) for x in eng.debug_counters()[:8]], flush=True)


if __name__ == "__main__":
    main()
