"""Time the vertex emission (k_vtx_tile) of one engine build on several
workloads: one JSON line per (library, workload).  The library is picked by
WGRAPH_LIB (a variant build of libwgraph.so, e.g. another tile size); run
once per variant.

usage: WGRAPH_LIB=path/to/lib.so python3 profiles/emit_variants.py [--steps 6] [--tag name]
           [--work wide16:1000000,linux:1300000]
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
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--tag", default=os.environ.get("WGRAPH_LIB", "default"))
    ap.add_argument("--work", default="wide16:1000000,linux:1300000")
    ap.add_argument("--checksum", action="store_true", help="also print the vertex buffer checksum")
    args = ap.parse_args()
    import torch
    import wgraph
    from wgraph import abi, synth
    dev = torch.device("cuda", 0)
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)
    for item in args.work.split(","):
        kind, n = item.split(":")
        d = synth.generate(kind, int(n))
        keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                       d.parent_oid.reshape(-1), d.flags, d.band)]
        c = abi.Commits()
        c.n_commits, c.n_parents = d.n, d.e
        c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
        c.residency = abi.WG_DEVICE
        eng = wgraph.Engine(0)
        eng.build(commits=c)
        eng.row_geometry(device_ptr=keep[5].data_ptr())
        for _ in range(2):
            eng.emit_vertices(0, d.n, selected=7, palette=pal)
        torch.cuda.synchronize()
        eng._check(wgraph.lib().wg_set_option(eng._ctx, 4, 1))   # WG_OPT_TIMING_EMIT_ONLY
        eng.enable_timing(True, reserve=64 * (args.steps + 1))
        for _ in range(args.steps):
            eng.emit_vertices(0, d.n, selected=7, palette=pal)
        torch.cuda.synchronize()
        ms = [t for name, t in eng.timings() if name == "vtx_emit"]
        eng.enable_timing(False)
        vs = eng.vertex_summary()
        gb = vs.n_vertices * 24 / 1e9
        out = {"tag": args.tag, "work": item, "vertices": int(vs.n_vertices), "emit_ms": round(float(np.median(ms)), 4),
               "emit_ms_min": round(float(np.min(ms)), 4), "write_TBps": round(gb / (float(np.median(ms)) * 1e-3) / 1e3, 3)}
        if args.checksum:
            out["checksum"] = hex(int(vs.checksum))
        print(json.dumps(out), flush=True)
        eng.close()
        del keep


if __name__ == "__main__":
    main()
