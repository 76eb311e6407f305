"""The emission's two rates: a time series of emission-only
calls in one process, to set beside a clock / power log taken at the same
time by another process (profiles/emit_modes.sh).  Each line: wall time
since start, the call's k_vtx_tile time by HIP events (ms).
With a second argument E > 1 it instead builds E engines (each with its own
vertex and frame buffers) in the one process and times their emission in
turn, to see whether the rate follows the buffers' placement; a third argument
"placeK" gives the odd-numbered engines WG_OPT_VTX_PLACE = K (the even ones one
plain allocation); "realloc" (plain allocations) reallocates every engine's vertex
buffer alone half-way through (inputs and frame buffers stay put).
usage: python3 profiles/emit_modes.py [seconds] [engines] [placeK|realloc] > gpurun_out/<tag>_emit_series.jsonl"""
import ctypes
import json
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
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    dev = torch.device("cuda", 0)
    d = synth.generate("wide16", 1_000_000)
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1), d.flags, d.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    n_eng = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    engs = []
    contig = sys.argv[3] if len(sys.argv) > 3 else ""
    realloc = contig == "realloc"
    for k in range(n_eng):
        eng = wgraph.Engine(0)
        eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        if contig.startswith("place"):   # odd engines K candidates, even ones a plain allocation
            eng._check(wgraph.lib().wg_set_option(eng._ctx, 15, int(contig[5:]) if k % 2 else 1))   # WG_OPT_VTX_PLACE
        elif contig == "realloc":
            eng._check(wgraph.lib().wg_set_option(eng._ctx, 15, 1))
        eng.build_frame(commits=c, device_ptr=keep[5].data_ptr())
        eng.emit_vertices(0, d.n, selected=7)
        engs.append(eng)
    torch.cuda.synchronize()
    t0 = time.time()
    views = []
    for eng in engs:
        v = eng.device_views()
        views.append({k: int(getattr(v, k) or 0) for k, _ in type(v)._fields_})
        n_p, kept, pms = ctypes.c_uint32(), ctypes.c_uint32(), (ctypes.c_float * 8)()
        eng._check(wgraph.lib().wg_vertex_placement_get(eng._ctx, ctypes.byref(n_p), ctypes.byref(kept), pms))
        views[-1]["place"] = [n_p.value, kept.value, [round(x, 4) for x in pms[:n_p.value]]]
    print(json.dumps({"t0_unix": t0, "engines": n_eng, "mode": contig, "n_vertices": int(engs[0].vertex_summary().n_vertices),
                      "views": views}), flush=True)
    phase = 0
    while time.time() - t0 < secs:
        if phase == 0 and realloc and time.time() - t0 > secs / 2:
            # phase 1: only the vertex buffers move (reallocated in reverse order), the inputs stay
            phase = 1
            for eng in reversed(engs):
                eng._check(wgraph.lib().wg_set_option(eng._ctx, 15, 1))   # frees the vertex buffer
                eng.emit_vertices(0, d.n, selected=7)
            torch.cuda.synchronize()
            print(json.dumps({"phase": 1, "vertices": [int(e.device_views().vertices or 0) for e in engs]}), flush=True)
        for k, eng in enumerate(engs):
            eng.enable_timing(True, reserve=64)
            for _ in range(10):
                eng.emit_vertices(0, d.n, selected=7)
            torch.cuda.synchronize()
            ms = [t for name, t in eng.timings() if name == "vtx_emit"]
            eng.enable_timing(False)
            print(json.dumps({"t": round(time.time() - t0, 3), "engine": k, "phase": phase,
                              "emit_ms": [round(x, 4) for x in ms]}), flush=True)
    for eng in engs:
        eng.close()


if __name__ == "__main__":
    main()
