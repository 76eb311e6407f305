"""Lane-replay chunk size sweep (WG_OPT_REPLAY_CHUNK) on the bench workload:
per chunk size, the build's lf_loop stage and the whole step.

usage: python3 profiles/tune_replay.py [--rows 1000000] [--kind wide16]
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
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--kind", default="wide16")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--chunks", default="64,128,192,256,384,512,1024",
                    help="chunk sizes, or chunk:warm pairs (WG_OPT_REPLAY_WARMUP)")
    args = ap.parse_args()
    import torch
    import wgraph
    from wgraph import abi, lib, synth
    dev = torch.device("cuda", 0)
    dag = synth.generate(args.kind, args.rows)
    keep = [torch.from_numpy(a).to(dev) for a in (dag.oid.reshape(-1), dag.time, dag.parent_off.view(np.int32),
                                                   dag.parent_oid.reshape(-1), dag.flags, dag.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = dag.n, dag.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    ref = None
    for spec in args.chunks.split(","):
        # "auto": the engine's own choice (short chunk, long after a slow list)
        auto = spec == "auto"
        ch, warm = (0, 0) if auto else ((int(v) for v in spec.split(":")) if ":" in spec else (int(spec), 0))
        # a fresh engine per chunk size: the replay's blind iteration count
        # adapts per context and must not carry over from another chunk size
        eng = wgraph.Engine(0)
        eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        if not auto:
            eng._check(lib().wg_set_option(eng._ctx, 2, ch))
            eng._check(lib().wg_set_option(eng._ctx, 6, warm))
        eng.set_defer_validation(True)

        def step():
            eng.build_frame(commits=c, device_ptr=keep[5].data_ptr())
            eng.emit_vertices(0, dag.n, selected=7)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        cold = (time.perf_counter() - t0) * 1e3
        for _ in range(2):
            step()
        torch.cuda.synchronize()
        eng.enable_timing(True, reserve=64 * (args.steps + 1))
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        st = {}
        for name, t in eng.timings():
            st[name] = st.get(name, 0.0) + t / args.steps
        eng.enable_timing(False)
        lane, _ = eng.lanes()
        same = True if ref is None else bool((lane == ref).all())
        ref = lane if ref is None else ref
        dbg = eng.debug_counters()
        print(json.dumps({"kind": args.kind, "rows": args.rows, "chunk": "auto" if auto else ch, "warm": warm,
                          "cold_ms": round(cold, 3), "step_ms": round(ms, 4), "lf_loop_ms": round(st.get("lf_loop", 0), 4),
                          "lanes_ms": round(st.get("lanes", 0), 4), "same_lanes": same,
                          "debug": [int(x) for x in dbg[:12]]}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
