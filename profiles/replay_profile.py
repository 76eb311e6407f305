"""Where does the lane-event replay (k_lf_replay) spend its time?  Runs the
bench step's build on BASELINE lists with a profiling build of the engine
(-DWG_REPLAY_PROFILE: per-iteration counters in the kernel) and prints, per
replay iteration of the last build: chunks, 64-event batches, batches that
took no scalar special event, scalar special events, of which merges with
more than two waiters, and the mean cycles per chunk spent in total / in the
scalar loop / in those merges.

usage: WGRAPH_LIB=profiles/librp_profile.so python3 profiles/replay_profile.py [kind rows]...
(profiles/librp_profile.so: hipcc ... -DWG_REPLAY_PROFILE -shared whisper-git_amd/csrc/*.hip)

The engine is held on the chunked replay (WG_OPT_REPLAY_MODE 1) at the long
chunk the auto mode would reach; the counters are per iteration modulo 64
(a replay of more iterations adds up in the same rows), so the totals over
all rows are what a long replay is judged by: events per chunk, scalar events
and cycles per replayed event, iterations (debug counter [3]).
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    import torch
    import wgraph
    from wgraph import abi, synth
    L = wgraph.lib()
    f = L.wg_debug_replay_profile
    f.argtypes = [ctypes.c_void_p, ctypes.c_int]
    args = sys.argv[1:] or ["wide16", "1000000", "linux", "1300000", "random13", "100000"]
    dev = torch.device("cuda", 0)
    out = {}
    for kind, n in zip(args[0::2], args[1::2]):
        d = synth.generate(kind, int(n))
        keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                       d.parent_oid.reshape(-1), d.flags)]
        c = abi.Commits()
        c.n_commits, c.n_parents = d.n, d.e
        c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep)
        c.residency = abi.WG_DEVICE
        eng = wgraph.Engine(0)
        eng.set_replay_mode(1)
        for _ in range(3):
            eng.build(commits=c)
        eng.synchronize()
        f(None, 1)
        eng.build(commits=c)
        eng.synchronize()
        buf = (ctypes.c_ulonglong * (64 * 8))()
        f(buf, 0)
        a = np.frombuffer(buf, dtype=np.uint64).reshape(64, 8)
        rows = []
        for it in range(64):
            if a[it, 0] == 0:
                continue
            ch = int(a[it, 0])
            rows.append({"iter": it, "chunks": ch, "batches": int(a[it, 1]), "no_scalar_batches": int(a[it, 2]),
                         "scalar_events": int(a[it, 3]), "merges_gt2": int(a[it, 4]),
                         "cycles_per_chunk": int(a[it, 5]) // ch, "scalar_cycles_per_chunk": int(a[it, 6]) // ch,
                         "merge_cycles_per_chunk": int(a[it, 7]) // ch})
        dc = eng.debug_counters()
        tot = a.sum(axis=0)
        ev = int(dc[4])
        out[f"{kind}/{n}"] = rec = {
            "list": kind, "rows": int(n), "events": ev, "replay_iterations": int(dc[3]), "n_slots": int(eng.layout_summary().n_slots),
            "chunks_run": int(tot[0]), "events_per_chunk": round(ev / max(1, int(rows[0]["chunks"]) if rows else 1), 1),
            "batches": int(tot[1]), "batches_without_scalar_events": int(tot[2]),
            "scalar_events": int(tot[3]), "merges_gt2": int(tot[4]),
            "cycles_total": int(tot[5]), "scalar_loop_cycles": int(tot[6]), "merge_cycles": int(tot[7]),
            "cycles_per_scalar_event": round(int(tot[6]) / max(1, int(tot[3])), 1),
            "iterations_first64": rows}
        print(json.dumps(rec), flush=True)
        eng.close()
        del keep


if __name__ == "__main__":
    main()
