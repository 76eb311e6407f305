"""Lane stage cost of the two lane paths on one GPU ("measure
the serial walk at 1M rows first").

For each list: a fresh engine builds it `steps` times on the parallel
(event-compressed) path — the replay in auto mode, held on the chunked fixed
point, and held on the single-wave serial pass (WG_OPT_REPLAY_MODE 0 / 1 / 2)
— and `steps` times forced onto the general single-wave walk
(WG_OPT_LANE_PATH = 1); prints one JSON line per (list, path, replay) with
the mean ms of the "lanes" stage and of the whole build, the path taken, the
replay used and the slot count.  python3 profiles/lane_paths.py [steps] [lists]
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))

LISTS = [("wide16", 1_000_000, {}), ("linux", 1_300_000, {}), ("skew", 1_000_000, {}),
         ("linuxwide", 1_000_000, {}), ("random13", 100_000, {}), ("anomaly", 20_000, {"p_dup_oid": 0.0})]


def main():
    import torch
    import wgraph
    from wgraph import synth
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None
    for kind, n, over in LISTS:
        if only and kind not in only:
            continue
        d = synth.generate(kind, n, **over)
        for general, mode in ((False, 0), (False, 1), (False, 2), (True, 0)):
            if general and only:
                continue
            eng = wgraph.Engine(0)
            eng.set_lane_path(general)
            eng.set_replay_mode(mode)
            eng.build(d)                      # sizes the buffers (cold build, not timed here)
            eng.synchronize()
            eng.enable_timing(True, reserve=64 * (steps + 1))
            t0 = time.perf_counter()
            for _ in range(steps):
                eng.build(d)
            eng.synchronize()
            wall = (time.perf_counter() - t0) / steps * 1e3
            st = {}
            for name, ms in eng.timings():
                st[name] = st.get(name, 0.0) + ms / steps
            s = eng.layout_summary()
            dc = eng.debug_counters()
            print(json.dumps({"list": kind, "rows": d.n, "forced_general": general, "replay_mode": mode,
                              "serial": int(dc[10]), "lane_path": int(s.lane_path),
                              "replay_iterations": int(dc[3]), "events": int(dc[4]),
                              "n_slots": int(s.n_slots), "max_lane": int(s.max_lane),
                              "lanes_ms": round(st.get("lanes", 0.0), 4), "build_wall_ms": round(wall, 4),
                              "stages_ms": {k: round(v, 4) for k, v in st.items()}}), flush=True)
            eng.close()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
