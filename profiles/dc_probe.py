"""The compacted lane replay (wg_lanes_dchunk.hip) on the BASELINE list
shapes: per list and replay mode a fresh engine builds the list `steps + 1`
times (the first exact, the rest speculative), every build's lanes, colours,
edges, max_lane and slot count compared with the C oracle; prints one JSON
line per (list, mode) with the form taken, the leaks struck out, the
iterations, and the mean "lanes" / "lf_loop" stage times of the timed builds.

python3 profiles/dc_probe.py [steps] [lists] [modes]   (research tool, not a test)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))

LISTS = [("skew", 1_000_000, {}), ("linux", 1_300_000, {}), ("linuxwide", 1_000_000, {}), ("wide16", 1_000_000, {}),
         ("random13", 100_000, {}), ("skewheavy", 300_000, {"p_clock_skew": 2e-3}),
         ("linux400", 200_000, {"max_lines": 400}), ("anomaly", 10_000, {"p_dup_oid": 0.0})]


def main():
    import numpy as np
    import torch
    import wgraph
    from wgraph import synth
    from oracle import oracle_c
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    only = sys.argv[2].split(",") if len(sys.argv) > 2 and sys.argv[2] else None
    modes = [int(m) for m in sys.argv[3].split(",")] if len(sys.argv) > 3 else [3, 0]
    for name, n, over in LISTS:
        if only and name not in only:
            continue
        kind = {"skewheavy": "skew", "linux400": "linux"}.get(name, name)
        d = synth.generate(kind, n, **over)
        o = oracle_c.OracleLayout(d)
        for mode in modes:
            eng = wgraph.Engine(0)
            eng.set_replay_mode(mode)
            bad = []
            forms = []
            t_wall = 0.0
            for it in range(steps + 1):
                if it == 1:
                    eng.synchronize()
                    eng.enable_timing(True, reserve=64 * (steps + 1))
                t0 = time.perf_counter()
                eng.build(d)
                eng.synchronize()
                if it >= 1:
                    t_wall += time.perf_counter() - t0
                s = eng.layout_summary()
                lane, color = eng.lanes()
                ok = (s.lane_path == 0 and (s.max_lane, s.n_slots) == (o.max_lane, o.n_slots)
                      and lane.tobytes() == o.lane.astype(np.uint32).tobytes() and color.tobytes() == o.color.tobytes()
                      and eng.edges().tobytes() == o.edges.tobytes())
                if not ok:
                    bad.append(it)
                dc = eng.debug_counters()
                forms.append(int(dc[12]))
            st = {}
            for nm, ms in eng.timings():
                st[nm] = st.get(nm, 0.0) + ms / steps
            dc = eng.debug_counters()
            print(json.dumps({"list": name, "rows": d.n, "mode": mode, "exact_all": not bad, "bad_builds": bad,
                              "forms": forms, "leaks": int(dc[13]), "warm": int(dc[14]), "iterations": int(dc[3]),
                              "events": int(dc[4]), "n_slots": int(o.n_slots), "lanes_ms": round(st.get("lanes", 0.0), 4),
                              "lf_loop_ms": round(st.get("lf_loop", 0.0), 4), "build_wall_ms": round(t_wall / steps * 1e3, 3),
                              "spec": [int(dc[6]), int(dc[7])]}), flush=True)
            eng.close()
        o.close()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
