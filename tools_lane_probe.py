import sys, numpy as np
sys.path.insert(0, 'whisper-git_amd'); sys.path.insert(0, '.')
import wgraph
from wgraph import synth
from oracle import oracle_c
e = wgraph.Engine(0)
e.enable_timing(True)
for kind, n in [("wide16", 1000000), ("random13", 1000000), ("linux", 1000000)]:
    d = synth.generate(kind, n)
    o = oracle_c.OracleLayout(d)
    for chunk in (128, 256, 512, 1024, 4096):
        e._check(wgraph.lib().wg_set_option(e._ctx, 2, chunk))
        for _ in range(2):
            e.enable_timing(True)
            e.build(d)
        t = dict(e.timings())
        c = e.debug_counters()
        lane, _ = e.lanes()
        ok = (lane == o.lane).all() and e.layout_summary().max_lane == o.max_lane
        print(f"{kind} chunk {chunk}: events {c[4]} iters {c[3]} lf_loop {t.get('lf_loop', -1):.3f} ms lanes {t.get('lanes',-1):.3f} ms exact {ok} path {e.layout_summary().lane_path}", flush=True)
