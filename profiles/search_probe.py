"""k_match timing probe: synthetic text with and without non-ASCII words,
several queries (which part of the per-row stream costs the time)."""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    import torch
    import wgraph
    from wgraph import synth
    n = 1_000_000
    d = synth.generate("wide16", n)
    eng = wgraph.Engine(0)
    eng.set_stream(torch.cuda.current_stream().cuda_stream)
    eng.build(d)
    for pu in (0.0, 0.15):
        summ, auth = synth.text_fields(n, p_unicode=pu)
        t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (summ[0], summ[1].view(np.int64),
                                                                          auth[0], auth[1].view(np.int64))]
        dev = ((t[0].data_ptr(), t[1].data_ptr()), (t[2].data_ptr(), t[3].data_ptr()))
        for q in ("Fix", "zzzz", "q", "the graph"):
            eng.match_rows(q.encode(), 0, n, device=dev)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                k = eng.match_rows(q.encode(), 0, n, device=dev)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 200
            print(f"p_unicode {pu} query {q!r}: {ms:.3f} ms/call, {k} matches, text bytes {len(summ[0]) + len(auth[0])}",
                  flush=True)


if __name__ == "__main__":
    main()
