"""k_match (wg_match_rows) on the bench's search leg: 1M rows of synthetic
summaries + authors (wgraph.synth.text_fields, ~15% non-ASCII words), query
"Fix" and a longer one; kernel time by HIP events, algorithmic bytes as
bench.py counts them, flags of the first 20k rows against the Python
restatement (oracle/search_oracle.py).  python3 profiles/match_probe.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ.get("WG_PKG_DIR") or os.path.join(ROOT, "whisper-git_amd"))   # (WG_PKG_DIR: an A/B copy)
sys.path.insert(0, ROOT)


def main():
    import torch
    import wgraph
    from wgraph import synth
    from oracle import search_oracle
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    dev = torch.device("cuda", 0)
    dag = synth.generate("wide16", n)
    eng = wgraph.Engine(0)
    eng.build(dag)
    (sb, so_), (ab, ao) = synth.text_fields(n)
    dt_ = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (sb, so_.view(np.int64), ab, ao.view(np.int64))]
    devp = ((dt_[0].data_ptr(), dt_[1].data_ptr()), (dt_[2].data_ptr(), dt_[3].data_ptr()))
    alg = int(so_[n] - so_[0]) + int(ao[n] - ao[0]) + n * (16 + 20 + 1 + 1)
    variants = [int(v) for v in os.environ.get("MATCH_THREADS", "0").split(",")]
    for rep in range(int(os.environ.get("MATCH_REPS", "1"))):
      for threads in variants:
       eng.set_match_threads(threads)
       for query in ("Fix", "refactor parser", "σοφ", "İ"):
        eng.match_rows(query, 0, n, device=devp)
        torch.cuda.synchronize()
        eng.enable_timing(True, reserve=64)
        for _ in range(10):
            nm = eng.match_rows(query, 0, n, device=devp)
        ms = [t for name, t in eng.timings() if name == "match"]
        eng.enable_timing(False)
        flags = eng.match_flags()
        m = 20_000
        want, _ = search_oracle.match_rows(dag, query.encode(), (sb, so_), (ab, ao), 0, m)
        ok = bool(np.array_equal(np.asarray(flags[:m], np.uint8), np.asarray(want, np.uint8)))
        k = float(np.mean(ms))
        print(json.dumps({"threads": threads, "rep": rep, "query": query, "rows": n, "matches": int(nm), "kernel_ms": round(k, 4),
                          "GBps": round(alg / (k * 1e-3) / 1e9, 1), "first_20k_equal_oracle": ok}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
