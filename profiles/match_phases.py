"""k_match per-phase latency inside a workgroup (r05 study): a build of the
kernel with clock64() stamps at each barrier (WG_PKG_DIR=profiles/ab_ph,
exporting wg_dbg_phases) on the probe's workload; prints per query the mean
and p90 cycles of each phase over the 3907 workgroups and the spread of their
start times, and the staging phase split per wave.  python3 profiles/match_phases.py"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.environ["WG_PKG_DIR"])
sys.path.insert(0, ROOT)


def main():
    import torch
    import wgraph
    from wgraph import synth
    n = 1_000_000
    dev = torch.device("cuda", 0)
    dag = synth.generate("wide16", n)
    eng = wgraph.Engine(0)
    eng.build(dag)
    (sb, so_), (ab, ao) = synth.text_fields(n)
    dt_ = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (sb, so_.view(np.int64), ab, ao.view(np.int64))]
    devp = ((dt_[0].data_ptr(), dt_[1].data_ptr()), (dt_[2].data_ptr(), dt_[3].data_ptr()))
    lib = ctypes.CDLL(wgraph.LIB_PATH)
    nb = (n + 255) // 256
    names = ["stage", "sigma", "lower", "match", "walk", "tail"]
    for query in ("Fix", "refactor parser", "σοφ", "İ"):
        for _ in range(3):
            eng.match_rows(query, 0, n, device=devp)
        torch.cuda.synchronize()
        buf = np.zeros((8192, 4, 14), np.uint64)
        assert lib.wg_dbg_phases(buf.ctypes.data_as(ctypes.c_void_p)) == 0
        w = buf[:nb].astype(np.int64)          # per wave
        b = w[:, 0]                            # wave 0
        d = np.diff(b[:, :7], axis=1)
        start = (b[:, 8] - b[:, 8].min()) / 100.0     # s_memrealtime: 100 MHz -> us
        life = (b[:, 9] - b[:, 8]) / 100.0
        out = {"query": query, "blocks": nb}
        for i, nm in enumerate(names):
            out[nm] = [int(d[:, i].mean()), int(np.percentile(d[:, i], 90))]
        # staging split per wave: start -> offsets -> first batch listed -> loop done -> barrier
        sp = np.stack([w[:, :, 10] - w[:, :, 0], w[:, :, 11] - w[:, :, 10], w[:, :, 12] - w[:, :, 11],
                       w[:, :, 1] - w[:, :, 12]], -1)
        out["stage_split_mean"] = [int(x) for x in sp.reshape(-1, 4).mean(0)]
        out["stage_split_p90"] = [int(x) for x in np.percentile(sp.reshape(-1, 4), 90, axis=0)]
        q = np.digitize(start, np.percentile(start, [25, 50, 75]))    # start-time quartile (round)
        out["by_round"] = {int(r): {"offsets": int(sp[q == r, :, 0].mean()), "batch1": int(sp[q == r, :, 1].mean()),
                                    "batch2": int(sp[q == r, :, 2].mean()), "sigma..tail": int(d[q == r, 1:].sum(1).mean()),
                                    "start_us": round(float(start[q == r].mean()), 1)} for r in range(4)}
        out["wave_start_spread"] = int((w[:, :, 0].max(1) - w[:, :, 0].min(1)).mean())
        out["wg_life_us_mean"] = round(float(life.mean()), 2)
        out["start_us_pct"] = [round(float(np.percentile(start, p)), 1) for p in (0, 25, 50, 75, 100)]
        out["end_us_max"] = round(float(((b[:, 9] - b[:, 8].min()) / 100.0).max()), 1)
        print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
