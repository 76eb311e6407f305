"""Golden per-shard results of BASELINE config C5 (8M-commit wide synthetic
DAG, <= 16 lanes, sharded 8x), made by the C oracle (oracle/wg_oracle.c,
test infrastructure).

The whole list is laid out by the oracle (GraphLayout::build +
row_geometry_with_bands with the preset's bands); each rank's contiguous row
range [n r / 8, n (r+1) / 8) is then emitted by the oracle in 100k-row pieces
and checksummed at its offset inside that rank's vertex buffer (WG-TESS-1
checksum; pieces add up mod 2^64).  Also per rank: its lanes' and colours'
sha256 and its vertex count.  tests/test_gpu_c5.py drives eight engine
contexts through the sharded protocol and compares.

Run:  python tests/golden/make_c5_golden.py     (writes tests/golden/c5_shards.json; ~2 min)
"""
from __future__ import annotations

import hashlib
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))
sys.path.insert(0, ROOT)

from wgraph import synth  # noqa: E402
from wgraph.shard import shard_rows  # noqa: E402
from oracle import oracle_c  # noqa: E402

N, WORLD, PIECE = 8_000_000, 8, 100_000
KIND, SEED = "wide16", synth.SEED_BASE + 5   # seed = 0x5EED + config id
SELECTED = N // 2 + 1


def main():
    t0 = time.time()
    d = synth.generate(KIND, N, seed=SEED)
    o = oracle_c.OracleLayout(d)
    g = o.row_geometry(d.band)
    ranks = []
    for r in range(WORLD):
        s, t = shard_rows(N, WORLD, r)
        total, first = 0, 0
        for a in range(s, t, PIECE):
            b = min(t, a + PIECE)
            ov, _ = o.emit_vertices(a, b, selected=SELECTED)
            total = (total + oracle_c.vertex_checksum(ov, first)) & 0xFFFFFFFFFFFFFFFF
            first += len(ov)
            del ov
        ranks.append({"rank": r, "row_begin": s, "row_end": t, "n_vertices": first, "checksum": f"{total:#018x}",
                      "lane_sha256": hashlib.sha256(o.lane[s:t].tobytes()).hexdigest(),
                      "color_sha256": hashlib.sha256(o.color[s:t].tobytes()).hexdigest(),
                      "row_top_end_bits": int(g["row_top"][t:t + 1].view("uint32")[0])})   # f32 bits of row_top_y[e]
        print(f"rank {r}: {first} vertices, {time.time() - t0:.0f} s", flush=True)
    out = {"config": "C5", "preset": KIND, "seed": SEED, "rows": N, "world": WORLD, "piece_rows": PIECE,
           "selected": SELECTED, "max_lane": int(o.max_lane), "n_slots": int(o.n_slots),
           "n_edges": int(len(o.edges)), "ranks": ranks}
    with open(os.path.join(HERE, "c5_shards.json"), "w") as f:
        json.dump(out, f, indent=1)
    o.close()
    print(f"done in {time.time() - t0:.0f} s")


if __name__ == "__main__":
    main()
