"""CPU oracle for the commit list's row order — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's CPU baseline may import
this module; the engine never calls it.

Restates (pure Python):
  commit_graph_with_orphans   git/mod.rs:761-775
      commits.extend(orphans); if orphans: commits.sort_by_key(Reverse(time))
      (Rust's sort_by_key is stable; so is Python's list.sort)
  insert_synthetics_sorted    git/mod.rs:234-242
      for each synthetic, in order: pos = first index with c.time <= s.time,
      else len; commits.insert(pos, s)
Result: perm[final row] = source row (walk rows, then orphans, then
synthetics).  Pinning: the reference holds no test or fixture for these two
functions (parity unpinned against reference output); the restatement is the
two functions' text, line by line.
"""
from __future__ import annotations

import numpy as np


def order_rows(walk_time, orphan_time=(), syn_time=()) -> np.ndarray:
    t = [int(x) for x in walk_time] + [int(x) for x in orphan_time]
    rows = list(range(len(t)))
    if len(orphan_time):
        rows.sort(key=lambda i: -t[i])          # stable, newest first (:771-772)
    ts = [int(x) for x in syn_time]
    tt = t + ts
    nb = len(t)
    for j, s in enumerate(ts):                  # :234-242
        pos = next((p for p, i in enumerate(rows) if tt[i] <= s), len(rows))
        rows.insert(pos, nb + j)
    return np.array(rows, np.uint32)
