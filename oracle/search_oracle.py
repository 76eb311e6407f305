"""CPU oracle for the search-match flags — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's CPU baseline may import
this module; the engine never calls it.

Restates (pure Python; small and medium sizes):
  history_view's match flags   commit_graph.rs:1320-1332
      query empty -> every row matches; else q = search_query.to_lowercase()
  commit_matches_query         commit_graph.rs:1509-1523
      summary.to_lowercase().contains(q) || author.to_lowercase().contains(q)
      || short_id.to_lowercase().contains(q)
      || id.to_string().to_lowercase().starts_with(q)
  short_id                     git/mod.rs:300 (first 7 hex digits); "" for
                               synthetic rows (git/mod.rs:360, 404)

Rust's str::to_lowercase and Python's str.lower() implement the same Unicode
default lowercase mapping (simple mappings, U+0130 -> "i̇", Final_Sigma), so
`str.lower()` is the restatement; bytes that are not well-formed UTF-8 go
through the `surrogateescape` round trip (copied unchanged, neither cased nor
case-ignorable).  Pinning: the reference holds no test or fixture for this
path (parity unpinned against reference output); the restatement is pinned
by the reference's own semantics (`str::to_lowercase` documentation cases in
tests/test_search_oracle.py) and Unicode's own data as this interpreter ships
it (unicodedata.unidata_version).
"""
from __future__ import annotations

import numpy as np


def to_lowercase(b: bytes) -> bytes:
    """Rust `str::to_lowercase` on UTF-8 bytes."""
    return b.decode("utf-8", "surrogateescape").lower().encode("utf-8", "surrogateescape")


def commit_matches_query(summary: bytes, author: bytes, oid: bytes, synthetic: bool, lower_query: bytes) -> bool:
    """commit_graph.rs:1509-1523 (lower_query already lowered, :1326)."""
    if lower_query in to_lowercase(summary):
        return True
    if lower_query in to_lowercase(author):
        return True
    hexid = oid.hex().encode()
    short_id = b"" if synthetic else hexid[:7]
    if lower_query in short_id:
        return True
    return hexid.startswith(lower_query)


def match_rows(dag, query: bytes, summaries=None, authors=None, row_begin: int = 0, row_end: int | None = None):
    """Match flags (uint8) of rows [row_begin, row_end) and their count
    (history_view, commit_graph.rs:1320-1332)."""
    n = dag.n if row_end is None else row_end
    rows = n - row_begin
    if not query:
        return np.ones(rows, np.uint8), rows
    q = to_lowercase(query)
    if not q:
        return np.ones(rows, np.uint8), rows

    def field(f, r):
        if f is None:
            return b""
        b, o = f
        return bytes(b[int(o[r]):int(o[r + 1])])

    out = np.zeros(rows, np.uint8)
    oid = dag.oid
    for r in range(row_begin, n):
        out[r - row_begin] = commit_matches_query(field(summaries, r), field(authors, r), bytes(oid[r]),
                                                  bool(dag.flags[r] & 2), q)
    return out, int(out.sum())
