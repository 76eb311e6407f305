"""CPU: the search-match oracle (commit_matches_query, commit_graph.rs:1509-1523)
and the engine's host-side str::to_lowercase (the query is lowered on the host,
:1326) against Python's str.lower over every code point."""
import numpy as np
import pytest

from oracle import search_oracle as so


def test_rust_to_lowercase_documented_cases():
    # the examples of Rust's str::to_lowercase documentation (semantics pins)
    assert so.to_lowercase("HELLO".encode()) == "hello".encode()
    assert so.to_lowercase("ὈΔΥΣΣΕΎΣ".encode()) == "ὀδυσσεύς".encode()        # final sigma
    assert so.to_lowercase("农历新年".encode()) == "农历新年".encode()
    assert so.to_lowercase("İ".encode()) == "i̇".encode()                  # SpecialCasing, unconditional


def _row(summary=b"", author=b"", oid=bytes(range(20)), synthetic=False):
    return summary, author, oid, synthetic


@pytest.mark.parametrize("query,expect", [
    (b"fix", True), (b"FIX", False),        # the query arrives lowered (:1326); fields are lowered
    (b"graph la", True), (b"linus", True), (b"torvalds", True),
    (b"0001020", True),                      # short id (7 hex digits, git/mod.rs:300)
    (b"0102", True),                         # inside the short id
    (b"00010203", True),                     # id prefix beyond the short id
    (b"0203040506", False),                  # inside the id but not a prefix and not in the short id
    (b"000102030405060708090a0b0c0d0e0f10111213", True),
    (b"000102030405060708090a0b0c0d0e0f1011121314", False),
])
def test_commit_matches_query(query, expect):
    s, a, oid, syn = _row(b"Fix Graph Layout", b"Linus Torvalds")
    assert so.commit_matches_query(s, a, oid, syn, query) == expect


def test_synthetic_rows_have_no_short_id_but_keep_the_id_prefix():
    oid = bytes.fromhex("ff" * 19 + "01")
    assert so.commit_matches_query(b"", b"", oid, True, b"fff")        # prefix of the id
    assert not so.commit_matches_query(b"", b"", oid, True, b"f01")
    assert so.commit_matches_query(b"", b"", bytes.fromhex("ab" * 20), False, b"bab")
    assert not so.commit_matches_query(b"", b"", bytes.fromhex("ab" * 20), True, b"bab")


def test_empty_query_matches_every_row():
    from wgraph import synth
    d = synth.generate("random13", 50)
    f, n = so.match_rows(d, b"")
    assert n == 50 and f.all()


def test_engine_lowercase_equals_str_lower_on_every_code_point():
    import wgraph
    cps = [cp for cp in range(0x110000) if not 0xD800 <= cp <= 0xDFFF]
    # every code point alone (between spaces: no Final_Sigma context) ...
    for i in range(0, len(cps), 4096):
        s = " ".join(chr(cp) for cp in cps[i:i + 4096]).encode()
        assert wgraph.to_lowercase(s) == so.to_lowercase(s), hex(cps[i])
    # ... and every code point as the context of a capital sigma, both sides
    for i in range(0, len(cps), 2048):
        chunk = cps[i:i + 2048]
        s = " ".join("a" + chr(cp) + "Σ" + chr(cp) + "a " + chr(cp) + "Σ" for cp in chunk).encode()
        assert wgraph.to_lowercase(s) == so.to_lowercase(s), hex(chunk[0])


def test_engine_lowercase_on_malformed_utf8():
    import wgraph
    rng = np.random.default_rng(7)
    pieces = [b"\xc3", b"\xc3\xa9", b"\xe2\x82", b"\xe2\x82\xac", b"\xed\xa0\x80", b"\xf4\x90\x80\x80", b"\xc0\xaf",
              b"\xe0\x80\xaf", b"\xf0\x9f\x9a\x80", b"\xce\xa3", b"A", b" ", b"\x80", b"\xff", b"\xce"]
    for _ in range(2000):
        s = b"".join(pieces[i] for i in rng.integers(0, len(pieces), rng.integers(0, 12)))
        assert wgraph.to_lowercase(s) == so.to_lowercase(s), s
