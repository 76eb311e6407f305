"""GPU search-match flags (commit_matches_query, commit_graph.rs:1509-1523;
history_view :1320-1332) against the oracle, bit for bit, through the C ABI:
ASCII and Unicode queries (final sigma, dotted I, Kelvin sign, titlecase
digraphs), short-id / id-prefix queries, synthetic rows, queries longer than
the LDS copy, rows too wide to stage, host and device text, row ranges —
and the search dimming of vertex and glyph emission (:1467, 1482)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN_DIR
from oracle import search_oracle as so
from wgraph import abi, synth

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def data():
    d = synth.generate("anomaly", 6000, seed=5)        # synthetic and orphan rows, duplicate ids
    summ, auth = synth.text_fields(d.n, seed=2)
    return d, summ, auth


def _queries(d):
    hexid = d.oid[123].tobytes().hex()
    return ["fix", "FIX", "Graph L", "ΣΟΦΙΑ", "σοφια", "όδος", "ας.", "ς", "σ", "İstanbul", "i̇", "STRASSE", "straße",
            "ǆ", "ǅemal", "K", "k", "ångström", "日本", "🚀", "dmitry", "дмитрий", " ", "a", "aab", "e e",
            hexid[:4], hexid[:7], hexid[2:6], hexid[:12], hexid, hexid + "0", "ʼn", "\xc3".encode("latin-1"),
            "x" * 3000, "remove " * 400]


@pytest.fixture(params=[512, 256], ids=["nt512", "nt256"])
def threads(engine, request):
    """The kernel's workgroup at 512 threads (default) and at 256: the same flags."""
    engine.set_match_threads(request.param)
    yield request.param
    engine.set_match_threads(0)


@pytest.mark.parametrize("residency", ["host", "device"])
def test_match_flags_equal_oracle(engine, data, residency, threads):
    import torch
    d, summ, auth = data
    engine.build(d)
    dev = None
    if residency == "device":
        t = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in (summ[0], summ[1].view(np.int64),
                                                                          auth[0], auth[1].view(np.int64))]
        dev = ((t[0].data_ptr(), t[1].data_ptr()), (t[2].data_ptr(), t[3].data_ptr()))
    try:
        for q in _queries(d):
            qb = q if isinstance(q, bytes) else q.encode()
            for rb, re_ in ((0, d.n), (777, 4321)):
                if dev is not None:
                    n = engine.match_rows(qb, rb, re_, device=dev)
                else:
                    n = engine.match_rows(qb, rb, re_, summaries=summ, authors=auth)
                want, wn = so.match_rows(d, qb, summ, auth, rb, re_)
                got = engine.match_flags()
                assert n == wn, (q, rb)
                assert (got == want).all(), (q, rb, np.flatnonzero(got != want)[:5])
    finally:
        engine.match_rows("")


def test_match_without_text_fields_and_wide_rows(engine):
    d = synth.generate("random13", 3000, seed=9)
    engine.build(d)
    # rows whose summaries are far too long for the 22 KiB LDS image (read from HBM instead)
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 400, d.n)
    lens[100:400] = 5000
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    words = np.frombuffer(b"abc Abd aBe ABF \xce\xa3\xce\x91\xce\xa3 ", np.uint8)
    body = np.resize(words, int(off[-1]))
    try:
        for q in ("abf", "σας", "σασ", "ab", d.oid[5].tobytes().hex()[:9]):
            n = engine.match_rows(q, summaries=(body, off))
            want, wn = so.match_rows(d, q.encode(), (body, off), None)
            assert n == wn and (engine.match_flags() == want).all(), q
        n = engine.match_rows(d.oid[7].tobytes().hex()[:5])          # id fields only
        want, wn = so.match_rows(d, d.oid[7].tobytes().hex()[:5].encode())
        assert n == wn and (engine.match_flags() == want).all()
    finally:
        engine.match_rows("")


def test_match_fuzz_bytes_unaligned(engine, threads):
    """Rows of random bytes from an alphabet of ASCII letters, lead and
    continuation bytes of two- to four-byte sequences (valid, truncated,
    overlong, stray), U+03A3 / U+0130 / U+1E9E / U+212A pieces, with the
    device text at byte offsets 0-3 (the LDS stage's edge words) and row
    ranges that start mid-word; queries cut from the lowered rows."""
    import torch
    d = synth.generate("random13", 2000, seed=3)
    engine.build(d)
    rng = np.random.default_rng(11)
    alpha = [b"A", b"a", b"Z", b"z", b" ", b".", b"'", b"\xce\xa3", b"\xcf\x83", b"\xc4\xb0", b"\xe1\xba\x9e",
             b"\xe2\x84\xaa", b"\xce", b"\xa3", b"\x80", b"\xc0\xaf", b"\xe0\x80\x80", b"\xf0\x9f\x9a\x80",
             b"\xf0\x9f", b"\xd0\x94", b"\xc7\x85", b"\xcc\x87", b"\xff", b"\xe6\x97\xa5", b"\x00", b"\x01"]
    try:
        # with raw 0xFF bytes in every 256-row range (specials left in place) and without (specials marked)
        for alph in (alpha, alpha[:22] + alpha[23:]):
            rows = [b"".join(alph[i] for i in rng.integers(0, len(alph), int(k))) for k in rng.integers(0, 24, d.n)]
            rows[50:60] = [b""] * 10
            off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint64)
            body = np.frombuffer(b"".join(rows), np.uint8)
            qs = [b"a", b"\xcf\x83", b"\xcf\x82", b"i\xcc\x87", b"\xc3\x9f", b"k", b"\x80", b"\xce", b"\xff", b"\x00",
                  b"a\x01", b"\xfe", b"i", b"\xcc\x87a"]
            for r in rng.integers(0, d.n, 12):
                lw = so.to_lowercase(rows[r])
                if len(lw) > 2:
                    a = int(rng.integers(0, len(lw) - 1))
                    qs.append(lw[a:a + int(rng.integers(1, 12))])
            for shift in range(4):
                buf = torch.zeros(len(body) + 8, dtype=torch.uint8, device="cuda")
                buf[shift:shift + len(body)] = torch.from_numpy(body.copy()).cuda()
                ot = torch.from_numpy(off.view(np.int64).copy()).cuda()
                dev = ((buf.data_ptr() + shift, ot.data_ptr()), None)
                for q in qs:
                    for rb, re_ in ((0, d.n), (333, 1501)):
                        n = engine.match_rows(q, rb, re_, device=dev)
                        want, wn = so.match_rows(d, q, (body, off), None, rb, re_)
                        got = engine.match_flags()
                        assert n == wn and (got == want).all(), (shift, q, rb, np.flatnonzero(got != want)[:5])
    finally:
        engine.match_rows("")


def test_match_dense_non_ascii_fields(engine, threads):
    """Fields with more non-ASCII code points per 256 rows than the kernel's
    lists hold (Cyrillic, Greek with final sigmas) and rows mixing them with
    length-changing code points: every path gives the oracle's flags."""
    d = synth.generate("random13", 1200, seed=4)
    engine.build(d)
    rng = np.random.default_rng(5)
    pieces = ["Дa", "Σa", "ΣΣ ", "İ", "ẞ", "σ", "ΟΣ "]
    rows = []
    for i in range(d.n):
        kind = (i // 256) % 3
        if kind == 0:
            rows.append(("Дa" * 20).encode())
        elif kind == 1:
            rows.append(("Σa" * 12 + ("ΟΣ " if i % 5 == 0 else "")).encode())
        else:
            rows.append("".join(pieces[j] for j in rng.integers(0, len(pieces), 9)).encode())
    off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint64)
    body = np.frombuffer(b"".join(rows), np.uint8)
    try:
        for q in ("да", "σa", "ς", "ας σ", "i̇", "ss", "σσ", "ος", "дaдaдaдaдaд"):
            n = engine.match_rows(q, summaries=(body, off), authors=(body, off))
            want, wn = so.match_rows(d, q.encode(), (body, off), (body, off))
            assert n == wn and (engine.match_flags() == want).all(), q
    finally:
        engine.match_rows("")


@pytest.mark.parametrize("sum_len,auth_len", [(60, 20), (60, 40), (80, 6), (0, 70)])
def test_match_fields_together_or_apart(engine, sum_len, auth_len, threads):
    """The kernel stages a workgroup's two fields into one LDS image when they
    fit together and in two passes when they do not (about 60 + 40 bytes per
    row is past the image, 60 + 20 is within it, 80 + 6 sits at the edge, an
    empty summary field leaves the authors alone): the same flags either way."""
    d = synth.generate("random13", 1500, seed=8)
    engine.build(d)
    rng = np.random.default_rng(sum_len * 7 + auth_len)
    words = ["ΣΟΦΙΑ", "İstanbul", "fix", "Graph", "STRAẞE", "ος", "kelvin", "Åse", "a", "ǅ"]

    def field(mean):
        rows = []
        for _ in range(d.n):
            s = ""
            target = int(rng.integers(max(0, mean - 8), mean + 9)) if mean else 0
            while len(s.encode()) < target:
                s += words[int(rng.integers(0, len(words)))] + " "
            rows.append(s.encode()[:target] if target else b"")
        off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint64)
        return np.frombuffer(b"".join(rows) or b"\0", np.uint8)[:int(off[-1])], off

    summ, auth = field(sum_len), field(auth_len)
    try:
        for q in ("fix", "σοφ", "i̇", "ος ", "ss", "å", "ǆ", "a a"):
            n = engine.match_rows(q, summaries=summ, authors=auth)
            want, wn = so.match_rows(d, q.encode(), summ, auth)
            assert n == wn and (engine.match_flags() == want).all(), (q, sum_len, auth_len)
    finally:
        engine.match_rows("")


def test_empty_query_matches_all_and_build_clears(engine, data):
    d, summ, auth = data
    engine.build(d)
    assert engine.match_rows("", summaries=summ, authors=auth) == d.n
    assert engine.match_flags().all()


def test_search_dimming_of_vertices_and_glyphs(engine, data):
    from oracle import oracle_c, text_oracle
    d, summ, auth = data
    engine.build(d)
    engine.row_geometry(d.band)
    o = oracle_c.OracleLayout(d)
    og = o.row_geometry(d.band)
    try:
        engine.match_rows("fix", 1000, 5000, summaries=summ, authors=auth)
        flags = engine.match_flags()
        assert 0 < flags.sum() < len(flags)
        engine.emit_vertices(500, 5500, selected=1003)
        want, _ = o.emit_vertices(500, 5500, selected=1003, match=flags, match_rb=1000)
        assert engine.vertex_summary().checksum == oracle_c.vertex_checksum(want)
        got = engine.vertices()
        assert got.tobytes() == want.tobytes()
        # glyph quads of the same rows
        z = np.load(os.path.join(GOLDEN_DIR, "font_regular.npz"), allow_pickle=False)
        p = abi.ATLAS_DEFAULTS
        engine.build_font_atlas(0)
        kw = dict(now=int(d.time.max()) + 86400)
        engine.emit_glyphs(900, 1200, summaries=summ, **kw)
        tv, _ = text_oracle.emit_glyphs(d, og["node_y"], z["glyphs"], p["width"], p["height"], p["spread"], p["em_px"],
                                        900, 1200, summaries=summ, match=flags, match_rb=1000, **kw)
        assert engine.glyph_vertices().view(np.float32).reshape(-1, 8).tobytes() == tv.tobytes()
        # empty query: no dimming
        engine.match_rows("")
        engine.emit_vertices(500, 5500, selected=1003)
        plain, _ = o.emit_vertices(500, 5500, selected=1003)
        assert engine.vertex_summary().checksum == oracle_c.vertex_checksum(plain)
    finally:
        engine.match_rows("")
        o.close()


@pytest.mark.parametrize("dense", ["summary", "author"])
def test_match_two_passes_with_an_overflowing_pass(engine, dense, threads):
    """a workgroup whose two fields do not fit one LDS image runs
    two passes; here one of them lists more non-ASCII leads than the kernel
    holds (LCAP 2560 per 256 rows: that pass takes the stream from HBM and
    skips its barriers uniformly) while the other pass walks rows with
    length-changing code points (U+1E9E, the Kelvin sign, U+0130) — with
    queries shorter than 8 bytes, between 9 and 16, and past 16 bytes (the KMP
    whole-row walk) that contain 'ß' / 'k'.  Each pass keeps its own counts
    (a slower wave of pass 0 must not see pass 1's cleared counters)."""
    d = synth.generate("random13", 1800, seed=21)
    engine.build(d)
    rng = np.random.default_rng(77 if dense == "summary" else 78)
    cyr = "ДмитрийСтрасБург"
    mixed = ["STRAẞE ", "straße ", "Kelvin ", "kelvin ", "İ ", "fix ", "Ölçek ", "a "]

    def rows_of(kind, target):
        rows = []
        for _ in range(d.n):
            s = ""
            if kind == "dense":
                while len(s.encode()) < target:
                    s += cyr[int(rng.integers(0, len(cyr)))]
            else:
                while len(s.encode()) < target:
                    s += mixed[int(rng.integers(0, len(mixed)))]
            b = s.encode()
            while len(b) > target:      # whole code points only
                s = s[:-1]
                b = s.encode()
            rows.append(b)
        off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint64)
        return np.frombuffer(b"".join(rows), np.uint8), off

    dense_f = rows_of("dense", 72)          # ~36 leads per row: 9k per 256 rows
    other_f = rows_of("mixed", 44)
    summ, auth = (dense_f, other_f) if dense == "summary" else (other_f, dense_f)
    qs = ["ß", "k", "дм", "straße kelvin", "strasse", "straße straße straße", "kelvin kelvin kelvin k",
          "i̇ fix a straße", "KELVIN KELVIN straẞe", "ийстрасбург", "рийстр"]
    try:
        for q in qs:
            n = engine.match_rows(q, summaries=summ, authors=auth)
            want, wn = so.match_rows(d, q.encode(), summ, auth)
            got = engine.match_flags()
            assert n == wn and (got == want).all(), (q, dense, np.flatnonzero(got != want)[:5])
    finally:
        engine.match_rows("")


def test_ascii_queries_across_the_ascii_lowering_code_points(engine, threads):
    """r06: an ASCII query lists only the leads of U+0130 (-> "i" U+0307) and
    U+212A (-> "k"), the two code points whose lowering holds an ASCII byte;
    every other code point is left unlowered in LDS.  Rows mixing both with
    other specials (U+1E9E, U+2126, U+212B), sigma and plain letters, with and
    without a raw 0xFF byte in the range (marks off): ASCII queries that match
    across the Kelvin sign and the dotted I, or must not, give the oracle's
    flags; non-ASCII queries still take the full lowering."""
    d = synth.generate("random13", 1300, seed=31)
    engine.build(d)
    rng = np.random.default_rng(9)
    pieces = ["K", "İ", "f", "x", "i", "k", "K", "ẞ", "Ω", "Å", "Σ", "é", "a", " "]
    qs = ["k", "xk", "kx", "fi", "fix", "i", "ik", "ki", "a k", "fa", "kki", "ix", "x" * 20 + "k", "fik",
          "σ", "ék", "ẞ"]
    try:
        for raw_ff in (False, True):
            rows = ["".join(pieces[j] for j in rng.integers(0, len(pieces), int(n))).encode()
                    for n in rng.integers(0, 30, d.n)]
            if raw_ff:
                rows[300] = rows[300] + b"\xff"
            off = np.concatenate([[0], np.cumsum([len(r) for r in rows])]).astype(np.uint64)
            body = np.frombuffer(b"".join(rows), np.uint8)
            for q in qs:
                n = engine.match_rows(q, summaries=(body, off))
                want, wn = so.match_rows(d, q.encode(), (body, off), None)
                got = engine.match_flags()
                assert n == wn and (got == want).all(), (q, raw_ff, np.flatnonzero(got != want)[:5])
    finally:
        engine.match_rows("")
