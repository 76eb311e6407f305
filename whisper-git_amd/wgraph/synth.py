"""Seeded synthetic commit DAGs (workload generator, ctypes over libwgsynth.so).

The generator itself is C (whisper-git_amd/synth/wg_synth.c).  Presets follow
SURVEY.md §8(d): LINEAR (C1), RANDOM13 (C3), LINUX (C4), WIDE16 (C5) and
ANOMALY (the edge cases GraphLayout::build tolerates), SKEW (LINUX with clock
skew and 100 reflog orphans, re-sorted by time as git/mod.rs:761-775 does)
and LINUXWIDE (LINUX with more than 100 concurrent lanes).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

LINEAR, RANDOM13, LINUX, WIDE16, ANOMALY, SKEW, LINUXWIDE = 0, 1, 2, 3, 4, 5, 6
PRESETS = {"linear": LINEAR, "random13": RANDOM13, "linux": LINUX, "wide16": WIDE16, "anomaly": ANOMALY,
           "skew": SKEW, "linuxwide": LINUXWIDE}
SEED_BASE = 0x5EED  # seed = 0x5EED + config id


class Params(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("max_lines", ctypes.c_int32),
                ("n", ctypes.c_uint64), ("seed", ctypes.c_uint64),
                ("p_merge", ctypes.c_double), ("p_octopus", ctypes.c_double),
                ("p_newtip", ctypes.c_double), ("p_fork", ctypes.c_double),
                ("main_weight", ctypes.c_double), ("p_dup_oid", ctypes.c_double),
                ("p_skew", ctypes.c_double), ("p_external", ctypes.c_double),
                ("p_self", ctypes.c_double), ("p_dup_parent", ctypes.c_double),
                ("p_orphan_flag", ctypes.c_double), ("band_frac", ctypes.c_double),
                ("truncated", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("p_feature", ctypes.c_double), ("p_clock_skew", ctypes.c_double),
                ("n_orphans", ctypes.c_uint64)]


_lib = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libwgsynth.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make synth` (or __graft_entry__.build())")
        lib = ctypes.CDLL(path)
        lib.wgs_preset.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_uint64, ctypes.POINTER(Params)]
        lib.wgs_generate.argtypes = [ctypes.POINTER(Params)]
        lib.wgs_generate.restype = ctypes.c_void_p
        lib.wgs_sizes.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        lib.wgs_copy.argtypes = [ctypes.c_void_p] + [ctypes.c_void_p] * 6
        lib.wgs_free.argtypes = [ctypes.c_void_p]
        _lib = lib
    return _lib


@dataclass
class Dag:
    """wg_commits as numpy arrays (+ the per-row pills band)."""
    oid: np.ndarray          # uint8 [N, 20]
    time: np.ndarray         # int64 [N]
    parent_off: np.ndarray   # uint32 [N+1]
    parent_oid: np.ndarray   # uint8 [E, 20]
    flags: np.ndarray        # uint8 [N]
    band: np.ndarray         # float32 [N]

    @property
    def n(self) -> int:
        return int(self.time.shape[0])

    @property
    def e(self) -> int:
        return int(self.parent_oid.shape[0])

    def slice_rows(self, n: int) -> "Dag":
        """First n rows (parents beyond the cut become out-of-list ids, as
        with the reference's COMMIT_LIMIT truncation, repo_tab.rs:105)."""
        e = int(self.parent_off[n])
        return Dag(self.oid[:n].copy(), self.time[:n].copy(), self.parent_off[:n + 1].copy(),
                   self.parent_oid[:e].copy(), self.flags[:n].copy(), self.band[:n].copy())


def params(kind: int, n: int, seed: int | None = None) -> Params:
    p = Params()
    rc = _load().wgs_preset(kind, n, SEED_BASE + kind if seed is None else seed, ctypes.byref(p))
    if rc != 0:
        raise ValueError(f"unknown preset {kind}")
    return p


def generate(kind: int | str, n: int, seed: int | None = None, **overrides) -> Dag:
    if isinstance(kind, str):
        kind = PRESETS[kind]
    p = params(kind, n, seed)
    for k, v in overrides.items():
        setattr(p, k, v)
    lib = _load()
    h = lib.wgs_generate(ctypes.byref(p))
    if not h:
        raise MemoryError("wgs_generate failed")
    try:
        nn, ee = ctypes.c_uint64(), ctypes.c_uint64()
        lib.wgs_sizes(h, ctypes.byref(nn), ctypes.byref(ee))
        N, E = nn.value, ee.value
        d = Dag(np.empty((N, 20), np.uint8), np.empty(N, np.int64), np.empty(N + 1, np.uint32),
                np.empty((E, 20), np.uint8), np.empty(N, np.uint8), np.empty(N, np.float32))
        lib.wgs_copy(h, d.oid.ctypes.data, d.time.ctypes.data, d.parent_off.ctypes.data,
                     d.parent_oid.ctypes.data, d.flags.ctypes.data, d.band.ctypes.data)
        return d
    finally:
        lib.wgs_free(h)


def prepend_commits(d: Dag, k: int, seed: int = 7) -> Dag:
    """The list after k new commits land on the current head (a refresh:
    apply_state_result -> rebuild_synthetic_entries, repo_tab.rs:790-861,
    973-979): rows 0..k-1 are a new first-parent chain, newest first, whose
    last commit's parent is the old row 0; every old row moves down by k."""
    rng = np.random.default_rng(seed)
    oid = rng.integers(0, 256, (k, 20), dtype=np.uint8)
    t0 = int(d.time[0]) if d.n else 1704067200
    time = (t0 + 60 * np.arange(k, 0, -1)).astype(np.int64)
    if d.n:
        new_par = np.concatenate([oid[1:], d.oid[:1]])
    else:
        new_par = oid[1:]
    m = len(new_par)   # k, or k - 1 on an empty base list (the last new commit has no parent)
    poff = np.concatenate([np.minimum(np.arange(k), m), d.parent_off.astype(np.int64) + m]).astype(np.uint32)
    return Dag(np.concatenate([oid, d.oid]), np.concatenate([time, d.time]), poff,
               np.concatenate([new_par, d.parent_oid]), np.concatenate([np.zeros(k, np.uint8), d.flags]),
               np.concatenate([np.zeros(k, np.float32), d.band]))


def save(d: Dag, path: str) -> None:
    np.savez_compressed(path, oid=d.oid, time=d.time, parent_off=d.parent_off,
                        parent_oid=d.parent_oid, flags=d.flags, band=d.band)


def load(path: str) -> Dag:
    z = np.load(path, allow_pickle=False)
    return Dag(z["oid"], z["time"], z["parent_off"], z["parent_oid"], z["flags"], z["band"])


_WORDS = (b"fix add remove update refactor merge branch into main for the of in to a with and bug test docs build "
          b"cache lane graph layout render atlas kernel shard commit parser stream buffer index config api client "
          b"server handle error path memory leak race speed up cleanup bump version deps revert wip tweak rename "
          b"move split support allow use make drop check ensure avoid guard") .split()


def summaries(n: int, seed: int = 0, mean_words: float = 6.0, p_empty: float = 0.02):
    """Synthetic commit summaries for n rows: (bytes uint8 array, offsets
    uint64 [n+1]).  Lowercase words, a capitalised first word, ~2% empty rows
    ("(no summary)") and ~1% non-ASCII bytes (drawn as '?')."""
    rng = np.random.default_rng(0xC0FFEE + seed)
    vocab = np.frombuffer(b"".join(_WORDS), np.uint8)
    vlen = np.array([len(w) for w in _WORDS], np.int64)
    vstart = np.concatenate([[0], np.cumsum(vlen)[:-1]])
    counts = rng.poisson(mean_words, n).clip(1, 14)
    counts[rng.random(n) < p_empty] = 0
    ids = rng.integers(0, len(_WORDS), int(counts.sum()))
    wl = vlen[ids] + 1                                  # word + separator
    row_of = np.repeat(np.arange(n), counts)
    row_bytes = np.zeros(n, np.int64)
    np.add.at(row_bytes, row_of, wl)
    row_bytes = np.maximum(row_bytes - (counts > 0), 0)  # no trailing space
    off = np.concatenate([[0], np.cumsum(row_bytes)]).astype(np.uint64)
    out = np.full(int(off[-1]) + int(counts.sum()) + 1, ord(" "), np.uint8)
    # place words at running positions within each row
    wstart_in_row = np.cumsum(wl) - wl
    first_word = np.concatenate([[0], np.cumsum(counts)[:-1]])
    wstart_in_row = wstart_in_row - np.repeat(wstart_in_row[first_word[counts > 0]], counts[counts > 0])
    pos = off[row_of].astype(np.int64) + wstart_in_row
    total = int(vlen[ids].sum())
    src = np.repeat(vstart[ids], vlen[ids]) + (np.arange(total) - np.repeat(np.cumsum(vlen[ids]) - vlen[ids], vlen[ids]))
    dst = np.repeat(pos, vlen[ids]) + (np.arange(total) - np.repeat(np.cumsum(vlen[ids]) - vlen[ids], vlen[ids]))
    out[dst] = vocab[src]
    out = out[:int(off[-1])]
    firsts = off[:-1][counts > 0].astype(np.int64)
    out[firsts] = np.where((out[firsts] >= 97) & (out[firsts] <= 122), out[firsts] - 32, out[firsts])
    odd = rng.random(out.size) < 0.01
    out[odd & (out != ord(" "))] = 0xC3
    return out, off


# Non-ASCII words for the search fields: Latin-1 / Extended-A letters, Greek
# with final-sigma contexts, Turkish dotted I, Kelvin / capital sharp s,
# titlecase digraphs, Cyrillic, CJK, an emoji, combining marks.
_UNI_WORDS = [w.encode() for w in (
    "Naïve", "FAÇADE", "Ørjan", "Ødegård", "ŁUKASZ", "Żółć", "Grüße", "STRAẞE", "İstanbul", "İİ", "ΣΟΦΙΑ", "ΌΔΟΣ",
    "Σ", "ΑΣ.", "ΑΣ'Σ", "ΣΑΣ:ΣΑ", "Οδυσσεύς", "ΦΩΣ", "ǅemal", "ǈubljana", "ᾼ", "Kelvin", "Ångström", "ДМИТРИЙ",
    "Москва", "日本語", "🚀", "éclair", "ΆͅΣ", "ΣΣ", "ⅫΣ")]
_NAMES = [w.encode() for w in (
    "Linus Torvalds", "Greg Kroah-Hartman", "José García", "Łukasz Nowak", "Ørjan Ødegård", "Σωκράτης ΠΑΠΑΔΟΠΟΥΛΟΣ",
    "İlker Yılmaz", "Дмитрий Иванов", "山田 太郎", "Zoë Ångström", "ǅemal Ǉubić", "dependabot[bot]", "Unknown",
    "ANNA-LENA MÜLLER", "Chloé Dubois", "Anders Ösäter")]


def _join_words(rng, n, vocab, counts, sep=b" "):
    """Rows of `counts[i]` words drawn from vocab joined by sep: (bytes, offsets)."""
    vb = np.frombuffer(b"".join(vocab), np.uint8)
    vlen = np.array([len(w) for w in vocab], np.int64)
    vstart = np.concatenate([[0], np.cumsum(vlen)[:-1]])
    ids = rng.integers(0, len(vocab), int(counts.sum()))
    wl = vlen[ids]
    row_of = np.repeat(np.arange(n), counts)
    row_bytes = np.zeros(n, np.int64)
    np.add.at(row_bytes, row_of, wl + len(sep))
    row_bytes = np.maximum(row_bytes - len(sep) * (counts > 0), 0)
    off = np.concatenate([[0], np.cumsum(row_bytes)]).astype(np.uint64)
    out = np.empty(int(off[-1]), np.uint8)
    if out.size:
        # word k of row i starts at off[i] + (sum of the earlier words of row i + separators)
        first = np.concatenate([[0], np.cumsum(counts)[:-1]])
        cum = np.cumsum(wl + len(sep)) - (wl + len(sep))
        start = off[row_of].astype(np.int64) + cum - np.repeat(cum[first[counts > 0]], counts[counts > 0])
        seps = start[np.concatenate([np.diff(row_of) == 0, [False]])] + wl[np.concatenate([np.diff(row_of) == 0, [False]])]
        for k, b in enumerate(sep):
            out[seps + k] = b
        tot = int(wl.sum())
        inner = np.arange(tot) - np.repeat(np.cumsum(wl) - wl, wl)
        out[np.repeat(start, wl) + inner] = vb[np.repeat(vstart[ids], wl) + inner]
    return out, off


def text_fields(n: int, seed: int = 0, p_unicode: float = 0.15):
    """Search fields for n rows (commit_matches_query, commit_graph.rs:1509-1523):
    summaries (ASCII words with ~p_unicode non-ASCII words, ~2% empty) and
    authors (a name pool with non-ASCII names), each as (bytes, offsets[n+1])."""
    rng = np.random.default_rng(0x5EA4C + seed)
    counts = rng.poisson(6.0, n).clip(1, 14)
    counts[rng.random(n) < 0.02] = 0
    ascii_words = [w.capitalize() if i % 7 == 0 else w for i, w in enumerate(_WORDS)]
    n_uni = max(1, int(round(len(ascii_words) * p_unicode / (1 - p_unicode))))
    vocab = ascii_words + [_UNI_WORDS[i % len(_UNI_WORDS)] for i in range(n_uni)]
    summ = _join_words(rng, n, vocab, counts)
    auth = _join_words(rng, n, _NAMES, np.ones(n, np.int64))
    return summ, auth
