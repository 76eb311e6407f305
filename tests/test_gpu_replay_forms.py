"""Every form of the lane replay, asserted by name (VERDICT r04 "next" #1).

The lane events (wg_lanes_fast.hip) are replayed by one of several kernels,
chosen per context from the list it built last:

* 100 + words: the chunked fixed point (wg_lanes_replay.hip), 1 / 4 / 16 words;
* 200 + words: the exact single-wave serial pass (wg_lanes_serial.hip) at 1,
  3, 4, 8 or 16 words of slots (63 / 191 / 255 / 511 / 1023), 264 = the
  16-wave workgroup (4095 slots); the 3- and 8-word forms are taken when the
  context's last list held at most 170 / 448 slots, and a list past their
  width is redone at the full width;
* 300 + words: the compacted fixed point (wg_lanes_dchunk.hip): the slots
  leaked by parents at earlier rows (commit_graph.rs:441-446; git/mod.rs:
  767-772 re-sorts reflog orphans by time) struck out of the slot order.

wg_debug_counters [12] names the form the last replay took.  Each case primes
a fresh context with the lists that set its state, then builds the list under
test (exactly, then speculatively), asserting the form of every build and
the results bit-exact against the C oracle: lanes, colours, edges, max_lane,
slot count (commit_graph.rs:276-320, 401-471).  The same sequences run on
row-sharded contexts (3 ranks in lockstep, the global replay on every rank).
"""
import os

import numpy as np
import pytest

from wgraph import synth

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_LISTS = {}


def _list(kind, n, **over):
    key = (kind, n, tuple(sorted(over.items())))
    if key not in _LISTS:
        d = synth.generate(kind, n, seed=515, **over)
        from oracle import oracle_c
        o = oracle_c.OracleLayout(d)
        want = dict(lane=o.lane.astype(np.uint32).copy(), color=o.color.copy(), edges=o.edges.copy(),
                    max_lane=int(o.max_lane), n_slots=int(o.n_slots))
        o.close()
        _LISTS[key] = (d, want)
    return _LISTS[key]


def _check(eng, want, tag):
    s = eng.layout_summary()
    assert s.lane_path == 0, f"{tag}: left the parallel lane path"
    assert (s.max_lane, s.n_slots) == (want["max_lane"], want["n_slots"]), tag
    lane, color = eng.lanes()
    assert lane.tobytes() == want["lane"].tobytes(), (tag, np.nonzero(lane != want["lane"])[0][:5])
    assert color.tobytes() == want["color"].tobytes(), tag
    assert eng.edges().tobytes() == want["edges"].tobytes(), tag


# (mode, [(list, expected form per build)]): the lists are (kind, n, overrides)
LIN = lambda m: ("linux", 60_000, {"max_lines": m})   # noqa: E731  (slots = max_lines on this shape)
WIDE = ("linuxwide", 60_000, {})                       # 160 slots
SKEW = ("skew", 200_000, {})                           # 1 word, leaked slots
SERIAL_SEQS = {
    "serial-1w": (2, [(SKEW, [201, 201])]),
    # fresh context: 1 -> 4 words (204); then the 3-word form (160 <= 170 slots)
    "serial-3w": (2, [(WIDE, [204, 203, 203])]),
    "serial-4w": (2, [(LIN(240), [204, 204])]),
    # 400 slots: 16 words first, then the 8-word form (400 <= 448)
    "serial-8w": (2, [(LIN(400), [216, 208, 208])]),
    "serial-16w": (2, [(LIN(600), [216, 216])]),
    "serial-workgroup": (2, [(("linux", 200_000, {"max_lines": 1500}), [264, 264])]),
    # a 3-word context (160 slots) meets 191 slots (the form's width: fits) and
    # 192 / 200 (past it: redone at the full 4 words); in between, 160 slots
    # again bring the 3-word form back
    "serial-3w-overflow": (2, [(WIDE, [204, 203]), (LIN(191), [203]), (WIDE, [204, 203]), (LIN(192), [204]),
                               (WIDE, [204, 203]), (LIN(200), [204, 204])]),
    # an 8-word context (400 slots) meets 511 slots (fits) and 512 / 600 (redone at 16 words)
    "serial-8w-overflow": (2, [(LIN(400), [216, 208]), (LIN(511), [208]), (LIN(400), [216, 208]), (LIN(512), [216]),
                               (LIN(400), [216, 208]), (LIN(600), [216])]),
    "chunked-1w": (1, [(("wide16", 200_000, {}), [101, 101])]),
    "chunked-4w": (1, [(WIDE, [104, 104])]),
    "compacted-1w": (3, [(SKEW, [301, 301, 301])]),
    # leaked slots struck out: 90 slots replayed in one word
    "compacted-leaky": (3, [(("skew", 100_000, {"p_clock_skew": 2e-3}), [301, 301])]),
    # 160 live slots: the compacted replay widens to 4 words of positions (1 -> 2 -> 4)
    "compacted-4w": (3, [(WIDE, [304, 304])]),
    # past 255 live positions the compacted replay does not apply: the serial pass
    "compacted-too-wide": (3, [(LIN(400), [216, 208])]),
}


def _run_single(mode, seq):
    import wgraph
    eng = wgraph.Engine(0)
    try:
        eng.set_replay_mode(mode)
        for (kind, n, over), forms in seq:
            d, want = _list(kind, n, **over)
            for i, form in enumerate(forms):
                tag = f"{kind}/{n}/{over} build {i}"
                eng.build(d)
                _check(eng, want, tag)
                got = int(eng.debug_counters()[12])
                assert got == form, f"{tag}: form {got}, expected {form}"
    finally:
        eng.close()


@pytest.mark.parametrize("name", list(SERIAL_SEQS))
def test_replay_form_single_gpu(name):
    mode, seq = SERIAL_SEQS[name]
    _run_single(mode, seq)


def _run_sharded(mode, seq, world=3):
    """The same sequence on `world` row-sharded engines in lockstep: every
    rank replays the global event stream; lanes of its rows, max_lane and the
    slot count equal the oracle's, the form is the same on every rank."""
    import ctypes

    import torch
    import wgraph
    from test_gpu_shard import _lockstep
    from wgraph import abi, lib
    from wgraph.shard import shard_rows

    dev = torch.device("cuda", 0)
    ts = torch.cuda.Stream(dev)
    ts.wait_stream(torch.cuda.current_stream(dev))
    stream_ctx = torch.cuda.stream(ts)
    stream_ctx.__enter__()
    engines = [wgraph.Engine(0) for _ in range(world)]
    try:
        for e in engines:
            e.set_stream(ts.cuda_stream)
            e.set_replay_mode(mode)
        for (kind, n, over), forms in seq:
            d, want = _list(kind, n, **over)
            keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                           d.parent_oid.reshape(-1), d.flags, d.band)]
            c = abi.Commits()
            c.n_commits, c.n_parents = d.n, d.e
            c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
            c.residency = abi.WG_DEVICE
            rng = [shard_rows(d.n, world, r) for r in range(world)]
            for i, form in enumerate(forms):
                tag = f"{kind}/{n}/{over} sharded build {i}"
                _lockstep(engines, lambda e, r, m: lib().wg_shard_build_frame_begin(
                    e._ctx, ctypes.byref(c), world, r, rng[r][0], rng[r][1], keep[5].data_ptr(), abi.WG_DEVICE, m))
                for r, e in enumerate(engines):
                    s, t = rng[r]
                    dc = e.debug_counters()
                    assert int(dc[5]) == 1, f"{tag} rank {r}: not sharded"
                    ls_ = e.layout_summary()
                    assert (ls_.max_lane, ls_.n_slots) == (want["max_lane"], want["n_slots"]), f"{tag} rank {r}"
                    lane, color = e.lanes()
                    assert lane.tobytes() == want["lane"][s:t].tobytes(), f"{tag} rank {r} lanes"
                    assert color.tobytes() == want["color"][s:t].tobytes(), f"{tag} rank {r} colours"
                    assert int(dc[12]) == form, f"{tag} rank {r}: form {int(dc[12])}, expected {form}"
            torch.cuda.synchronize()
            del keep
    finally:
        for e in engines:
            e.close()
        stream_ctx.__exit__(None, None, None)


SHARD_SEQS = {
    "serial-3w-overflow": (2, [(WIDE, [204, 203]), (LIN(200), [204])]),
    "serial-8w-overflow": (2, [(LIN(400), [216, 208]), (LIN(600), [216])]),
    "compacted-1w": (3, [(SKEW, [301, 301])]),
    "compacted-leaky": (3, [(("skew", 100_000, {"p_clock_skew": 2e-3}), [301, 301])]),
}


@pytest.mark.parametrize("name", list(SHARD_SEQS))
def test_replay_form_sharded(name):
    mode, seq = SHARD_SEQS[name]
    _run_sharded(mode, seq)


def test_auto_mode_forms_follow_the_list():
    """Auto mode on one context: wide16 stays on the chunked replay; the
    skewed list (leaked slots) moves to the compacted replay within one build
    and stays exact; 160 concurrent lanes (positions past one word, the fixed
    point still late after the warm-up) end on a serial or compacted form;
    wide16 of a very different length starts the choice over."""
    import wgraph
    eng = wgraph.Engine(0)
    try:
        seq = [(("wide16", 200_000, {}), 100), (("skew", 200_000, {}), 300), (("skew", 200_000, {}), 300),
               (WIDE, None), (WIDE, None), (("wide16", 20_000, {}), 100)]
        for (kind, n, over), fam in seq:
            d, want = _list(kind, n, **over)
            eng.build(d)
            _check(eng, want, f"{kind}/{n}")
            form = int(eng.debug_counters()[12])
            if fam is not None:
                assert form // 100 * 100 == fam, f"{kind}/{n}: form {form}"
            else:
                assert form // 100 in (2, 3), f"{kind}/{n}: form {form}"
    finally:
        eng.close()


def test_leak_free_compacted_choice_expires():
    """a context moved off the chunked replay by a skewed
    list does not keep later lists of the same length there for good: after
    16 compacted builds that struck out no leaked slot the chunked replay is
    tried again (and wide16 then stays on it)."""
    import wgraph
    eng = wgraph.Engine(0)
    try:
        d, want = _list("skew", 200_000)
        eng.build(d)
        eng.build(d)
        assert int(eng.debug_counters()[12]) // 100 == 3
        w, wwant = _list("wide16", 200_000)
        forms = []
        for _ in range(18):
            eng.build(w)
            _check(eng, wwant, "wide16 after skew")
            forms.append(int(eng.debug_counters()[12]))
        assert forms[0] // 100 == 3, forms
        assert forms[-1] == 101, forms
    finally:
        eng.close()
