"""WG-TEXT-1 oracle pieces on the CPU: format_relative_time thresholds
(git/mod.rs:34-49), short SHA (git/mod.rs:300), and the synthetic summaries."""
import numpy as np
import pytest

from oracle import text_oracle as to
from wgraph import synth

NOW = 1_700_000_000


@pytest.mark.parametrize("age,want", [
    (-5, b"just now"), (0, b"just now"), (59, b"just now"), (60, b"1m"), (3599, b"59m"), (3600, b"1h"),
    (86399, b"23h"), (86400, b"1d"), (604799, b"6d"), (604800, b"1w"), (2591999, b"4w"), (2592000, b"1mo"),
    (31535999, b"12mo"), (31536000, b"1y"), (10 * 31536000 + 5, b"10y")])
def test_relative_time_thresholds(age, want):
    assert to.relative_time(NOW, NOW - age) == want


def test_short_id_is_first_seven_hex_digits():
    oid = np.frombuffer(bytes.fromhex("0a1b2c3d4e5f60718293a4b5c6d7e8f901234567"), np.uint8)
    assert to.short_id(oid) == b"0a1b2c3"


def test_synthetic_summaries_shape():
    b, o = synth.summaries(5000, seed=2)
    assert o[0] == 0 and o[-1] == len(b) and (np.diff(o.astype(np.int64)) >= 0).all()
    lens = np.diff(o.astype(np.int64))
    assert 0 < (lens == 0).mean() < 0.06
    assert 20 < lens[lens > 0].mean() < 60
    assert (b == 0xC3).any()
