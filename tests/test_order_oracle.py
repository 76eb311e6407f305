"""CPU: the row-order oracle (commit_graph_with_orphans git/mod.rs:761-775,
insert_synthetics_sorted git/mod.rs:234-242) on hand-checked cases."""
import numpy as np

from oracle.order_oracle import order_rows


def test_no_orphans_keeps_the_walk_order():
    # no orphans: no re-sort, even when the walk is not time-ordered (clock skew)
    assert order_rows([5, 9, 1, 7]).tolist() == [0, 1, 2, 3]


def test_orphans_trigger_a_stable_sort_newest_first():
    # equal times keep their relative order (Rust sort_by_key is stable)
    assert order_rows([5, 4, 4, 3], [4, 6]).tolist() == [5, 0, 1, 2, 4, 3]


def test_synthetics_go_before_the_first_row_not_newer():
    # s0 (t=4) before walk row 1; s1 (t=4) before s0 (s0 already qualifies);
    # s2 (t=9) at the top; s3 (t=0) appended
    assert order_rows([5, 4, 4, 3], [4, 6], [4, 4, 9, 0]).tolist() == [8, 5, 0, 7, 6, 1, 2, 4, 3, 9]


def test_synthetic_into_an_unsorted_walk_uses_the_first_qualifying_row():
    assert order_rows([5, 9, 1, 7], [], [6]).tolist() == [4, 0, 1, 2, 3]   # 5 <= 6 already at row 0
    assert order_rows([], [], [3, 1, 2]).tolist() == [0, 2, 1]


def test_empty():
    assert order_rows([]).size == 0
