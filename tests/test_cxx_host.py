"""The C++ host side (whisper-git_amd/host/graph_layout.hpp): GraphLayout,
compute_row_heights and the reference's types over the C ABI, exercised by
the compiled test binary tests/cpp/test_graph_layout (built by `make`).

CPU: the binary lists its tests and, with no GPU, GraphLayout refuses with
WG_E_NODEVICE (no host fallback).  GPU: every test — the reference's known
answers at the GraphLayout boundary and bit-exact parity with the oracle."""
import os
import subprocess

import pytest

from conftest import ROOT

BIN = os.path.join(ROOT, "tests", "cpp", "test_graph_layout")


def run(*args, timeout=300):
    assert os.path.exists(BIN), "tests/cpp/test_graph_layout not built (make)"
    return subprocess.run([BIN, *args], capture_output=True, text=True, timeout=timeout)


def test_cxx_tests_listed():
    p = run("--list")
    assert p.returncode == 0
    names = p.stdout.split()
    for kat in ("compute_row_heights_clamps_to_min_for_dense_commits",
                "compute_row_heights_saturates_at_max_for_long_gaps",
                "decompose_same_lane_emits_top_full_bottom_verticals",
                "decompose_cross_lane_emits_one_curve_per_spanned_row",
                "decompose_cross_lane_segment_y_spans_row_strip",
                "cubic_t_at_y_recovers_endpoints", "cubic_subcurve_endpoints_match_y_at"):
        assert kat in names
    assert sum(n.startswith("parity_") for n in names) >= 5


def test_cxx_graph_layout_refuses_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    p = run("--no-device")
    assert p.returncode == 0, p.stdout + p.stderr
    assert "status -6" in p.stdout


@pytest.mark.gpu
def test_cxx_graph_layout_on_gpu():
    p = run()
    assert p.returncode == 0, p.stdout[-4000:] + p.stderr[-2000:]
    assert "FAIL" not in p.stdout
