"""Row-sharded multi-GPU build against the oracle.

world ranks (gloo group, all on cuda:0 of the test box) each build their
contiguous row shard through the C ABI's exchange protocol; every shard's
lanes, edges, heights, both geometries and vertex buffers must equal the
oracle's whole-list results restricted to the shard, bit for bit.  The
anomaly preset (duplicate ids, skewed parents) exercises the whole-list
fallback, which must give the same answers.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(world, cases, tmp_path):
    out = tmp_path / f"w{world}"
    out.mkdir()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.join(ROOT, "tests", "shard_worker.py"), "--cases", cases, "--out", str(out)]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=ROOT, env=env, timeout=600, capture_output=True, text=True)
    results = []
    for r in range(world):
        f = out / f"rank{r}.json"
        assert f.exists(), f"rank {r} wrote nothing; rc={p.returncode}\n{p.stderr[-3000:]}"
        results.append(json.loads(f.read_text()))
    for r, res in enumerate(results):
        assert res["ok"], f"rank {r}: " + "\n".join(res["errors"])
    return results


def test_two_shards(tmp_path):
    run_world(2, "wide16:60000:3,random13:30000:4,linux:40000:5,linear:5000:6,anomaly:3000:7,wide16:3:8", tmp_path)


def test_three_shards(tmp_path):
    run_world(3, "random13:20000:11,wide16:1000:12,linux:25000:13", tmp_path)


def test_two_shards_row_top_beyond_2_25(tmp_path):
    """1.4M linux-shaped rows: rank 1's row_top prefix crosses 2^24 and 2^25
    (transducer walk over super-chunks) and its shard sums past 2^25."""
    run_world(2, "linux:1400000:31", tmp_path)


def test_four_shards_small(tmp_path):
    run_world(4, "wide16:4000:21,random13:64:22", tmp_path)
