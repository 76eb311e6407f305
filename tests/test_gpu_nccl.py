"""RCCL transport of the row-sharded build (bench.py --gpus N > 1): a
world-1 "nccl" process group on the test box's GPU drives ShardComm through
both slot paths.  (Several ranks on one GPU is not an RCCL configuration;
the multi-rank protocol itself is covered over gloo in test_gpu_shard.py.)"""
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


def test_rccl_shard_transport(tmp_path):
    out = tmp_path / "rank0.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={free_port()}",
           os.path.join(ROOT, "tests", "nccl_worker.py"), str(out)]
    p = subprocess.run(cmd, cwd=ROOT, timeout=240, capture_output=True, text=True)
    assert out.exists(), f"worker wrote nothing; rc={p.returncode}\n{p.stderr[-3000:]}"
    res = json.loads(out.read_text())
    assert res["ok"], "\n".join(res["errors"])
    assert res["exchanges"] == 12 and res["collectives"] > 12   # overflowing messages were re-sent
