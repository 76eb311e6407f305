"""All-gather plumbing for row-sharded builds (include/wgraph.h, wg_shard_*).

The engine packs one message per exchange point; every rank's message is
all-gathered over a torch.distributed group (backend "nccl" = RCCL over xGMI
on MI355X, or "gloo" on the host) and handed back to the engine as one
device buffer: rank r's message at r * stride.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

__all__ = ["ShardComm", "shard_rows"]


def shard_rows(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous row shard of rank `rank`: [n*rank/world, n*(rank+1)/world)."""
    return n * rank // world, n * (rank + 1) // world


class ShardComm:
    """Variable-length byte all-gather.

    device: the CUDA (HIP) device the engine runs on; the gathered buffer is
    always returned there.  With a gloo group the exchange itself runs on host
    tensors (copied in and out), with nccl it stays in HBM.
    """

    def __init__(self, device: torch.device, group=None):
        self.device = device
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.on_device = dist.get_backend(group) == "nccl"
        self.exchanges = 0
        self.bytes_sent = 0

    @staticmethod
    def layout(sizes: list[int]) -> int:
        """Stride of the gathered buffer: the largest message, 16-byte aligned (>= 16)."""
        m = max(max(sizes), 16)
        return (m + 15) // 16 * 16

    def allgather(self, nbytes: int, fill):
        """fill(ptr) writes this rank's nbytes-long message to ptr (device or
        host memory).  Returns (gathered device tensor, stride, sizes)."""
        dev = self.device if self.on_device else torch.device("cpu")
        n = torch.tensor([nbytes], dtype=torch.int64, device=dev)
        ns = [torch.empty_like(n) for _ in range(self.world)]
        dist.all_gather(ns, n, group=self.group)
        sizes = [int(x.item()) for x in ns]
        stride = self.layout(sizes)
        send = torch.zeros(stride, dtype=torch.uint8, device=dev)
        if nbytes:
            fill(send.data_ptr())
        out = torch.empty(self.world * stride, dtype=torch.uint8, device=dev)
        if self.on_device:
            dist.all_gather_into_tensor(out, send, group=self.group)
            torch.cuda.current_stream(self.device).synchronize()
        else:
            dist.all_gather(list(out.view(self.world, stride).unbind(0)), send, group=self.group)
            if self.device.type != "cpu":
                out = out.to(self.device)
                torch.cuda.synchronize(self.device)
        self.exchanges += 1
        self.bytes_sent += nbytes
        return out, stride, sizes
