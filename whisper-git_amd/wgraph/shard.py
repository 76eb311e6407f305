"""All-gather plumbing for row-sharded builds (include/wgraph.h, wg_shard_*).

The engine packs one message per exchange point; every rank's message is
all-gathered over a torch.distributed group (backend "nccl" = RCCL over xGMI
on MI355X, or "gloo" on the host) and handed back to the engine as one
device buffer: rank r's message at r * stride.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["ShardComm", "shard_rows"]


def shard_rows(n: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous row shard of rank `rank`: [n*rank/world, n*(rank+1)/world)."""
    return n * rank // world, n * (rank + 1) // world


class ShardComm:
    """Variable-length byte all-gather, one collective per exchange.

    device: the CUDA (HIP) device the engine runs on; the gathered buffer is
    always returned there.  With a gloo group the exchange itself runs on host
    tensors (copied in and out), with nccl it stays in HBM.

    Every message travels in a slot of `cap + 16` bytes: a 16-byte header
    holding its length, then the payload.  `cap` is remembered per exchange
    point (the engine numbers them), so steady-state steps move each
    message with ONE all-gather; a message longer than the slot makes every
    rank (they all see the same lengths) repeat that exchange with a larger
    slot.
    """

    HDR = 16

    def __init__(self, device: torch.device, group=None, initial_cap: int = 4096, device_transport: bool | None = None):
        """device_transport: gather device-resident slots (default: only on an
        "nccl" group).  True on a gloo group moves HIP tensors through gloo,
        which lets several ranks on ONE GPU (RCCL refuses a duplicate GPU)
        exercise the stream-ordered slot path bench.py takes over RCCL."""
        self.device = device
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.on_device = self.backend == "nccl" if device_transport is None else bool(device_transport)
        if self.on_device and device.type == "cpu":
            raise ValueError("a device transport needs a HIP device")
        self.initial_cap = self.round_cap(initial_cap)   # wg_shard_pack_slot takes caps of 16k bytes, k >= 1
        self.caps: dict[int, int] = {}
        self.exchanges = 0
        self.collectives = 0
        self.bytes_sent = 0
        # seam-exchange timing (set_timing): host seconds inside allgather (the
        # wait for the producing kernels, the collective and the heads) and,
        # on a device transport, HIP events around every collective on the stream
        self.timing = False
        self.host_s = 0.0
        self._events = []
        self._x0 = 0
        self.heads = None   # host copy of every message's first 16 bytes (uint32 [world, 4]), last exchange

    def set_timing(self, on: bool):
        """Start (True: counters reset) or stop recording the exchange times."""
        self.timing = on
        if on:
            self.host_s = 0.0
            self._events = []
            self._x0 = self.exchanges

    def timing_report(self) -> dict:
        """{'exchanges', 'host_ms', 'collective_ms'} since set_timing(True);
        collective_ms (device transport) sums the collectives' own GPU time."""
        coll = None
        if self._events:
            torch.cuda.synchronize(self.device)
            coll = sum(a.elapsed_time(b) for a, b in self._events)
        return {"exchanges": self.exchanges - self._x0, "host_ms": self.host_s * 1e3, "collective_ms": coll}

    @staticmethod
    def round_cap(n: int) -> int:
        """Slot payload capacity for an n-byte message: 16-byte aligned, >= 16."""
        m = max(n, 16)
        return (m + 15) // 16 * 16

    def allgather(self, nbytes: int, fill, step: int = 0, pack=None, read_heads=None):
        """fill(ptr) writes this rank's nbytes-long message to ptr (device or
        host memory); or, on a device transport, pack(slot_ptr, cap) writes the
        whole slot (header + message) in stream order on the current stream,
        and read_heads(ptr, stride) (optional) returns every slot's length and
        message header as a (world, 3) uint64 array, read in stream order.
        Returns (gathered device tensor, payload offset, stride, sizes): rank
        r's message starts at offset + r * stride."""
        import time
        t_host = time.perf_counter() if self.timing else 0.0
        dev = self.device if self.on_device else torch.device("cpu")
        cap = self.caps.get(step, self.initial_cap)
        while True:
            stride = cap + self.HDR
            if self.on_device and pack is not None:
                send = torch.empty(stride, dtype=torch.uint8, device=dev)
                pack(send.data_ptr(), cap)
            else:
                send = torch.zeros(stride, dtype=torch.uint8, device=dev)
                send[:8].view(torch.int64)[0] = nbytes
                if nbytes and nbytes <= cap:
                    fill(send.data_ptr() + self.HDR)
            out = torch.empty(self.world * stride, dtype=torch.uint8, device=dev)
            if self.on_device and self.backend == "nccl":
                if self.timing:
                    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    ev[0].record()
                dist.all_gather_into_tensor(out, send, group=self.group)
                if self.timing:
                    ev[1].record()
                    self._events.append(ev)
            else:
                dist.all_gather(list(out.view(self.world, stride).unbind(0)), send, group=self.group)
            self.collectives += 1
            # one device->host read: every slot's length and its message's 16-byte header
            if self.on_device and read_heads is not None:
                h = read_heads(out.data_ptr(), stride)
                sizes = [int(x) for x in h[:, 0]]
                self.heads = np.ascontiguousarray(h[:, 1:3]).view(np.uint32).reshape(self.world, 4)
            else:
                head = out.view(self.world, stride)[:, :32].cpu().numpy()
                sizes = [int(x) for x in head[:, :8].copy().view(np.int64).reshape(-1)]
                self.heads = np.ascontiguousarray(head[:, 16:32]).view(np.uint32).reshape(self.world, 4)
            if max(sizes) <= cap:
                break
            cap = self.round_cap(max(sizes))
        self.caps[step] = cap
        if not self.on_device and self.device.type != "cpu":
            out = out.to(self.device)
        if self.device.type != "cpu" and not self.on_device:
            torch.cuda.current_stream(self.device).synchronize()   # the H2D copy above
        self.exchanges += 1
        self.bytes_sent += sizes[self.rank]   # nbytes is 0 when the length lives on the device
        if self.timing:
            self.host_s += time.perf_counter() - t_host
        return out, self.HDR, stride, sizes
