"""Host cost of one ShardComm exchange over a world-1 RCCL group (launch with
torch.distributed.run --nproc-per-node=1): pack path, 4 KiB messages, the
same calls bench.py's sharded step makes per exchange, timed end to end."""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))


def main():
    import torch
    import torch.distributed as dist
    from wgraph.shard import ShardComm
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend="nccl", init_method="env://", device_id=dev)
    comm = ShardComm(dev)
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
    stream = torch.cuda.current_stream().cuda_stream

    def pack(slot, cap):   # stand-in for wg_shard_pack_slot: one async device write on the stream
        hip.hipMemsetAsync(ctypes.c_void_p(slot), 0, 32, ctypes.c_void_p(stream))

    for _ in range(20):
        comm.allgather(0, None, step=1, pack=pack)
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        g, off, stride, sizes = comm.allgather(0, None, step=1, pack=pack)
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / n * 1e6
    print(f"ShardComm.allgather world=1 nccl: {us:.1f} us per exchange (pack path, header read to host)", flush=True)
    import numpy as np
    import wgraph
    eng = wgraph.Engine(0)
    eng.set_stream(stream)

    def read_heads(ptr, stride):   # the engine's polled read (what Engine._shard_loop passes)
        h = np.empty(3 * comm.world, np.uint64)
        rc = wgraph.lib().wg_shard_slot_heads(eng._ctx, ptr, stride, comm.world, h.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"wg_shard_slot_heads: {rc}")
        return h.reshape(comm.world, 3)

    for _ in range(20):
        comm.allgather(0, None, step=1, pack=pack, read_heads=read_heads)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        comm.allgather(0, None, step=1, pack=pack, read_heads=read_heads)
    torch.cuda.synchronize()
    print(f"ShardComm.allgather world=1 nccl, heads by wg_shard_slot_heads: "
          f"{(time.perf_counter() - t0) / n * 1e6:.1f} us per exchange", flush=True)
    x = torch.zeros(4096, dtype=torch.uint8, device=dev)
    out = torch.empty(4096, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        dist.all_gather_into_tensor(out, x)
    torch.cuda.synchronize()
    print(f"bare all_gather_into_tensor (no host read): {(time.perf_counter() - t0) / n * 1e6:.1f} us", flush=True)
    t0 = time.perf_counter()
    for _ in range(n):
        dist.all_gather_into_tensor(out, x)
        out[:32].cpu()
    print(f"all_gather + 32-byte host read: {(time.perf_counter() - t0) / n * 1e6:.1f} us", flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
