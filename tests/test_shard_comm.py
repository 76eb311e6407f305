"""Host plumbing of the row-sharded build: the variable-length all-gather
(wgraph.shard.ShardComm) over a world-size-2 gloo group on the CPU, and the
shard partition.  The engine side runs in tests/test_gpu_shard.py."""
import ctypes
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from wgraph.shard import ShardComm, shard_rows


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = ShardComm(torch.device("cpu"), initial_cap=64)
        got = []
        # lengths below, at and above the slot; the last two reuse step 3's grown slot
        for step, length in enumerate([0, 5, 37 + 11 * rank, 4096 * (rank + 1), 10, 3000]):
            payload = bytes((rank * 31 + step + i) & 0xFF for i in range(length))
            out, off, stride, sizes = comm.allgather(length, lambda ptr: ctypes.memmove(ptr, payload, length),
                                                     step=min(step, 3))
            got.append((stride, sizes, [bytes(out[off + r * stride:off + r * stride + sizes[r]].numpy())
                                        for r in range(world)], comm.heads.tobytes()))
        q.put((rank, got, (comm.exchanges, comm.collectives)))
    finally:
        dist.destroy_process_group()


def test_allgather_world2_gloo():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, n)) for r, g, n in (q.get(timeout=120) for _ in procs))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    lengths = [lambda r: 0, lambda r: 5, lambda r: 37 + 11 * r, lambda r: 4096 * (r + 1), lambda r: 10,
               lambda r: 3000]
    for step, length_of in enumerate(lengths):
        for rank in range(world):
            stride, sizes, msgs, heads = res[rank][0][step]
            assert sizes == [length_of(r) for r in range(world)]
            # host copy of each message's first 16 bytes (zero padded), handed to wg_shard_exchange
            assert heads == b"".join((msgs[r][:16] + bytes(16))[:16] for r in range(world))
            assert stride % 16 == 0 and stride >= max(max(sizes), 16)
            for r in range(world):
                assert msgs[r] == bytes((r * 31 + step + i) & 0xFF for i in range(length_of(r)))
    # one collective per exchange, plus one retry where the 64-byte slot had to grow (step 3)
    assert res[0][1] == (6, 7)


@pytest.mark.parametrize("n,world", [(0, 2), (1, 2), (7, 3), (1_000_000, 8), (8_000_000, 8)])
def test_shard_rows_partition(n, world):
    bounds = [shard_rows(n, world, r) for r in range(world)]
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    for (a, b), (c, d) in zip(bounds, bounds[1:]):
        assert b == c and a <= b
    assert max(b - a for a, b in bounds) - min(b - a for a, b in bounds) <= 1


@pytest.mark.parametrize("initial,want", [(0, 16), (1, 16), (15, 16), (16, 16), (17, 32), (4096, 4096), (4100, 4112)])
def test_initial_slot_is_a_valid_pack_capacity(initial, want):
    """wg_shard_pack_slot takes capacities that are multiples of 16, >= 16 (its
    header kernel writes 32 bytes): the first exchange uses the rounded cap."""
    port = _free_port()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        assert ShardComm(torch.device("cpu"), initial_cap=initial).initial_cap == want
        with pytest.raises(ValueError):
            ShardComm(torch.device("cpu"), device_transport=True)
    finally:
        dist.destroy_process_group()
