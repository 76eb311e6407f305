"""One rank of a world-1 RCCL job (tests/test_gpu_nccl.py): ShardComm over
the "nccl" backend — the transport bench.py uses for N > 1 — through both the
stream-ordered slot path (pack, heads read by the engine's polled
wg_shard_slot_heads) and the copy-out path (fill), with messages that
overflow the slot (the retry grows it), checked byte for byte."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))


def main():
    import numpy as np
    import torch
    import torch.distributed as dist
    import wgraph
    from wgraph.shard import ShardComm

    out = sys.argv[1]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group(backend="nccl", init_method="env://", device_id=dev)
    # torch's HIP runtime (already loaded under this SONAME): raw device copies
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

    def d2d(dst, src_ptr, n):
        torch.cuda.current_stream().synchronize()
        if n and hip.hipMemcpy(ctypes.c_void_p(dst), ctypes.c_void_p(src_ptr), n, 3) != 0:
            raise RuntimeError("hipMemcpy failed")

    errors = []
    try:
        comm = ShardComm(dev, initial_cap=64)
        # a non-default stream shared with torch (its collectives and slot
        # buffers): handle 0, the default stream, would give the engine one of its own
        ts = torch.cuda.Stream(dev)
        ts.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(ts)
        eng = wgraph.Engine(0)
        eng.set_stream(ts.cuda_stream)

        def read_heads(ptr, stride):
            h = np.empty(3 * comm.world, np.uint64)
            rc = wgraph.lib().wg_shard_slot_heads(eng._ctx, ptr, stride, comm.world, h.ctypes.data)
            if rc != 0:
                raise RuntimeError(f"wg_shard_slot_heads: {rc}")
            return h.reshape(comm.world, 3)
        if not comm.on_device:
            errors.append("nccl group not on device")
        rng = np.random.default_rng(1)
        comm.set_timing(True)   # bench.py's seam-exchange breakdown over RCCL
        for use_pack in (True, False):
            for step, n in enumerate([0, 5, 64, 200, 4096, 100]):   # 200 / 4096 overflow the slot
                msg = torch.from_numpy(rng.integers(0, 256, max(n, 1), dtype=np.uint8)).to(dev)

                def fill(ptr):
                    d2d(ptr, msg.data_ptr(), n)

                def pack(slot, cap):   # wg_shard_pack_slot's layout: u64 length, zeros, payload
                    head = np.zeros(32, np.uint8)
                    head[:8] = np.frombuffer(np.int64(n).tobytes(), np.uint8)
                    h = torch.from_numpy(head).to(dev)
                    d2d(slot, h.data_ptr(), 32)
                    if n and n <= cap:
                        d2d(slot + 16, msg.data_ptr(), n)

                g, off, stride, sizes = comm.allgather(n, fill, step=step + (100 if use_pack else 0),
                                                       pack=pack if use_pack else None,
                                                       read_heads=read_heads if use_pack else None)
                tag = f"{'pack' if use_pack else 'fill'} step {step} n {n}"
                if sizes != [n]:
                    errors.append(f"{tag}: sizes {sizes}")
                got = g[off:off + n].cpu().numpy().tobytes() if n else b""
                want = msg[:n].cpu().numpy().tobytes() if n else b""
                if got != want:
                    errors.append(f"{tag}: payload differs")
                if comm.heads.tobytes() != (want + bytes(16))[:16]:
                    errors.append(f"{tag}: heads differ")
        rep = comm.timing_report()
        if rep["exchanges"] != 12 or not (rep["collective_ms"] or 0) > 0 or not rep["host_ms"] > 0:
            errors.append(f"timing report {rep}")
        res = {"ok": not errors, "errors": errors, "collectives": comm.collectives, "exchanges": comm.exchanges}
    except Exception:   # report, do not hang the launcher
        import traceback
        res = {"ok": False, "errors": errors + [traceback.format_exc()]}
    with open(out, "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
