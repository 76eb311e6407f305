"""Frame pipelining probe: the bench step (build + banded geometry + vertex
emission of a 1M-row wide16 list) run K times
  seq        one engine on one stream (bench.py's step, one after the other);
  pipe2      two engines, each on its own stream, step i on engine i % 2;
  split*     two engines; build + geometry on a build stream, emission on an
             emission stream (event-ordered both ways), so step i's emission
             (HBM-write-bound, ~1 ms) can run beside step i+1's build
             (latency-bound small kernels and host waits):
    split      plain streams
    split_prio build streams high priority
    split_mK   emission streams CU-masked off the first K mask bits
    split_bK   ... and build streams restricted to those K bits
  emit_mK    emission alone on a CU-masked stream (bandwidth it loses)
usage: python3 profiles/pipeline_probe.py [steps]
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))


def main():
    import torch
    import wgraph
    from wgraph import abi, synth

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    props = torch.cuda.get_device_properties(dev)
    ncu = props.multi_processor_count
    print("CUs", ncu, flush=True)

    def masked_stream(off_bits=0, only_bits=None, prio=0):
        words = (ncu + 31) // 32
        m = np.zeros(words, np.uint32)
        for b in range(ncu):
            on = (b < only_bits) if only_bits is not None else (b >= off_bits)
            if on:
                m[b // 32] |= np.uint32(1 << (b % 32))
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), m.ctypes.data_as(ctypes.c_void_p))
        assert rc == 0, rc
        return torch.cuda.ExternalStream(s.value, device=dev)

    dag = synth.generate("wide16", 1_000_000)
    keep = [torch.from_numpy(a).to(dev) for a in (dag.oid.reshape(-1), dag.time, dag.parent_off.view(np.int32),
                                                   dag.parent_oid.reshape(-1), dag.flags, dag.band)]
    c = abi.Commits()
    c.n_commits, c.n_parents = dag.n, dag.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
    c.residency = abi.WG_DEVICE
    band = keep[5].data_ptr()
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)
    res = {}
    engines = [wgraph.Engine(0) for _ in range(2)]

    def timed(label, step, n_eng):
        for i in range(4):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            step(i)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / steps
        sums = {e.vertex_summary().checksum for e in engines[:n_eng]}
        res[label] = {"ms_per_step": round(ms, 4), "distinct_checksums": len(sums)}
        print(label, res[label], flush=True)

    def plain(label, streams):
        for e, s in zip(engines, streams):
            e.set_stream(s.cuda_stream)

        def step(i):
            e = engines[i % len(streams)]
            e.build(commits=c)
            e.row_geometry(device_ptr=band)
            e.emit_vertices(0, dag.n, selected=7, palette=pal)
        timed(label, step, len(streams))

    def split(label, bstreams, estreams):
        done = [None, None]

        def step(i):
            k = i % 2
            e, bs, es = engines[k], bstreams[k], estreams[k]
            if done[k] is not None:
                bs.wait_event(done[k])          # geometry buffers: the previous emission has read them
            e.set_stream(bs.cuda_stream)
            e.build(commits=c)
            e.row_geometry(device_ptr=band)
            ev = torch.cuda.Event()
            ev.record(bs)
            es.wait_event(ev)
            e.set_stream(es.cuda_stream)
            e.emit_vertices(0, dag.n, selected=7, palette=pal)
            done[k] = torch.cuda.Event()
            done[k].record(es)
        timed(label, step, 2)

    plain("seq", [torch.cuda.current_stream(dev)])
    plain("pipe2", [torch.cuda.Stream(dev), torch.cuda.Stream(dev)])
    split("split", [torch.cuda.Stream(dev) for _ in range(2)], [torch.cuda.Stream(dev) for _ in range(2)])
    split("split_prio", [torch.cuda.Stream(dev, priority=-1) for _ in range(2)],
          [torch.cuda.Stream(dev) for _ in range(2)])
    for k in (16, 32, 64):
        split(f"split_m{k}", [torch.cuda.Stream(dev, priority=-1) for _ in range(2)],
              [masked_stream(off_bits=k) for _ in range(2)])
        split(f"split_b{k}", [masked_stream(only_bits=k) for _ in range(2)],
              [masked_stream(off_bits=k) for _ in range(2)])
    for k in (0, 16, 32, 64):
        s = masked_stream(off_bits=k)
        e = engines[0]
        e.set_stream(s.cuda_stream)
        e.build(commits=c)
        e.row_geometry(device_ptr=band)
        e.emit_vertices(0, dag.n, selected=7, palette=pal)
        e.enable_timing(True, reserve=64)
        for _ in range(10):
            e.emit_vertices(0, dag.n, selected=7, palette=pal)
        torch.cuda.synchronize()
        t = [ms for n, ms in e.timings() if n == "vtx_emit"]
        e.enable_timing(False)
        res[f"emit_m{k}"] = round(float(np.mean(t)), 4)
        print(f"emit_m{k}", res[f"emit_m{k}"], flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
