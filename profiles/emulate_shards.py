"""Emulate the N-GPU row-sharded bench step on ONE GPU, rank by rank.

The driver runs the real multi-GPU bench (`torch.distributed.run ... bench.py
--gpus N`); this script answers "what does each rank's step cost" before an
8-GPU node is available.  N engines (one per emulated rank, each on its own
stream and thread) run the same wg_shard_* protocol as bench.py's sharded
step, but a lock lets only one rank use the GPU at a time: every segment of
a rank's step (from one exchange to the next, ending in a stream sync) is
timed alone.  The all-gathers are emulated by device copies outside the
timed segments; their cost on xGMI is NOT measured here, only counted
(exchanges per step, bytes per exchange).

  rank time  = sum of its segments (build + geometry + emission)
  step bound = max over ranks + exchanges x (RCCL all-gather latency)

usage: python3 profiles/emulate_shards.py [--world 8] [--rows-per-rank 1000000]
           [--kind wide16] [--steps 3] [--out profiles/r01_shard_emulation.json]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "whisper-git_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rows-per-rank", type=int, default=1_000_000)
    ap.add_argument("--kind", default="wide16")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--stage-events", action="store_true", help="record every stage's HIP events (stages_ms)")
    ap.add_argument("--no-defer", action="store_true", help="validate each speculative pass before the call returns")
    ap.add_argument("--replay", default=None, help="CHUNK:WARM: fixed replay chunk / warm-up (options 2 and 6)")
    ap.add_argument("--no-spec-replay", action="store_true", help="WG_OPT_SHARD_SPEC_REPLAY 0: X3 checks its replay")
    ap.add_argument("--replay-mode", type=int, default=None, help="WG_OPT_REPLAY_MODE (0 auto, 1 chunked, 2 serial)")
    ap.add_argument("--no-isolated", action="store_true", help="skip the isolated per-rank replay")
    ap.add_argument("--two-calls", action="store_true",
                    help="shard_build + shard_geometry (two geometry passes) instead of shard_build_frame (3 exchanges either way)")
    args = ap.parse_args()

    import torch
    import wgraph
    from wgraph import abi, synth
    from wgraph.shard import ShardComm

    W, R = args.world, args.rows_per_rank
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    dag = synth.generate(args.kind, W * R)
    print(f"generated {args.kind} {dag.n} rows in {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
    keep = [torch.from_numpy(a).to(dev) for a in (dag.oid.reshape(-1), dag.time, dag.parent_off.view(np.int32),
                                                   dag.parent_oid.reshape(-1), dag.flags, dag.band)]
    commits = abi.Commits()
    commits.n_commits, commits.n_parents = dag.n, dag.e
    commits.oid, commits.time, commits.parent_off, commits.parent_oid, commits.flags = (t.data_ptr() for t in keep[:5])
    commits.residency = abi.WG_DEVICE
    band_ptr = keep[5].data_ptr()
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)

    gpu = threading.Lock()
    bar = threading.Barrier(W)
    captured = [[] for _ in range(W)]     # per rank: the last step's gathered exchanges (isolated replay)
    capture_on = [False]
    slots: list = [None] * W
    seg = [[] for _ in range(W)]          # per rank: (label, seconds)
    xlog = []                             # per exchange: (step, bytes per rank)

    class EmuComm:
        """Lock-step stand-in for ShardComm.allgather between W threads."""

        def __init__(self, rank, eng, stream):
            self.rank, self.eng, self.stream = rank, eng, stream
            self.t = None
            self.label = ""
            self.on_device, self.device = True, dev   # slots packed in stream order, as over RCCL
            self.world = W

        held = False

        def start(self, label):
            gpu.acquire()
            self.held = True
            self.label = label
            self.t = time.perf_counter()

        def stop(self, final=False):
            # between exchanges only the engine's main stream is drained (as
            # wg_shard_copy_msg does); side-stream work may run on
            if final:
                self.eng.synchronize()
            else:
                self.stream.synchronize()
            seg[self.rank].append((self.label, time.perf_counter() - self.t))
            self.held = False
            gpu.release()

        caps: dict = {}

        def allgather(self, nbytes, fill, step=0, pack=None, read_heads=None):
            # (read_heads: the heads come from the host copy below, as with a gloo transport)
            with torch.cuda.stream(self.stream):
                if pack is not None:
                    # the slot header carries the length (set on the device when
                    # the engine left it there): read after the timed segment,
                    # repacked with a larger slot if the message did not fit
                    cap = self.caps.get(step, 4096)
                    slot = torch.empty(cap + ShardComm.HDR, dtype=torch.uint8, device=dev)
                    pack(slot.data_ptr(), cap)
                else:
                    cap = ShardComm.round_cap(nbytes)
                    send = torch.zeros(cap, dtype=torch.uint8, device=dev)
                    if nbytes:
                        fill(send.data_ptr())
            self.stop()
            if pack is not None:
                with torch.cuda.stream(self.stream):
                    nbytes = int(slot[:8].cpu().view(torch.int64).item())
                    if nbytes > cap:
                        cap = ShardComm.round_cap(nbytes)
                        slot = torch.empty(cap + ShardComm.HDR, dtype=torch.uint8, device=dev)
                        pack(slot.data_ptr(), cap)
                    self.stream.synchronize()
                self.caps[step] = cap
                send = slot[ShardComm.HDR:]
            slots[self.rank] = (send, nbytes)
            bar.wait()
            stride = ShardComm.round_cap(max(s[1] for s in slots)) + ShardComm.HDR
            if self.rank == 0:
                xlog.append((step, [s[1] for s in slots]))
            with gpu:
                with torch.cuda.stream(self.stream):
                    out = torch.zeros(W * stride, dtype=torch.uint8, device=dev)
                    for r, (b, n) in enumerate(slots):
                        if n:
                            out[r * stride + ShardComm.HDR: r * stride + ShardComm.HDR + n].copy_(b[:n])
                    # ShardComm brings every message's 16-byte header to the host with the sizes
                    self.heads = np.ascontiguousarray(out.view(W, stride)[:, 16:32].cpu().numpy()).view(np.uint32)
                self.stream.synchronize()
            sizes = [s[1] for s in slots]
            if capture_on[0]:
                captured[self.rank].append((out.clone(), stride, list(sizes), self.heads.copy()))
            bar.wait()
            self.start(self.label)
            return out, ShardComm.HDR, stride, sizes

    engines, streams = [], []
    for r in range(W):
        e = wgraph.Engine(0)
        s = torch.cuda.Stream(dev)
        e.set_stream(s.cuda_stream)
        e.set_defer_validation(not args.no_defer)   # as bench.py
        e.set_shard_spec_replay(not args.no_spec_replay)
        if args.replay_mode is not None:
            e.set_replay_mode(args.replay_mode)
        if args.replay:
            ch, wm = (int(x) for x in args.replay.split(":"))
            e._check(wgraph.lib().wg_set_option(e._ctx, 2, ch))
            e._check(wgraph.lib().wg_set_option(e._ctx, 6, wm))
        engines.append(e)
        streams.append(s)

    stage_ms = [dict() for _ in range(W)]
    errors = []

    def rank_main(r):
        with torch.cuda.stream(streams[r]):   # the engine's stream is the transport's stream
            rank_body(r)

    def rank_body(r):
        comm = None
        try:
            eng = engines[r]
            comm = EmuComm(r, eng, streams[r])
            s0, s1 = r * R, min(dag.n, (r + 1) * R)
            for it in range(args.steps + 1):
                if it == args.steps:
                    captured[r].clear()
                    if r == 0:
                        capture_on[0] = True
                    bar.wait()
                if it == 1:
                    # per-stage events only with --stage-events: each costs a few us of
                    # GPU time, which would inflate the segments against the
                    # uninstrumented single-GPU step
                    wgraph.lib().wg_set_option(eng._ctx, 4, 0 if args.stage_events else 1)
                    eng.enable_timing(True, reserve=64 * (args.steps + 1))
                comm.start("build")
                if args.two_calls:
                    eng.shard_build(commits, W, r, s0, s1, comm)
                    comm.stop()
                    comm.start("geometry")
                    eng.shard_geometry(comm, device_ptr=band_ptr)
                else:
                    eng.shard_build_frame(commits, W, r, s0, s1, comm, device_ptr=band_ptr)
                comm.stop()
                comm.start("emit")
                eng.emit_vertices(s0, s1, selected=s0 + 7, palette=pal)
                comm.stop(final=True)
                if it == 0:
                    seg[r].clear()
                    if r == 0:
                        xlog.clear()
                if r == 0:
                    print(f"step {it} done", file=sys.stderr, flush=True)
                bar.wait()
            for name, ms in eng.timings():
                stage_ms[r][name] = stage_ms[r].get(name, 0.0) + ms / args.steps
            eng.enable_timing(False)
        except Exception as ex:   # surface worker failures in the main thread
            errors.append((r, repr(ex)))
            if comm is not None and comm.held:   # let the other ranks run into the aborted barrier
                comm.held = False
                gpu.release()
            bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(W)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    if errors:
        raise SystemExit(f"emulated rank failed: {errors}")

    capture_on[0] = False

    # Isolated replay (r06): each rank's whole step alone on the GPU — its main
    # and side streams overlapping each other as on a GPU of its own, no other
    # rank's work beside it — with every exchange answered from the buffers
    # the lockstep run gathered for the same step (the exchanges themselves
    # cost nothing here; the collectives' time is not measured).  The lockstep
    # segments above run one rank at a time, so a rank's side-stream work
    # lands under the next rank's segments instead of its own.
    class IsoComm:
        def __init__(self, rank, stream):
            self.rank, self.stream, self.k = rank, stream, 0
            self.on_device, self.device, self.world = True, dev, W
            self.heads = None
            self.held = False

        def allgather(self, nbytes, fill, step=0, pack=None, read_heads=None):
            out, stride, sizes, heads = captured[self.rank][self.k]
            with torch.cuda.stream(self.stream):
                if pack is not None:   # (the rank packs its message as it would; the answer is the recorded one)
                    cap = stride - ShardComm.HDR
                    slot = torch.empty(cap + ShardComm.HDR, dtype=torch.uint8, device=dev)
                    pack(slot.data_ptr(), cap)
                elif nbytes:
                    send = torch.zeros(ShardComm.round_cap(nbytes), dtype=torch.uint8, device=dev)
                    fill(send.data_ptr())
            self.k += 1
            self.heads = heads
            return out, ShardComm.HDR, stride, sizes

    iso_ms = []
    iso_err = None
    try:
      if not args.no_isolated and all(captured[r] for r in range(W)):
        for r in range(W):
            eng, st = engines[r], streams[r]
            s0, s1 = r * R, min(dag.n, (r + 1) * R)
            ts = []
            with torch.cuda.stream(st):
                for it in range(args.steps + 1):
                    comm = IsoComm(r, st)
                    eng.synchronize()
                    t0 = time.perf_counter()
                    eng.shard_build_frame(commits, W, r, s0, s1, comm, device_ptr=band_ptr)
                    eng.emit_vertices(s0, s1, selected=s0 + 7, palette=pal)
                    eng.synchronize()
                    if it:
                        ts.append(time.perf_counter() - t0)
            iso_ms.append(round(1e3 * float(np.median(ts)), 4))
    except Exception as ex:   # (the lockstep figures stand without it)
        iso_err = repr(ex)
        iso_ms = []

    counters = [int(e.debug_counters()[5]) for e in engines]
    dcs = [e.debug_counters() for e in engines]   # [1] lane slots of the global replay, [10] serial replay

    # rank 0's emission again on its sharded geometry, alone on the GPU (no other
    # rank's segments interleaved): separates the shard data from the emulation
    reemit_ms = None
    if args.stage_events:
        e0 = engines[0]
        with torch.cuda.stream(streams[0]):
            e0.synchronize()
            wgraph.lib().wg_set_option(e0._ctx, 4, 0)
            e0.enable_timing(True, reserve=64 * args.steps)
            for _ in range(args.steps):
                e0.emit_vertices(0, R, selected=7, palette=pal)
            e0.synchronize()
            reemit_ms = round(sum(ms for n, ms in e0.timings() if n == "vtx_emit") / args.steps, 4)
            e0.enable_timing(False)

    # the single-GPU step on an R-row list of the same kind, for comparison
    single = wgraph.Engine(0)
    single.set_defer_validation(not args.no_defer)   # as bench.py
    dag1 = synth.generate(args.kind, R)
    k1 = [torch.from_numpy(a).to(dev) for a in (dag1.oid.reshape(-1), dag1.time, dag1.parent_off.view(np.int32),
                                                 dag1.parent_oid.reshape(-1), dag1.flags, dag1.band)]
    c1 = abi.Commits()
    c1.n_commits, c1.n_parents = dag1.n, dag1.e
    c1.oid, c1.time, c1.parent_off, c1.parent_oid, c1.flags = (t.data_ptr() for t in k1[:5])
    c1.residency = abi.WG_DEVICE

    def one(eng=None):
        eng = eng or single
        if args.two_calls:
            eng.build(commits=c1)
            eng.row_geometry(device_ptr=k1[5].data_ptr())
        else:
            eng.build_frame(commits=c1, device_ptr=k1[5].data_ptr())
        eng.emit_vertices(0, R, selected=7, palette=pal)
        eng.synchronize()
    one()
    times = []
    for _ in range(args.steps):
        t0 = time.perf_counter()
        one()
        times.append(time.perf_counter() - t0)
    single_ms = 1e3 * float(np.median(times))
    single_stages = {}
    if args.stage_events:   # the same stage events on the single-GPU step, for a side-by-side table
        wgraph.lib().wg_set_option(single._ctx, 4, 0)
        single.enable_timing(True, reserve=64 * args.steps)
        for _ in range(args.steps):
            one()
        for name, ms in single.timings():
            single_stages[name] = round(single_stages.get(name, 0.0) + ms / args.steps, 4)
        single.enable_timing(False)
        # the same single-GPU step on rank 0's engine (its buffers were sized by the sharded steps)
        e0 = engines[0]
        one(e0)
        wgraph.lib().wg_set_option(e0._ctx, 4, 0)
        e0.enable_timing(True, reserve=64 * args.steps)
        for _ in range(args.steps):
            one(e0)
        single_stages["rank0_engine_vtx_emit"] = round(sum(ms for n, ms in e0.timings() if n == "vtx_emit") / args.steps, 4)
        e0.enable_timing(False)

    per_rank = []
    for r in range(W):
        tot = {}
        nseg = len(seg[r]) // args.steps
        for k in range(nseg):   # per segment: median over the steps
            lab = seg[r][k][0]
            tot[lab] = tot.get(lab, 0.0) + 1e3 * float(np.median([seg[r][k + j * nseg][1] for j in range(args.steps)]))
        per_rank.append({"rank": r, "ms": round(sum(tot.values()), 4),
                         **{k: round(v, 4) for k, v in tot.items()},
                         "segments_per_step": len(seg[r]) // args.steps,
                         "segment_ms": [round(1e3 * float(np.median([seg[r][k + j * (len(seg[r]) // args.steps)][1]
                                                                   for j in range(args.steps)])), 4)
                                        for k in range(len(seg[r]) // args.steps)],
                         "mode": counters[r], "lane_slots": int(dcs[r][1]), "serial_replay": int(dcs[r][10]),
                         "replay_iterations": int(dcs[r][3]), "events": int(dcs[r][4]),
                         "stages_ms": {k: round(v, 4) for k, v in sorted(stage_ms[r].items())}})
    n_x = len(xlog) // args.steps
    xbytes = {}
    for step, sizes in xlog[:n_x]:
        xbytes[f"X{step}" if step not in xbytes else f"X{step}b"] = sizes
    worst = max(p["ms"] for p in per_rank)
    res = {"world": W, "rows_per_rank": R, "kind": args.kind, "steps": args.steps,
           "single_gpu_step_ms": round(single_ms, 4), "single_gpu_stages_ms": single_stages,
           "rank0_reemit_vtx_emit_ms": reemit_ms,
           "max_rank_ms_without_collectives": round(worst, 4),
           "exchanges_per_step": n_x, "exchange_bytes_per_rank": xbytes,
           "efficiency_without_collectives": round(single_ms / worst, 4),
           "isolated_rank_ms": iso_ms, "isolated_error": iso_err,
           "max_rank_isolated_ms": max(iso_ms) if iso_ms else None,
           "efficiency_isolated": round(single_ms / max(iso_ms), 4) if iso_ms else None,
           "isolated_note": ("each rank's whole step replayed alone on the GPU (main and side streams overlapping "
                             "as on its own GPU) with the exchanges answered from the gathered buffers the lockstep "
                             "run recorded; collective time not included"),
           "ranks": per_rank}
    print(json.dumps(res, indent=1))
    if args.out:
        with open(args.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
