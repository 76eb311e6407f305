"""Benchmark: commit-rows/s to vertex buffers (BASELINE.json metric).

One step = the whole hot path over one batch of device-resident commits:
GraphLayout::build (hash join, lane assignment, edges, heights) and the
frame's row_geometry_with_bands (pills bands) in one call
(wg_layout_build_frame: the build's geometry pass takes the bands, which is
what history_view's first frame after a refresh computes) -> graph_cell
vertex emission for every row of this rank's shard (WG-TESS-1 SplineVertex
buffers written to HBM).  Workload: the WIDE16 synthetic DAG (C5 shape,
<= 16 lanes), 1M commit-rows per GPU (weak scaling: N GPUs = an
N-million-row DAG, each rank emits its contiguous 1M-row shard);
--total-rows T gives strong scaling instead (one T-row DAG over N GPUs).

Multi-GPU: every rank holds the whole DAG in HBM and builds
only its contiguous shard (wg_shard_* C ABI): parent ids, crossing
references, chain tokens and the lane-event stream are all-gathered over
RCCL (torch.distributed "nccl" group) at the exchange points of DESIGN.md
§6 (four per step with wg_shard_build_frame_begin), then each rank emits
its own rows' vertex buffers.
Launched per the driver contract:
  python bench.py --gpus 1 --steps K --warmup W
  python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.environ.get("WG_PKG_DIR") or os.path.join(ROOT, "whisper-git_amd"))   # (WG_PKG_DIR: an A/B build)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--rows-per-gpu", type=int, default=1_000_000,
                    help="weak scaling (the default): each GPU builds and emits this many rows of an N x that DAG")
    ap.add_argument("--total-rows", type=int, default=0,
                    help="strong scaling: one DAG of this many rows split over the N GPUs (e.g. 1000000 at "
                         "--gpus 8 = 125000 rows per GPU); overrides --rows-per-gpu")
    ap.add_argument("--kind", default="wide16")
    ap.add_argument("--cpu-rows", type=int, default=1_000_000, help="rows of the CPU-baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the side measurements (host-input rate, glyph quads, font atlas)")
    ap.add_argument("--no-events", action="store_true",
                    help="diagnostic: no HIP timing events inside the timed region (no roofline launch time)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (RCCL over xGMI) or gloo (host rehearsal)")
    ap.add_argument("--same-device", action="store_true", help="all ranks on cuda:0 (rehearsal on a 1-GPU box)")
    ap.add_argument("--device-transport", action="store_true",
                    help="gloo rehearsal: move HIP-resident slots through gloo (the stream-ordered slot path of RCCL)")
    ap.add_argument("--no-defer", action="store_true",
                    help="validate every speculative build before build() returns (WG_OPT_DEFER_VALIDATION off)")
    ap.add_argument("--vtx-tile", type=int, default=0, help="vertices per emission tile (1024, 2048; 0 = auto)")
    ap.add_argument("--no-fused-read", action="store_true", help="the emission's host read by a read kernel (A/B)")
    ap.add_argument("--join-fused", action="store_true",
                    help="the id table's place pass inside the window probe, settle on the main stream (A/B; default: beside it)")
    ap.add_argument("--slice", action="store_true",
                    help="row-slice the geometry lists under the emission (WG_OPT_SLICE_LISTS 1; default off)")
    ap.add_argument("--no-build-frame", action="store_true",
                    help="separate build() and row_geometry() calls instead of wg_layout_build_frame")
    ap.add_argument("--all-stage-events", action="store_true",
                    help="record every stage's HIP events inside the timed region (default: only the emission "
                         "kernel's, for the roofline; the stage breakdown comes from a separate pass)")
    return ap.parse_args()


def host_threads() -> int:
    """Threads this process may use on the host (the GPU box gives a 16-CPU
    share while os.cpu_count() reports the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(16, n))


def host_cpu() -> dict:
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"model": model, "logical_cpus": os.cpu_count(), "threads_used_mt": host_threads()}


def cpu_baseline(dag, rows, log, min_seconds=10.0, max_reps=4):
    """The CPU oracle (faithful single-thread restatement of commit_graph.rs)
    timed on this host over the first `rows` rows of the same workload; the
    sample is repeated until it has run >= min_seconds (mean rate reported)."""
    sys.path.insert(0, ROOT)
    from oracle import oracle_c   # checker / baseline only
    d = dag.slice_rows(min(rows, dag.n))
    total, reps, nv = 0.0, 0, 0
    while reps < max_reps and (reps == 0 or total < min_seconds):
        t0 = time.perf_counter()
        o = oracle_c.OracleLayout(d)
        o.row_geometry(d.band)
        step = 50_000
        nv = 0
        for r0 in range(0, d.n, step):
            v, _ = o.emit_vertices(r0, min(d.n, r0 + step), selected=7 if r0 == 0 else -1)
            nv += len(v)
        total += time.perf_counter() - t0
        reps += 1
        o.close()
    log(f"cpu baseline: {d.n} rows x {reps} in {total:.2f}s ({nv} vertices per pass)")
    return {"value": d.n * reps / total, "unit": "commit-rows/s", "cores": 1, "kind": "port",
            "sample": f"first {d.n} rows of the same workload, {reps} passes: oracle build + "
                      f"row_geometry_with_bands + vertex emission, 1 thread, {total:.1f}s total"}


def cpu_baseline_threads(dag, log, threads=None, min_seconds=5.0, max_reps=6):
    """The OpenMP CPU port (oracle/cpu_mt.c, bit-exact with the single-thread
    oracle: tests/test_cpu_mt.py) on the whole workload: concurrent id table,
    the sequential greedy lane walk and f32 row_top prefix the reference's
    semantics require, per-edge decomposition over owned row ranges merged in
    edge order, rows emitted in parallel into a vertex buffer reused across
    passes (as the engine reuses its HBM buffers).  threads: the host share
    this process may use (host_threads(): the GPU box gives 16 CPUs per GPU)."""
    sys.path.insert(0, ROOT)
    from oracle import cpu_mt   # baseline only
    threads = threads or host_threads()
    m = cpu_mt.MtLayout(dag, threads)
    m.row_geometry(dag.band)
    nv = m.emit_vertices(0, dag.n, selected=7, copy=False)[0]   # the vertex count (an untimed pass)
    m.close()
    dst = np.zeros(nv + 1, cpu_mt.abi.VERTEX_DTYPE)   # first touch outside the timed passes
    off = np.zeros(dag.n + 1, np.uint64)
    total, reps, phases = 0.0, 0, {}
    while reps < max_reps and (reps == 0 or total < min_seconds):
        t0 = time.perf_counter()
        m = cpu_mt.MtLayout(dag, threads)
        m.row_geometry(dag.band)
        got = m.emit_vertices_into(0, dag.n, dst, off, selected=7)
        total += time.perf_counter() - t0
        reps += 1
        for k, v in cpu_mt.phase_ms().items():
            phases[k] = phases.get(k, 0.0) + v
        m.close()
    assert got == nv
    phases = {k: round(v / reps, 2) for k, v in phases.items()}
    log(f"cpu baseline (OpenMP, {threads} threads): {dag.n} rows x {reps} in {total:.2f}s, phases ms {phases}")
    return {"value": dag.n * reps / total, "unit": "commit-rows/s", "cores": threads, "kind": "port",
            "sample": f"the whole workload ({dag.n} rows, {nv} vertices), {reps} passes: build + "
                      f"row_geometry_with_bands + vertex emission on {threads} OpenMP threads "
                      f"(oracle/cpu_mt.c; lane walk and row_top sequential), {total:.1f}s total",
            "phases_ms": phases,
            "threads_note": "threads = this process's CPU share (16 per GPU on the GPU box, which sets "
                            "OMP_NUM_THREADS=16 and asks jobs to stay within it), not the machine's logical CPUs"}


def extra_measurements(eng, dag, dev, torch, r0, r1, args, log):
    """Side measurements beside the headline metric (never `value`):
    glyph quads (A13) for the same rows with synthetic summaries, and the
    Roboto Regular+Bold 1024^2 SDF atlas build (A14, BASELINE config C2) on
    the GPU beside the CPU restatement."""
    from wgraph import abi, synth
    out = {}
    b, o = synth.summaries(dag.n)
    t_b = torch.from_numpy(b).to(dev)
    t_o = torch.from_numpy(o.view(np.int64)).to(dev)
    # atlas (C2): both fonts, GPU wall time incl. the host TrueType parse
    eng.build_font_atlas(0)
    eng.build_font_atlas(1)
    torch.cuda.synchronize()
    reps = 5
    eng.enable_timing(True, reserve=64)
    t0 = time.perf_counter()
    for _ in range(reps):
        eng.build_font_atlas(0)
        eng.build_font_atlas(1)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / reps
    ev = {}
    for name, ms in eng.timings():
        ev[name] = ev.get(name, 0.0) + ms / reps
    # cold: the first build of each font at new parameters (the case a font
    # or monitor-scale change hits): TrueType parse, outline flattening and the
    # uploads, then the same kernels; each timed build follows a build of the
    # same slot at another em size, so nothing of the timed one is cached
    cold = []
    for _ in range(reps):
        eng.build_font_atlas(0, em_px=95.0)
        eng.build_font_atlas(1, em_px=95.0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.build_font_atlas(0)
        eng.build_font_atlas(1)
        torch.cuda.synchronize()
        cold.append((time.perf_counter() - t0) * 1e3)
    atlas = {"config": "Roboto Regular+Bold, 1024x1024 R8 SDF, 96 px/em, spread 8, ASCII 32-126",
             "gpu_ms": round(wall, 3), "warm_ms": round(wall, 3), "cold_ms": round(float(np.median(cold)), 3),
             "gpu_kernel_ms": round(ev.get("font_atlas", 0.0), 4),
             "edt_ms": round(ev.get("font_edt", 0.0), 4), "coverage_ms": round(ev.get("font_coverage", 0.0), 4),
             "note": ("warm_ms (= gpu_ms): rebuilds of the same font at the same parameters, which skip the TrueType "
                      "parse and uploads (the device inputs stand); cold_ms: the first build at new parameters "
                      "(parse + flatten + upload + kernels, median of 5). The EDT passes touch ~10 MB per font "
                      "(1024^2 u8 coverage and SDF + four u16 distance planes), so they run out of the 256 MB Infinity Cache: "
                      "edt_ms is a cache-resident figure, not an HBM rate.")}
    if not args.no_cpu:
        # C2's CPU leg: an exact Felzenszwalb-Huttenlocher EDT in
        # C (oracle/edt_cpu.c, OpenMP) over the same two coverages, 1 thread and
        # all the threads this box gives us; its SDF bytes must equal the GPU's
        sys.path.insert(0, ROOT)
        from oracle import edt_cpu   # baseline only
        covs = [eng.atlas(slot) for slot in (0, 1)]
        spread = int(abi.ATLAS_DEFAULTS["spread"])
        mt = host_threads()
        for label, th in (("cpu_edt_ms_1t", 1), ("cpu_edt_ms_mt", mt)):
            edt_cpu.edt_sdf(covs[0]["cov"], spread, th)   # warm (pages, OpenMP pool)
            reps_c = 5
            t0 = time.perf_counter()
            for _ in range(reps_c):
                res = [edt_cpu.edt_sdf(a["cov"], spread, th) for a in covs]
            atlas[label] = round((time.perf_counter() - t0) * 1e3 / reps_c, 2)
        atlas["cpu_edt_threads_mt"] = mt
        atlas["cpu_edt_sdf_equals_gpu"] = bool(all((r[2] == a["sdf"]).all() for r, a in zip(res, covs)))
        atlas["cpu_kind"] = ("native C exact Felzenszwalb-Huttenlocher EDT + SDF bytes (oracle/edt_cpu.c, -O3), both "
                             "fonts, from the GPU atlas's coverage; compare with edt_ms (the GPU's two EDT passes)")
    out["font_atlas"] = atlas
    # glyph quads over the rank's rows
    eng.row_geometry(dag.band)
    kw = dict(now=int(dag.time.max()) + 86400)
    eng.emit_glyphs(r0, r1, device=(t_b.data_ptr(), t_o.data_ptr()), **kw)
    torch.cuda.synchronize()
    eng.enable_timing(True, reserve=64 * 6)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.emit_glyphs(r0, r1, device=(t_b.data_ptr(), t_o.data_ptr()), **kw)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    ev = {}
    for name, ms in eng.timings():
        ev.setdefault(name, []).append(ms)
    eng.enable_timing(False)
    gs = eng.glyph_summary()
    quad_ms = float(np.mean(ev.get("text_quads", [float("nan")])))
    rows_ms = float(np.mean(ev.get("text_rows", [float("nan")])))
    out["glyph_quads"] = {"rows": int(r1 - r0), "quads": int(gs.n_quads), "ms_per_call": round(dt * 1e3, 4),
                          "rows_per_s": round((r1 - r0) / dt, 1), "text_rows_ms": round(rows_ms, 4),
                          "text_quads_ms": round(quad_ms, 4),
                          "text_quads_GBps": round(gs.n_quads * (192 + 16) / (quad_ms * 1e-3) / 1e9, 1),
                          "data": "synthetic summaries (wgraph.synth.summaries), relative times vs max(time)+1d"}
    # search-match flags (commit_matches_query, commit_graph.rs:1509-1523) over the same rows
    (sb, so_), (ab, ao) = synth.text_fields(dag.n)
    dt_ = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (sb, so_.view(np.int64), ab, ao.view(np.int64))]
    devp = ((dt_[0].data_ptr(), dt_[1].data_ptr()), (dt_[2].data_ptr(), dt_[3].data_ptr()))
    query = "Fix"
    eng.match_rows(query, r0, r1, device=devp)
    torch.cuda.synchronize()
    eng.enable_timing(True, reserve=64 * 2)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        nm = eng.match_rows(query, r0, r1, device=devp)
    dt = (time.perf_counter() - t0) / args.steps
    ev = [ms for name, ms in eng.timings() if name == "match"]
    eng.enable_timing(False)
    eng.match_rows("")
    kms = float(np.mean(ev)) if ev else float("nan")
    text_bytes = int(so_[r1] - so_[r0]) + int(ao[r1] - ao[r0])
    alg = text_bytes + 16 * (r1 - r0) + (r1 - r0) * (20 + 1 + 1)   # text + offsets + id + flags + flag out
    srch = {"rows": int(r1 - r0), "query": query, "matches": int(nm), "ms_per_call": round(dt * 1e3, 4),
            "kernel_ms": round(kms, 4), "kernel_GBps": round(alg / (kms * 1e-3) / 1e9, 1),
            "algorithmic_bytes": alg, "data": "synthetic summaries + authors (wgraph.synth.text_fields), ~15% non-ASCII words"}
    if not args.no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import search_oracle   # baseline only
        m = min(100_000, r1 - r0)
        t0 = time.perf_counter()
        search_oracle.match_rows(dag, query.encode(), (sb, so_), (ab, ao), r0, r0 + m)
        srch["cpu_rows_per_s"] = round(m / (time.perf_counter() - t0), 1)
        srch["cpu_kind"] = f"port (Python str.lower restatement, 1 thread, first {m} rows)"
    out["search"] = srch
    # row order (commit_graph_with_orphans + insert_synthetics_sorted) of the same list
    rng = np.random.default_rng(11)
    orph = np.sort(rng.choice(dag.time, 100))[::-1].copy()
    syn = rng.choice(dag.time, 4)
    t_w, t_o, t_s = (torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (dag.time, orph, syn))
    perm_d = torch.empty(dag.n + 104, dtype=torch.int32, device=dev)
    devo = ((t_w.data_ptr(), dag.n), (t_o.data_ptr(), 100), (t_s.data_ptr(), 4))
    eng.order_rows(None, device=devo, out_device_ptr=perm_d.data_ptr())
    eng.enable_timing(True, reserve=64 * 2)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.order_rows(None, device=devo, out_device_ptr=perm_d.data_ptr())
    dt = (time.perf_counter() - t0) / args.steps
    ev = [ms for name, ms in eng.timings() if name == "order"]
    eng.enable_timing(False)
    order = {"rows": int(dag.n + 104), "orphans": 100, "synthetics": 4, "ms_per_call": round(dt * 1e3, 4),
             "gpu_ms": round(float(np.mean(ev)), 4) if ev else None}
    if not args.no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import order_oracle   # baseline only
        t0 = time.perf_counter()
        order_oracle.order_rows(dag.time, orph, syn)
        order["cpu_ms"] = round((time.perf_counter() - t0) * 1e3, 1)
        order["cpu_kind"] = "port (Python stable sort + list inserts, 1 thread)"
    out["order"] = order
    out["frames"] = frame_rates(eng, dag, dev, torch, args)
    out["builds"] = build_lifecycle(dag, dev, torch, args, np.ascontiguousarray(abi.DEFAULT_PALETTE))
    out["baseline_configs"] = config_rates(eng, dev, torch, args)
    log("extras:", json.dumps(out))
    return out


def frame_rates(eng, dag, dev, torch, args):
    """Per-frame geometry (history_view recomputes
    row_geometry_with_bands every frame, commit_graph.rs:1419-1421) on the
    bench list: bands unchanged (one compare pass), one band changed at 90%
    of the list (rows and curves from there on), one band changed at row 0
    (the whole pass); device-resident bands, ms per frame."""
    from wgraph import abi
    keep = [torch.from_numpy(a).to(dev) for a in (dag.oid.reshape(-1), dag.time, dag.parent_off.view(np.int32),
                                                   dag.parent_oid.reshape(-1), dag.flags)]
    c = abi.Commits()
    c.n_commits, c.n_parents = dag.n, dag.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep)
    c.residency = abi.WG_DEVICE
    eng.build(commits=c)
    band = torch.from_numpy(dag.band.copy()).to(dev)
    eng.row_geometry(device_ptr=band.data_ptr())
    res = {}
    for name, row in (("unchanged", None), ("changed_at_90pct", int(dag.n * 0.9)), ("changed_at_row0", 0)):
        times = []
        for k in range(args.steps):
            if row is not None:
                band[row] = float(30.0 if k % 2 == 0 else 0.0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.row_geometry(device_ptr=band.data_ptr())
            torch.cuda.synchronize()
            times.append(time.perf_counter() - t0)
        res[name + "_ms"] = round(1e3 * float(np.median(times)), 4)
    res["rows"] = int(dag.n)
    del keep
    return res


def config_rates(eng, dev, torch, args):
    """The same step (build + banded geometry + emission, inputs in HBM) on
    BASELINE.json's other single-GPU DAG configs: C3 (100k commits, 1.3
    parents on average) and C4 (Linux-kernel-shaped 1.3M commits; its vertex
    buffer checksum equals the CPU oracle's in tests/test_gpu_parity.py)."""
    from wgraph import abi, synth
    res = {}
    # C1: the 10k-commit linear repo on the reference's CPU path (the oracle,
    # 1 thread: build + row_geometry_with_bands + graph_cell emission; the
    # headless screenshot_mode itself needs Vulkan + Rust), and the same step here
    d1 = synth.generate("linear", 10_000)
    c1 = {"workload": "linear synthetic repo, 10000 commits"}
    if not args.no_cpu:
        sys.path.insert(0, ROOT)
        from oracle import oracle_c   # baseline only
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            o = oracle_c.OracleLayout(d1)
            o.row_geometry(d1.band)
            o.emit_vertices(0, d1.n, selected=7)
            o.close()
        cms = (time.perf_counter() - t0) * 1e3 / reps
        c1.update({"cpu_ms_per_step": round(cms, 3), "cpu_rows_per_s": round(d1.n / cms * 1e3, 1), "cpu_cores": 1,
                   "cpu_kind": "port (oracle/wg_oracle.c, 1 thread)"})
    res["C1"] = c1
    import wgraph
    for cid, kind, n in (("C1", "linear", 10_000), ("C3", "random13", 100_000), ("C4", "linux", 1_300_000),
                         ("skew", "skew", 1_000_000), ("linuxwide", "linuxwide", 1_000_000)):
        # a context of its own per list (a repository tab's GraphLayout): the
        # bench list's buffers would size the speculative grids (capacities)
        eng = wgraph.Engine(dev.index)
        eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
        eng.set_defer_validation(not args.no_defer)
        eng.set_slice_lists(1 if args.slice else 0)
        eng.set_join_fused(args.join_fused)
        eng.set_vtx_tile(args.vtx_tile)
        eng.set_fused_read(not args.no_fused_read)
        d = synth.generate(kind, n)
        keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                       d.parent_oid.reshape(-1), d.flags, d.band)]
        c = abi.Commits()
        c.n_commits, c.n_parents = d.n, d.e
        c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
        c.residency = abi.WG_DEVICE

        def step():
            if args.no_build_frame:
                eng.build(commits=c)
                eng.row_geometry(device_ptr=keep[5].data_ptr())
            else:
                eng.build_frame(commits=c, device_ptr=keep[5].data_ptr())
            eng.emit_vertices(0, d.n, selected=7)
        for _ in range(5):   # (the replay's blind count adapts over the first builds)
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / args.steps
        ls = eng.layout_summary()
        r = res.setdefault(cid, {})
        if cid == "C1":
            r.update({"gpu_ms_per_step": round(ms, 4), "gpu_rows_per_s": round(n / ms * 1e3, 1)})
        else:
            r.update({"workload": f"{kind} synthetic DAG, {n} commits", "ms_per_step": round(ms, 4),
                      "rows_per_s": round(n / ms * 1e3, 1)})
        r.update({"vertices": int(eng.vertex_summary().n_vertices), "max_lane": int(ls.max_lane),
                  "n_slots": int(ls.n_slots), "lane_path": int(ls.lane_path)})
        if cid == "skew":
            r["note"] = ("LINUX shape + clock skew + 100 reflog orphans stable-sorted by time (git/mod.rs:761-775): "
                         "parents at earlier rows, leaked slots")
        if cid == "linuxwide":
            r["note"] = "LINUX shape with > 100 concurrent lanes (4-word replay occupancy)"
        eng.close()
        del keep
    return res


def build_lifecycle(dag, dev, torch, args, pal):
    """The builds the reference runs besides the warm steady state
    (GraphLayout::build on every refresh with a changed list, repo_tab.rs:
    790-861, 973-979): a cold step on a fresh context (first allocation of
    every buffer), then a refresh step whose list has 50 new commits
    prepended (new head chain on the old tips: every row shifts by 50), then
    the same refreshed list again (warm).  ms per step (build + banded
    geometry + emission) and wg_debug_counters [6..8] (speculative builds,
    lanes / geometry redone by the exact stages)."""
    import wgraph
    from wgraph import abi, synth

    def upload(d):
        keep = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
                (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32), d.parent_oid.reshape(-1), d.flags, d.band)]
        c = abi.Commits()
        c.n_commits, c.n_parents = d.n, d.e
        c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep[:5])
        c.residency = abi.WG_DEVICE
        return keep, c

    fresh = synth.prepend_commits(dag, 50)
    k0, c0 = upload(dag)
    k1, c1 = upload(fresh)
    eng = wgraph.Engine(dev.index)
    eng.set_stream(torch.cuda.current_stream(dev).cuda_stream)
    eng.set_defer_validation(not args.no_defer)
    eng.set_slice_lists(1 if args.slice else 0)
    eng.set_join_fused(args.join_fused)
    eng.set_vtx_tile(args.vtx_tile)
    eng.set_fused_read(not args.no_fused_read)

    def step(k, c, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if args.no_build_frame:
            eng.build(commits=c)
            eng.row_geometry(device_ptr=k[5].data_ptr())
        else:
            eng.build_frame(commits=c, device_ptr=k[5].data_ptr())
        eng.emit_vertices(0, n, selected=7, palette=pal)
        torch.cuda.synchronize()
        return round((time.perf_counter() - t0) * 1e3, 4)

    out = {"rows": int(dag.n), "cold_ms": step(k0, c0, dag.n)}
    warm = [step(k0, c0, dag.n) for _ in range(3)]
    out["warm_ms"] = float(np.median(warm))
    out["refresh_ms"] = step(k1, c1, fresh.n)
    out["refresh_again_ms"] = step(k1, c1, fresh.n)
    dc = eng.debug_counters()
    out.update({"spec_builds": int(dc[6]), "spec_lanes_redone": int(dc[7]), "spec_geometry_redone": int(dc[8]),
                "note": "refresh = 50 commits prepended (new ids, rows shifted by 50); cold = first step of a fresh "
                        "context, incl. its device allocations"})
    eng.close()
    del k0, k1
    return out


def pmc_traffic(args, workload):
    """Latest profiles/<tag>_pmc.json collected on this exact workload (or None).
    Tags run r<round><a..z, aa..az, ba..>: ordered by round, then suffix length,
    then suffix (so r06o < r06af < r06bf)."""
    import glob
    import re

    def order(f):
        m = re.match(r"r(\d+)([a-z]*)_pmc\.json$", os.path.basename(f))
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (-1, 0, os.path.basename(f))

    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")), key=order):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") == workload and "hbm_bytes_per_launch" in d:
            if "hbm_bytes_per_emission" in d:   # (a two-part emission: both parts)
                d["hbm_bytes_per_launch"] = d["hbm_bytes_per_emission"]
            d["_file"] = os.path.relpath(f, ROOT)
            best = d
    return best


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    log = (lambda *a: print(*a, file=sys.stderr, flush=True)) if (args.verbose or rank == 0) else (lambda *a: None)

    import torch
    import torch.distributed as dist
    dev_idx = 0 if args.same_device else local_rank
    torch.cuda.set_device(dev_idx)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group(backend="nccl", init_method="env://", device_id=torch.device("cuda", dev_idx))
        else:
            dist.init_process_group(backend=args.dist_backend, init_method="env://")

    import wgraph
    from wgraph import abi, synth

    strong = args.total_rows > 0
    if strong:   # a fixed DAG over the N GPUs (the last shard may be shorter)
        args.rows_per_gpu = (args.total_rows + world - 1) // world
        rows_total = args.total_rows
    else:
        rows_total = args.rows_per_gpu * world
    workload = (f"{args.kind} synthetic DAG (C5 shape), "
                + (f"{rows_total} commit-rows over {world} GPU(s) (strong scaling)" if strong
                   else f"{args.rows_per_gpu} commit-rows per GPU")
                + ", full path: layout build + banded geometry + SplineVertex emission")
    t0 = time.perf_counter()
    dag = synth.generate(args.kind, rows_total)
    log(f"generated {args.kind} DAG: {dag.n} rows, {dag.e} parent refs in {time.perf_counter() - t0:.1f}s")
    shard0 = rank * args.rows_per_gpu
    shard1 = min(rows_total, shard0 + args.rows_per_gpu)

    # device-resident inputs (the timed region starts from HBM)
    dev = torch.device("cuda", dev_idx)
    t_oid = torch.from_numpy(dag.oid.reshape(-1)).to(dev)
    t_time = torch.from_numpy(dag.time).to(dev)
    t_poff = torch.from_numpy(dag.parent_off.view(np.int32)).to(dev)
    t_poid = torch.from_numpy(dag.parent_oid.reshape(-1)).to(dev)
    t_flags = torch.from_numpy(dag.flags).to(dev)
    t_band = torch.from_numpy(dag.band).to(dev)
    commits = abi.Commits()
    commits.n_commits, commits.n_parents = dag.n, dag.e
    commits.oid, commits.time = t_oid.data_ptr(), t_time.data_ptr()
    commits.parent_off, commits.parent_oid = t_poff.data_ptr(), t_poid.data_ptr()
    commits.flags, commits.residency = t_flags.data_ptr(), abi.WG_DEVICE

    # one non-default stream for the engine, the events and the collectives:
    # the default stream's handle is 0, which wg_set_stream takes as "a stream
    # of the engine's own" (then the device-packed exchange slots could not be
    # ordered with RCCL, and ShardComm falls back to host copies)
    stream = torch.cuda.Stream(dev)
    stream.wait_stream(torch.cuda.current_stream(dev))
    torch.cuda.set_stream(stream)
    eng = wgraph.Engine(dev_idx)
    eng.set_stream(stream.cuda_stream)
    # a step's build is validated with its emission's vertex-total read (one
    # host wait per step, while the emission runs) instead of mid-step
    eng.set_defer_validation(not args.no_defer)
    eng.set_slice_lists(1 if args.slice else 0)
    eng.set_join_fused(args.join_fused)
    eng.set_vtx_tile(args.vtx_tile)
    eng.set_fused_read(not args.no_fused_read)
    pal = np.ascontiguousarray(abi.DEFAULT_PALETTE)
    selected = shard0 + 7
    comm = None
    if world > 1:
        from wgraph.shard import ShardComm
        comm = ShardComm(dev, device_transport=True if args.device_transport else None)

    def step():
        if comm is None and args.no_build_frame:
            eng.build(commits=commits)
            eng.row_geometry(device_ptr=t_band.data_ptr())
        elif comm is None:   # the same two calls, the build's geometry pass taking the bands
            eng.build_frame(commits=commits, device_ptr=t_band.data_ptr())
        elif not args.no_build_frame:   # sharded: 3 exchanges (X1-X3), one geometry pass instead of two
            eng.shard_build_frame(commits, world, rank, shard0, shard1, comm, device_ptr=t_band.data_ptr())
        else:
            eng.shard_build(commits, world, rank, shard0, shard1, comm)
            eng.shard_geometry(comm, device_ptr=t_band.data_ptr())
        eng.emit_vertices(shard0, shard1, selected=selected, palette=pal)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # HIP events on the engine's stream, logged across the whole timed region
    # and read back only after it (no per-step readback): the emission kernel's
    # (the roofline's launch duration) and, with --all-stage-events, every
    # stage's; the stage breakdown is otherwise a separate pass below
    lib_opt = wgraph.lib().wg_set_option
    eng._check(lib_opt(eng._ctx, 4, 0 if args.all_stage_events else 1))   # WG_OPT_TIMING_EMIT_ONLY
    eng.enable_timing(not args.no_events, reserve=64 * (args.steps + 1))

    if comm is not None:
        comm.set_timing(True)
    # timed region: barrier + sync on both sides, exactly K steps
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    exchange = None
    if comm is not None:   # seam exchanges: max over ranks, per step
        rep = comm.timing_report()
        comm.set_timing(False)
        vals = torch.tensor([rep["host_ms"], rep["collective_ms"] or 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        exchange = {"exchanges_per_step": rep["exchanges"] / args.steps,
                    "collective_ms_per_step": round(float(vals[1]) / args.steps, 4) if rep["collective_ms"] is not None else None,
                    "host_wait_ms_per_step": round(float(vals[0]) / args.steps, 4),
                    "note": "collective_ms: the all-gathers' own GPU time (HIP events on the stream); host_wait_ms: "
                            "host time inside ShardComm.allgather, i.e. waiting for the producing kernels, the "
                            "collective and the slot heads (max over ranks)"}
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    stage_ms, launches = {}, {}
    for name, ms in eng.timings():   # a stage may run twice per step (build + banded geometry)
        stage_ms[name] = stage_ms.get(name, 0.0) + ms / args.steps
        launches.setdefault(name, []).append(ms)
    eng.enable_timing(False)
    if not args.all_stage_events:   # stage breakdown: a few more steps with every stage's events
        eng._check(lib_opt(eng._ctx, 4, 0))
        nb = min(args.steps, 5)
        eng.enable_timing(True, reserve=64 * (nb + 1))
        for _ in range(nb):
            step()
        torch.cuda.synchronize()
        stage_ms = {}
        for name, ms in eng.timings():
            stage_ms[name] = stage_ms.get(name, 0.0) + ms / nb
        eng.enable_timing(False)

    # the emission alone, back to back with no timing events, by the host's
    # clock (each call: the offsets kernel, the total's read, the launch):
    # a check on the event-timed launch duration the roofline uses
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ne = min(args.steps, 10)
    for _ in range(ne):
        eng.emit_vertices(shard0, shard1, selected=selected, palette=pal)
    torch.cuda.synchronize()
    emit_only_ms = (time.perf_counter() - t1) * 1e3 / ne

    ms_per_step = elapsed * 1e3 / args.steps
    rows_done = rows_total  # all ranks together emit every row once per step
    value = rows_done * args.steps / elapsed

    # roofline of the dominant kernel (vertex emission), from live HIP events
    vs = eng.vertex_summary()
    gs = eng.geometry_summary()
    sliced_emits = int(eng.debug_counters()[11])
    n_rows_shard = shard1 - shard0
    # one emission per step: one k_vtx_tile launch, or two when the geometry
    # lists are row-sliced under it (WG_OPT_SLICE_LISTS) — then
    # the span from part 1's start to the end of both parts
    vtx_ms = float(np.mean(launches.get("vtx_emit", [float("nan")])))
    g = eng.geometry()   # this rank's rows (the whole list at N=1)
    r0, r1 = (shard0, shard1) if world == 1 else (0, shard1 - shard0)
    nvert_shard = int(g["vert_off"][r1]) - int(g["vert_off"][r0])
    ncurve_shard = int(g["curve_off"][r1]) - int(g["curve_off"][r0])
    # algorithmic bytes of one vtx_emit launch: vertices written + geometry read
    bytes_w = 24 * vs.n_vertices
    bytes_r = 4 * nvert_shard + 33 * ncurve_shard + n_rows_shard * (8 + 4 + 4 + 4 + 4 + 4 + 1)
    achieved = (bytes_w + bytes_r) / (vtx_ms * 1e-3) / 1e9
    roofline = {"kernel": "k_vtx_tile (vtx_emit)", "bound": "hbm", "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None, "algorithmic_bytes_per_launch": int(bytes_w + bytes_r),
                "avg_launch_ms": round(vtx_ms, 4),
                "launches_per_emission": 2 if sliced_emits else 1,
                # the host clock over emission-only calls (no events): launch + offsets kernel + the total's read
                "emit_only_wall_ms_per_call": round(emit_only_ms, 4)}
    pmc = pmc_traffic(args, workload)
    if pmc is not None:
        # HBM bytes per launch from the committed PMC passes of this same command
        # (profiles/collect.sh), over the live launch duration -> GB/s like `achieved`
        roofline["traffic"] = round(pmc["hbm_bytes_per_launch"] / (vtx_ms * 1e-3) / 1e9, 1)
        roofline["traffic_bytes_per_launch"] = int(pmc["hbm_bytes_per_launch"])
        roofline["traffic_source"] = pmc["_file"]

    # host-resident variant (reported beside `value`, never as it): the commit
    # SoA and bands start in pinned-less host memory, so the step includes the
    # PCIe H2D copies; vertex buffers still land in HBM
    host_rate = None
    if rank == 0 and world == 1 and not args.no_extras:
        host_commits = abi.commits_struct(dag)
        band_host = np.ascontiguousarray(dag.band)

        def host_step():
            eng.build(commits=host_commits)
            eng.row_geometry(band_host)
            eng.emit_vertices(shard0, shard1, selected=selected, palette=pal)
        host_step()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(3):
            host_step()
        torch.cuda.synchronize()
        host_rate = rows_total * 3 / (time.perf_counter() - t1)

    # the vertex buffer's placement (WG_OPT_VTX_PLACE): read
    # before the side measurements, which emit other lists into the buffer
    import ctypes
    pn, pk, pms = ctypes.c_uint32(), ctypes.c_uint32(), (ctypes.c_float * 8)()
    eng._check(wgraph.lib().wg_vertex_placement_get(eng._ctx, ctypes.byref(pn), ctypes.byref(pk), pms))
    placement = {"candidates_probed": pn.value, "kept": pk.value, "probe_ms": [round(x, 4) for x in pms[:pn.value]]}

    extras = {}
    if rank == 0 and world == 1 and not args.no_extras:
        extras = extra_measurements(eng, dag, dev, torch, shard0, shard1, args, log)

    stages = {k: round(float(v), 4) for k, v in stage_ms.items()}
    log("stage ms (mean over timed steps):", json.dumps(stages))
    log(f"rows {rows_total}, shard {n_rows_shard}, vertices {vs.n_vertices}, vert {gs.n_vert}, curves {gs.n_curve}, "
        f"max_lane {eng.layout_summary().max_lane}, lane_path {eng.layout_summary().lane_path}, "
        f"build mode {int(eng.debug_counters()[5])}" + (f", exchanges/step {comm.exchanges / (args.steps + args.warmup):.1f}"
                                                         if comm else ""))

    cpu = cpu_mt = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(dag, args.cpu_rows, log)
        cpu_mt = cpu_baseline_threads(dag, log)

    if rank == 0:
        out = {"metric": "commit-rows/sec to vertex buffers, 1M-commit synthetic DAG per GPU",
               "value": round(value, 1), "unit": "commit-rows/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
               "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
               "config": {"workload": workload,
                          "rows_total": rows_total, "rows_per_gpu": args.rows_per_gpu,
                          "vertices_per_gpu": int(vs.n_vertices), "parallelism": f"row-shard x{world}"},
               "stages_ms": stages, "host_input_rows_per_s": None if host_rate is None else round(host_rate, 1),
               "roofline": roofline, "vtx_placement": placement,
               "cpu_baseline": cpu, "cpu_baseline_threads": cpu_mt, "host_cpu": host_cpu(),
               **extras}
        if exchange is not None:
            out["seam_exchange"] = exchange
        print(json.dumps(out), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
