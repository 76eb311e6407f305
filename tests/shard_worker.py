"""One rank of a row-sharded build, checked against the oracle.

Launched by tests/test_gpu_shard.py through torch.distributed.run (gloo
process group; every rank drives its own engine context, all on cuda:0 of
the test box).  For each case: build the shard, compare the shard's slice of
lanes / edges / heights / both geometries / vertex buffers with the C oracle
over the whole list, and write the verdict to <out>/rank<r>.json.
"""
import argparse
import json
import os
import sys
import traceback

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "whisper-git_amd"))
sys.path.insert(0, ROOT)


def u32rows(e):
    return np.ascontiguousarray(e).view(np.uint32).reshape(-1, 5) if len(e) else np.zeros((0, 5), np.uint32)


def geometry_slice(g, s, e):
    vo, co = g["vert_off"].astype(np.int64), g["curve_off"].astype(np.int64)
    return {"height": g["height"][s:e], "node_y": g["node_y"][s:e], "row_top": g["row_top"][s:e + 1],
            "vert_off": (vo[s:e + 1] - vo[s]).astype(np.uint32), "vert": g["vert"][vo[s]:vo[e]],
            "curve_off": (co[s:e + 1] - co[s]).astype(np.uint32), "curve": g["curve"][co[s]:co[e]],
            "curve_color": g["curve_color"][co[s]:co[e]]}


def run_case(eng, comm, torch, kind, n, seed, world, rank, errors):
    from oracle import oracle_c
    from wgraph import abi, synth
    from wgraph.shard import shard_rows

    def same(name, got, want):
        got, want = np.ascontiguousarray(got), np.ascontiguousarray(want)
        if got.shape != want.shape or got.tobytes() != want.tobytes():
            errors.append(f"{kind}/{n}/w{world} rank {rank}: {name} differs "
                          f"(shape {got.shape} vs {want.shape})")

    d = synth.generate(kind, n, seed=seed)
    dev = comm.device
    keep = [torch.from_numpy(a).to(dev) for a in (d.oid.reshape(-1), d.time, d.parent_off.view(np.int32),
                                                   d.parent_oid.reshape(-1) if d.e else d.oid.reshape(-1), d.flags)]
    c = abi.Commits()
    c.n_commits, c.n_parents = d.n, d.e
    c.oid, c.time, c.parent_off, c.parent_oid, c.flags = (t.data_ptr() for t in keep)
    c.residency = abi.WG_DEVICE
    s, e = shard_rows(d.n, world, rank)
    eng.shard_build(c, world, rank, s, e, comm)
    o = oracle_c.OracleLayout(d)
    mode = int(eng.debug_counters()[5])
    want_mode = 2 if (kind == "anomaly" or world == 1) else 1
    if mode != want_mode:
        errors.append(f"{kind}/{n}/w{world} rank {rank}: build mode {mode}, expected {want_mode}")
    ls = eng.layout_summary()
    if ls.max_lane != o.max_lane:
        errors.append(f"{kind}/{n}/w{world} rank {rank}: max_lane {ls.max_lane} vs {o.max_lane}")
    if np.float32(ls.graph_width) != np.float32(o.graph_width):
        errors.append(f"{kind}/{n}/w{world} rank {rank}: graph_width")
    if ls.row_begin != s or ls.n_rows != e - s:
        errors.append(f"{kind}/{n}/w{world} rank {rank}: summary rows {ls.row_begin}+{ls.n_rows}")
    lane, color = eng.lanes()
    same("lane", lane, o.lane[s:e])
    same("color", color, o.color[s:e])
    oe = u32rows(o.edges)
    same("edges", u32rows(eng.edges()), oe[(oe[:, 0] >= s) & (oe[:, 0] < e)])
    same("heights", eng.row_heights(), o.heights[s:e])
    got = eng.geometry()
    for k, v in geometry_slice(o.geometry, s, e).items():
        same("build_" + k, got[k], v)
    eng.shard_geometry(comm, band=d.band)
    og = o.row_geometry(d.band)
    got = eng.geometry()
    for k, v in geometry_slice(og, s, e).items():
        same("band_" + k, got[k], v)
    if n <= 100_000:   # fractional bands: the rounding regime of row_top inside every shard
        fb = np.random.default_rng(seed).uniform(0, 40, d.n).astype(np.float32)
        eng.shard_geometry(comm, band=fb)
        ogf = o.row_geometry(fb)
        got = eng.geometry()
        for k, v in geometry_slice(ogf, s, e).items():
            same("fband_" + k, got[k], v)
        eng.shard_geometry(comm, band=d.band)
        og = o.row_geometry(d.band)
    sel = (s + e) // 2 if e > s else -1
    eng.emit_vertices(s, e, selected=sel)
    ov, ooff = o.emit_vertices(s, e, selected=sel)
    same("vtx_off", eng.vertex_offsets(), ooff)
    if eng.vertex_summary().checksum != oracle_c.vertex_checksum(ov):
        gv = eng.vertices()
        gw = np.ascontiguousarray(gv).view(np.uint32).reshape(len(gv), -1)
        ow = np.ascontiguousarray(ov).view(np.uint32).reshape(len(ov), -1)
        bad = np.nonzero((gw != ow).any(axis=1))[0] if gw.shape == ow.shape else np.array([0])
        i = int(bad[0]) if len(bad) else -1
        row = s + int(np.searchsorted(ooff.astype(np.int64), i, side="right")) - 1 if i >= 0 else -1
        errors.append(f"{kind}/{n}/w{world} rank {rank}: vertex checksum; {len(bad)} vertices differ, first {i} "
                      f"(row {row}, sel {sel}): got {gw[i].view(np.float32) if i >= 0 else None} "
                      f"want {ow[i].view(np.float32) if i >= 0 else None}")
    # build + banded frame in one sharded call (wg_shard_build_frame_begin): X1, X2, X3
    x0 = comm.exchanges
    eng.shard_build_frame(c, world, rank, s, e, comm, band=d.band)
    frame_x = comm.exchanges - x0
    if world > 1 and want_mode == 1 and frame_x != 3:
        errors.append(f"{kind}/{n}/w{world} rank {rank}: build_frame took {frame_x} exchanges, expected 3")
    lane, color = eng.lanes()
    same("frame lane", lane, o.lane[s:e])
    same("frame color", color, o.color[s:e])
    same("frame edges", u32rows(eng.edges()), oe[(oe[:, 0] >= s) & (oe[:, 0] < e)])
    got = eng.geometry()
    for k, v in geometry_slice(og, s, e).items():
        same("frame_" + k, got[k], v)
    eng.emit_vertices(s, e, selected=sel)
    if eng.vertex_summary().checksum != oracle_c.vertex_checksum(ov):
        errors.append(f"{kind}/{n}/w{world} rank {rank}: build_frame vertex checksum")
    o.close()
    del keep


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", required=True, help="kind:n:seed,...")
    ap.add_argument("--out", required=True)
    ap.add_argument("--transport", choices=("host", "device"), default="host",
                    help="device: HIP tensors through gloo, slots packed in stream order and their heads read by "
                         "the engine's polled wg_shard_slot_heads (the path bench.py takes over RCCL)")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    errors = []
    try:
        import wgraph
        from wgraph.shard import ShardComm
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        # a non-default stream shared with torch (its collectives and slot
        # buffers): handle 0, the default stream, would give the engine one of its own
        ts = torch.cuda.Stream(dev)
        ts.wait_stream(torch.cuda.current_stream(dev))
        torch.cuda.set_stream(ts)
        eng = wgraph.Engine(0)
        eng.set_stream(ts.cuda_stream)
        comm = ShardComm(dev, initial_cap=16, device_transport=args.transport == "device")
        for case in args.cases.split(","):
            kind, n, seed = case.split(":")
            run_case(eng, comm, torch, kind, int(n), int(seed), world, rank, errors)
        result = {"ok": not errors, "errors": errors[:20], "exchanges": comm.exchanges,
                  "collectives": comm.collectives, "on_device": comm.on_device}
        eng.close()
    except Exception:
        result = {"ok": False, "errors": errors[:20] + [traceback.format_exc()]}
    with open(os.path.join(args.out, f"rank{rank}.json"), "w") as f:
        json.dump(result, f)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
