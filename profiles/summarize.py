"""Summarise one round's rocprofv3 output (profiles/collect.sh) into files
that are committed under profiles/:

  <tag>_kernel_stats.csv  the rocprofv3 --stats table (kernel names shortened)
  <tag>_kernels.md        top kernels, per-step GPU busy/idle split
  <tag>_pmc.json          k_vtx_tile HBM traffic per launch from FETCH_SIZE /
                          WRITE_SIZE, corrected per MI355X_MICROARCH.md §HBM
                          (FETCH_SIZE counts half the bytes of wide streaming
                          reads on gfx950 -> doubled; units are KiB)

usage: python3 profiles/summarize.py <prof_dir> <tag> [dest_dir]
"""
from __future__ import annotations

import csv
import json
import os
import re
import sys
from collections import defaultdict

KERNEL = "k_vtx_tile"


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)


def is_kernel(name: str) -> bool:
    """KERNEL, plain or as a template instance (void k_vtx_tile<1024>, r05)."""
    s = short(name)
    return s == KERNEL or re.fullmatch(r"(void )?" + KERNEL + r"<[^>]*>", s) is not None


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def bench_line(path):
    try:
        for line in open(path):
            line = line.strip()
            if line.startswith("{"):
                return json.loads(line)
    except OSError:
        pass
    return None


def main():
    src, tag = sys.argv[1], sys.argv[2]
    dest = sys.argv[3] if len(sys.argv) > 3 else src
    os.makedirs(dest, exist_ok=True)
    stats = read_csv(os.path.join(src, "trace", "run_kernel_stats.csv"))
    trace = read_csv(os.path.join(src, "trace", "run_kernel_trace.csv"))
    bench = bench_line(os.path.join(src, "trace.json"))

    with open(os.path.join(dest, f"{tag}_kernel_stats.csv"), "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for r in stats:
            w.writerow([short(r["Name"]), r["Calls"], r["TotalDurationNs"], r["AverageNs"], r["Percentage"],
                        r["MinNs"], r["MaxNs"]])

    # per-step windows: from one build's first kernel to the next (the
    # emission may be two k_vtx_tile launches: row-sliced geometry lists)
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in trace)
    first = "k_probe_near" if any(n == "k_probe_near" for _, _, n in ev) else "k_hash_place"
    ends = [s for s, e, n in ev if n == first]
    windows = []
    for a, b in zip(ends[:-1], ends[1:]):
        iv = sorted((max(s, a), min(e, b)) for s, e, n in ev if e > a and s < b)
        busy, cur_s, cur_e, nk = 0, None, None, 0
        for s, e in iv:
            nk += 1
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            busy += cur_e - cur_s
        windows.append((b - a, busy, nk))
    # whole steps only (bench.py ends with emission-only calls: windows of a few
    # launches), and the timed ones: the last five whole steps are the
    # stage-breakdown pass, whose per-stage events add gaps
    # (windows run from one build's first kernel to the next build's: the
    # timed steps are the five shortest whole ones — the stage-breakdown pass
    # adds event gaps, the last window holds the emission-only calls)
    full = [w for w in windows[:-1] if w[2] >= 20]
    timed = sorted(full)[:5]

    vtx = next((r for r in stats if is_kernel(r["Name"])), None)
    lines = [f"# {tag}: rocprofv3 --kernel-trace --stats of `bench.py --steps 5 --warmup 2 --no-cpu --no-extras`", ""]
    if bench:
        lines += [f"bench line under the profiler: value {bench['value']:.4g} {bench['unit']}, "
                  f"{bench['ms_per_step']} ms/step, workload: {bench['config']['workload']}", ""]
    if timed:
        span = sum(w[0] for w in timed) / len(timed) / 1e6
        busy = sum(w[1] for w in timed) / len(timed) / 1e6
        nk = sum(w[2] for w in timed) / len(timed)
        lines += [f"Per step (build start to build start, {len(timed)} timed steps): span {span:.3f} ms, "
                  f"GPU busy {busy:.3f} ms ({100 * busy / span:.1f}%), idle {span - busy:.3f} ms, "
                  f"{nk:.0f} kernel launches.", ""]
    lines += ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in stats[:30]:
        lines.append(f"| {short(r['Name'])} | {r['Calls']} | {int(r['TotalDurationNs']) / 1e6:.3f} | "
                     f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")

    pmc = {"kernel": KERNEL, "tag": tag}
    for cname, sub in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write")):
        p = os.path.join(src, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        per = defaultdict(float)
        for r in read_csv(p):
            if r["Counter_Name"] == cname and is_kernel(r["Kernel_Name"]):
                per[r["Dispatch_Id"]] += float(r["Counter_Value"])
        if per:
            pmc[cname.lower() + "_kib_per_launch"] = sum(per.values()) / len(per)
            pmc[cname.lower() + "_launches"] = len(per)
    if "fetch_size_kib_per_launch" in pmc and "write_size_kib_per_launch" in pmc:
        rd = 2.0 * pmc["fetch_size_kib_per_launch"] * 1024   # gfx950: FETCH_SIZE = 1/2 of streamed bytes
        wr = pmc["write_size_kib_per_launch"] * 1024
        pmc["hbm_read_bytes_per_launch"] = rd
        pmc["hbm_write_bytes_per_launch"] = wr
        pmc["hbm_bytes_per_launch"] = rd + wr
        if vtx:
            pmc["trace_avg_launch_ns"] = float(vtx["AverageNs"])
        if bench:
            pmc["workload"] = bench["config"]["workload"]
            pmc["rows_per_gpu"] = bench["config"]["rows_per_gpu"]
            pmc["algorithmic_bytes_per_launch"] = bench["roofline"]["algorithmic_bytes_per_launch"]
            # one emission = launches_per_emission k_vtx_tile launches (two
            # when the geometry lists are row-sliced): its HBM bytes
            lpe = int(bench["roofline"].get("launches_per_emission", 1))
            pmc["launches_per_emission"] = lpe
            pmc["hbm_bytes_per_emission"] = (rd + wr) * lpe
        lines += ["", f"PMC ({KERNEL}, per launch): FETCH_SIZE {pmc['fetch_size_kib_per_launch']:.0f} KiB "
                      f"(x2 gfx950 correction -> {rd / 1e9:.3f} GB read), WRITE_SIZE "
                      f"{pmc['write_size_kib_per_launch']:.0f} KiB ({wr / 1e9:.3f} GB written)"
                      + (f"; algorithmic {pmc['algorithmic_bytes_per_launch'] / 1e9:.3f} GB" if bench else "")]
    side = os.path.join(src, "side", "run_kernel_stats.csv")
    if os.path.exists(side):
        sb = bench_line(os.path.join(src, "side.json"))
        sl = [f"# {tag}: kernel statistics of the full bench (`bench.py --steps 2 --warmup 1 --no-cpu`, "
              "side measurements included: glyph quads, font atlas, search, order)", "",
              "| kernel | calls | avg us |", "|---|---:|---:|"]
        for r in read_csv(side):
            sl.append(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} |")
        if sb:
            for k in ("glyph_quads", "font_atlas", "search", "order"):
                if k in sb:
                    sl += ["", f"{k}: `{json.dumps(sb[k])}`"]
        with open(os.path.join(dest, f"{tag}_side_kernels.md"), "w") as f:
            f.write("\n".join(sl) + "\n")
    for name in ("store_ceiling", "store_sweep"):
        sc = os.path.join(src, f"{name}.jsonl")
        if os.path.exists(sc):
            with open(sc) as f_in, open(os.path.join(dest, f"{tag}_{name}.jsonl"), "w") as f_out:
                f_out.write(f_in.read())
    with open(os.path.join(dest, f"{tag}_pmc.json"), "w") as f:
        json.dump(pmc, f, indent=1)
    with open(os.path.join(dest, f"{tag}_kernels.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
