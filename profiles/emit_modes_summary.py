"""Summary of profiles/emit_modes.sh runs: per engine (and phase) the median
and min k_vtx_tile time, the vertex buffer's address and placement record, and
the rocm-smi clocks / power over the run (median sclk, mclk, package power).
usage: python3 profiles/emit_modes_summary.py <dir> <tag>... > summary.json"""
import json
import re
import statistics as st
import sys
from collections import defaultdict


def summarize(d, tag):
    lines = [json.loads(x) for x in open(f"{d}/{tag}_emit_series.jsonl")]
    head, out = lines[0], {"tag": tag}
    ms = defaultdict(list)
    for s in lines[1:]:
        if "emit_ms" in s:
            ms[(s.get("engine", 0), s.get("phase", 0))].extend(s["emit_ms"])
        elif "vertices" in s:
            out["phase1_vertices"] = [hex(v) for v in s["vertices"]]
    out["mode"] = head.get("mode", head.get("contig", ""))
    out["engines"] = []
    for (k, ph), v in sorted(ms.items()):
        e = {"engine": k, "phase": ph, "calls": len(v), "median_ms": round(st.median(v), 4), "min_ms": round(min(v), 4)}
        if "views" in head:
            e["vertices"] = hex(head["views"][k]["vertices"])
            if "place" in head["views"][k]:
                e["place"] = head["views"][k]["place"]
        out["engines"].append(e)
    smi = defaultdict(list)
    for x in open(f"{d}/{tag}_smi.jsonl"):
        for key, name in (("sclk", "sclk clock speed:"), ("mclk", "mclk clock speed:"),
                          ("power_w", "Current Socket Graphics Package Power (W)")):
            m = re.search(re.escape(name) + r'": "\(?([0-9.]+)', x)
            if m:
                smi[key].append(float(m.group(1)))
    out["smi_busy_median"] = {k: st.median(sorted(v)[len(v) // 4:]) for k, v in smi.items() if v}
    return out


if __name__ == "__main__":
    print(json.dumps([summarize(sys.argv[1], t) for t in sys.argv[2:]], indent=1))
