"""Summarise an ab_lib.sh run: python3 profiles/ab_summary.py <tag>"""
import glob
import json
import os
import re
import sys

tag = sys.argv[1]
out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
res = {}
for f in sorted(glob.glob(os.path.join(out, f"{tag}_[ab][0-9]*_*.json"))):
    m = re.search(r"_([ab])(\d+)_(\w+)\.json$", f)
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
    except Exception:
        continue
    v, i, cfg = m.group(1), m.group(2), m.group(3)
    st = d.get("stages_ms", {})
    res.setdefault(cfg, {}).setdefault(v, []).append((d["ms_per_step"], st.get("vtx_emit", 0.0)))
for cfg, vv in res.items():
    for v, xs in sorted(vv.items()):
        print(f"{cfg:5s} {v}: ms/step " + " ".join(f"{x[0]:.4f}" for x in xs)
              + "   pre-emission " + " ".join(f"{x[0] - x[1]:.4f}" for x in xs))
