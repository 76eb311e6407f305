#!/bin/bash
# Summary of a profiles/cycle.sh run (here, after gpurun merged gpurun_out/<tag>)
TAG=${1:?tag}
D=gpurun_out/$TAG
grep -E "passed|failed|FAILED|Error" "$D/t.log" | tail -5
python3 - "$D" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1] + "/bench.json").read().strip().splitlines()[-1])
print({k: d[k] for k in ["value", "ms_per_step"]}, "emit", d["roofline"]["avg_launch_ms"], "frac", d["roofline"]["frac"])
print("stages", json.dumps(d.get("stages_ms")))
bc = d.get("baseline_configs", {})
print({k: (v.get("ms_per_step") or v.get("gpu_ms_per_step")) for k, v in bc.items()})
print("builds", d.get("builds"))
EOF
python3 profiles/gaps.py "$D/trace/run_kernel_trace.csv" 2.0 5 > "$D/timeline.txt" && head -1 "$D/timeline.txt" && tail -1 "$D/timeline.txt"
