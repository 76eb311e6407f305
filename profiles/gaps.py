"""Per-step kernel timeline from a rocprofv3 --kernel-trace CSV: kernels of
one step (from a build's first kernel to the next build's; t = 0 at the end
of the previous step's last kernel), their durations and the idle gap
before each one (host synchronisations show up as gaps).

usage: python3 profiles/gaps.py <run_kernel_trace.csv> [min_gap_us] [step]
  step: which step (from 0); default the last complete one.  bench.py's last steps are its stage-breakdown
        pass, whose per-stage HIP events show up as ~10 us gaps: pick a step
        of the timed region (after the warmup) to see the timed step.
"""
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1], newline="")))
    min_gap = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                  re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))) for r in rows))
    # a step starts at its build's first kernel (the near probe; the hash
    # place on lists built another way); the emission may be two launches
    first = "k_probe_near" if any(k[2] == "k_probe_near" for k in ks) else "k_hash_place"
    starts = [i for i, k in enumerate(ks) if k[2] == first] + [len(ks)]
    if len(sys.argv) > 3:
        st = int(sys.argv[3])
    else:
        st = len(starts) - 3
    a, b = starts[st], starts[st + 1]
    step = ks[a:b]
    t0 = max(e for _, e, _ in ks[:a]) if a else step[0][0]
    busy = sum(e - s for s, e, _ in step)
    span = step[-1][1] - t0
    print(f"step span {span / 1e3:.1f} us, busy {busy / 1e3:.1f} us, {len(step)} kernels")
    prev = t0
    idle_total = 0
    for s, e, n in step:
        gap = (s - prev) / 1e3
        if gap > 0:
            idle_total += gap
        mark = "  <-- gap" if gap >= min_gap else ""
        print(f"{(s - t0) / 1e3:9.1f} {gap:7.1f} {(e - s) / 1e3:8.1f}  {n}{mark}")
        prev = max(prev, e)
    print(f"idle {idle_total:.1f} us")


if __name__ == "__main__":
    main()
