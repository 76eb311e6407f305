"""Print a rocprofv3 run_kernel_stats.csv as a short table: python3 profiles/kstats.py <csv> [regex]"""
import csv
import re
import sys

pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
for r in csv.DictReader(open(sys.argv[1], newline="")):
    n = re.sub(r"\(.*", "", r["Name"].replace("(anonymous namespace)::", ""))[:64]
    if pat and not pat.search(n):
        continue
    print("%-64s %6s %10.1f us" % (n, r["Calls"], float(r["AverageNs"]) / 1e3))
