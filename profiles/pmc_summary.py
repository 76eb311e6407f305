"""Summarise rocprofv3 --pmc counter CSVs: per-dispatch totals, averaged."""
import collections, csv, glob, sys
root = sys.argv[1]
for f in sorted(glob.glob(f"{root}/*/run_counter_collection.csv")):
    rows = list(csv.DictReader(open(f)))
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for r in rows:
        agg[r['Counter_Name']] += float(r['Counter_Value'])
        disp[r['Counter_Name']].add(r['Dispatch_Id'])
    for k, v in agg.items():
        print(f"{k:24s} per-dispatch {v / len(disp[k]):.6g}  ({len(disp[k])} dispatches)")
