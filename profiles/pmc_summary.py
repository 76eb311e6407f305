"""Per-kernel, per-wave SQ counter summary of a rocprofv3 --pmc run
(run_counter_collection.csv): instructions by kind, wave cycles and wait
cycles per wave, averaged over the dispatches of each kernel.
usage: python3 profiles/pmc_summary.py <run_counter_collection.csv>"""
import collections
import csv
import re
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    meta = {}
    for r in rows:
        name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", ""))
        key = (name, int(r["Dispatch_Id"]))
        d[key][r["Counter_Name"]] += float(r["Counter_Value"])
        meta[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, r["VGPR_Count"], r["Workgroup_Size"]
    byk = collections.defaultdict(list)
    for (k, disp), v in d.items():
        byk[k].append((disp, v, meta[(k, disp)]))
    cols = ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
            "SQ_WAIT_INST_ANY"]
    short = ["valu", "salu", "vmrd", "vmwr", "lds", "cycles", "wait"]
    print(f"{'kernel':28s} {'disp':>4s} {'us':>7s} {'vgpr':>4s} {'waves':>7s} " + " ".join(f"{s:>8s}" for s in short))
    for k, lst in sorted(byk.items()):
        for disp, v, (us, vgpr, wg) in sorted(lst)[-3:]:
            w = v.get("SQ_WAVES", 1.0) or 1.0
            print(f"{k:28s} {disp:4d} {us:7.1f} {vgpr:>4s} {int(w):7d} " +
                  " ".join(f"{v.get(c, 0) / w:8.0f}" for c in cols))


if __name__ == "__main__":
    main()
