"""Summary of profiles/pmc_step.sh: per kernel, averaged over its dispatches,
HBM-side bytes (FETCH_SIZE raw and x2 per the gfx950 correction for wide
streaming reads — uncalibrated for the narrow random reads of the hash join
and the replay, so both are printed), WRITE_SIZE, the L2 hit rate, the rate
those bytes make over the launch, and SQ counters per wave.

usage: python3 profiles/pmc_step_summary.py gpurun_out/pmc_step_<tag>
"""
import collections
import csv
import glob
import os
import re
import sys


def load(d):
    """kernel -> {counter: [per-dispatch values]}, kernel -> [durations us]"""
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    dur = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f, newline="")):
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("(anonymous namespace)::", "")).strip()
            name = re.sub(r"^void ", "", name)
            disp = int(r["Dispatch_Id"])
            vals[name][disp][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[name][disp] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    return vals, dur


def avg(xs):
    xs = list(xs)
    return sum(xs) / len(xs) if xs else float("nan")


def main():
    root = sys.argv[1]
    passes = {p: load(os.path.join(root, p)) for p in ("fetch", "write", "tcc", "sq")}
    kernels = sorted(set().union(*(set(v[0]) for v in passes.values())))
    print("| kernel | disp | us | FETCH KB (raw) | read GB/s (x2) | WRITE KB | write GB/s | L2 hit | waves | VALU/w | SALU/w | VMEM/w | LDS/w | cycles/w | wait_any/w | wait_inst/w |")
    print("|---|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|")
    for k in kernels:
        fv, fd = passes["fetch"][0].get(k, {}), passes["fetch"][1].get(k, {})
        wv, wd = passes["write"][0].get(k, {}), passes["write"][1].get(k, {})
        tv = passes["tcc"][0].get(k, {})
        sv, sd = passes["sq"][0].get(k, {}), passes["sq"][1].get(k, {})
        us = avg(list(fd.values()) + list(wd.values()) + list(sd.values()))
        fetch = avg(x.get("FETCH_SIZE", 0.0) for x in fv.values())
        write = avg(x.get("WRITE_SIZE", 0.0) for x in wv.values())
        hit = avg(x.get("TCC_HIT_sum", 0.0) for x in tv.values())
        miss = avg(x.get("TCC_MISS_sum", 0.0) for x in tv.values())
        waves = avg(x.get("SQ_WAVES", 0.0) for x in sv.values()) or float("nan")

        def per_wave(c):
            return avg(x.get(c, 0.0) for x in sv.values()) / waves
        rd_gbs = fetch * 2 * 1024 / (us * 1e3) if us == us and us > 0 else float("nan")
        wr_gbs = write * 1024 / (us * 1e3) if us == us and us > 0 else float("nan")
        hr = hit / (hit + miss) if hit + miss > 0 else float("nan")
        ndisp = max(len(fv), len(wv), len(sv))
        print(f"| {k} | {ndisp} | {us:.1f} | {fetch:.0f} | {rd_gbs:.0f} | {write:.0f} | {wr_gbs:.0f} | {hr:.2f} | {waves:.0f} | "
              f"{per_wave('SQ_INSTS_VALU'):.0f} | {per_wave('SQ_INSTS_SALU'):.0f} | {per_wave('SQ_INSTS_VMEM'):.0f} | "
              f"{per_wave('SQ_INSTS_LDS'):.0f} | {per_wave('SQ_WAVE_CYCLES'):.0f} | {per_wave('SQ_WAIT_ANY'):.0f} | "
              f"{per_wave('SQ_WAIT_INST_ANY'):.0f} |")
    print()
    print("FETCH_SIZE / WRITE_SIZE in KiB per dispatch (rocprofv3); read GB/s doubles FETCH_SIZE per the gfx950 "
          "correction (exact for 16-B streaming reads, uncalibrated for narrow random reads). SQ cycle counters are "
          "quad-cycles (MI355X_MICROARCH.md).")


if __name__ == "__main__":
    main()
