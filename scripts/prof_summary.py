"""Summarise rocprofv3 output for profiles/: kernel-trace stats and PMC (FETCH_SIZE / WRITE_SIZE) per launch.

usage: python3 scripts/prof_summary.py <trace_dir> <fetch_dir> <write_dir> <out.json> [pmc_cycles]

pmc_cycles: the allocate cycles the PMC passes ran (bench.py --steps 1 --warmup 0 --no-timing: the step and the
host-split cycle after it = 2); with it, each kernel's PMC dispatch count makes the cycle's measured traffic
(bench.py pmc_cycle_traffic: bytes per dispatch x dispatches / cycles, summed over the cycle's kernels).

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch. On gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read (MI355X_MICROARCH.md, HBM section), so `hbm_read_bytes` doubles it; WRITE_SIZE is taken
as is. Both count memory-side L2 requests (Infinity-Cache hits included).
"""
import csv
import glob
import json
import os
import re
import sys


def short(name):
    m = re.search(r"kbgpu::(\w+)", name)
    return m.group(1) if m else name.split("(")[0]


def kernel_stats(d):
    out = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row["Name"])
                e = out.setdefault(k, {"calls": 0, "total_ns": 0})
                e["calls"] += int(row["Calls"])
                e["total_ns"] += int(float(row["TotalDurationNs"]))
    for e in out.values():
        e["avg_us"] = round(e["total_ns"] / max(1, e["calls"]) / 1e3, 3)
    return out


def counters(d, counter):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                k = short(row.get("Kernel_Name", ""))
                disp = row.get("Dispatch_Id", "")
                e = per.setdefault(k, {})
                e[disp] = e.get(disp, 0.0) + float(row["Counter_Value"])
    return {k: {"dispatches": len(v), "avg_kib": sum(v.values()) / max(1, len(v))} for k, v in per.items()}


def main():
    trace, fetch, write, out = sys.argv[1:5]
    cycles = int(sys.argv[5]) if len(sys.argv) > 5 else None
    ks = kernel_stats(trace)
    fs = counters(fetch, "FETCH_SIZE")
    ws = counters(write, "WRITE_SIZE")
    res = {"kernels": {}, **({"pmc_cycles": cycles} if cycles else {})}
    for k in sorted(set(ks) | set(fs) | set(ws)):
        e = dict(ks.get(k, {}))
        if k in fs:
            e["fetch_size_kib_per_launch"] = round(fs[k]["avg_kib"], 2)
            e["pmc_dispatches"] = fs[k]["dispatches"]
            e["hbm_read_bytes_per_launch"] = round(2 * fs[k]["avg_kib"] * 1024, 1)
        if k in ws:
            e["write_size_kib_per_launch"] = round(ws[k]["avg_kib"], 2)
            e["hbm_write_bytes_per_launch"] = round(ws[k]["avg_kib"] * 1024, 1)
        if "hbm_read_bytes_per_launch" in e and "hbm_write_bytes_per_launch" in e:
            e["hbm_bytes_per_launch"] = e["hbm_read_bytes_per_launch"] + e["hbm_write_bytes_per_launch"]
        res["kernels"][k] = e
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
