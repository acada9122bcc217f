"""The fed engine's write accounting (scripts/write_account.sh runs the passes; DESIGN.md §4 has the table).

usage: python3 scripts/write_account.py <out_dir>

1. Calibration: the wcal kernels' WRITE_SIZE per dispatch against the bytes they store (wcal.log's JSON line) gives
   the counted bytes per store lane for each store form the engine uses.
2. The C2 cycle's engine dispatch (fed_engine_kernel, one per allocate cycle of 1,000 jobs): measured WRITE_SIZE per
   job, in the production pass and the A/B passes (no level records, no committed-row write-back).
3. The per-writer table: each writer's store count per job (from the C2 cycle's shape: its nodes, the placements
   per job and the distinct nodes each job commits to, taken from the oracle's frozen C2 digest) times the
   calibrated bytes of its store form, summed and set against the measured bytes per job.
"""
import csv
import glob
import json
import os
import re
import statistics
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)


def short(name):
    m = re.search(r"kbgpu::(\w+)", name) or re.search(r"(\w+)\(", name)
    return m.group(1) if m else name.split("(")[0]


def counter_per_kernel(d, counter="WRITE_SIZE"):
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
    return {k: sorted(v.values()) for k, v in per.items()}  # KiB per dispatch


def main():
    out = sys.argv[1]
    # ---- 1. calibration ----
    known = None  # wcal.log: {kernel: [stored bytes, store lanes]}
    with open(os.path.join(out, "wcal.log")) as f:
        for line in f:
            if line.startswith("{"):
                known = json.loads(line)
    cal = counter_per_kernel(os.path.join(out, "wcal"))
    per_lane = {}
    cal_rows = {}
    for k, (nbytes, lanes) in known.items():
        v = cal.get(k)
        if not v:
            continue
        kib = statistics.median(v)
        per_lane[k] = kib * 1024 / lanes
        cal_rows[k] = {"stored_bytes": nbytes, "lanes": lanes, "write_size_bytes": round(kib * 1024),
                       "counted_per_stored": round(kib * 1024 / nbytes, 3), "counted_bytes_per_lane": round(per_lane[k], 2)}
    # ---- 2. the engine's measured bytes per job ----
    jobs_per_cycle = 1000  # C2: 1,000 gang jobs, each one engine unit
    meas = {}
    for v in ("prod", "nolvl", "norows", "noacq", "noswrows", "noswst"):
        c = counter_per_kernel(os.path.join(out, v)).get("fed_engine_kernel")
        if c:
            meas[v] = {"dispatches": len(c), "kib_per_dispatch": [round(x, 1) for x in c],
                       "bytes_per_job": round(statistics.median(c) * 1024 / jobs_per_cycle)}
    fetch = counter_per_kernel(os.path.join(out, "fetch"), "FETCH_SIZE").get("fed_engine_kernel")
    # ---- 3. store counts per job (C2) ----
    from scheduler_amd import synth
    snap = synth.c2_snapshot()
    z = np.load(os.path.join(ROOT, "tests", "golden", "digest-C2.npz"))
    tj = np.asarray(snap.s_task_job)[z["event_task"]]
    pairs = len(set(zip(tj.tolist(), z["event_node"].tolist())))
    n = int(snap.n_nodes)
    c = pairs / jobs_per_cycle        # distinct nodes a job commits to
    T = len(z["event_task"]) / jobs_per_cycle  # placements per job
    nsw_group = 21                    # C2: 42 resident sweepers in two groups (engine.sweepers in the bench line)
    fac = lambda k: cal_rows[k]["counted_per_stored"] if k in cal_rows else 1.0
    rows = [
        # writer, store form (its calibrated counted / stored bytes), stored bytes per job
        ("sweepers: level-0 keys (4 B per node, plain)", "w_plain4", 4 * n),
        ("sweepers: static cache (8 B per node, plain)", "w_plain8", 8 * n),
        ("sweepers: level records (32 B per feasible node, 4-B stores)", "w_plain4_rec", 32 * n),
        ("sweepers: ring counter adds + relay words (single words)", "w_at8_scatter", 8 * (nsw_group + 10)),
        ("selector: candidate entries (16 words x T, agent atomic)", "w_at8", 8 * 16 * T),
        ("selector: B static caches + command words + head", "w_at8", 8 * (T + 17)),
        ("placer: published set (T words) + head / done", "w_at8", 8 * (T + 2)),
        ("placer: committed rows (7 columns per node, one line each)", "w_at8_scatter", 8 * 7 * c),
        ("placer: commit list (4 B per node, agent atomic)", "w_at4", 4 * c),
        ("placer: placements + job state to pinned host memory", "w_plain4", 8 * T + 256),
    ]
    table = []
    total = 0.0
    for name, form, stored in rows:
        b = stored * fac(form)
        total += b
        table.append({"writer": name, "form": form, "stored_bytes_per_job": round(stored),
                      "counted_per_stored": fac(form), "bytes_per_job": round(b)})
    res = {"calibration": cal_rows, "measured": meas,
           "fetch_bytes_per_job": round(statistics.median(fetch) * 1024 * 2 / jobs_per_cycle) if fetch else None,
           "c2_shape": {"nodes": n, "placements_per_job": T, "distinct_nodes_per_job": round(c, 2)},
           "model": table, "model_bytes_per_job": round(total)}
    if "prod" in meas:
        m = meas["prod"]["bytes_per_job"]
        res["model_over_measured"] = round(total / m, 3) if m else None
        lv = [r for r in table if "level records" in r["writer"]][0]["bytes_per_job"]
        rw = [r for r in table if "committed rows" in r["writer"]][0]["bytes_per_job"]
        if "nolvl" in meas:
            res["ab_level_records"] = {"measured": m - meas["nolvl"]["bytes_per_job"], "model": lv}
        if "norows" in meas:
            res["ab_committed_rows"] = {"measured": m - meas["norows"]["bytes_per_job"], "model": rw}
        for v, what in (("noacq", "sweepers' per-job acquire"), ("noswrows", "sweepers' row loads"),
                        ("noswst", "sweepers' key / static-cache stores")):
            if v in meas:
                res["ab_" + v] = {"what": what, "measured": m - meas[v]["bytes_per_job"]}
    print(json.dumps(res, indent=1))
    with open(os.path.join(out, "write_account.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
