"""CPU baselines for every BASELINE.json configuration, on the host this runs on.

The Go reference cannot be built here (no Go toolchain), so the baseline is the oracle: the C++ restatement
of the reference's allocate action (oracle/oracle.cpp), structured like it -- a full predicate chain and a
full re-score of every node per task, fanned out over a pool of worker threads the way
workqueue.ParallelizeUntil(ctx, 16, N, fn) does (vendor/k8s.io/client-go/util/workqueue/parallelizer.go:
38-71). Each config runs a bounded sample (the first `sample` task attempts of its allocate cycle) with 16
workers (the reference's ParallelizeUntil width and the GPU box's CPU share) and with 1 worker; the full
cycle time is extrapolated from the sample's rate and labelled as such.

usage: python3 scripts/cpu_baselines.py [out.json]
"""
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle  # noqa: E402
from scheduler_amd import synth  # noqa: E402

# config -> (generator kwargs, sampled task attempts, total pods of the full cycle)
PLAN = {
    "C1": (dict(), 5000, 5000),  # the reference's CPU-runnable case: the whole cycle
    "C2": (dict(), 3000, 100000),
    "C3": (dict(), 1000, 200000),
    "C4": (dict(), 300, 100000),
    # C5: the per-task cost is the 50k-node sweep; 100 jobs (the first jobs in the cycle's order are the same
    # with 10k) keep the million-pod session out of the sample's session open
    "C5": (dict(n_nodes=50000, n_jobs=100, tasks_per_job=100), 300, 1000000),
}


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    res = {"host": {"cpu": cpu_model(), "os_cpu_count": os.cpu_count(),
                    "affinity_cpus": len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else None},
           "kind": "port (oracle/oracle.cpp, reference-structured: full predicate chain + full re-score per task)",
           "configs": {}}
    for cfg, (kw, sample, total) in PLAN.items():
        gen = synth.c2 if cfg == "C5" else synth.CONFIGS[cfg]
        t0 = time.time()
        cl = gen(**kw)
        gen_s = time.time() - t0
        row = {"sample_attempts": sample, "cycle_pods": total}
        for workers in (16, 1):
            if workers == 1 and cfg in ("C4", "C5"):
                s = max(50, sample // 4)  # one thread: a smaller sample keeps the run bounded
            else:
                s = sample
            o = pyoracle.allocate(cl, workers=workers, max_tasks=s)
            secs = o["elapsed_ms"] / 1e3
            placed = len(o["events"])
            rate = placed / secs if secs > 0 else None
            row[f"workers{workers}"] = {
                "attempts": o["attempts"], "placed": placed, "seconds": round(secs, 3),
                "pods_per_s": round(rate, 1) if rate else None,
                "extrapolated_cycle_s": round(total / rate, 1) if rate else None,
                "extrapolated": s < total}
            print(cfg, workers, row[f"workers{workers}"], flush=True)
        row["generate_s"] = round(gen_s, 1)
        res["configs"][cfg] = row
    js = json.dumps(res, indent=1)
    if out_path:
        with open(out_path, "w") as f:
            f.write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
