"""Full-size placement digests: the oracle's allocate outcome on BASELINE.json's
configurations at full size, frozen as data so the GPU test can compare the HIP path against the oracle at
the sizes the bench runs, without re-running the oracle on the GPU box.

For each config: digest-<cfg>.npz holds the placement sequence (session-task index, node index, kind per
event, in the cycle's order) plus every job's failing task, and digest-<cfg>.json the sha256 of those
arrays, the counts and the FitErrors of the failed jobs. Indices follow export.Snapshot of the same
seeded cluster (synth.CONFIGS[cfg]() with the generator defaults).

Run from the repo root:  python tests/golden/make_digests.py C1 C2 [C3 C4]   (oracle on 8 threads;
C2 takes about 1.5 minutes here, C3 several)
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from helpers import digest_arrays  # noqa: E402
from oracle import pyoracle  # noqa: E402
from scheduler_amd import export as E  # noqa: E402
from scheduler_amd import synth  # noqa: E402

KIND = {"allocate": 1, "pipeline": 2}


# C5-head: the first placements of a 300-job C5-shaped cluster (the sharded 3-rank test compares a prefix)
HEADS = {"C5-head": (dict(n_nodes=50000, n_jobs=300, tasks_per_job=100), 3000),
         # past the resident engine's node ceiling on one GPU (4 range selectors x 20,480 nodes): 100k C2-shaped
         # nodes, the whole cycle of 30 jobs (test_gpu_big.py runs it on the per-commit re-key path)
         "X100k-head": (dict(n_nodes=100000, n_jobs=30, tasks_per_job=100), 3000)}
# BASELINE.json configs[4] at full size: the C2 shape at 50k nodes x 1M pods (10k jobs)
SHAPES = {"C5": dict(n_nodes=50000, n_jobs=10000, tasks_per_job=100)}


def cluster_of(cfg):
    if cfg in HEADS:
        return synth.c2(**HEADS[cfg][0])
    if cfg in SHAPES:
        return synth.c2(**SHAPES[cfg])
    return synth.CONFIGS[cfg]()


def make(cfg, workers=int(os.environ.get("DIGEST_WORKERS", "8"))):
    cl = cluster_of(cfg)
    snap = E.Snapshot(cl)
    max_tasks = HEADS[cfg][1] if cfg in HEADS else -1
    t0 = time.time()
    out = pyoracle.allocate(cl, workers=workers, max_tasks=max_tasks)
    secs = time.time() - t0
    uid = {t["uid"]: i for i, t in enumerate(snap.session_tasks)}
    nidx = snap.node_index
    ev = out["events"]
    event_task = np.array([uid[e["task"]] for e in ev], np.int32)
    event_node = np.array([nidx[e["node"]] for e in ev], np.int32)
    event_kind = np.array([KIND[e["kind"]] for e in ev], np.int8)
    job_fail = np.full(len(snap.jobs), -1, np.int32)
    jidx = {j["uid"]: i for i, j in enumerate(snap.jobs)}
    for ju, tf in out["fit_errors"].items():
        for tu in tf:
            job_fail[jidx[ju]] = uid[tu]
    np.savez_compressed(os.path.join(HERE, f"digest-{cfg}.npz"), event_task=event_task, event_node=event_node,
                        event_kind=event_kind, job_fail=job_fail)
    shape = HEADS[cfg][0] if cfg in HEADS else SHAPES.get(cfg)
    meta = {"config": cfg, "generator": ("synth.c2(**%r)" % (shape,) if shape is not None else
                                         "synth.CONFIGS[%r]() defaults" % cfg) + " (seed %d)" % synth.SEED,
            "max_tasks": max_tasks,
            "nodes": snap.n_nodes, "pods": len(snap.session_tasks), "events": len(ev),
            "failed_jobs": int((job_fail >= 0).sum()), "sha256": digest_arrays(event_task, event_node, event_kind,
                                                                              job_fail),
            "fit_errors": out["fit_errors"], "oracle_seconds": round(secs, 1), "oracle_workers": workers,
            "source": "oracle/oracle.cpp (CPU restatement) via tests/golden/make_digests.py"}
    with open(os.path.join(HERE, f"digest-{cfg}.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
        f.write("\n")
    print(cfg, "events", len(ev), "oracle", round(secs, 1), "s", meta["sha256"][:16], flush=True)


if __name__ == "__main__":
    for c in sys.argv[1:] or ["C1", "C2"]:
        make(c)
