"""Probe: one allocate cycle of C2 (10k x 100k) on a node-sharded context with a one-rank RCCL communicator
(the pipelined sharded path: sweep, proposal, ncclAllGather, merge + commit per job, no host round trip
between jobs), against the serial kb_place_job-per-job driver (KB_NO_PIPELINE=1 in a second run)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scheduler_amd import runtime, synth  # noqa: E402

snap = synth.c2_snapshot(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=synth.SEED)
ctx = runtime.Context(0, timing=True)
ctx.set_shard(0, 1, snap.n_nodes, rccl_id=runtime.comm_unique_id())
ctx.upload(snap)
ctx.allocate(snap)
ctx.stats(reset=True)
ts = []
for _ in range(3):
    ctx.restore()
    t0 = time.perf_counter()
    out = ctx.allocate(snap)
    ts.append(time.perf_counter() - t0)
st = ctx.stats()
k = runtime.KERNELS
per = {k[i]: round(st["kernel_ms"][i] * 1e3 / st["launches"][i], 2) for i in range(len(k)) if st["launches"][i]}
print(json.dumps({"pipeline": os.environ.get("KB_NO_PIPELINE") is None, "cycle_ms": round(min(ts) * 1e3, 2),
                  "pods_per_s": round(int(out["n_events"]) / min(ts), 1), "us_per_launch": per}))
ctx.close()
