"""Probe: allocate cycles of C2 (10k x 100k) on a node-sharded context with one rank, per exchange kind:
  peer -- the node-sharded fed engine (kb_set_shard_peer): the resident engine proposes, exchanges through the
          inboxes and merges on the device, one launch per cycle plus one sweep per job;
  rccl -- the pipelined launch path (sweep, proposal, ncclAllGather, merge + commit per job);
  none -- the unsharded fed engine on the same box, for comparison.
Usage: python3 scripts/shard_pipeline_probe.py [--opt no_pipeline,...] [peer|rccl ...]   (no_pipeline: the serial
driver)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scheduler_amd import runtime, synth  # noqa: E402


def probe(kind, snap, opts):
    ctx = runtime.Context(0, timing=True, options=opts)
    if kind == "peer":
        ctx.set_shard(0, 1, snap.n_nodes, allgather=lambda b: b, peer=True)
    elif kind == "rccl":
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
    jobs = st["job_calls"] / 3
    print(json.dumps({"exchange": kind, "pipeline": not opts.get("no_pipeline"),
                      "cycle_ms": round(min(ts) * 1e3, 2), "us_per_job": round(min(ts) * 1e6 / jobs, 2),
                      "pods_per_s": round(int(out["n_events"]) / min(ts), 1), "sharded_engine_cycles":
                      st["fed_sharded"], "us_per_launch": per}), flush=True)
    ctx.close()


def main():
    snap = synth.c2_snapshot(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=synth.SEED)
    args = sys.argv[1:]
    opts = {}
    if args[:1] == ["--opt"]:
        opts, args = runtime.parse_options(args[1]), args[2:]
    for kind in args or ["none", "peer", "rccl"]:
        probe(kind, snap, opts)


if __name__ == "__main__":
    main()
