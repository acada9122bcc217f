"""Benchmark: kube-batch allocate cycles on MI355X (BASELINE.json metric).

metric : pods placed/sec (+ p50 allocate-cycle ms) at 10k nodes x 100k pods (BASELINE.json configs[1], "C2")
step   : one allocateAction.Execute (actions/allocate/allocate.go:42-193) over the C2 session snapshot:
         re-open the session from the snapshot already resident in HBM (kb_restore_nodes, device-to-device),
         then kb_allocate (host ordering plugins + per-job device sweep/argmax/commit). The snapshot is
         uploaded once before the timed region; value = pods placed / second over the timed steps.

Multi-GPU (N > 1, one process per GPU): every rank schedules its own independent C2 cluster (a partition of the
fleet with its own seed; no collective on the data path: torch.distributed only for the barriers and the
max-over-ranks time) -- `value` = all ranks' pods / the max-over-ranks time, scaling "weak", the same per-GPU
workload as the N = 1 line. One allocate cycle is a sequential chain of jobs, so GPUs add throughput by serving
partitions. Beside it, "sharded": BASELINE.json configs[4], C5 -- ONE cluster of 50k C2-shaped nodes x 1M pods
whose node table is split across the N ranks: every rank's resident engine proposes its first T picks per job and
writes them into every rank's inbox over xGMI (kb_set_shard_peer: device memory mapped across the GPUs), then
merges them on the device -- no host round trip or collective launch per job. `--mode shard` makes that the line.
`python bench.py --gpus N` without torchrun's environment starts the N ranks itself (before any GPU call).
One GPU also runs C5 whole: `--config C5` (the split fed engine with range selectors).

Extra JSON fields: roofline (dominant kernel, HIP events on the library's stream during the timed region),
eval_roofline (the fit/score sweep kb_eval at 256 specs x 50k nodes: the HBM-bound kernel), and cpu_baseline
(the oracle's C++ restatement of the reference algorithm on a bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
# per configuration: generator defaults, algorithmic node-table bytes per (task, node) evaluation
# (the row bytes the enabled predicate / score stages read) and the workload line
CONFIGS = {
    "C1": dict(nodes=1000, jobs=100, tasks=50, row_bytes=76,
               workload="C1: 1k nodes x 5k pods in 100 gang jobs (the reference's CPU-runnable case)"),
    "C2": dict(nodes=10000, jobs=1000, tasks=100, row_bytes=76,
               workload="C2: 10k homogeneous nodes x 100k pods in 1k gang jobs, resource-fit + "
                        "LeastRequested/Balanced (default tiers)"),
    "C3": dict(nodes=20000, jobs=2000, tasks=100, row_bytes=124,
               workload="C3: 20k heterogeneous nodes x 200k pods, GPU scalars, taints/tolerations, node affinity"),
    "C4": dict(nodes=10000, jobs=1000, tasks=100, row_bytes=88,
               workload="C4: 10k nodes x 100k pods, inter-pod (anti)affinity over hostname / zone / rack"),
    "C5": dict(nodes=50000, jobs=10000, tasks=100, row_bytes=76,
               workload="C5: 50k nodes x 1M pods (C2 shape), node table sharded across the GPUs"),
}
ARRAY_CONFIGS = ("C2", "C5")  # built by synth.c2_snapshot (numpy) instead of per-pod objects


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="BASELINE.json configuration (default: C2, the headline metric's; C5 node-sharded at N>1)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--tasks-per-job", type=int, default=None)
    ap.add_argument("--cpu-sample-tasks", type=int, default=3000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events (roofline unavailable)")
    ap.add_argument("--path", default="select", choices=["select", "engine", "trajectory", "rekey"],
                    help="device path for the runs (scheduler_amd.runtime.PATHS)")
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "shard"],
                    help="N>1: shard = ONE cluster, node table split across the ranks, one RCCL all-gather per run "
                         "segment; replicas = every rank schedules its own cluster (no collective). auto = shard "
                         "(C5) as the line, plus a short replicas measurement beside it")
    ap.add_argument("--side-steps", type=int, default=5, help="cycles of the side measurement (auto, N>1)")
    ap.add_argument("--no-eval", action="store_true", help="skip the kb_eval roofline measurement (N=1)")
    ap.add_argument("--timing-every", type=int, default=8,
                    help="HIP events around the launches of every Nth job call of the timed region")
    args = ap.parse_args()
    args.mode_auto = args.mode == "auto"

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)  # torchrun's environment is missing: start the ranks (no GPU touched yet)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    mode = args.mode if args.mode != "auto" else "replicas"
    args.mode = mode
    args.config = args.config or ("C5" if mode == "shard" and world > 1 else "C2")
    cfg = CONFIGS[args.config]
    args.nodes = args.nodes or cfg["nodes"]
    args.jobs = args.jobs or cfg["jobs"]
    args.tasks_per_job = args.tasks_per_job or cfg["tasks"]
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # KB_BENCH_SAME_GPU=1: rehearse N ranks on one GPU (gloo process group; with KB_FED_PLAIN_LAUNCH=1, see
    # scripts/rehearse_multi.sh)
    same_gpu = os.environ.get("KB_BENCH_SAME_GPU") == "1"
    device = 0 if same_gpu else local_rank
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        torch.cuda.set_device(device)
        dist_mod.init_process_group("nccl" if torch.cuda.is_available() and not same_gpu else "gloo")
        dist = dist_mod

    from scheduler_amd import export, runtime, synth

    shard = args.mode == "shard" and world > 1
    # replicas: each rank an independent cluster partition (different seed per rank); shard: one cluster
    seed = synth.SEED + (0 if shard else rank)
    cl = None
    walk_ms = None
    e0 = time.perf_counter()
    if args.config in ARRAY_CONFIGS:  # the numpy session builder (equal to the exporter: test_export.py)
        snap = synth.c2_snapshot(n_nodes=args.nodes, n_jobs=args.jobs, tasks_per_job=args.tasks_per_job, seed=seed)
        export_kind = "synth.c2_snapshot (numpy arrays)"
    else:
        from scheduler_amd import columns
        cl = synth.CONFIGS[args.config](n_nodes=args.nodes, n_jobs=args.jobs, tasks_per_job=args.tasks_per_job,
                                        seed=seed)
        w0 = time.perf_counter()
        cols = columns.columns_of(cl)  # stands in for the Go shim's walk over ssn.Nodes / ssn.Jobs
        walk_ms = (time.perf_counter() - w0) * 1e3
        e0 = time.perf_counter()
        snap = columns.build(cols)
        export_kind = ("columns.build (vectorised over the session's columns; equal to export.Snapshot array by "
                       "array: tests/test_columns.py)")
    export_ms = (time.perf_counter() - e0) * 1e3
    ctx = runtime.Context(device, timing=not args.no_timing, timing_every=args.timing_every, path=args.path)
    if shard:
        ctx.set_shard(rank, world, snap.n_nodes, **shard_exchange(dist, rank, device))
    ctx.upload(snap)

    def step():
        ctx.restore()
        return ctx.allocate(snap)

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        step()
    ctx.stats(reset=True)
    barrier()
    t0 = time.perf_counter()
    times, placed = [], 0
    for _ in range(args.steps):
        s0 = time.perf_counter()
        out = step()
        times.append((time.perf_counter() - s0) * 1e3)
        placed += int(out["n_events"])
    barrier()
    elapsed = time.perf_counter() - t0
    st = ctx.stats()
    # SURVEY.md §8 d1 also asks for the cycle WITH the snapshot upload: time re-uploads of the same snapshot
    # (kb_set_config + kb_upload_nodes + kb_upload_specs [+ affinity tables]; host arrays -> HBM), after the
    # timed region so they do not disturb it
    up = []
    if not shard:
        for _ in range(3):
            u0 = time.perf_counter()
            ctx.upload(snap)
            up.append((time.perf_counter() - u0) * 1e3)

    total_placed = placed
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=tensor_device(dist, device))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        if not shard:  # replicas place their own pods; sharded ranks all report the same placements
            p = torch.tensor([placed], dtype=torch.float64, device=tensor_device(dist, device))
            dist.all_reduce(p, op=dist.ReduceOp.SUM)
            total_placed = int(p.item())
    side = None
    if world > 1 and mode == "shard":
        side = {"replicas": replicas_side(args, dist, rank, world, device)}
    elif world > 1 and args.mode_auto:
        side = {"sharded": shard_side(args, dist, rank, world, device)}
    ev = None
    if world == 1 and rank == 0 and not args.no_eval:
        ev = eval_side(device)

    roofline = roofline_of(st, args, cfg)
    engine = engine_of(st, args) if st["launches"][runtime.KERNELS.index("fed_engine_kernel")] else None

    workload = cfg["workload"]
    if (args.nodes, args.jobs, args.tasks_per_job) != (cfg["nodes"], cfg["jobs"], cfg["tasks"]):
        workload = f"{args.config} shape at {args.nodes} nodes x {args.jobs * args.tasks_per_job} pods"
    result = None
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            if cl is None:  # the oracle runs on the cluster objects of the same workload
                cl = synth.CONFIGS.get(args.config, synth.c2)(n_nodes=args.nodes, n_jobs=args.jobs,
                                                            tasks_per_job=args.tasks_per_job, seed=seed)
            cpu = cpu_baseline(cl, args.cpu_sample_tasks, args.config)
        result = {
            "metric": "pods placed/sec + p50 allocate-cycle ms at 10k nodes x 100k pods",
            "value": round(total_placed / elapsed, 1), "unit": "pods/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "p50_cycle_ms": round(statistics.median(times), 3),
            **({"upload_ms": round(statistics.median(up), 3),
                "p50_cycle_with_upload_ms": round(statistics.median(times) + statistics.median(up), 3)} if up else {}),
            # session open: building the exported snapshot from the cluster objects (the Go shim's
            # exportSnapshot twin) + its upload; the reference's counterpart is cache.Snapshot + OnSessionOpen
            "session_open": {"export_ms": round(export_ms, 1), "export": export_kind,
                             "upload_ms": round(statistics.median(up), 3) if up else None,
                             **({"shim_walk_ms": round(walk_ms, 1),
                                 "shim_walk": "columns.columns_of: the per-pod walk into columns, in Python here "
                                              "(the Go shim's work; not part of the export)"}
                                if walk_ms is not None else {})},
            "higher_is_better": True, "scaling": "strong" if shard else "weak", "vs_baseline": None,
            "dtype": "int64", "data": f"synthetic (seeded {args.config} generator, SURVEY.md §8 d2)",
            "config": {"workload": workload,
                       "nodes": args.nodes, "pods": args.jobs * args.tasks_per_job, "jobs": args.jobs,
                       "pods_placed_per_cycle": placed // max(1, args.steps),
                       "parallelism": f"node_shard{world}" if shard else f"replicas{world}"},
            "device_ms_per_step": round(st["device_ms"] / args.steps, 3),
            **({"diag_place_phases": diag_summary(st["diag"], placed, "fed_engine_kernel" if engine is not None
                                                  else roofline["kernel"])}
               if any(st["diag"]) else {}),
            "job_calls_per_step": st["job_calls"] / args.steps,
            "roofline": roofline,
            **({"engine": engine} if engine is not None else {}),
            "cpu_baseline": cpu,
            **({"shard_exchange_us_per_segment": exchange_us(st),
                "shard_segments_per_step": st["launches"][runtime.KERNELS.index("shard_exchange")] / args.steps}
               if shard else {}),
            **(side if side is not None else {}),
            **({"eval_roofline": ev} if ev is not None else {}),
        }
        print(json.dumps(result), flush=True)
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


SWEEP_OUT_BYTES = 12  # the level-0 sweep's output per node: 4 B key + 8 B static cache


def roofline_of(st, args, cfg, streaming=False):
    """The roofline of the cycle's HBM-streaming kernel. Fed-engine cycles: the per-job level-0 sweep
    (sel_sweep_kernel on the sweep stream: every node's row read and its key written once per job -- the hot
    path's fit/score evaluation of every (job spec, node) pair); the resident engine itself is a latency-bound
    chain and is reported beside it ("engine"). Other cycles: the kernel with the most event time. achieved =
    algorithmic bytes per launch (the row bytes of each (task, node) evaluation the launch makes,
    plus the sweep's output) / the launch's average HIP-event duration on the stream it runs on; traffic = the
    same kernel's measured HBM bytes per launch from this configuration's committed rocprofv3 PMC pass."""
    from scheduler_amd import runtime
    K = runtime.KERNELS
    fed = st["launches"][K.index("fed_engine_kernel")] > 0
    if fed or (streaming and st["launches"][K.index("sel_sweep_kernel")]):  # streaming: node-sharded cycles
        k = K.index("sel_sweep_kernel")
    else:
        kern_ms = [0.0 if K[i] in ("shard_exchange", "fed_engine_kernel") else v for i, v in enumerate(st["kernel_ms"])]
        k = int(np.argmax(kern_ms)) if any(kern_ms) else 0
    launches = max(1, st["launches"][k])
    avg_ms = st["kernel_ms"][k] / launches
    per_eval = cfg["row_bytes"] + (SWEEP_OUT_BYTES if K[k] == "sel_sweep_kernel" else 0)
    bytes_per_launch = st["pairs"][k] * per_eval / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    out = {"bound": "hbm", "kernel": K[k], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "traffic_source": None,
           "avg_launch_us": round(avg_ms * 1e3, 3), "timed_launches": st["launches"][k],
           "timing": (f"HIP events on the sweep stream around every {args.timing_every}th job's sweep launch in the "
                      f"timed region" if K[k] == "sel_sweep_kernel" else
                      f"HIP events on the library stream around every launch of every {args.timing_every}th job "
                      f"call in the timed region"),
           "algorithmic_bytes_per_launch": round(bytes_per_launch, 1),
           "algorithmic_bytes_note": (f"{cfg['row_bytes']} B row read + {SWEEP_OUT_BYTES} B key/static cache written "
                                      f"per node, every node once per job" if K[k] == "sel_sweep_kernel" else
                                      f"{cfg['row_bytes']} B row per (task, node) evaluation (SURVEY.md §8 d3)"),
           "avg_us_per_launch": {K[i]: round(st["kernel_ms"][i] * 1e3 / st["launches"][i], 3)
                                 for i in range(len(K)) if st["launches"][i]},
           "measured_frac": None}
    full = (args.nodes, args.jobs, args.tasks_per_job) == (cfg["nodes"], cfg["jobs"], cfg["tasks"])
    tr = pmc_traffic(K[k], args.config) if full else None
    if tr is not None:
        out["traffic"] = tr["bytes_per_launch"]
        out["traffic_source"] = tr["source"] + f": {K[k]} " + (
            "(the same kernel and launch size; counters taken on the per-job launch path, KB_NO_FED=1, because "
            "counter collection serialises dispatches and the resident engine waits on the sweeps)" if fed else
            "(this kernel, this configuration)")
        if avg_ms > 0:
            out["measured_frac"] = round(tr["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)
    return out


def engine_of(st, args):
    """The resident fed engine (one launch per allocate cycle): a latency-bound chain of dependent LDS round
    trips per job inside one placer workgroup fed by selector workgroups -- not an HBM roofline kernel. Its
    launch spans the cycle; the per-job time and the committed KB_DIAG phase split (busy vs waiting) are what
    bound it."""
    from scheduler_amd import runtime
    K = runtime.KERNELS
    k = K.index("fed_engine_kernel")
    launches = max(1, st["launches"][k])
    us = st["kernel_ms"][k] * 1e3 / launches
    jobs = st["job_calls"] / launches
    return {"kernel": "fed_engine_kernel", "bound": "latency (per-job dependent chain in one workgroup)",
            "avg_launch_us": round(us, 3), "launches": st["launches"][k], "jobs_per_launch": round(jobs, 1),
            "us_per_job": round(us / max(1.0, jobs), 3)}


def tensor_device(dist, device):
    return "cpu" if dist is not None and dist.get_backend() == "gloo" else f"cuda:{device}"


def shard_exchange(dist, rank, device):
    """Context.set_shard keywords: the node-sharded fed engine's device exchange (kb_set_shard_peer), whose inbox
    IPC handles travel once through an all-gather over the torch process group (RCCL, or gloo when the ranks share
    one GPU in a rehearsal); that all-gather also serves any job the engine does not run."""
    import torch
    world = dist.get_world_size()
    dev = "cpu" if dist.get_backend() == "gloo" else f"cuda:{device}"

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8, device=dev)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.cpu().tolist()) for o in outs)
    return {"allgather": allgather, "peer": True}


def exchange_us(st):
    from scheduler_amd import runtime
    k = runtime.KERNELS.index("shard_exchange")
    return round(st["kernel_ms"][k] * 1e3 / st["launches"][k], 2) if st["launches"][k] else None


def replicas_side(args, dist, rank, world, device):
    """Beside the sharded line: every rank schedules its own independent C2 cluster (different seed per rank,
    no collective), `side_steps` cycles; pods/s over all ranks at the max-over-ranks time."""
    import torch
    from scheduler_amd import runtime, synth
    try:
        c = CONFIGS["C2"]
        snap = synth.c2_snapshot(n_nodes=c["nodes"], n_jobs=c["jobs"], tasks_per_job=c["tasks"], seed=synth.SEED + rank)
        ctx = runtime.Context(device)
        ctx.upload(snap)
        ctx.allocate(snap)  # warm-up cycle
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        placed = 0
        for _ in range(args.side_steps):
            ctx.restore()
            placed += int(ctx.allocate(snap)["n_events"])
        dist.barrier()
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tensor_device(dist, device))
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        p = torch.tensor([placed], dtype=torch.float64, device=tensor_device(dist, device))
        dist.all_reduce(p, op=dist.ReduceOp.SUM)
        ctx.close()
        return {"workload": f"C2 replicas: {world} independent 10k x 100k clusters, one per rank (no collective)",
                "value": round(float(p.item()) / float(el.item()), 1), "unit": "pods/s", "steps": args.side_steps,
                "scaling": "weak", "ms_per_step": round(float(el.item()) / args.side_steps * 1e3, 3)}
    except Exception as e:  # the side measurement never takes the main line down
        return {"error": repr(e)[:300]}


def shard_side(args, dist, rank, world, device):
    """Beside the replicas line (N > 1): BASELINE.json configs[4], C5 -- ONE cluster of 50k C2-shaped nodes x 1M
    pods whose node table is split across the N ranks (contiguous blocks; per job every rank's engine proposes,
    writes its proposal into every rank's inbox over xGMI and merges all of them; every rank commits its own rows).
    `side_steps` cycles after one warm-up; pods/s at the max-over-ranks time."""
    import torch
    from scheduler_amd import runtime, synth
    try:
        c = CONFIGS["C5"]
        nodes = c["nodes"]
        snap = synth.c2_snapshot(n_nodes=nodes, n_jobs=c["jobs"], tasks_per_job=c["tasks"], seed=synth.SEED)
        ctx = runtime.Context(device, timing=True, timing_every=args.timing_every)
        ctx.set_shard(rank, world, snap.n_nodes, **shard_exchange(dist, rank, device))
        ctx.upload(snap)
        ctx.allocate(snap)  # warm-up cycle
        ctx.stats(reset=True)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        placed = 0
        for _ in range(args.side_steps):
            ctx.restore()
            placed = int(ctx.allocate(snap)["n_events"])
        dist.barrier()
        torch.cuda.synchronize()
        el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=tensor_device(dist, device))
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        st = ctx.stats()
        ctx.close()
        a = argparse.Namespace(**vars(args))
        a.config, a.nodes, a.jobs, a.tasks_per_job = "C5", nodes, c["jobs"], c["tasks"]
        elapsed = float(el.item())
        out = {"workload": c["workload"], "value": round(placed * args.side_steps / elapsed, 1), "unit": "pods/s",
               "steps": args.side_steps, "scaling": "strong", "ms_per_step": round(elapsed / args.side_steps * 1e3, 3),
               "sharded_engine_cycles": st["fed_sharded"], "roofline": roofline_of(st, a, c, streaming=True)}
        if st["launches"][runtime.KERNELS.index("fed_engine_kernel")]:
            out["engine"] = engine_of(st, a)
        else:  # (a cycle the engine does not serve: the per-job launch path with the host-staged exchange)
            out["exchange_us_per_segment"] = exchange_us(st)
        return out
    except Exception as e:  # the side measurement never takes the main line down
        return {"error": repr(e)[:300]}


EVAL_SPECS, EVAL_NODES = 256, 50000
EVAL_OUT_BYTES = 8  # kb_eval32: u32 reason mask + i32 score per (spec, node)


def eval_side(device):
    """The fit/score sweep on its own (kb_eval): reasons + scores of EVAL_SPECS specs x
    EVAL_NODES nodes (a C2-shaped table, one spec per job), through kb_eval32. HIP events around the kernel;
    algorithmic bytes = the output (4 B reason mask + 4 B score per pair) + one read of every node row (76 B),
    the least HBM traffic the sweep needs. Measured HBM bytes come from the committed rocprofv3 PMC pass."""
    from scheduler_amd import runtime, synth
    try:
        snap = synth.c2_snapshot(n_nodes=EVAL_NODES, n_jobs=EVAL_SPECS, tasks_per_job=1, seed=synth.SEED)
        ctx = runtime.Context(device, timing=True)
        ctx.upload(snap)
        ids = (np.arange(EVAL_SPECS) % len(snap.spec_arr)).astype(np.int32)  # (equal requests share a spec)
        ctx.eval32(ids)  # warm-up
        ctx.stats(reset=True)
        for _ in range(5):
            ctx.eval32(ids)
        st = ctx.stats()
        ctx.close()
        k = runtime.KERNELS.index("eval_kernel")
        us = st["kernel_ms"][k] * 1e3 / max(1, st["launches"][k])
        pairs = len(ids) * EVAL_NODES
        alg = pairs * EVAL_OUT_BYTES + EVAL_NODES * 76
        # (a batch of plain specs, as here, runs eval_plain_kernel: DESIGN.md §4)
        kname = "eval_plain_kernel" if snap_plain(snap, ids) else "eval_kernel"
        out = {"kernel": kname, "bound": "hbm", "specs": len(ids), "nodes": EVAL_NODES,
               "avg_launch_us": round(us, 3), "algorithmic_bytes_per_launch": alg,
               "achieved": round(alg / (us * 1e-6) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
               "frac": round(alg / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "traffic": None, "measured_frac": None}
        tr = pmc_traffic(kname, "C2")  # the C2 PMC pass carries this side measurement
        if tr is not None:
            out["traffic"], out["traffic_source"] = tr["bytes_per_launch"], tr["source"]
            out["measured_frac"] = round(tr["bytes_per_launch"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
        return out
    except Exception as e:
        return {"error": repr(e)[:300]}


def snap_plain(snap, ids):
    """Every spec of the batch is plain (kb_ctx::spec_plain in kbgpu_host.cpp)."""
    from scheduler_amd import export as E
    a = snap.spec_arr[np.asarray(ids)]
    bad = (E.SPEC_HAS_SELECTOR | E.SPEC_HAS_REQUIRED | E.SPEC_INIT_HAS_MAP | E.SPEC_NA_ERROR | E.SPEC_POD_AFFINITY |
           E.SPEC_IPA_ERROR)
    lim = 1 << 49
    ok = (((a["flags"] & bad) == 0) & (a["pref_term_cnt"] == 0) & (a["port_cnt"] == 0) & (a["aff_class"] < 0) &
          (a["init_cpu"] >= 0) & (a["init_cpu"] < lim) & (a["init_mem"] >= 0) & (a["init_mem"] < lim) &
          (a["nz_cpu"] >= 0) & (a["nz_cpu"] < lim) & (a["nz_mem"] >= 0) & (a["nz_mem"] < lim))
    return bool(ok.all()) and snap.tolerates.shape[1] == 1 and bool(snap.tolerates[:, 0].all())


def spawn_ranks(n):
    """`bench.py --gpus N` outside torchrun: run N ranks as `torch.distributed.run` children (one process per
    GPU, rendezvous on 127.0.0.1) and exit with their code. Nothing here has touched the GPU."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC pass of this configuration
    (profiles/*_<config>_prof_summary.json: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section), or
    None when none is committed."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_prof_summary.json")), reverse=True)
    for f in files:
        try:
            with open(f) as fh:
                e = json.load(fh)["kernels"].get(kernel, {})
        except (OSError, ValueError, KeyError):
            continue
        if "hbm_bytes_per_launch" in e:
            return {"bytes_per_launch": e["hbm_bytes_per_launch"], "source": os.path.relpath(f, ROOT)}
    return None


DIAG_PHASES = {
    "traj_place_kernel": ["argmax", "commit", "rereduce", "lmax", "prefetch_store", "loop", "fill"],
    "sel_place_kernel": ["key_load", "node_select", "node_setup", "e_sequences", "winners_order", "stop_commit",
                         "nofit_hist"],
    "fed_engine_kernel": ["key_load_patch", "node_select", "node_setup", "e_sequences", "winners_order",
                          "commit_publish_nofit", "wait_for_command"],
    "cls_place_kernel": ["prologue_rest", "minmax_keys_argmax", "commit", "rescan_counts", "prologue_loads",
                         "stop_flush", "hot_switches_x1000"],
    "aff_place_kernel": ["prologue", "live_loads_minmax", "keys_argmax", "commit", "table_incr_fence", "stop_flush",
                         "nofit_hist"],
}


def diag_summary(d, tasks, kernel):
    """Per-task shader cycles of each place-kernel phase (KB_DIAG builds) and the implied clock."""
    names = DIAG_PHASES.get(kernel, [f"phase{i}" for i in range(7)])
    clock_mhz = d[7] and (sum(d[:7]) / (d[7] / 100.0))
    return {"cycles_per_task": {n: round(d[i] / max(1, tasks), 1) for i, n in enumerate(names)},
            "fill_cycles_total": d[6],
            "clock_mhz": round(clock_mhz, 1) if clock_mhz else None}


def cpu_baseline(cluster, sample_tasks, config):
    """The oracle (C++ restatement of the reference, ParallelizeUntil-style pool) on the first
    `sample_tasks` placements of the same workload."""
    from oracle import pyoracle
    cores = min(16, os.cpu_count() or 1)
    try:
        aff = len(os.sched_getaffinity(0))
        cores = min(cores, aff)
    except AttributeError:
        pass
    out = pyoracle.allocate(cluster, workers=cores, max_tasks=sample_tasks)
    placed = len(out["events"])
    secs = out["elapsed_ms"] / 1e3
    return {"value": round(placed / secs, 1) if secs > 0 else None, "unit": "pods/s", "cores": cores,
            "kind": "port", "sample": f"first {out['attempts']} task placements of the {config} cycle "
                                      f"({placed} placed in {secs:.2f} s, {cores} worker threads, "
                                      f"reference-structured full predicate+score sweep per task)"}


if __name__ == "__main__":
    sys.exit(main() or 0)
