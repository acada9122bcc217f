"""Benchmark: kube-batch allocate cycles on MI355X (BASELINE.json metric).

metric : pods placed/sec (+ p50 allocate-cycle ms) at 10k nodes x 100k pods (BASELINE.json configs[1], "C2")
step   : one allocateAction.Execute (actions/allocate/allocate.go:42-193) over the C2 session snapshot:
         re-open the session from the snapshot already resident in HBM (kb_restore_nodes, device-to-device),
         then kb_allocate (host ordering plugins + the device's sweep / argmax / commit per job). The snapshot is
         uploaded once before the timed region; value = pods placed / second over the timed steps.

Multi-GPU (N > 1, one process per GPU): the SAME workload as N = 1 -- ONE C2 cluster (10k nodes x 100k pods) whose
node table is split into N contiguous blocks, one per rank (`scaling: "strong"`): every rank's resident engine
proposes its first T picks per job, writes them into every rank's inbox over xGMI (kb_set_shard_peer: device
memory mapped across the GPUs) and merges all proposals on the device -- no host round trip or collective launch
per job. `shard_exchange_us_per_job` is the engines' own stamp of the inbox wait per job. Beside the line:
"replicas" (every rank its own C2 cluster, no collective: weak scaling) and "sharded_C5" (BASELINE.json
configs[4]: 50k nodes x 1M pods split N ways). `--mode replicas` makes the replicas the line.
`python bench.py --gpus N` without torchrun's environment starts the N ranks itself (before any GPU call).

Extra JSON fields: roofline (the dominant kernel: the resident fed engine on C1/C2/C3/C5, the class loop on C4;
SURVEY.md §8 d3's bytes per (task, node) over its HIP-event duration, and the cycle's measured HBM bytes from the
committed rocprofv3 PMC pass), sweep_roofline (the per-job level-0 sweep, measured in a separate cycle), the
session open, eval_roofline (kb_eval at 256 specs x 50k nodes) and cpu_baseline (the oracle's C++ restatement of
the reference algorithm on a bounded sample).
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
    # not a BASELINE.json configuration: VERDICT r04's mixed cycle (C2 plus ~2% two-template jobs and ~2% jobs with
    # inter-pod anti-affinity), to hold against the C2 line per job
    "C2M": dict(nodes=10000, jobs=1000, tasks=100, row_bytes=80,
                workload="C2M: C2's 10k nodes x 100k pods with ~2% PS/worker (two-template) jobs and ~2% jobs with "
                         "required pod anti-affinity over hostname (a mixed cycle)"),
}
ARRAY_CONFIGS = ("C2", "C5")  # built by synth.c2_snapshot (numpy) instead of per-pod objects


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default=None, choices=sorted(CONFIGS),
                    help="BASELINE.json configuration (default: C2, the headline metric's, at every N)")
    ap.add_argument("--nodes", type=int, default=None)
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--tasks-per-job", type=int, default=None)
    ap.add_argument("--cpu-sample-tasks", type=int, default=3000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-timing", action="store_true", help="no per-kernel HIP events (roofline unavailable)")
    ap.add_argument("--path", default="select", choices=["select", "engine", "trajectory", "rekey"],
                    help="device path for the runs (scheduler_amd.runtime.PATHS)")
    ap.add_argument("--mode", default="auto", choices=["auto", "replicas", "shard"],
                    help="N>1: shard (auto) = ONE cluster of the configuration, its node table split across the ranks; "
                         "replicas = every rank schedules its own cluster (no collective)")
    ap.add_argument("--side-steps", type=int, default=5, help="cycles of each side measurement (N>1)")
    ap.add_argument("--no-side", action="store_true", help="N>1: no replicas / sharded-C5 side measurements")
    ap.add_argument("--no-eval", action="store_true", help="skip the kb_eval roofline measurement (N=1)")
    ap.add_argument("--timing-every", type=int, default=8,
                    help="per-job launch paths: HIP events around the launches of every Nth job call of the timed "
                         "region (fed-engine cycles time the engine's one launch per cycle only)")
    ap.add_argument("--opt", default="",
                    help="context options (runtime.make_opts: no_fed, fed_plain_launch, ...), for the profiler's "
                         "passes and the shared-GPU rehearsal; the default is the production path")
    ap.add_argument("--same-gpu", action="store_true",
                    help="N>1 rehearsal: every rank on GPU 0 (gloo group; engines launched plainly)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)  # torchrun's environment is missing: start the ranks (no GPU touched yet)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    args.mode = "shard" if args.mode == "auto" else args.mode
    args.config = args.config or "C2"
    cfg = CONFIGS[args.config]
    args.nodes = args.nodes or cfg["nodes"]
    args.jobs = args.jobs or cfg["jobs"]
    args.tasks_per_job = args.tasks_per_job or cfg["tasks"]
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # --same-gpu: rehearse N ranks on one GPU (gloo process group; plain engine launches: cooperative launches from
    # several processes take turns on one card; scripts/rehearse_multi.sh)
    from scheduler_amd import runtime as _rt
    args.options = _rt.parse_options(args.opt)
    if args.same_gpu and world > 1:
        args.options.setdefault("fed_plain_launch", True)
    device = 0 if args.same_gpu else local_rank
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        torch.cuda.set_device(device)
        dist_mod.init_process_group("nccl" if torch.cuda.is_available() and not args.same_gpu else "gloo")
        dist = dist_mod

    from scheduler_amd import runtime, synth

    shard = args.mode == "shard" and world > 1
    # replicas: each rank an independent cluster partition (different seed per rank); shard: one cluster
    seed = synth.SEED + (0 if shard else rank)
    snap, sess = session_snapshot(args, seed)

    exch = {"kind": "peer"}  # node-sharded: the device exchange, or the host-staged one if its pre-flight fails

    def make_ctx(every):
        def fresh():
            return runtime.Context(device, timing=not args.no_timing, timing_every=every, path=args.path,
                                   options=args.options)
        return sharded_context(fresh, dist, rank, world, device, snap.n_nodes, exch) if shard else fresh()

    # fed-engine cycles: the engine's one launch per cycle is timed (per-job sweep events would add barrier packets
    # on the sweep queue and host calls to every job); per-job launch paths: every Nth job's launches
    ctx = make_ctx(1 << 30)
    u0 = time.perf_counter()
    ctx.upload(snap)
    sess["upload_ms"] = round((time.perf_counter() - u0) * 1e3, 3)

    last = {}

    def step():  # (the result arrays of the previous cycle are reused, as a serving loop would)
        ctx.restore()
        last["out"] = ctx.allocate(snap, out=last.get("out"))
        return last["out"]

    def barrier():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()

    def warm():
        for _ in range(args.warmup):
            step()
    if shard and exch["kind"] == "peer" and args.warmup:
        # a cycle on the device exchange that fails on any rank (a peer that stops answering: the engines' idle
        # bound) moves every rank to the host-staged exchange before the timed region, and the line says so
        err = None
        try:
            warm()
        except runtime.KbError as e:
            err = str(e)[:300]
        if not all_ranks_ok(dist, device, err is None):
            exch.update(kind="host", peer_error=err or "a warm-up cycle on the peer exchange failed on another rank")
            ctx.close()
            ctx = make_ctx(1 << 30)
            ctx.upload(snap)
            warm()
    else:
        warm()
    if args.warmup and not ctx.stats()["fed_cycles"] and not args.no_timing and not shard:
        ctx.close()  # per-job launch paths: time every Nth job's launches
        ctx = make_ctx(args.timing_every)
        ctx.upload(snap)
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
    # where a step's host time goes (after the timed region): the session re-open and the kb_allocate call
    host = host_split(ctx, snap, out)
    # SURVEY.md §8 d1 also asks for the cycle WITH the snapshot upload: time re-uploads of the same snapshot
    # (kb_set_config + kb_upload_nodes + kb_upload_specs [+ affinity tables]; host arrays -> HBM), after the
    # timed region so they do not disturb it
    up = []
    if not shard:
        for _ in range(3):
            u0 = time.perf_counter()
            ctx.upload(snap)
            up.append((time.perf_counter() - u0) * 1e3)
        sess["upload_ms"] = round(statistics.median(up), 3)
    sess["total_ms"] = round(sess["build_ms"] + sess["upload_ms"], 3)
    ctx.close()

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
    side = {}
    if world == 1 and rank == 0 and not args.no_timing:
        side["sweep_roofline"] = sweep_side(args, cfg, snap, device)
    if world > 1 and not args.no_side:
        if shard:
            side["replicas"] = replicas_side(args, dist, rank, world, device)
            side["sharded_C5"] = shard_side(args, dist, rank, world, device)
        else:
            side["sharded"] = shard_side(args, dist, rank, world, device, config=args.config)
    if world == 1 and rank == 0 and not args.no_eval:
        side["eval_roofline"] = eval_side(device)

    roofline = roofline_of(st, args, cfg)
    engine = engine_of(st) if st["launches"][runtime.KERNELS.index("fed_engine_kernel")] else None

    workload = cfg["workload"]
    if (args.nodes, args.jobs, args.tasks_per_job) != (cfg["nodes"], cfg["jobs"], cfg["tasks"]):
        workload = f"{args.config} shape at {args.nodes} nodes x {args.jobs * args.tasks_per_job} pods"
    if shard:
        workload += f", node table split into {world} blocks (one per rank)"
    if rank == 0:
        ms = elapsed / args.steps * 1e3
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cl = synth.CONFIGS.get(args.config, synth.c2)(n_nodes=args.nodes, n_jobs=args.jobs,
                                                        tasks_per_job=args.tasks_per_job, seed=seed)
            cpu = cpu_baseline(cl, args.cpu_sample_tasks, args.config)
        result = {
            "metric": "pods placed/sec + p50 allocate-cycle ms at 10k nodes x 100k pods",
            "value": round(total_placed / elapsed, 1), "unit": "pods/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "p50_cycle_ms": round(statistics.median(times), 3),
            **({"upload_ms": round(statistics.median(up), 3),
                "p50_cycle_with_upload_ms": round(statistics.median(times) + statistics.median(up), 3)} if up else {}),
            "session_open": sess,
            "higher_is_better": True, "scaling": "strong" if shard else "weak", "vs_baseline": None,
            "dtype": "int64", "data": f"synthetic (seeded {args.config} generator, SURVEY.md §8 d2)",
            "config": {"workload": workload,
                       "nodes": args.nodes, "pods": args.jobs * args.tasks_per_job, "jobs": args.jobs,
                       "pods_placed_per_cycle": placed // max(1, args.steps),
                       "parallelism": f"node_shard{world}" if shard else f"replicas{world}"},
            "host_ms_per_step": host,
            "device_ms_per_step": round(st["device_ms"] / args.steps, 3),
            **({"diag_place_phases": diag_summary(st["diag"], placed, "fed_engine_kernel" if engine is not None
                                                  else roofline["kernel"])}
               if any(st["diag"]) else {}),
            "job_calls_per_step": st["job_calls"] / args.steps,
            "roofline": roofline,
            **({"engine": engine} if engine is not None else {}),
            "cpu_baseline": cpu,
            **({**shard_fields(st, args), "shard_exchange": exch} if shard else {}),
            **side,
        }
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def session_snapshot(args, seed):
    """The session snapshot of the configuration and its open cost: C2 / C5 from the numpy
    builder; C1 / C3 / C4 from the generator's columns (synth.COLUMNS: per node and per job, no per-pod objects --
    the Go shim's columnar walk) through columns.build. build_ms = the snapshot build; the upload
    is added once the context exists."""
    from scheduler_amd import synth
    if args.config in ARRAY_CONFIGS:  # the numpy session builder (equal to the exporter: test_export.py)
        e0 = time.perf_counter()
        snap = synth.c2_snapshot(n_nodes=args.nodes, n_jobs=args.jobs, tasks_per_job=args.tasks_per_job, seed=seed)
        return snap, {"build_ms": round((time.perf_counter() - e0) * 1e3, 1),
                      "build": "synth.c2_snapshot (numpy arrays, equal to export.Snapshot: tests/test_export.py)"}
    from scheduler_amd import columns
    cols = synth.COLUMNS[args.config](n_nodes=args.nodes, n_jobs=args.jobs, tasks_per_job=args.tasks_per_job,
                                      seed=seed)
    e0 = time.perf_counter()
    snap = columns.build(cols)
    return snap, {"build_ms": round((time.perf_counter() - e0) * 1e3, 1),
                  "build": "columns.build over the session's columns (vectorised per pod; equal to export.Snapshot "
                           "array by array: tests/test_columns.py); the columns come straight from the generator "
                           "(synth.COLUMNS, no per-pod walk)"}


def host_split(ctx, snap, out):
    """One more step after the timed region, split: kb_restore_nodes (the session re-open) and the kb_allocate call
    (its own elapsed time, and the Python binding around it)."""
    r0 = time.perf_counter()
    ctx.restore()
    r1 = time.perf_counter()
    o = ctx.allocate(snap)
    r2 = time.perf_counter()
    return {"restore": round((r1 - r0) * 1e3, 3), "allocate_call": round((r2 - r1) * 1e3, 3),
            "kb_allocate": round(float(o["elapsed_ms"]), 3)}


SWEEP_OUT_BYTES = 12  # the level-0 sweep's output per node: 4 B key + 8 B static cache
# kernels of the allocate cycle whose PMC bytes make up the cycle's traffic (not the eval side measurement, not the
# upload / restore copies)
CYCLE_KERNELS = ("sel_sweep_kernel", "sel_place_kernel", "fed_engine_kernel", "fed_cmd_sweep_kernel", "cls_sweep_kernel",
                 "cls_place_kernel", "aff_commit_kernel", "aff_place_kernel", "aff_reg_kernel", "ipa_minmax_kernel",
                 "traj_sweep_kernel", "traj_place_kernel", "sweep_keys_kernel", "place_loop_kernel",
                 "shard_propose_kernel", "shard_commit_kernel")


def roofline_of(st, args, cfg):
    """The roofline of the cycle's dominant kernel: the resident fed engine where it ran (one launch per cycle, the
    whole placement chain), else the kernel with the most HIP-event time (C4: the class loop, cls_place_kernel).
    achieved = SURVEY.md §8 d3's algorithmic bytes -- the row bytes of every (task, node) evaluation the launch
    stands for (76 B C1/C2/C5, 124 B C3, 88 B C4) -- over the launch's average HIP-event duration on the stream it
    runs on. The kernels read far fewer bytes than that (the selection reads each node's row once per job, not once
    per task): traffic = the HBM bytes the cycle moved per launch of the kernel, from this configuration's committed
    rocprofv3 PMC pass (every cycle kernel's FETCH_SIZE x 2 + WRITE_SIZE per dispatch x its dispatches per cycle;
    MI355X_MICROARCH.md's gfx950 correction), and measured_frac = traffic / duration / peak."""
    from scheduler_amd import runtime
    K = runtime.KERNELS
    fed = st["launches"][K.index("fed_engine_kernel")] > 0
    if fed:
        k = K.index("fed_engine_kernel")
    else:
        kern_ms = [0.0 if K[i] in ("shard_exchange",) else v for i, v in enumerate(st["kernel_ms"])]
        k = int(np.argmax(kern_ms)) if any(kern_ms) else 0
    launches = max(1, st["launches"][k])
    avg_ms = st["kernel_ms"][k] / launches
    bytes_per_launch = st["pairs"][k] * cfg["row_bytes"] / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    out = {"bound": "hbm", "kernel": K[k], "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None, "traffic_source": None,
           "avg_launch_us": round(avg_ms * 1e3, 3), "timed_launches": st["launches"][k],
           "timing": ("HIP events on the library stream around the engine's one launch per cycle, every cycle of the "
                      "timed region" if fed else
                      f"HIP events on the library stream around every launch of every {args.timing_every}th job call "
                      f"in the timed region"),
           "algorithmic_bytes_per_launch": round(bytes_per_launch, 1),
           "algorithmic_bytes_note": (f"SURVEY.md §8 d3: {cfg['row_bytes']} B of node row per (task, node) "
                                      f"evaluation x the (task, node) pairs the launch decides "
                                      f"({st['pairs'][k] / launches:.4g}); the kernel itself reads each row once per "
                                      f"job at most (see traffic)"),
           "avg_us_per_launch": {K[i]: round(st["kernel_ms"][i] * 1e3 / st["launches"][i], 3)
                                 for i in range(len(K)) if st["launches"][i]},
           "measured_frac": None,
           "frac_meaning": ("definitional, not bandwidth: SURVEY.md §8 d3's row bytes of every (task, node) "
                            "evaluation the launch decides, over its duration; the kernel reads each row at most once "
                            "per job (the selection's algorithmic saving, DESIGN.md §3), so frac counts avoided work and "
                            "can exceed 1 (C5). The bandwidth figure is measured_frac (traffic / duration / peak)")}
    full = (args.nodes, args.jobs, args.tasks_per_job) == (cfg["nodes"], cfg["jobs"], cfg["tasks"])
    tr = pmc_cycle_traffic(args.config, K[k]) if full and args.gpus == 1 else None
    if tr is not None:
        out["traffic"] = tr["bytes_per_launch"]
        out["traffic_source"] = tr["source"]
        out["traffic_is_proxy"] = tr.get("proxy", fed)
        out["cycle_traffic_bytes"] = tr["cycle_bytes"]
        if avg_ms > 0:
            out["measured_frac"] = round(tr["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 6)
    return out


def engine_of(st):
    """The resident fed engine (one launch per allocate cycle): its per-job time and the shader clock over its
    launches (kb_stats fed_clock_ticks / fed_real_ticks: s_memtime against the 100 MHz s_memrealtime)."""
    from scheduler_amd import runtime
    K = runtime.KERNELS
    k = K.index("fed_engine_kernel")
    launches = max(1, st["launches"][k])
    us = st["kernel_ms"][k] * 1e3 / launches
    jobs = st["job_calls"] / launches
    clk = 100.0 * st["fed_clock_ticks"] / st["fed_real_ticks"] if st["fed_real_ticks"] else None
    place = [{"xcc": int(v) >> 32, "se": (int(v) >> 13) & 7, "cu": (int(v) >> 8) & 15} if v else None
             for v in st.get("fed_wg_place", [0, 0])]
    return {"kernel": "fed_engine_kernel", "bound": "latency (per-job dependent chain in one workgroup)",
            "avg_launch_us": round(us, 3), "launches": st["launches"][k], "jobs_per_launch": round(jobs, 1),
            "us_per_job": round(us / max(1.0, jobs), 3), "clock_mhz": round(clk, 1) if clk else None,
            "placement": {"placer": place[0], "selector": place[1]},
            "depth": st["fed_last_depth"], "sweepers": st["fed_last_sweepers"],
            "mispredicts_per_step": round(st["fed_mispredicts"] / launches, 2),
            "skipped_per_step": round(st["fed_skipped"] / launches, 2),
            "nofit_predicted_per_step": round(st["nofit_predicted"] / launches, 2),
            "units_per_step": round(st["fed_units"] / launches, 1)}


def shard_fields(st, args):
    """Node-sharded line: the engines' own stamp of the exchange (the placer's wait from writing its record into
    the peers' inboxes to holding every peer's record) per job, and the launch-path exchanges if any."""
    from scheduler_amd import runtime
    out = {"sharded_engine_cycles_per_step": st["fed_sharded"] / args.steps,
           "shard_exchange_us_per_job": (round(st["shard_wait_ticks"] / 100.0 / st["shard_xchg"], 3)
                                         if st["shard_xchg"] else None),
           "shard_exchanges_per_step": st["shard_xchg"] / args.steps}
    ph = st.get("shard_phase_ticks")
    if ph is not None and st["shard_xchg"]:  # the placer's s_memrealtime per phase of a sharded job (kb_stats)
        names = ("proposal", "xgmi_write", "peer_wait", "merge_stop_rules", "commit", "nofit_round")
        out["shard_phase_us_per_job"] = {nm: round(float(ph[i]) / 100.0 / st["shard_xchg"], 3)
                                         for i, nm in enumerate(names)}
    k = runtime.KERNELS.index("shard_exchange")
    if st["launches"][k]:
        out["launch_path_exchange_us_per_segment"] = round(st["kernel_ms"][k] * 1e3 / st["launches"][k], 2)
    return out


def sweep_side(args, cfg, snap, device):
    """The per-job level-0 sweep on its own (sel_sweep_kernel: every node's row read and its 32-bit key and static
    cache written once per job), from one more cycle with HIP events around every job's sweep (kept out of the
    timed region: the events add barrier packets to the sweep queue). Algorithmic bytes n x (row + 12 B)."""
    from scheduler_amd import runtime
    try:
        ctx = runtime.Context(device, timing=True, timing_every=1, path=args.path, options=args.options)
        ctx.upload(snap)
        ctx.allocate(snap)
        ctx.restore()
        ctx.stats(reset=True)
        ctx.allocate(snap)
        st = ctx.stats()
        ctx.close()
        K = runtime.KERNELS
        k = K.index("sel_sweep_kernel")
        if not st["launches"][k]:
            return None
        avg_ms = st["kernel_ms"][k] / st["launches"][k]
        alg = st["pairs"][k] / st["launches"][k] * (cfg["row_bytes"] + SWEEP_OUT_BYTES)
        out = {"kernel": "sel_sweep_kernel", "avg_launch_us": round(avg_ms * 1e3, 3), "launches": st["launches"][k],
               "algorithmic_bytes_per_launch": round(alg, 1), "achieved": round(alg / (avg_ms * 1e-3) / 1e9, 2),
               "frac": round(alg / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5), "traffic": None, "measured_frac": None}
        tr = pmc_traffic("sel_sweep_kernel", args.config)
        if tr is not None:
            out["traffic"], out["traffic_source"] = tr["bytes_per_launch"], tr["source"]
            out["measured_frac"] = round(tr["bytes_per_launch"] / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
        return out
    except Exception as e:  # the side measurement never takes the main line down
        return {"error": repr(e)[:300]}


def tensor_device(dist, device):
    return "cpu" if dist is not None and dist.get_backend() == "gloo" else f"cuda:{device}"


def sharded_context(fresh, dist, rank, world, device, n_total, exch):
    """A node-sharded context (this rank's block of n_total nodes) on the engines' device exchange
    (kb_set_shard_peer). If a peer mapping or the pre-flight round trip fails on any rank, every rank takes the
    host-staged exchange (kb_set_shard) instead and `exch` records why -- the line still measures the sharded cycle
    rather than ending the run. exch["kind"] == "host" on entry skips the peer attempt."""
    from scheduler_amd import runtime
    c = fresh()
    kw = shard_exchange(dist, rank, device)
    if exch.get("kind", "peer") == "peer":
        err = None
        try:
            c.set_shard(rank, world, n_total, **kw)
        except runtime.KbError as e:  # (the pre-flight's outcome is all-gathered: every rank fails alike)
            err = str(e)[:300]
        if all_ranks_ok(dist, device, err is None):
            exch["kind"] = "peer"
            return c
        exch.update(kind="host", peer_error=err or "the peer pre-flight failed on another rank")
        c.close()
        c = fresh()
    c.set_shard(rank, world, n_total, **{**kw, "peer": False})
    return c


def all_ranks_ok(dist, device, ok):
    """True on every rank iff `ok` holds on every rank (one MIN all-reduce over the process group)."""
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=tensor_device(dist, device))
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


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


def replicas_side(args, dist, rank, world, device):
    """Beside the sharded line: every rank schedules its own independent C2 cluster (different seed per rank,
    no collective), `side_steps` cycles; pods/s over all ranks at the max-over-ranks time (weak scaling)."""
    import torch
    from scheduler_amd import runtime, synth
    try:
        c = CONFIGS["C2"]
        snap = synth.c2_snapshot(n_nodes=c["nodes"], n_jobs=c["jobs"], tasks_per_job=c["tasks"], seed=synth.SEED + rank)
        ctx = runtime.Context(device, options=args.options)
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


def shard_side(args, dist, rank, world, device, config="C5"):
    """Beside the line (N > 1): a node-sharded cycle of `config` -- by default BASELINE.json configs[4], C5: ONE
    cluster of 50k C2-shaped nodes x 1M pods whose node table is split across the N ranks (contiguous blocks; per
    job every rank's engine proposes, writes its proposal into every rank's inbox over xGMI and merges all of them;
    every rank commits its own rows). `side_steps` cycles after one warm-up; pods/s at the max-over-ranks time."""
    import torch
    from scheduler_amd import runtime, synth
    try:
        c = CONFIGS[config]
        snap = synth.c2_snapshot(n_nodes=c["nodes"], n_jobs=c["jobs"], tasks_per_job=c["tasks"], seed=synth.SEED)
        exch = {"kind": "peer"}
        ctx = sharded_context(lambda: runtime.Context(device, timing=True, timing_every=1 << 30, options=args.options),
                              dist, rank, world, device, snap.n_nodes, exch)
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
        a.config, a.nodes, a.jobs, a.tasks_per_job, a.steps = config, c["nodes"], c["jobs"], c["tasks"], args.side_steps
        elapsed = float(el.item())
        out = {"workload": c["workload"] + f", node table split into {world} blocks",
               "value": round(placed * args.side_steps / elapsed, 1), "unit": "pods/s",
               "steps": args.side_steps, "scaling": "strong", "ms_per_step": round(elapsed / args.side_steps * 1e3, 3),
               "roofline": roofline_of(st, a, c), **shard_fields(st, a), "shard_exchange": exch}
        if st["launches"][runtime.KERNELS.index("fed_engine_kernel")]:
            out["engine"] = engine_of(st)
        return out
    except Exception as e:  # the side measurement never takes the main line down
        return {"error": repr(e)[:300]}


EVAL_SPECS, EVAL_NODES = 256, 50000
EVAL_OUT_BYTES = 8  # kb_eval32: u32 reason mask + i32 score per (spec, node)


EVAL_WARMUP, EVAL_TIMED = 200, 200


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
        # warm-up long enough for the card's power management to leave the idle memory / clock state the allocate
        # cycles left it in (a few launches after the cycles ran 47 us against 33-36 us in a process that ran
        # kb_eval only: DESIGN.md §4), then the timed launches
        for _ in range(EVAL_WARMUP):
            ctx.eval32(ids)
        ctx.stats(reset=True)
        for _ in range(EVAL_TIMED):
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


def _prof_summaries(config):
    import glob
    return sorted(glob.glob(os.path.join(ROOT, "profiles", f"*_{config}_prof_summary.json")), reverse=True)


def pmc_traffic(kernel, config):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC pass of this configuration
    (profiles/*_<config>_prof_summary.json: FETCH_SIZE x2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section), or
    None when none is committed."""
    for f in _prof_summaries(config):
        try:
            with open(f) as fh:
                e = json.load(fh)["kernels"].get(kernel, {})
        except (OSError, ValueError, KeyError):
            continue
        if "hbm_bytes_per_launch" in e:
            return {"bytes_per_launch": e["hbm_bytes_per_launch"], "source": os.path.relpath(f, ROOT)}
    return None


def pmc_cycle_traffic(config, kernel):
    """The allocate cycle's measured HBM bytes from the newest committed PMC pass of this configuration that counts
    dispatches (scripts/prof_summary.py: every cycle kernel's bytes per dispatch x its dispatches, over the pass's
    cycles), expressed per launch of `kernel`: the whole cycle for the fed engine (one launch per cycle), else
    `kernel`'s own bytes per launch. The fed engine's pass runs the per-job launch path (option no_fed: counter
    collection serialises dispatches, and the resident engine waits on sweeps of another stream), whose kernels
    read and write what the engine's jobs do."""
    for f in _prof_summaries(config):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):
            continue
        ks, cycles = d.get("kernels", {}), d.get("pmc_cycles")
        if not cycles or not any("pmc_dispatches" in e for e in ks.values()):
            continue
        cyc = sum(e["hbm_bytes_per_launch"] * e["pmc_dispatches"] for k, e in ks.items()
                  if k in CYCLE_KERNELS and "hbm_bytes_per_launch" in e and "pmc_dispatches" in e) / cycles
        src = os.path.relpath(f, ROOT)
        fe = ks.get("fed_engine_kernel", {})
        if kernel == "fed_engine_kernel" and "hbm_bytes_per_launch" in fe:
            # round 5: the engine's own counters (its resident sweepers take the commands from a pinned ring, so
            # the profiler's dispatch serialisation has no other-stream sweep to stall: scripts/profile_round.sh
            # FEDPMC=1) -- one dispatch per cycle
            return {"bytes_per_launch": fe["hbm_bytes_per_launch"], "cycle_bytes": round(cyc, 1), "proxy": False,
                    "source": f"{src}: the engine's own PMC counts (FETCH_SIZE x2 + WRITE_SIZE), one dispatch per "
                              f"cycle"}
        if kernel == "fed_engine_kernel":
            return {"bytes_per_launch": round(cyc, 1), "cycle_bytes": round(cyc, 1),
                    "source": f"PROXY, not the engine's own counters: {src}: the same cycle on the per-job launch path "
                              f"(option no_fed; counter collection serialises dispatches, so the resident engine cannot "
                              f"be fed under it), every cycle kernel's bytes per dispatch x dispatches per cycle, summed "
                              f"= one engine launch"}
        e = ks.get(kernel, {})
        if "hbm_bytes_per_launch" in e:
            return {"bytes_per_launch": e["hbm_bytes_per_launch"], "cycle_bytes": round(cyc, 1),
                    "source": f"{src}: {kernel}'s own bytes per launch"}
    return None


DIAG_PHASES = {
    "traj_place_kernel": ["argmax", "commit", "rereduce", "lmax", "prefetch_store", "loop", "fill"],
    "sel_place_kernel": ["key_load", "node_select", "node_setup", "e_sequences", "winners_order", "stop_commit",
                         "nofit_hist"],
    "fed_engine_kernel": ["key_load_patch", "node_select", "node_setup", "e_sequences", "winners_order",
                          "commit_publish_nofit", "wait_for_command"],
    "cls_place_kernel": ["prologue", "per_task_path", "phase_setup", "phase_rounds", "phase_picks",
                         "phase_deep_keys_writeback", "counts_picks_1e6rounds_1e12deep"],
    "aff_place_kernel": ["prologue", "live_loads_minmax", "keys_argmax", "commit", "table_incr_fence", "stop_flush",
                         "nofit_hist"],
}


def diag_summary(d, tasks, kernel):
    """Per-task shader cycles of each place-kernel phase (KB_DIAG builds) and the implied clock."""
    names = DIAG_PHASES.get(kernel, [f"phase{i}" for i in range(7)])
    clock_mhz = d[7] and (sum(d[:7]) / (d[7] / 100.0))
    return {"cycles_per_task": {n: round(d[i] / max(1, tasks), 1) for i, n in enumerate(names)}, "totals": list(d),
            "fill_cycles_total": d[6],
            "clock_mhz": round(clock_mhz, 1) if clock_mhz else None}


def cgroup_cpus():
    """CPUs granted by the cgroup's CPU quota (cgroup v2 cpu.max, else v1 cfs quota / period), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0 and per > 0:
            return max(1, -(-q // per))
    except (OSError, ValueError):
        pass
    return None


def cpu_baseline(cluster, sample_tasks, config):
    """The oracle (C++ restatement of the reference, ParallelizeUntil-style pool) on the first `sample_tasks`
    placements of the same workload: 16 workers (the reference's ParallelizeUntil(..., 16, ...)), and beside it the
    same sample on every core this process may run on ("Also report an all-cores run")."""
    from oracle import pyoracle
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    # the cores this process may actually use: its affinity, capped by the cgroup's CPU quota (the GPU box shows all
    # 256 CPUs of the host but grants 16; 256 workers there thrashed: 80 pods/s against 2,280 on 16, r05j)
    quota = cgroup_cpus()
    if not quota and os.environ.get("OMP_NUM_THREADS", "").isdigit():
        quota = int(os.environ["OMP_NUM_THREADS"])  # (the pool's stated CPU share when no cgroup quota is visible)
    avail = min(affinity, quota) if quota else affinity
    label = "CPU restatement of the reference algorithm (oracle/oracle.cpp), not the Go reference"

    def run(workers):
        out = pyoracle.allocate(cluster, workers=workers, max_tasks=sample_tasks)
        placed = len(out["events"])
        secs = out["elapsed_ms"] / 1e3
        return out, placed, secs

    cores = min(16, avail)
    out, placed, secs = run(cores)
    res = {"value": round(placed / secs, 1) if secs > 0 else None, "unit": "pods/s", "cores": cores,
           "kind": "port", "label": label,
           "sample": f"first {out['attempts']} task placements of the {config} cycle "
                     f"({placed} placed in {secs:.2f} s, {cores} worker threads, "
                     f"reference-structured full predicate+score sweep per task)",
           "host": {"nproc_visible": os.cpu_count(), "affinity_cpus": affinity, "cgroup_cpu_quota": quota}}
    if avail > cores:
        out2, placed2, secs2 = run(avail)
        res["all_cores"] = {"value": round(placed2 / secs2, 1) if secs2 > 0 else None, "unit": "pods/s",
                            "cores": avail, "sample": f"the same {out2['attempts']} placements on {avail} worker "
                                                      f"threads ({secs2:.2f} s)"}
    else:
        res["all_cores"] = {"value": res["value"], "cores": cores,
                            "sample": f"this process may run on no more than the {cores} cores above (affinity "
                                      f"{affinity}, cgroup quota {quota})"}
    return res


if __name__ == "__main__":
    sys.exit(main() or 0)
