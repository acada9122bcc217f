"""The node-sharded engine across consecutive contexts of one process: allocate cycles on W ranks
sharing one GPU, peer exchange, every fed job issue / finish traced per rank (KB_HOST_TRACE) into
gpurun_out/<tag>_rank<r>.err. Cases: one parity cluster, "all" (the sharded parity test's sequence, repeated),
"fresh" (each context in processes of its own), "big" (C2-shaped clusters of 4k+ nodes). Usage: scripts/shard_small_probe.py <tag> [world] [case]"""
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def rank_main(rank, world, port, tag, case):
    os.environ["KB_HOST_TRACE"] = "1"
    fd = os.open(os.path.join(ROOT, "gpurun_out", f"{tag}_rank{rank}.err"), os.O_WRONLY | os.O_CREAT | os.O_TRUNC)
    os.dup2(fd, 2)
    import torch
    import torch.distributed as dist
    from scheduler_amd import export as E, runtime
    from helpers import backfill_cluster, parity_clusters
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)
    names = ["C1-parity", "C2-parity", "C2-fill0.9", "C3-parity", "C2-nogang", "edge-mixed"]
    if case == "all":  # the sharded parity test's sequence of contexts, repeated
        cases = [n for _ in range(int(os.environ.get("PROBE_REPEAT", "3"))) for n in names + ["backfill"]]
    else:
        cases = [case]
    if case == "big":  # C2-shaped clusters (1.3k+ nodes per rank), several contexts per process
        cases = [f"c2big{i}" for i in range(int(os.environ.get("PROBE_REPEAT", "8")))]
    pcs = dict(parity_clusters())
    from scheduler_amd import synth
    for i in range(16):
        pcs[f"c2big{i}"] = None
    bad = 0
    for name in cases:
        if name.startswith("c2big"):
            k = int(name[5:])
            snap = synth.c2_snapshot(n_nodes=4000 + 300 * k, n_jobs=60, tasks_per_job=40 + k, seed=30 + k,
                                     fill=0.9 if k % 3 == 2 else None)
        else:
            snap = E.Snapshot(backfill_cluster() if name == "backfill" else pcs[name])
        ctx = runtime.Context(0, options={"fed_plain_launch": True})
        try:
            ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=True)
            ctx.upload(snap)
            out = ctx.allocate(snap)
            print(f"rank {rank} {name}: ok n_events={out['n_events']} fed_sharded={ctx.stats()['fed_sharded']}",
                  flush=True)
        except Exception as e:
            bad += 1
            print(f"rank {rank} {name}: {e!r}", flush=True)
        finally:
            ctx.close()
        if bad:
            break
    dist.destroy_process_group()


if __name__ == "__main__":
    import torch.multiprocessing as mp
    tag = sys.argv[1] if len(sys.argv) > 1 else "ssp"
    world = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    case = sys.argv[3] if len(sys.argv) > 3 else "backfill"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctxm = mp.get_context("spawn")
    if case == "fresh":  # every context in processes of its own (no earlier context in the process)
        names = ["C1-parity", "C2-parity", "C2-fill0.9", "C3-parity", "C2-nogang", "edge-mixed", "backfill"]
        runs = [n for _ in range(int(os.environ.get("PROBE_REPEAT", "3"))) for n in names]
    else:
        runs = [case]
    for i, name in enumerate(runs):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        procs = [ctxm.Process(target=rank_main, args=(r, world, port, f"{tag}_{i}" if case == "fresh" else tag, name))
                 for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=120)
    sys.exit(0)
