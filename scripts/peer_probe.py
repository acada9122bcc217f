"""Probe: the node-sharded fed engine (kb_set_shard_peer) with W ranks as processes sharing one GPU (gloo for the
one-time handle exchange): per-cycle times and the one-GPU comparison of a C2-shaped cycle.
Usage: python3 scripts/peer_probe.py W [nodes jobs tasks cycles]"""
import os
import socket
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def _rank(rank, world, port, shape, q):
    import torch
    import torch.distributed as dist
    from scheduler_amd import runtime, synth
    from test_gpu_shard import _summary
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)
    try:
        n, jobs, tasks, cycles = shape
        snap = synth.c2_snapshot(n_nodes=n, n_jobs=jobs, tasks_per_job=tasks, seed=21)
        ctx = runtime.Context(0)
        ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=True)
        ctx.upload(snap)
        ts, outs = [], []
        for _ in range(cycles):
            ctx.restore()
            dist.barrier()
            t0 = time.perf_counter()
            outs.append(_summary(ctx.allocate(snap)))
            ts.append(round((time.perf_counter() - t0) * 1e3, 1))
        st = ctx.stats()
        ctx.close()
        q.put((rank, ts, outs, st["fed_sharded"], None))
    except Exception as e:
        q.put((rank, None, None, None, repr(e)))
    finally:
        dist.destroy_process_group()


def main():
    import torch.multiprocessing as mp
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    shape = tuple(int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (2100 * world + 300, 40, 60, 2)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    procs = [ctxm.Process(target=_rank, args=(r, world, port, shape, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
    from scheduler_amd import runtime, synth
    from test_gpu_shard import _summary
    n, jobs, tasks, cycles = shape
    snap = synth.c2_snapshot(n_nodes=n, n_jobs=jobs, tasks_per_job=tasks, seed=21)
    ctx = runtime.Context(0)
    ctx.upload(snap)
    ref = _summary(ctx.allocate(snap))
    ctx.close()
    for rank, ts, outs, n_sh, err in sorted(res, key=lambda x: x[0]):
        same = err is None and all(o == ref for o in outs)
        print(f"rank {rank}/{world} shape {shape} plain_launch={os.environ.get('KB_FED_PLAIN_LAUNCH', '0')}: "
              f"cycle ms {ts} sharded_cycles {n_sh} equal_to_one_gpu {same} err {err}", flush=True)


if __name__ == "__main__":
    main()
