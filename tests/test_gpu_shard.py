"""Node sharding across GPUs against one GPU holding the whole table.

Each rank holds a contiguous block of the canonical node table; per run segment the ranks exchange their
proposals (one all-gather) and commit their own rows. Here the ranks are processes sharing one GPU and the
exchange is host-staged over gloo; the RCCL exchange is exercised with a one-rank communicator. The bar
is identical placements, statuses and FitErrors histograms -- and, through test_gpu_parity, the oracle's.
"""
import os
import socket

import numpy as np
import pytest

from scheduler_amd import export as E
from scheduler_amd import runtime, synth

from helpers import parity_clusters

pytestmark = pytest.mark.gpu

NAMES = ["C1-parity", "C2-parity", "C2-fill0.9", "C3-parity", "C2-nogang", "edge-mixed"]


def _clusters():
    return {name: cl for name, cl in parity_clusters() if name in NAMES}


def _summary(out):
    n = int(out["n_events"])
    return {"task_node": out["task_node"].tolist(), "event_task": out["event_task"][:n].tolist(),
            "task_status": out["task_status"].tolist(), "job_fail_task": out["job_fail_task"].tolist(),
            "job_reason_hist": out["job_reason_hist"].tolist()}


def _rank_main(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)

    res = {}
    try:
        for name, cl in _clusters().items():
            snap = E.Snapshot(cl)
            ctx = runtime.Context(0)
            try:
                ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather)
                ctx.upload(snap)
                res[name] = _summary(ctx.allocate(snap))
            finally:
                ctx.close()
        q.put((rank, res, None))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_one_gpu(world):
    import torch.multiprocessing as mp
    ref = {}
    for name, cl in _clusters().items():
        snap = E.Snapshot(cl)
        ctx = runtime.Context(0)
        try:
            ctx.upload(snap)
            ref[name] = _summary(ctx.allocate(snap))
        finally:
            ctx.close()
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=240)
        assert err is None, f"rank {rank}: {err}"
        got[rank] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        for name in ref:
            assert got[r][name] == ref[name], (world, r, name)


def test_rccl_exchange_one_rank():
    """The RCCL path (ncclAllGather on the library stream) with a one-rank communicator, on C2 at 2k nodes."""
    snap = synth.c2_snapshot(n_nodes=2000, n_jobs=200, tasks_per_job=30, seed=13)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        ref = _summary(ctx.allocate(snap))
    finally:
        ctx.close()
    ctx = runtime.Context(0)
    try:
        ctx.set_shard(0, 1, snap.n_nodes, rccl_id=runtime.comm_unique_id())
        ctx.upload(snap)
        got = _summary(ctx.allocate(snap))
    finally:
        ctx.close()
    assert got == ref
