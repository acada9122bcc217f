"""The node-sharded fed engine (kb_set_shard_peer): every rank's resident engine proposes its first T picks,
writes them into every rank's inbox (device memory mapped across the ranks through IPC handles) and merges all of
them on the device -- no host round trip and no collective launch per job. Parity bar: the placements, statuses
and FitErrors of one unsharded GPU context on the same snapshot (itself oracle- and digest-checked), cycle after
cycle (the engine's tags carry the cycle number). Multi-rank runs are processes sharing the one GPU of the box."""
import os
import socket
import time

import numpy as np
import pytest

from scheduler_amd import runtime, synth

from test_gpu_shard import _summary

pytestmark = pytest.mark.gpu


def _cases(world):
    """Fed-eligible cycles (one <= 100-task run per job): full gangs, half gangs whose jobs are popped again, a cycle
    that runs out of room (NO_FIT), blocks of fewer nodes than one key group."""
    n = 2100 * world + 300
    half = synth.c2_snapshot(n_nodes=n, n_jobs=90, tasks_per_job=40, seed=23)
    half.s_job_min = np.full_like(half.s_job_min, 20)  # ready at half the job: popped again for the rest
    return {
        "c2-gang": synth.c2_snapshot(n_nodes=n, n_jobs=120, tasks_per_job=60, seed=21),
        "c2-nofit": synth.c2_snapshot(n_nodes=n, n_jobs=60, tasks_per_job=100, seed=22, fill=2.5),
        "c2-halfgang": half,
        # every rank's block under one key group (2048 nodes): the sharded engine's two-group instance (8 ranks
        # split C2's 10k nodes into 1,250-node blocks)
        "c2-small": synth.c2_snapshot(n_nodes=1200 * world + 100, n_jobs=50, tasks_per_job=50, seed=24),
    }


def _reference(snap, cycles):
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out = []
        for _ in range(cycles):
            ctx.restore()
            out.append(_summary(ctx.allocate(snap)))
        return out
    finally:
        ctx.close()


def _sharded(snap, rank, world, allgather, cycles, barrier=None, options=None):
    ctx = runtime.Context(0, options=options)
    try:
        ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=True)
        ctx.upload(snap)
        out = []
        for c in range(cycles):
            ctx.restore()
            if barrier is not None:
                barrier()
            t0 = time.perf_counter()
            out.append(_summary(ctx.allocate(snap)))
            print(f"rank {rank}/{world} cycle {c}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
        return out, ctx.stats()
    finally:
        ctx.close()


def test_peer_engine_one_rank():
    """world 1: the sharded engine's exchange through its own inbox; three cycles (the tags' cycle halves)."""
    for name, snap in _cases(1).items():
        print(f"one rank: {name}", flush=True)
        ref = _reference(snap, 3)
        got, st = _sharded(snap, 0, 1, lambda b: b, 3)
        assert st["fed_sharded"] == 3 and st["fed_abandon"] == 0, (name, st)
        assert got == ref, name


def _rank_main(rank, world, port, q, cycles=2, options=None, names=None):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    # (the engine is a plain launch since ABI 14; fed_plain_launch stays accepted)
    options = dict(options or {})
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)

    res = {}
    try:
        for name, snap in _cases(world).items():
            if names is not None and name not in names:
                continue
            print(f"rank {rank}/{world}: {name}", flush=True)
            got, st = _sharded(snap, rank, world, allgather, cycles, barrier=dist.barrier, options=options)
            res[name] = (got, st["fed_sharded"], st["fed_abandon"], st["shard_rezero"], st["peer_checks"])
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
def test_peer_engine_ranks_equal_one_gpu(world):
    """2 and 3 ranks (processes on the one GPU, inboxes IPC-mapped between them): every rank reports the one-GPU
    outcome, two cycles each, and every cycle ran on the sharded engine."""
    import torch.multiprocessing as mp
    ref = {name: _reference(snap, 2) for name, snap in _cases(world).items()}
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            assert err is None, f"rank {rank}: {err}"
            got[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
    for r in range(world):
        for name in ref:
            out, n_sharded, n_abandon, _, n_checks = got[r][name]
            assert n_sharded == 2 and n_abandon == 0, (world, r, name)
            # the pre-flight: a hello and an answer from every peer arrived intact
            assert n_checks == 2 * (world - 1), (world, r, name, n_checks)
            assert out == ref[name], (world, r, name)


EPOCH_WRAP = 1 << 12  # kShardEpochBits of the cycle epoch in an inbox word's tag (kbgpu_device.h)


def test_peer_engine_one_rank_epoch_wrap():
    """The inbox tags keep 12 bits of the cycle epoch, so every 4096 cycles the ranks re-zero their inboxes between
    two host barriers (a word an earlier cycle left -- a no-fit histogram, a longer record -- must never read as
    current). One rank started just below the wrap: four cycles across it, every one a NO_FIT cycle, equal to one
    unsharded GPU, with exactly one re-zeroing."""
    snap = _cases(1)["c2-nofit"]
    ref = _reference(snap, 4)
    got, st = _sharded(snap, 0, 1, lambda b: b, 4, options={"shard_epoch0": EPOCH_WRAP - 2})
    assert st["fed_sharded"] == 4 and st["fed_abandon"] == 0 and st["shard_rezero"] == 1, st
    assert got == ref


def test_peer_engine_two_ranks_epoch_wrap():
    """Two ranks across the epoch wrap (the re-zeroing's two barriers run through the all-gather callback)."""
    import torch.multiprocessing as mp
    world, cycles = 2, 4
    ref = {name: _reference(snap, cycles) for name, snap in _cases(world).items() if name == "c2-nofit"}
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_rank_main, args=(r, world, port, q, cycles, {"shard_epoch0": EPOCH_WRAP - 2},
                                                   ["c2-nofit"])) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            assert err is None, f"rank {rank}: {err}"
            got[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
    for r in range(world):
        out, n_sharded, n_abandon, n_rezero, _ = got[r]["c2-nofit"]
        assert n_sharded == cycles and n_abandon == 0 and n_rezero == 1, (r, n_sharded, n_abandon, n_rezero)
        assert out == ref["c2-nofit"], r


def _badtag_main(rank, world, port, q, bad_rank):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)
    try:
        ctx = runtime.Context(0, options={"test_peer_badtag": rank == bad_rank})
        try:
            ctx.set_shard(rank, world, 4000, allgather=allgather, peer=True)
            q.put((rank, None))
        except runtime.KbError as e:
            q.put((rank, (e.code, str(e))))
        finally:
            ctx.close()
    except Exception as e:
        q.put((rank, (-1, repr(e))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_peer_preflight_fails_loudly(world):
    """kb_set_shard_peer's pre-flight round trip: when one rank's words arrive wrong (forced here: rank 1 stores a
    bad tag), EVERY rank's kb_set_shard_peer fails with KB_E_STATE naming the rank pair -- before any cycle, instead
    of a 10 s engine timeout in the first one."""
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_badtag_main, args=(r, world, port, q, 1)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, err = q.get(timeout=120)
            got[rank] = err
    finally:
        for p in procs:
            p.join(timeout=60)
    for r in range(world):
        assert got[r] is not None, f"rank {r} passed the pre-flight"
        code, msg = got[r]
        assert code == runtime.KB_E_STATE and "pre-flight" in msg and "from rank 1" in msg, (r, msg)


def _mixed_rank_main(rank, world, port, q, cluster, options=None):
    import torch
    import torch.distributed as dist
    from scheduler_amd import export as E
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)
    try:
        snap = E.Snapshot(cluster)
        ctx = runtime.Context(0, options=options)
        try:
            ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=True)
            ctx.upload(snap)
            out = []
            for _ in range(2):
                ctx.restore()
                dist.barrier()
                r = runtime.result_dict(snap, ctx.allocate(snap))
                out.append({k: r[k] for k in ("events", "binds", "fit_errors")})
            st = ctx.stats()
        finally:
            ctx.close()
        q.put((rank, (out, st["fed_sharded"], st["fed_pauses"], st["off_engine_units"], st["fed_abandon"],
                      st["fed_aff_units"]), None))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("aff_path", ["engine", "pause"])
def test_peer_engine_mixed_cycle_two_ranks(aff_path):
    """A node-sharded mixed cycle (C2M shape: two-template jobs, which stay on the engine as units, and jobs with
    required anti-affinity over hostname): both ranks equal the oracle, twice. engine: the anti-affinity jobs are
    cap-1 units of the peer engine too (every rank commits every placement's table increments), no
    pause. pause (option fed_no_aff): they pause every rank's engine and run through the host-staged exchange, and
    every rank pauses at the same units -- the pause's bound is a unit count, not a rank's own clock, so no rank
    relaunches its engine (a new exchange epoch) while a peer resumes."""
    import torch.multiprocessing as mp
    from oracle import pyoracle
    world = 2
    cl = synth.c2m(n_nodes=2100 * world + 300, n_jobs=50, tasks_per_job=30, seed=62, frac_multi=0.15, frac_aff=0.2)
    ref = pyoracle.allocate(cl)
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    opts = {"fed_no_aff": aff_path == "pause"}
    procs = [ctxm.Process(target=_mixed_rank_main, args=(r, world, port, q, cl, opts)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(world):
            rank, res, err = q.get(timeout=240)
            assert err is None, f"rank {rank}: {err}"
            got[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
    for r in range(world):
        out, n_sharded, n_pauses, n_off, n_abandon, n_aff = got[r]
        assert n_abandon == 0 and n_sharded >= 2, (r, n_sharded, n_pauses, n_off)
        if aff_path == "pause":
            assert n_off > 0 and n_aff == 0, (r, n_sharded, n_pauses, n_off, n_aff)
        else:
            assert n_off == 0 and n_pauses == 0 and n_aff > 0, (r, n_sharded, n_pauses, n_off, n_aff)
        assert got[r][1:] == got[0][1:], (r, got[r][1:], got[0][1:])
        for c in out:
            for k in ("events", "binds", "fit_errors"):
                assert c[k] == ref[k], (r, k)
