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

from helpers import backfill_cluster, parity_clusters

pytestmark = pytest.mark.gpu

NAMES = ["C1-parity", "C2-parity", "C2-fill0.9", "C3-parity", "C2-nogang", "edge-mixed"]


# ranks sharing one GPU: plain engine launches (cooperative launches from several processes take turns on the card,
# DESIGN.md §5; one process per GPU, as deployed, keeps the cooperative launch)
SHARED_GPU = {}  # (ranks sharing one GPU: since ABI 14 every engine launch is plain, the default)


def _clusters():
    return {name: cl for name, cl in parity_clusters() if name in NAMES}


def _summary(out):
    n = int(out["n_events"])
    s = {"task_node": out["task_node"].tolist(), "event_task": out["event_task"][:n].tolist(),
         "task_status": out["task_status"].tolist(), "job_fail_task": out["job_fail_task"].tolist(),
         "job_reason_hist": out["job_reason_hist"].tolist()}
    if "backfill_fit" in out:  # backfill: first fit with every score equal; FitErrors merged over the ranks
        s["backfill_fit"] = {j: {t: dict(h) for t, h in tf.items()} for j, tf in out["backfill_fit"].items()}
    return s


def _run(name, snap, ctx):
    ctx.upload(snap)
    out = ctx.allocate(snap)
    if name == "backfill":
        out = ctx.backfill(snap, out)
    return _summary(out)


def _cases():
    return dict(_clusters(), backfill=backfill_cluster())


def _rank_main(rank, world, port, q, peer=False):
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
    name = None
    try:
        for name, cl in _cases().items():
            snap = E.Snapshot(cl)
            ctx = runtime.Context(0, options=SHARED_GPU if peer else None)
            try:
                ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=peer)
                res[name] = _run(name, snap, ctx)
            finally:
                ctx.close()
        q.put((rank, res, None))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, None, f"{name}: {e!r}"))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("exchange", ["host", "peer"])
@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_one_gpu(world, exchange):
    """Parity clusters on 2 and 3 ranks, one context per cluster in the same processes. host: the launch-path
    exchange for every job; peer: kb_set_shard_peer contexts -- the node-sharded engine on 8-100-node blocks, and the
    host-staged exchange for the cycles it does not take."""
    import torch.multiprocessing as mp
    ref = {}
    for name, cl in _cases().items():
        ctx = runtime.Context(0)
        try:
            ref[name] = _run(name, E.Snapshot(cl), ctx)
        finally:
            ctx.close()
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_rank_main, args=(r, world, port, q, exchange == "peer")) for r in range(world)]
    for p in procs:
        p.start()
    got, errs = {}, []
    for _ in range(world):  # every rank's outcome before judging (a stalled peer shows in the others' errors)
        rank, res, err = q.get(timeout=240)
        if err is not None:
            errs.append(f"rank {rank}: {err}")
        got[rank] = res
    for p in procs:
        p.join(timeout=60)
    assert not errs, "\n".join(errs)
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


@pytest.mark.parametrize("frac", [1.0, 0.5, 0.34])
def test_rccl_pipelined_matches_oracle(frac):
    """A sharded context with the RCCL exchange runs kb_allocate pipelined (job k+1 issued, guarded on job k's
    predicted outcome, before job k is read). minMember below the job size makes jobs stop READY mid-way, so
    predictions fail and guarded sharded jobs skip (sweep, proposal and commit no-ops; the exchange still runs).
    One-rank communicator; placements, statuses and FitErrors equal the oracle's."""
    from oracle import pyoracle
    cl = synth.c2(n_nodes=160, n_jobs=36, tasks_per_job=20, seed=41)
    for pg in cl.pod_groups:
        pg.min_member = max(1, int(pg.min_member * frac))
    ref = pyoracle.allocate(cl)
    snap = E.Snapshot(cl)
    ctx = runtime.Context(0)
    try:
        ctx.set_shard(0, 1, snap.n_nodes, rccl_id=runtime.comm_unique_id())
        ctx.upload(snap)
        got = runtime.result_dict(snap, ctx.allocate(snap))
    finally:
        ctx.close()
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    assert got["fit_errors"] == ref["fit_errors"]


def _c5_rank(rank, world, port, q):
    import torch.distributed as dist
    import torch
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)
    try:
        snap = synth.c2_snapshot(n_nodes=50000, n_jobs=300, tasks_per_job=100, seed=synth.SEED)
        ctx = runtime.Context(0, timing=True)
        try:
            ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather)
            ctx.upload(snap)
            out = _summary(ctx.allocate(snap))
            st = ctx.stats()
        finally:
            ctx.close()
        k = runtime.KERNELS.index("shard_exchange")
        q.put((rank, (out, st["launches"][k]), None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_c5_sharded_matches_one_gpu_and_oracle_prefix():
    """BASELINE.json configs[4] shape (C5: C2 nodes at 50k) with 300 jobs: 3 ranks sharing the GPU (each
    ~16.7k rows, the selection path per shard, one exchange per run segment over gloo) give the placements
    of one GPU holding all 50k rows (the split fed engine with three range selectors), and that cycle's
    first 3000 placements are the oracle's (tests/golden/digest-C5-head)."""
    import json
    import torch.multiprocessing as mp
    from helpers import digest_arrays
    snap = synth.c2_snapshot(n_nodes=50000, n_jobs=300, tasks_per_job=100, seed=synth.SEED)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
    finally:
        ctx.close()
    ref = _summary(out)
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(golden, "digest-C5-head.json")) as f:
        meta = json.load(f)
    want = np.load(os.path.join(golden, "digest-C5-head.npz"), allow_pickle=False)
    k = meta["events"]
    et = np.asarray(ref["event_task"][:k], np.int32)
    assert np.array_equal(et, want["event_task"])
    assert np.array_equal(np.asarray(ref["task_node"])[et].astype(np.int32), want["event_node"])
    assert digest_arrays(et, want["event_node"], want["event_kind"], want["job_fail"]) == meta["sha256"]
    world = 3
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_c5_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=300)
        assert err is None, f"rank {rank}: {err}"
        got[rank] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        summary, exchanges = got[r]
        assert summary == ref, r
        assert exchanges >= 300  # at least one all-gather per job


def _diverge_rank(rank, world, port, q):
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
        snap = synth.c2_snapshot(n_nodes=400, n_jobs=6, tasks_per_job=10, seed=17)
        ctx = runtime.Context(0)
        try:
            ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather)
            ctx.upload(snap)
            try:  # the overlay's verdicts would be rank-local
                ctx.set_host_overlay(0, fail=np.zeros(ctx.n_nodes, np.uint8))
                res["overlay"] = "accepted"
            except runtime.KbError as e:
                res["overlay"] = e.code
            try:  # rank r issues a job of spec r: the exchanged segment tags differ
                ctx.place_job([rank % len(snap.spec_arr)] * 5, ready_num=0, min_available=5)
                res["diverged"] = "no error"
            except runtime.KbError as e:
                res["diverged"] = e.code
        finally:
            ctx.close()
        q.put((rank, res, None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_ranks_that_diverge_fail_loudly():
    """every rank must issue the same segments. Ranks whose drivers issue different jobs get
    KB_E_STATE from the exchanged segment tags (ShardRec::tag) instead of committing a mixed merge (or, with a
    collective count mismatch, hanging later); the host overlay is refused on a sharded context."""
    import torch.multiprocessing as mp
    world = 2
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_diverge_rank, args=(r, world, port, q)) for r in range(world)]
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
        assert got[r] == {"overlay": runtime.KB_E_UNSUPPORTED, "diverged": runtime.KB_E_STATE}, (r, got[r])


def _c5_full_rank(rank, world, port, q, peer=False):
    import torch
    import torch.distributed as dist
    from helpers import digest_arrays
    os.environ["MASTER_ADDR"], os.environ["MASTER_PORT"] = "127.0.0.1", str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def allgather(b):
        t = torch.tensor(list(b), dtype=torch.uint8)
        outs = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(outs, t)
        return b"".join(bytes(o.tolist()) for o in outs)
    try:
        snap = synth.c2_snapshot(n_nodes=50000, n_jobs=10000, tasks_per_job=100, seed=synth.SEED)
        ctx = runtime.Context(0, options=SHARED_GPU if peer else None)
        try:
            ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=peer)
            ctx.upload(snap)
            out = ctx.allocate(snap)
            if peer and ctx.stats()["fed_sharded"] != 1:
                raise AssertionError("the cycle did not run on the node-sharded engine")
        finally:
            ctx.close()
        k = int(out["n_events"])
        et = out["event_task"][:k].astype(np.int32)
        en = out["task_node"][et].astype(np.int32)
        ek = np.where(out["task_status"][et] == E.ST["Pipelined"], 2, 1).astype(np.int8)
        jf = out["job_fail_task"][:10000].astype(np.int32)
        q.put((rank, (k, digest_arrays(et, en, ek, jf)), None))
    except Exception as e:
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("exchange", ["host", "peer"])
def test_c5_full_eight_ranks_match_oracle_digest(exchange):
    """BASELINE.json configs[4] at its stated size and split: 50k nodes x 1M pods, the node table sharded 8 ways
    (8 ranks sharing the GPU). host: one host-staged all-gather over gloo per run segment; peer: the node-sharded
    fed engine (kb_set_shard_peer), every job's proposals exchanged between the ranks' resident engines through
    IPC-mapped inboxes. Every rank's whole cycle equals the oracle's (tests/golden/digest-C5: 1,000,000
    placements, 7,373 s of oracle time)."""
    import json
    import torch.multiprocessing as mp
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(golden, "digest-C5.json")) as f:
        meta = json.load(f)
    world = 8
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_c5_full_rank, args=(r, world, port, q, exchange == "peer")) for r in range(world)]
    for p in procs:
        p.start()
    import queue
    import time
    got = {}
    t0 = time.time()
    while len(got) < world:
        try:
            rank, res, err = q.get(timeout=30)
        except queue.Empty:  # a heartbeat for runs without output capture (the whole cycle takes minutes)
            print(f"c5 eight ranks: {len(got)}/{world} done after {time.time() - t0:.0f} s", flush=True)
            assert time.time() - t0 < 900, "ranks did not finish"
            continue
        assert err is None, f"rank {rank}: {err}"
        got[rank] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        assert got[r] == (meta["events"], meta["sha256"]), r


# ---- inter-pod affinity, node-sharded (SURVEY.md §8 e1 with interpod_affinity.go:119-241) ----
def _aff_cases():
    from helpers import affinity_clusters
    return dict(affinity_clusters())


def _aff_rank_main(rank, world, port, q, peer=False):
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
        for name, cl in _aff_cases().items():
            snap = E.Snapshot(cl)
            ctx = runtime.Context(0, options=SHARED_GPU if peer else None)
            try:
                ctx.set_shard(rank, world, snap.n_nodes, allgather=allgather, peer=peer)
                ctx.upload(snap)
                r = runtime.result_dict(snap, ctx.allocate(snap))
                res[name] = {k: r[k] for k in ("events", "binds", "fit_errors")}
                res[name]["fed_aff_units"] = ctx.stats()["fed_aff_units"]
            finally:
                ctx.close()
        q.put((rank, res, None))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, None, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,exchange", [(2, "host"), (3, "host"), (2, "peer")])
def test_sharded_affinity_matches_oracle(world, exchange):
    """Replicated count tables and histograms, one whole-cluster IPA min / max per run (or per task), every
    commit applied on every rank: the oracle's events, binds and FitErrors on every affinity cluster (C4 shapes,
    the edge clusters, the self-affinity clusters whose specs run one task per segment or as cap-1 runs). peer: the
    affinity units the node-sharded engine takes run on it (each rank commits every placement's
    table increments; the histogram specs' min / max reduced over the ranks before the launch)."""
    import torch.multiprocessing as mp
    from oracle import pyoracle
    ref = {name: pyoracle.allocate(cl) for name, cl in _aff_cases().items()}
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    port = _free_port()
    procs = [ctxm.Process(target=_aff_rank_main, args=(r, world, port, q, exchange == "peer")) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=300)
        assert err is None, f"rank {rank}: {err}"
        got[rank] = res
    for p in procs:
        p.join(timeout=60)
    for r in range(world):
        for name, o in ref.items():
            for k in ("events", "binds", "fit_errors"):
                assert got[r][name][k] == o[k], (world, r, name, k)
            assert got[r][name]["fed_aff_units"] == got[0][name]["fed_aff_units"], (r, name)
    if exchange == "peer":
        assert sum(v["fed_aff_units"] for v in got[0].values()) > 0, {k: v["fed_aff_units"] for k, v in got[0].items()}
