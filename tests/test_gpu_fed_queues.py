"""Forward progress of the resident fed engine in a crowded process (the N > 1 bench's situation).

The engine (one launch per allocate cycle) waits for per-job sweep kernels issued on a second stream. If that
stream shared a hardware queue with the engine's, a sweep would queue behind the engine and the engine would
wait out its idle bound (1 s) before the cycle finished on the launch path. The library creates the sweep stream
with a CU mask (a hardware queue of its own; the engine is a plain launch on the library's main stream after a
residency check, ABI 14), so that cannot happen whatever other streams the process holds: here a torch process group with
its communicator streams, torch's stream pool, and 0..7 raw HIP streams created between the library's own
streams. Every cycle must finish on the engine (fed_abandon == 0) with the oracle's placements
(allocate.go:95-192: one cycle must not stall).
"""
import ctypes
import os
import socket

import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import runtime, synth

from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu


def _child(q, shared, kernel_sweeps):
    """One fresh process: torch's HIP runtime first (as in bench.py's ranks), then the library's."""
    try:
        # a stall shows as an abandon within the test's time; shared: the sweep stream without its own queue;
        # kernel_sweeps: the per-job sweep kernels on that stream (else the engine's resident sweepers)
        options = {"fed_idle_ms": 300, "fed_shared_queues": shared, "fed_kernel_sweeps": kernel_sweeps}
        import torch
        import torch.distributed as dist
        with socket.socket() as sk:
            sk.bind(("127.0.0.1", 0))
            port = sk.getsockname()[1]
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        t = torch.ones(1024, device="cuda:0")
        dist.all_reduce(t)  # the communicator and its streams exist from here on
        pool = [torch.cuda.Stream() for _ in range(8)]  # torch's stream pool, with work on each
        for s in pool:
            with torch.cuda.stream(s):
                torch.ones(4096, device="cuda:0").sum()
        torch.cuda.synchronize()
        hip = ctypes.CDLL("libamdhip64.so")
        cl = synth.c2(n_nodes=3000, n_jobs=40, tasks_per_job=40, seed=51)
        snap = E.Snapshot(cl)
        res, raw = [], []
        for extra in range(8):
            ctx = runtime.Context(0, options=options)
            try:
                for _ in range(extra):  # between the library's main stream and its sweep stream
                    s = ctypes.c_void_p()
                    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
                    raw.append(s)
                ctx.upload(snap)
                out = ctx.allocate(snap)
                st = ctx.stats()
            finally:
                ctx.close()
            res.append((extra, st["fed_cycles"], st["fed_abandon"], runtime.result_dict(snap, out)))
        for s in raw:
            hip.hipStreamDestroy(s)
        dist.destroy_process_group()
        q.put((res, None))
    except Exception as e:  # report, do not hang the parent
        q.put((None, repr(e)))


def _run(shared, kernel_sweeps=True):
    import torch.multiprocessing as mp
    ctxm = mp.get_context("spawn")
    q = ctxm.Queue()
    p = ctxm.Process(target=_child, args=(q, shared, kernel_sweeps))
    p.start()
    res, err = q.get(timeout=240)
    p.join(timeout=60)
    assert err is None, err
    return res


@pytest.mark.parametrize("kernel_sweeps", [True, False], ids=["sweep-kernels", "resident-sweepers"])
def test_fed_engine_progress_beside_other_streams(kernel_sweeps):
    """Both ways the split engine gets its sweeps: the per-job sweep kernels on the CU-masked stream, and the
    engine's resident sweepers (no per-job launch at all)."""
    ref = pyoracle.allocate(synth.c2(n_nodes=3000, n_jobs=40, tasks_per_job=40, seed=51), workers=8)
    for extra, cycles, abandon, got in _run(shared=False, kernel_sweeps=kernel_sweeps):
        assert cycles == 1 and abandon == 0, (extra, cycles, abandon)
        _compare(ref, got)


def test_shared_queues_hazard_is_real():
    """The same process layout with the sweep kernels' stream from the shared pool
    (options fed_shared_queues, fed_kernel_sweeps): the hazard is observable -- some layouts stall the engine into its idle exit --
    and the cycle still ends with the oracle's placements on the launch path (correct, 300 ms slower)."""
    ref = pyoracle.allocate(synth.c2(n_nodes=3000, n_jobs=40, tasks_per_job=40, seed=51), workers=8)
    res = _run(shared=True)
    for extra, cycles, abandon, got in res:
        _compare(ref, got)
    assert any(abandon for _, _, abandon, _ in res), [(e, a) for e, _, a, _ in res]
