"""GPU parity past one workgroup's key plan: the split fed engine with range selectors (kbgpu_device.hip
fed_nsel: tables above 20,480 nodes are split into up to four node ranges, one selector workgroup each, and
the placer merges their candidate lists), and the streamed no-fit histogram over a table too large for LDS.

The reference has no node-count limit (util/scheduler_helper.go:34-158), so neither may the fast path.
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import model as m
from scheduler_amd import runtime, synth

from test_gpu_parity import _compare

pytestmark = pytest.mark.gpu

GI = 1024 ** 3
WORKERS = 16


def _pool_cluster(n_nodes=24700, n_pool=150, seed=61):
    """Mostly plain C2-shaped nodes with random load; a small pool labelled pool=a in the last range.
    Jobs: plain gangs (their best nodes spread over every selector's range), then gangs restricted to the
    pool by a node selector: those stop NO_FIT, with every other node failing the selector (the streamed
    histogram over the whole table, with the rows of the last three jobs re-keyed)."""
    rng = np.random.default_rng(seed)
    cl = m.Cluster()
    for i in range(n_nodes):
        cpu = int(rng.integers(8, 65)) * 1000
        labels = {"pool": "a"} if i >= n_nodes - n_pool else {"pool": "b"}
        cl.nodes.append(m.Node(name=f"node-{i:05d}", alloc={m.CPU: cpu, m.MEMORY: 256 * GI, m.PODS: 110},
                               labels=labels))
    cl.queues.append(m.Queue(name="default", weight=1))
    jobs = [("plain", {}, 100, 1000)] * 6 + [("pool", {"pool": "a"}, 100, 30000)] * 4 + [("plain", {}, 60, 500)] * 3
    for j, (kind, sel, n, cpu) in enumerate(jobs):
        name = f"{kind}{j:02d}"
        cl.pod_groups.append(m.PodGroup(ns="ns", name=name, queue="default", min_member=n))
        for t in range(n):
            cl.pods.append(m.Pod(ns="ns", name=f"{name}-{t:03d}", uid=f"ns-{name}-{t:03d}", group=name,
                                 node_selector=dict(sel),
                                 containers=[m.Container(req={m.CPU: cpu, m.MEMORY: 2 * GI})]))
    # running pods: random load, so the best nodes are scattered over the whole table
    cl.pod_groups.append(m.PodGroup(ns="ns", name="run", queue="default", min_member=1, phase="Running"))
    for t in range(3000):
        node = int(rng.integers(0, n_nodes))
        cl.pods.append(m.Pod(ns="ns", name=f"run-{t:04d}", uid=f"ns-run-{t:04d}", group="run",
                             node=f"node-{node:05d}", phase="Running",
                             containers=[m.Container(req={m.CPU: 1000, m.MEMORY: GI})]))
    return cl


BIG = [
    ("pool-24700", _pool_cluster()),                                  # two ranges
    ("C3-41000", synth.c3(n_nodes=41000, n_jobs=12, tasks_per_job=100, seed=62)),  # two ranges, taints/GPUs
    ("pool-61000", _pool_cluster(n_nodes=61000, n_pool=120, seed=63)),  # three ranges
]


@pytest.mark.parametrize("name,cluster", BIG, ids=[c[0] for c in BIG])
def test_range_selectors_match_oracle(name, cluster):
    ref = pyoracle.allocate(cluster, workers=WORKERS)
    snap = E.Snapshot(cluster)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        st = ctx.stats()
    finally:
        ctx.close()
    assert st["fed_cycles"] == 1 and st["fed_split"] == 1 and st["fed_abandon"] == 0, st
    got = runtime.result_dict(snap, out)
    _compare(ref, got)
    assert len(got["events"]) > 0
    if name.startswith("pool"):
        assert ref["fit_errors"], "the pool jobs stop NO_FIT"


def test_c5_one_gpu_matches_oracle_prefix():
    """BASELINE.json configs[4]'s node table (50k C2-shaped nodes, three ranges) with 300 jobs on ONE GPU: the
    cycle's first 3,000 placements are the oracle's (tests/golden/digest-C5-head)."""
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(golden, "digest-C5-head.json")) as f:
        meta = json.load(f)
    want = np.load(os.path.join(golden, "digest-C5-head.npz"), allow_pickle=False)
    snap = synth.c2_snapshot(n_nodes=50000, n_jobs=300, tasks_per_job=100, seed=synth.SEED)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        st = ctx.stats()
    finally:
        ctx.close()
    assert st["fed_cycles"] == 1 and st["fed_split"] == 1 and st["fed_abandon"] == 0, st
    k = meta["max_tasks"]
    et = out["event_task"][:k].astype(np.int32)
    assert np.array_equal(et, want["event_task"])
    assert np.array_equal(out["task_node"][et].astype(np.int32), want["event_node"])
    kinds = np.where(out["task_status"][et] == E.ST["Pipelined"], 2, 1).astype(np.int8)
    assert np.array_equal(kinds, want["event_kind"])


def test_100k_nodes_one_gpu_matches_oracle_head():
    """Past the resident engine's node ceiling on one GPU (four range selectors of 20,480 nodes): 100k C2-shaped
    nodes x 30 jobs of 100 tasks. The cycle runs on the per-job launch path with 64-bit keys and a re-key per commit
    (sweep_keys_kernel + place_loop_kernel); all 3,000 placements are the oracle's (tests/golden/digest-X100k-head)."""
    golden = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    with open(os.path.join(golden, "digest-X100k-head.json")) as f:
        meta = json.load(f)
    want = np.load(os.path.join(golden, "digest-X100k-head.npz"), allow_pickle=False)
    snap = synth.c2_snapshot(n_nodes=100000, n_jobs=30, tasks_per_job=100, seed=synth.SEED)
    ctx = runtime.Context(0, timing=True)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        st = ctx.stats()
    finally:
        ctx.close()
    assert st["fed_cycles"] == 0, st  # (beyond the engine: the launch path)
    k = meta["max_tasks"]
    assert int(out["n_events"]) == meta["events"] == k
    et = out["event_task"][:k].astype(np.int32)
    assert np.array_equal(et, want["event_task"])
    assert np.array_equal(out["task_node"][et].astype(np.int32), want["event_node"])
    kinds = np.where(out["task_status"][et] == E.ST["Pipelined"], 2, 1).astype(np.int8)
    assert np.array_equal(kinds, want["event_kind"])
    K = runtime.KERNELS
    print({K[i]: (st["launches"][i], round(st["kernel_ms"][i], 2)) for i in range(len(K)) if st["launches"][i]},
          "cycle ms", round(out["elapsed_ms"], 1), flush=True)
