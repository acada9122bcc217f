"""kb_apply: rows changed by commits made outside the device.

A Go-side commit (backfill, a preempt / reclaim eviction, another plugin's bookkeeping) runs
NodeInfo.AddTask / RemoveTask and the plugins' schedulercache AddPod / RemovePod on the session's nodes
(api/node_info.go:165-221; cache/node_info.go:498-630). kb_apply replays those row deltas on the device
table. The check: cluster A = cluster B plus some pods bound to nodes; B uploaded + the pods' deltas must
be the same table as A uploaded (CPU, on the exporter's arrays), and an allocate cycle over it must place
exactly what the oracle places on A (GPU).
"""
import copy

import numpy as np
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import model as m
from scheduler_amd import runtime, synth

from helpers import edge_cluster

GI = 1024 ** 3


def _pair(seed):
    """(A, B, extra pods of A, their node names): A has extra running / releasing pods with host ports and
    scalars outside any session job; B is A without them."""
    a = edge_cluster(seed)
    rng = np.random.default_rng(seed)
    names = sorted(n.name for n in a.nodes)
    fpga = {n.name for n in a.nodes if "example.com/fpga" in n.alloc}
    extra = []
    for i in range(10):
        node = names[int(rng.integers(0, len(names)))]
        req = {m.CPU: 250 * int(rng.integers(1, 5)), m.MEMORY: GI // 4 * int(rng.integers(1, 5))}
        if node in fpga:  # (a scalar request on a node without the resource panics: util/assert)
            req["example.com/fpga"] = 500
        p = m.Pod(ns="ext", name=f"x{i}", uid=f"ext-x{i}", node=node, phase="Running", deleting=(i % 4 == 1),
                  containers=[m.Container(req=req, ports=[{"hostPort": 8080}] if i == 5 else [])])
        extra.append(p)
    b = copy.deepcopy(a)
    a.pods = list(a.pods) + extra
    return a, b, extra


@pytest.mark.parametrize("seed", [3, 4, 5])
def test_pod_deltas_rebuild_the_table(seed):
    a, b, extra = _pair(seed)
    sa, sb = E.Snapshot(a), E.Snapshot(b)
    assert sa.node_names() == sb.node_names() and sa.scalars == sb.scalars
    rows = [E.pod_delta(sb, p, sb.node_index[p.node]) for p in extra]
    d, sc, ports = E.row_deltas(rows)
    cols = {k: v.copy() for k, v in sb.cols.items()}
    S, n = len(sb.scalars), sb.n_nodes
    for i, r in enumerate(d):  # what apply_kernel does, in numpy
        w = r["node"]
        for k in ("idle_cpu", "idle_mem", "rel_cpu", "rel_mem", "nz_cpu", "nz_mem"):
            cols[k][w] += r[k]
        cols["pod_count"][w] += r["pods"]
        cols["flags"][w] |= r["flags_set"]
        if r["sc_off"] != 0xffffffff:
            for q in range(S):
                cols["idle_sc"][q, w] += sc[r["sc_off"] + q]
                cols["rel_sc"][q, w] += sc[r["sc_off"] + S + q]
        for s_id, ip in ports[r["port_off"]:r["port_off"] + r["port_cnt"]]:
            cols["port_used"][s_id, w] |= np.uint64(1 << int(ip))
    for k, v in sa.cols.items():
        assert np.array_equal(cols[k], v), k


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [3, 4, 5])
def test_apply_then_allocate_matches_oracle(seed):
    a, b, extra = _pair(seed)
    ref = pyoracle.allocate(a)
    sb = E.Snapshot(b)
    ctx = runtime.Context(0)
    try:
        ctx.upload(sb)
        ctx.apply(*E.row_deltas([E.pod_delta(sb, p, sb.node_index[p.node]) for p in extra]))
        out = ctx.allocate(sb)
    finally:
        ctx.close()
    got = runtime.result_dict(sb, out)
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    assert got["fit_errors"] == ref["fit_errors"]


@pytest.mark.gpu
def test_apply_removal_is_the_inverse():
    """AddTask then RemoveTask deltas of the same pods leave the device table as uploaded."""
    cl = synth.c4(n_nodes=200, n_jobs=10, tasks_per_job=10, seed=8, n_zones=4, n_racks=20, n_pre=200,
                  pre_job_size=20)
    snap = E.Snapshot(cl)
    pods = [p for p in cl.pods if p.node][:30]
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        before = ctx.read_nodes(snap.n_nodes)
        rows = [E.pod_delta(snap, p, snap.node_index[p.node]) for p in pods if p.node in snap.node_index]
        ctx.apply(*E.row_deltas(rows))
        mid = ctx.read_nodes(snap.n_nodes)
        rows = [E.pod_delta(snap, p, snap.node_index[p.node], remove=True) for p in pods if p.node in snap.node_index]
        ctx.apply(*E.row_deltas(rows))
        after = ctx.read_nodes(snap.n_nodes)
    finally:
        ctx.close()
    assert any(not np.array_equal(before[k], mid[k]) for k in before)
    for k in before:
        assert np.array_equal(before[k], after[k]), k
