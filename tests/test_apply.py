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


# ---- kb_apply_affinity: inter-pod affinity tables for pods outside the pending specs ----
def _aff_pair(seed):
    """(A, B, bound, evicted): A = affinity_edge_cluster(seed) plus loose pods (no PodGroup: scored, not listed)
    that copy the running pods' labels and terms, with one running lister task of B evicted (Releasing: it leaves
    the lister, stays on its node); B is A without the loose pods and without the eviction."""
    from helpers import affinity_edge_cluster
    b = affinity_edge_cluster(seed)
    a = copy.deepcopy(b)
    rng = np.random.default_rng(seed)
    names = sorted(n.name for n in a.nodes)
    src = [p for p in a.pods if p.node and p.affinity]
    bound = []
    for i in range(8):
        s = src[int(rng.integers(0, len(src)))]
        p = m.Pod(ns=s.ns, name=f"loose-x{i}", uid=f"{s.ns}-loose-x{i}", node=names[int(rng.integers(0, len(names)))],
                  phase="Running", labels=dict(s.labels), affinity=copy.deepcopy(s.affinity),
                  containers=[m.Container(req={m.CPU: 100, m.MEMORY: GI // 8})])
        bound.append(p)
    a.pods = list(a.pods) + bound
    victim = next(p for p in a.pods if p.group == "db")
    victim.deleting = True
    before = next(p for p in b.pods if p.uid == victim.uid)
    return a, b, bound, (before, victim)


def _aff_deltas(sb, bound, evicted):
    tb = sb.aff
    rows, ad = [], []
    for p in bound:
        w = sb.node_index[p.node]
        rows.append(E.pod_delta(sb, p, w))
        ad += tb.pod_deltas(p, w, existing=1)
    before, after = evicted
    w = sb.node_index[before.node]
    rows += [E.pod_delta(sb, before, w, remove=True), E.pod_delta(sb, after, w)]
    ad += tb.pod_deltas(before, w, lister=-1)  # Running -> Releasing: out of the lister, still on the node
    return rows, runtime.aff_delta_array(ad)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_pod_affinity_deltas_rebuild_the_tables(seed):
    a, b, bound, evicted = _aff_pair(seed)
    sa, sb = E.Snapshot(a), E.Snapshot(b)
    for f in ("topo_dom", "table_arr", "spec_arr", "check_arr", "lister_arr", "hist_arr", "incr_arr"):
        assert np.array_equal(getattr(sa.aff, f), getattr(sb.aff, f)), f  # the same layout
    _, ad = _aff_deltas(sb, bound, evicted)
    assert len(ad) and (ad["table"] >= 0).any() and (ad["table"] < 0).any()
    cnt, tot, h = sb.aff.counters.copy(), sb.aff.totals.copy(), sb.aff.h.copy()
    for e in ad:  # what apply_aff_kernel does, in numpy
        if e["table"] >= 0:
            slot, off = sb.aff.table_arr[e["table"]]
            d = sb.aff.topo_dom[slot, e["node"]]
            if d >= 0:
                cnt[off + d] += e["weight"]
            tot[e["table"]] += e["weight"]
        else:
            d = sb.aff.topo_dom[e["slot"], e["node"]]
            if d >= 0:
                h[e["h_off"] + d] += e["weight"]
    assert np.array_equal(cnt, sa.aff.counters)
    assert np.array_equal(tot, sa.aff.totals)
    assert np.array_equal(h, sa.aff.h)
    assert not np.array_equal(h, sb.aff.h) and not np.array_equal(tot, sb.aff.totals)


def test_pod_affinity_deltas_refuse_new_tables():
    """A bound pod whose terms score a spec on a topology key the spec has no histogram for is refused."""
    b = __import__("helpers").affinity_edge_cluster(11)
    sb = E.Snapshot(b)
    p = m.Pod(ns="ns", name="odd", uid="ns-odd", node=sb.node_names()[0], phase="Running", labels={"app": "odd"},
              affinity={"podAffinity": {"preferred": [{"weight": 5, "podAffinityTerm": {
                  "labelSelector": {"matchLabels": {"job": "plain"}}, "topologyKey": "brand-new-key"}}]}},
              containers=[m.Container(req={m.CPU: 100})])
    with pytest.raises(E.Unsupported):
        sb.aff.pod_deltas(p, 0, existing=1)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [11, 12, 13])
def test_apply_affinity_then_allocate_matches_oracle(seed):
    a, b, bound, evicted = _aff_pair(seed)
    ref = pyoracle.allocate(a)
    sa, sb = E.Snapshot(a), E.Snapshot(b)
    rows, ad = _aff_deltas(sb, bound, evicted)
    ctx = runtime.Context(0)
    try:
        ctx.upload(sb)
        ctx.apply(*E.row_deltas(rows))
        ctx.apply_affinity(ad)
        out = ctx.allocate(sa)  # the host's session state is A's (the eviction changed the job's ready count)
    finally:
        ctx.close()
    got = runtime.result_dict(sa, out)
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    assert got["fit_errors"] == ref["fit_errors"]
