"""backfill (actions/backfill/backfill.go:40-90): BestEffort tasks take the first node, in the canonical
node order, that passes Session.PredicateFn; allocate skips them (allocate.go:116-122).

CPU: the oracle against a hand-derived case. GPU: runtime.allocate_backfill (kb_allocate, then one-task
kb_place_job calls with the node order off) against the oracle, bit-exact."""
import pytest

from oracle import pyoracle
from scheduler_amd import model as m
from scheduler_amd import runtime

from helpers import GI, affinity_clusters, affinity_error_clusters, backfill_cluster, parity_clusters


def _first_fit_cluster():
    cl = m.Cluster(tiers=m.default_tiers())
    for name in ("a", "b", "c"):
        cl.nodes.append(m.Node(name=name, alloc={m.CPU: 4000, m.MEMORY: 8 * GI, m.PODS: 2}, labels={},
                               unschedulable=(name == "c")))
    cl.queues.append(m.Queue(name="q", weight=1))
    cl.pod_groups.append(m.PodGroup(ns="ns", name="pg", queue="q", min_member=1))
    for i in range(5):
        cl.pods.append(m.Pod(ns="ns", name=f"p{i}", uid=f"u{i}", group="pg", containers=[m.Container(req={})]))
    return cl


def test_oracle_first_fit_hand_derived():
    cl = _first_fit_cluster()
    assert pyoracle.allocate(cl)["events"] == []  # allocate leaves BestEffort tasks alone
    r = pyoracle.allocate_backfill(cl)
    assert [(e["task"], e["node"]) for e in r["events"]] == [("u0", "a"), ("u1", "a"), ("u2", "b"), ("u3", "b")]
    assert r["binds"] == {f"ns/p{i}": n for i, n in enumerate("aabb")}  # min_member 1: dispatched at once
    assert r["backfill_fit_errors"] == {"ns/pg": {"u4": {"node(s) pod number exceeded": 2,
                                                          "node(s) were unschedulable": 1}}}
    assert r["status"]["u4"] == "Pending"


def test_oracle_backfill_skips_invalid_and_nonempty():
    r = pyoracle.allocate_backfill(backfill_cluster())
    for t in range(3):  # gang job below minMember: JobValid fails (gang.go:48-69)
        assert r["status"][f"b-beg-{t}"] == "Pending"
    placed = {e["task"] for e in r["events"]}
    # a task with empty Resreq but an init container request is not backfilled (backfill.go:87-89)
    assert not any(u.startswith("e-g07") for u in placed)
    ports = [e["node"] for e in r["events"] if e["task"].startswith("b-be2-")]
    assert len(ports) == len(set(ports))  # one hostPort 9090 per node


def _with_best_effort(cl, n=6, sel=None):
    """cl plus a job of BestEffort pods (backfill candidates)."""
    cl.pod_groups.append(m.PodGroup(ns="ns", name="be", queue=cl.queues[0].name, min_member=1))
    for i in range(n):
        cl.pods.append(m.Pod(ns="ns", name=f"be-{i}", uid=f"ns-be-{i}", group="be", labels={"role": "be"},
                             node_selector=dict(sel or {}), containers=[m.Container(req={})]))
    return cl


def _error_backfill_cases():
    """Inputs where backfill's PredicateFn returns the inter-pod predicate's error on nodes (the device's
    host-evaluated bucket): an invalid lister pod at session open, and one arising from the cycle's commits."""
    errs = dict(affinity_error_clusters())
    return [("be-err-existing-anti", _with_best_effort(errs["err-existing-anti"])),
            ("be-err-dynamic", _with_best_effort(errs["err-existing-anti-dynamic"]))]


CASES = [("first-fit", _first_fit_cluster()), ("backfill-edge", backfill_cluster())] + \
    parity_clusters()[-2:] + affinity_clusters()[:2] + _error_backfill_cases()


@pytest.mark.gpu
@pytest.mark.parametrize("name,cluster", CASES, ids=[c[0] for c in CASES])
def test_backfill_parity(name, cluster):
    ref = pyoracle.allocate_backfill(cluster)
    got = runtime.allocate_backfill(cluster)
    assert got["nodes"] == ref["nodes"]
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    assert got["fit_errors"] == ref["fit_errors"]
    assert got["backfill_fit_errors"] == ref["backfill_fit_errors"]
    for uid, st in got["status"].items():  # the oracle also lists pods outside any job
        assert ref["status"][uid] == st, uid


@pytest.mark.gpu
def test_backfill_overlay_strings():
    """A node the host overlay rejects fails a backfill task with the overlay plugin's own reason string
    (fe.SetNodeError, backfill.go:84-86), never an unnamed bucket."""
    from scheduler_amd import export as E
    cl = _with_best_effort(_first_fit_cluster(), n=3, sel=None)
    snap = E.Snapshot(cl)
    names = snap.node_names()
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        fail = [1, 1, 0]  # a, b rejected; c is unschedulable: nothing fits
        for sp in range(len(snap.spec_arr)):
            ctx.set_host_overlay(sp, fail=fail, reason=lambda node: f"plugin says no to {node}")
        out = ctx.backfill(snap, ctx.allocate(snap))
    finally:
        ctx.close()
    fit = out["backfill_fit"]
    assert fit, "every BestEffort task fails"
    for tasks in fit.values():
        for h in tasks.values():
            assert None not in h
            assert h == {"plugin says no to a": 1, "plugin says no to b": 1, "node(s) were unschedulable": 1}, h
    assert names == ["a", "b", "c"]
