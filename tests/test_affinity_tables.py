"""The exporter's inter-pod affinity tables against the oracle (CPU): the lookups the device does
(tests/aff_emul.py) must give the oracle's affinity reasons and InterPodAffinity scores, at session open
and after the oracle's own placements are applied through the tables' increment lists."""
import copy

import numpy as np
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import model as m

from aff_emul import Tables
from helpers import affinity_clusters

CLUSTERS = affinity_clusters()
AFF_BITS = (1 << 12) | (1 << 13) | (1 << 14) | (1 << 15)


def _with_pa_weight(cl, w):
    cl = copy.deepcopy(cl)
    for t in cl.tiers:
        for p in t["plugins"]:
            if p["name"] == "nodeorder":
                p["arguments"] = dict(p.get("arguments") or {}, **{"podaffinity.weight": str(w)})
    return cl


def _check(snap, tabs, cluster, specs_uids):
    """Compare emulated affinity reasons / IPA with the oracle for (spec, representative uid) pairs."""
    uids = [u for _, u in specs_uids]
    ref = pyoracle.evaluate(cluster, uids)
    ref0 = pyoracle.evaluate(_with_pa_weight(cluster, 0), uids)
    assert ref["nodes"] == snap.node_names()
    checked = 0
    for i, (s, u) in enumerate(specs_uids):
        rs = tabs.reasons(s)
        ipa = tabs.ipa(s)
        for n in range(snap.n_nodes):
            want = set(ref["tasks"][i]["reasons"][n])
            idx = {E.REASONS.index(r) for r in want if r in E.REASONS}
            assert len(idx) == len(want), want
            other = {b for b in idx if not (AFF_BITS >> b) & 1}
            if other:
                continue  # an earlier predicate failed: the affinity stage is not reached
            got = {b for b in range(16) if (int(rs[n]) >> b) & 1}
            assert got == idx, (u, n, sorted(got), sorted(idx))
            checked += 1
        diff = np.array(ref["tasks"][i]["score"]) - np.array(ref0["tasks"][i]["score"])
        assert list(diff) == list(ipa), (u, list(diff), list(ipa))
    return checked


def _reps(snap):
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t["uid"]
    return sorted(reps.items())


@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_tables_at_session_open(name, cluster):
    snap = E.Snapshot(cluster)
    assert snap.aff is not None
    assert _check(snap, Tables(snap), cluster, _reps(snap)) > 0


@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_tables_after_commits(name, cluster):
    """Apply the oracle's Allocate placements through the increment lists; compare with the oracle
    evaluated on the cluster where those pods are bound (Bound is an allocated status too)."""
    snap = E.Snapshot(cluster)
    out = pyoracle.allocate(cluster, workers=2)
    events = []
    for e in out["events"]:
        if e["kind"] != "allocate":
            break  # Pipelined has no pod phase to rebuild the post-state from
        events.append(e)
    events = events[: max(1, len(events) * 2 // 3)]
    tabs = Tables(snap)
    uid_spec = {t["uid"]: t["spec"] for t in snap.session_tasks if "spec" in t}
    node_idx = snap.node_index
    post = copy.deepcopy(cluster)
    by_uid = {p.uid: p for p in post.pods}
    for e in events:
        tabs.commit(uid_spec[e["task"]], node_idx[e["node"]], True)
        by_uid[e["task"]].node = e["node"]
    placed = {e["task"] for e in events}
    left = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["uid"] not in placed and t["spec"] not in left:
            left[t["spec"]] = t["uid"]
    if not left:
        pytest.skip("every pending task placed")
    assert _check(snap, tabs, post, sorted(left.items())) > 0


def test_unsupported_inputs_fail_loudly():
    """What the device path still refuses (export.Unsupported, never a CPU fallback): a lister pod on a node
    outside the session (the predicate's node lookup errors), and a pending pod with invalid score terms that
    could commit (later scores would error mid-cycle)."""
    base = affinity_clusters()[2][1]
    bad = copy.deepcopy(base)
    p = next(p for p in bad.pods if p.name == "db-1")
    p.node = "elsewhere"  # a node the cache does not know
    with pytest.raises(E.Unsupported):
        E.Snapshot(bad)
    # no pod runs anywhere, so the pod's own score cannot error (nothing to process its terms against)
    bad = m.Cluster(nodes=[m.Node(name=f"n{i}", alloc={m.CPU: 8000, m.MEMORY: 16 * 2 ** 30, m.PODS: 10},
                                  labels={"zone": "z"}) for i in range(3)], queues=[m.Queue(name="q")])
    bad.pod_groups.append(m.PodGroup(ns="ns", name="g", queue="q", min_member=1))
    bad.pods.append(m.Pod(ns="ns", name="g-0", uid="ns-g-0", group="g", containers=[m.Container(req={m.CPU: 100})],
                          affinity={"podAntiAffinity": {"preferred": [{"weight": 1, "podAffinityTerm": {
                              "labelSelector": {"matchExpressions": [{"key": "a", "operator": "In", "values": []}]},
                              "topologyKey": "zone"}}]}}))
    with pytest.raises(E.Unsupported):
        E.Snapshot(bad)


def test_spec_signature_splits_on_identity():
    """Pods that differ only in labels / namespace get different specs once affinity is in play."""
    snap = E.Snapshot(affinity_clusters()[2][1])
    specs = {}
    for t in snap.session_tasks:
        if "spec" in t:
            specs.setdefault(t["pod"].group, set()).add(t["spec"])
    assert all(len(v) == 1 for v in specs.values())
    assert len({next(iter(v)) for v in specs.values()}) == len(specs)
