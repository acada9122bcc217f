"""preempt's use of the sweep: PredicateNodes with Session.PredicateFn alone, PrioritizeNodes,
SortNodes (actions/preempt/preempt.go:187-195; util/scheduler_helper.go:132-144) -- the whole feasible list
in descending score order, lowest index first among equal scores -- on the device (kb_sort_nodes) against the
oracle's restatement, at session open and after an allocate cycle's commits."""
import copy

import numpy as np
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import runtime

from helpers import affinity_clusters, affinity_error_clusters, parity_clusters

CLUSTERS = parity_clusters() + affinity_clusters() + affinity_error_clusters()[:3]


def _reps(snap):
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t["uid"]
    return sorted(reps.items())


def test_oracle_sort_skips_the_resource_check():
    """CPU: a task too big for every node still gets every node passing PredicateFn (preempt makes room)."""
    from helpers import edge_cluster
    cl = edge_cluster()
    big = next(p for p in cl.pods if p.containers and p.containers[0].req.get("cpu") == 9000)
    ev = pyoracle.evaluate(cl, [big.uid])
    assert all("node(s) resource fit failed" in r for r in ev["tasks"][0]["reasons"])
    srt = pyoracle.sort_nodes(cl, [big.uid])["tasks"][0]
    assert len(srt["order"]) > 0
    sc = srt["score"]
    assert all(a >= b for a, b in zip(sc, sc[1:]))


@pytest.mark.gpu
@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_sort_nodes_parity(name, cluster):
    snap = E.Snapshot(cluster)
    reps = _reps(snap)
    ref = pyoracle.sort_nodes(cluster, [u for _, u in reps])
    names = snap.node_names()
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        for i, (s, u) in enumerate(reps):
            order, scores = ctx.sort_nodes(s)
            assert [names[k] for k in order] == ref["tasks"][i]["order"], u
            assert scores.tolist() == ref["tasks"][i]["score"], u
            # reclaim's set (reclaim.go:122-126): the PredicateFn-feasible nodes and the others' FitErrors
            feas, hist = ctx.predicate_nodes(s)
            assert [names[k] for k in feas] == ref["tasks"][i]["feasible"], u
            if not any(r not in E.REASONS for r in ref["tasks"][i]["fit_errors"]):
                assert {E.REASONS[b]: int(c) for b, c in enumerate(hist) if c} == ref["tasks"][i]["fit_errors"], u
        # after a cycle: the table the device holds vs the oracle on the cluster with those pods bound
        out = ctx.allocate(snap)
        got = runtime.result_dict(snap, out)
        if not got["events"] or any(e["kind"] != "allocate" for e in got["events"]):
            return  # Pipelined has no pod phase to rebuild the post-state from
        post = copy.deepcopy(cluster)
        by_uid = {p.uid: p for p in post.pods}
        for e in got["events"]:
            by_uid[e["task"]].node = e["node"]
        left = [(s, u) for s, u in reps if by_uid[u].node == ""]
        if not left:
            return
        ref2 = pyoracle.sort_nodes(post, [u for _, u in left])
        for i, (s, u) in enumerate(left):
            order, scores = ctx.sort_nodes(s)
            assert [names[k] for k in order] == ref2["tasks"][i]["order"], u
            assert scores.tolist() == ref2["tasks"][i]["score"], u
    finally:
        ctx.close()


@pytest.mark.gpu
def test_sort_nodes_at_50k_nodes():
    """The bitonic sort past one LDS tile (2^16 keys, global stages): sorted, complete, index-ordered ties."""
    from scheduler_amd import synth
    snap = synth.c2_snapshot(n_nodes=50000, n_jobs=4, tasks_per_job=1, seed=5)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        ctx.allocate(snap)
        order, scores = ctx.sort_nodes(0)
        r, sc = ctx.eval([0])
    finally:
        ctx.close()
    # the PredicateFn-feasible set: every node the device's mask passes apart from the resource check
    feasible = np.nonzero((r[0] & ~np.uint32(1)) == 0)[0]
    assert sorted(order.tolist()) == feasible.tolist()
    assert (np.diff(scores) <= 0).all()
    for a, b, sa, sb in zip(order, order[1:], scores, scores[1:]):
        assert sa > sb or a < b
