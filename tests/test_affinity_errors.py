"""Inter-pod affinity inputs the reference answers with a plain error, and the per-node Go fallback.

Where InterPodAffinityMatches returns an error instead of failure reasons (an invalid label selector, a
required term with an empty topologyKey), the predicates plugin returns it and PredicateNodes records the
error's own string per node (plugins/predicates/predicates.go:285-289; api/unschedule_info.go:40-54). The
device evaluates those cases with KB_AFF_ERROR table checks and reports KB_R_HOST_ERROR; the host composes
the strings (affinity.Tables.host_error_string) from the per-node masks kb_allocate hands to the NO_FIT
hook. An invalid selector the InterPodAffinity score meets makes PrioritizeNodes return no scores and
SelectBestNode panic (scheduler_helper.go:101-105,147-158): KB_SPEC_IPA_ERROR -> KB_E_PANIC.

CPU tests pin the tables + strings against the oracle's literal restatement; GPU tests run whole cycles.
"""
import numpy as np
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import model as m
from scheduler_amd import runtime

from aff_emul import Tables
from helpers import affinity_error_clusters, ipa_error_clusters

ERR = affinity_error_clusters()
IPA = ipa_error_clusters()
AFF_BITS = (1 << 12) | (1 << 13) | (1 << 14) | (1 << 15) | (1 << 16)


def _reps(snap):
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t
    return sorted(reps.items())


@pytest.mark.parametrize("name,cluster", ERR, ids=[c[0] for c in ERR])
def test_error_tables_at_session_open(name, cluster):
    """Per (spec, node), the emulated table checks + host strings == the oracle's literal predicate."""
    snap = E.Snapshot(cluster)
    tabs = Tables(snap)
    reps = _reps(snap)
    ref = pyoracle.evaluate(cluster, [t["uid"] for _, t in reps], literal_affinity=True)
    names = snap.node_names()
    assert ref["nodes"] == names
    checked = host = 0
    for i, (s, t) in enumerate(reps):
        rs = tabs.reasons(s)
        for n in range(snap.n_nodes):
            want = sorted(ref["tasks"][i]["reasons"][n])
            known = [r for r in want if r in E.REASONS]
            if any(not (AFF_BITS >> E.REASONS.index(r)) & 1 for r in known):
                continue  # an earlier predicate failed: the affinity stage is not reached
            r = int(rs[n])
            if (r >> 16) & 1:
                got = [snap.aff.host_error_string(t["pod"], s, names[n], [])]
                host += 1
            else:
                got = sorted(E.REASONS[b] for b in range(16) if (r >> b) & 1)
            assert got == want, (t["uid"], names[n], got, want)
            checked += 1
    assert checked > 0
    if name not in ("err-empty-key-anti", "err-existing-anti-dynamic", "err-own-anti"):
        assert host > 0  # the case really produces error strings at session open


@pytest.mark.parametrize("name,cluster", IPA, ids=[c[0] for c in IPA])
def test_ipa_error_flag_matches_oracle(name, cluster):
    """KB_SPEC_IPA_ERROR is set exactly for the specs whose InterPodAffinity score the oracle errors on."""
    snap = E.Snapshot(cluster)
    reps = _reps(snap)
    ref = pyoracle.evaluate(cluster, [t["uid"] for _, t in reps])
    for i, (s, t) in enumerate(reps):
        flagged = bool(snap.spec_arr["flags"][s] & E.SPEC_IPA_ERROR)
        assert flagged == ref["tasks"][i]["batch_error"], t["uid"]
    assert any(r["batch_error"] for r in ref["tasks"])


# ---- GPU ------------------------------------------------------------------------------------------------
def _compare(ref, got):
    assert got["nodes"] == ref["nodes"]
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    assert got["fit_errors"] == ref["fit_errors"]
    for uid, st in got["status"].items():
        assert ref["status"][uid] == st, uid


@pytest.mark.gpu
@pytest.mark.parametrize("name,cluster", ERR, ids=[c[0] for c in ERR])
def test_error_inputs_allocate_parity(name, cluster, monkeypatch):
    """Whole allocate cycles over error inputs: placements, statuses and FitErrors (with the reference's
    error strings per node) match the oracle."""
    ref = pyoracle.allocate(cluster)
    got = runtime.allocate(cluster)
    _compare(ref, got)


@pytest.mark.gpu
@pytest.mark.parametrize("name,cluster", IPA, ids=[c[0] for c in IPA])
def test_ipa_error_panics_like_the_reference(name, cluster):
    ref = pyoracle.allocate(cluster)
    assert ref["error"].startswith("panic")
    with pytest.raises(runtime.KbError) as e:
        runtime.allocate(cluster)
    assert e.value.code == runtime.KB_E_PANIC


@pytest.mark.gpu
def test_host_overlay_matches_an_oracle_plugin():
    """kb_set_host_overlay standing in for a Go plugin the device does not express: its per-node verdict is
    ANDed into the predicate chain and its score added to the order score (session_plugins.go:372-389,
    443-469). The oracle runs the same plugin restated in expressible terms -- a NoSchedule taint nobody
    tolerates on the nodes it rejects, a preferred node-affinity term worth its score -- and the placements
    and statuses must agree (the FitErrors differ by design: the overlay's stage is last, the taint's is not)."""
    from helpers import edge_cluster
    cl = edge_cluster()
    snap = E.Snapshot(cl)
    names = snap.node_names()
    reject = {n for i, n in enumerate(names) if i % 5 == 2}
    bonus = {n: (i % 4) * 3 for i, n in enumerate(names)}
    # oracle side: the plugin as a NoSchedule taint nobody tolerates and a labelled preference per bonus level
    ref_cl = cl.copy()
    for nd in ref_cl.nodes:
        if nd.name in reject:
            nd.taints = list(nd.taints) + [{"key": "gofallback", "value": "x", "effect": "NoSchedule"}]
        nd.labels = dict(nd.labels, bonus=str(bonus[nd.name]))
    for p in ref_cl.pods:
        if p.group:
            aff = dict(p.affinity or {})
            na = dict(aff.get("nodeAffinity") or {})
            na["preferred"] = list(na.get("preferred") or []) + [
                {"weight": b, "preference": {"matchExpressions": [{"key": "bonus", "operator": "In",
                                                                    "values": [str(b)]}]}} for b in (3, 6, 9)]
            aff["nodeAffinity"] = na
            p.affinity = aff
    ref = pyoracle.allocate(ref_cl)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        fail = np.array([n in reject for n in names], np.uint8)
        score = np.array([bonus[n] for n in names], np.int64)
        for s in range(len(snap.spec_arr)):
            ctx.set_host_overlay(s, fail, score, reason="node(s) had taints that the pod didn't tolerate")
        out = ctx.allocate(snap)
        got = runtime.result_dict(snap, out)
    finally:
        ctx.close()
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    for uid, st in got["status"].items():
        assert ref["status"][uid] == st, uid
    assert len(got["events"]) > 0
