"""Runner for the reference's e2e scheduling expectations (tests/golden/ref-e2e-*.json, made by
tests/golden/make_e2e.py from test/e2e/nodeorder.go and test/e2e/predicates.go).

A scenario is a sequence of steps on one cluster: create a job (a PodGroup and its pods), taint / untaint every
node, or run one scheduling cycle (allocate then backfill: config/kube-batch-conf.yaml). Pods a cycle binds run on
their node from then on (the next cycle's snapshot lists them Running there); pods it leaves Pending stay pending.
After each cycle the spec's assertions are checked on the cycle's binds.
"""
import json
import os

from scheduler_amd import model as m

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
HOST = "kubernetes.io/hostname"
NS = "e2e"


def load(name):
    with open(os.path.join(HERE, f"ref-e2e-{name}.json")) as f:
        return json.load(f)["scenarios"]


def _cluster(nodes, jobs, bound):
    cl = m.Cluster(tiers=m.default_tiers())
    for n in nodes:
        cl.nodes.append(m.Node(name=n["name"], alloc=dict(n["alloc"]), labels={HOST: n["name"]},
                               taints=[dict(t) for t in n["taints"]]))
    cl.queues.append(m.Queue(name="default", weight=1))
    for j in jobs:
        cl.pod_groups.append(m.PodGroup(ns=NS, name=j["name"], queue="default", min_member=j["min"],
                                        priority=j["priority"]))
        for i in range(j["rep"]):
            name = f"{j['name']}-{i}"
            ports = [{"hostPort": j["hostport"], "protocol": "TCP"}] if j["hostport"] else []
            node = bound.get(f"{NS}/{name}", "")
            cl.pods.append(m.Pod(ns=NS, name=name, uid=f"{NS}-{name}", group=j["name"], node=node,
                                 phase="Running" if node else "Pending", labels=dict(j["labels"]),
                                 containers=[m.Container(req=dict(j["req"]), ports=ports)],
                                 affinity=j["affinity"]))
    return cl


def _check(expect, jobs, bound, where):
    by_name = {j["name"]: j for j in jobs}
    for e in expect:
        if e.get("any"):
            continue
        j = by_name[e["job"]]
        on = [bound[f"{NS}/{j['name']}-{i}"] for i in range(j["rep"]) if f"{NS}/{j['name']}-{i}" in bound]
        assert len(on) == e["bound"], (where, e, on)
        if "pending" in e:
            assert j["rep"] - len(on) == e["pending"], (where, e, on)
        if "all_on" in e:
            assert all(n == e["all_on"] for n in on), (where, e, on)
        if "none_on" in e:
            assert not set(on) & set(e["none_on"]), (where, e, on)
        if e.get("same_node"):
            assert len(set(on)) == 1, (where, e, on)
        if e.get("distinct_nodes"):
            assert len(set(on)) == len(on), (where, e, on)
        if "with_job" in e:
            other = by_name[e["with_job"]]
            theirs = {bound[f"{NS}/{other['name']}-{i}"] for i in range(other["rep"])
                      if f"{NS}/{other['name']}-{i}" in bound}
            assert set(on) <= theirs, (where, e, on, theirs)


def run(scenario, allocate_backfill):
    """Play the scenario with `allocate_backfill(cluster) -> {"binds": {ns/name: node}, ...}`; returns the binds
    of every cycle (the trace both implementations must share)."""
    nodes = [dict(n, taints=list(n["taints"])) for n in scenario["nodes"]]
    jobs, bound, trace = [], {}, []
    for k, step in enumerate(scenario["steps"]):
        if "create" in step:
            jobs.append(step["create"])
        elif "taint_all" in step:
            for n in nodes:
                n["taints"] = n["taints"] + [dict(step["taint_all"])]
        elif "untaint_all" in step:
            for n in nodes:
                n["taints"] = [t for t in n["taints"] if t["key"] != step["untaint_all"]]
        elif "cycle" in step:
            out = allocate_backfill(_cluster(nodes, jobs, bound))
            new = {p: n for p, n in out["binds"].items() if p not in bound}
            bound.update(new)
            trace.append(sorted(new.items()))
            _check(step["cycle"], jobs, bound, f"{scenario['name']} step {k}")
    return trace
