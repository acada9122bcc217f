"""The oracle's precomputed inter-pod affinity forms against its literal restatement (CPU).

The device path and the oracle's default mode both use reformulations of the reference's inter-pod
affinity code: the predicate with the lister scan hoisted out of the node loop (what predicateMetadata
does, vendor/.../algorithm/predicates/metadata.go:115-165) and the InterPodAffinity priority as per-key
domain histograms. The oracle also keeps line-by-line restatements of the reference's slow paths
(literal_affinity=True): satisfiesExistingPodsAntiAffinity / satisfiesPodsAffinityAntiAffinity with
meta == nil (vendor/.../predicates/predicates.go:1293-1333, 1367-1465) and the O(P*N) processTerm loop
of CalculateInterPodAffinityPriority (vendor/.../priorities/interpod_affinity.go:86-241). These tests
show the two agree -- per (task, node) reason sets and scores, and whole allocate cycles -- so the
histogram / table form the GPU is checked against is the reference's algorithm.
"""
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import model as m
from scheduler_amd import synth

from helpers import affinity_clusters

GI = 1024 ** 3


def _seeded_c4(seed):
    """Small C4 shapes with varied topology sizes, lister sizes and job counts."""
    n_nodes = 20 + 7 * (seed % 9)
    n_zones = 1 + seed % 4
    return synth.c4(n_nodes=n_nodes, n_jobs=4 + seed % 5, tasks_per_job=2 + seed % 6, n_zones=n_zones,
                    n_racks=max(n_zones, 2 + seed % 11), n_pre=n_nodes * (1 + seed % 3) // 2,
                    pre_job_size=5 + seed % 7, seed=1000 + seed)


CASES = affinity_clusters() + [(f"c4-seed{s}", _seeded_c4(s)) for s in range(20)]


def _pending_reps(cl):
    snap = E.Snapshot(cl)
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t["uid"]
    return [reps[s] for s in sorted(reps)]


@pytest.mark.parametrize("name,cluster", CASES, ids=[c[0] for c in CASES])
def test_literal_equals_fast_evaluate(name, cluster):
    uids = _pending_reps(cluster)
    fast = pyoracle.evaluate(cluster, uids)
    lit = pyoracle.evaluate(cluster, uids, literal_affinity=True)
    assert fast["nodes"] == lit["nodes"]
    for a, b in zip(fast["tasks"], lit["tasks"]):
        assert a["task"] == b["task"]
        assert [sorted(r) for r in a["reasons"]] == [sorted(r) for r in b["reasons"]], a["task"]
        assert a["score"] == b["score"], a["task"]
        assert a["batch_error"] == b["batch_error"]


@pytest.mark.parametrize("name,cluster", CASES, ids=[c[0] for c in CASES])
def test_literal_equals_fast_allocate(name, cluster):
    fast = pyoracle.allocate(cluster)
    lit = pyoracle.allocate(cluster, literal_affinity=True)
    for k in ("events", "binds", "fit_errors", "status"):
        assert fast[k] == lit[k], k
    assert len(fast["events"]) > 0


# --- hand-derived KATs ---------------------------------------------------------------
def _weights(**w):
    args = {"leastrequested.weight": "0", "balancedresource.weight": "0", "nodeaffinity.weight": "0",
            "podaffinity.weight": "0"}
    args.update({k: str(v) for k, v in w.items()})
    return [{"plugins": [m.plugin("predicates"), m.plugin("nodeorder", args)]}]


@pytest.mark.parametrize("literal", [False, True])
def test_interpod_affinity_priority_kat(literal):
    """CalculateInterPodAffinityPriority normalisation (interpod_affinity.go:219-235): counts {3, 0, 7},
    min 0, max 7 -> int(10 * 3/7) = 4, 0, 10. The incoming pod prefers (weight 1, hostname) pods labelled
    app=x; n0 runs 3 of them, n1 none, n2 seven."""
    nodes = [m.Node(name=f"n{i}", alloc={m.CPU: 64000, m.MEMORY: 256 * GI, m.PODS: 110},
                    labels={"kubernetes.io/hostname": f"n{i}"}) for i in range(3)]
    pods = []
    for node, k in (("n0", 3), ("n2", 7)):
        for i in range(k):
            pods.append(m.Pod(ns="x", name=f"{node}-{i}", uid=f"x-{node}-{i}", node=node, phase="Running",
                              labels={"app": "x"}, containers=[m.Container(req={m.CPU: 100})]))
    aff = {"podAffinity": {"preferred": [{"weight": 1, "podAffinityTerm": {
        "labelSelector": {"matchLabels": {"app": "x"}}, "topologyKey": "kubernetes.io/hostname"}}]}}
    pods.append(m.Pod(ns="x", name="t", uid="x-t", group="g", affinity=aff,
                      containers=[m.Container(req={m.CPU: 1000, m.MEMORY: GI})]))
    c = m.Cluster(nodes=nodes, pods=pods, pod_groups=[m.PodGroup(ns="x", name="g", queue="q")],
                  queues=[m.Queue(name="q")], tiers=_weights(**{"podaffinity.weight": 1}))
    out = pyoracle.evaluate(c, ["x-t"], literal_affinity=literal)
    assert out["nodes"] == ["n0", "n1", "n2"]
    assert out["tasks"][0]["score"] == [4, 0, 10]
    # preferred anti-affinity (weight -1) to the seven pods on n2: counts {3, 0, -7}, min -7, max 3
    for p in c.pods:
        if p.node == "n2":
            p.labels = {"app": "y"}
    anti = {"podAntiAffinity": {"preferred": [{"weight": 1, "podAffinityTerm": {
        "labelSelector": {"matchLabels": {"app": "y"}}, "topologyKey": "kubernetes.io/hostname"}}]}}
    c.pods[-1].affinity = dict(aff, **anti)
    out = pyoracle.evaluate(c, ["x-t"], literal_affinity=literal)
    assert out["tasks"][0]["score"] == [10, 7, 0]  # int(10*10/10), int(10*7/10), int(10*0/10)


def _one_node(node_kw, pod_kw, tiers=None):
    node = m.Node(name="n", alloc={m.CPU: 8000, m.MEMORY: 16 * GI, m.PODS: 10}, **node_kw)
    pod = m.Pod(ns="x", name="t", uid="x-t", group="g", containers=[m.Container(req={m.CPU: 1000, m.MEMORY: GI},
                                                                                 ports=pod_kw.pop("ports", []))],
                **pod_kw)
    return m.Cluster(nodes=[node], pods=[pod], pod_groups=[m.PodGroup(ns="x", name="g", queue="q")],
                     queues=[m.Queue(name="q")], tiers=tiers or m.default_tiers())


TAINTS = "node(s) had taints that the pod didn't tolerate"


@pytest.mark.parametrize("taint,tols,fits", [  # PodToleratesNodeTaints (predicates.go:1489-1518),
    # Toleration.ToleratesTaint (vendor/k8s.io/api/core/v1/toleration.go:37-56)
    ({"key": "k", "value": "v", "effect": "NoSchedule"}, [], False),
    ({"key": "k", "value": "v", "effect": "PreferNoSchedule"}, [], True),  # only NoSchedule/NoExecute count
    ({"key": "k", "value": "v", "effect": "NoExecute"}, [{"key": "k", "operator": "Equal", "value": "v"}], True),
    ({"key": "k", "value": "v", "effect": "NoSchedule"}, [{"key": "k", "value": "w"}], False),  # value differs
    ({"key": "k", "value": "v", "effect": "NoSchedule"}, [{"key": "k", "operator": "Exists"}], True),
    ({"key": "k", "value": "v", "effect": "NoSchedule"}, [{"operator": "Exists"}], True),  # empty key: all keys
    ({"key": "k", "value": "v", "effect": "NoSchedule"},
     [{"key": "k", "operator": "Exists", "effect": "NoExecute"}], False),  # effect differs
    ({"key": "k", "value": "v", "effect": "NoSchedule"},
     [{"key": "k", "operator": "Exists", "effect": "NoSchedule"}], True),
    ({"key": "k", "value": "", "effect": "NoSchedule"}, [{"key": "k"}], True),  # "" op = Equal, "" == ""
    ({"key": "k", "value": "v", "effect": "NoSchedule"}, [{"key": "k", "operator": "Bogus", "value": "v"}], False),
])
def test_taint_toleration_kat(taint, tols, fits):
    c = _one_node(dict(taints=[taint]), dict(tolerations=tols))
    out = pyoracle.evaluate(c, ["x-t"])
    assert out["tasks"][0]["reasons"] == [[] if fits else [TAINTS]]


PORTS = "node(s) didn't have free ports for the requested pod ports"


@pytest.mark.parametrize("used,want,fits", [  # PodFitsHostPorts (predicates.go:1031-1052),
    # HostPortInfo.CheckConflict (cache/host_ports.go:96-125): "" ip = 0.0.0.0, "" protocol = TCP
    ({"hostPort": 80}, {"hostPort": 80}, False),
    ({"hostPort": 80}, {"hostPort": 81}, True),
    ({"hostPort": 80, "protocol": "UDP"}, {"hostPort": 80}, True),
    ({"hostPort": 80, "hostIP": "10.0.0.1"}, {"hostPort": 80, "hostIP": "10.0.0.2"}, True),
    ({"hostPort": 80, "hostIP": "10.0.0.1"}, {"hostPort": 80}, False),  # 0.0.0.0 conflicts with any ip
    ({"hostPort": 80}, {"hostPort": 80, "hostIP": "10.0.0.2"}, False),  # any ip conflicts with 0.0.0.0
    ({"hostPort": 80, "hostIP": "10.0.0.1"}, {"hostPort": 80, "hostIP": "10.0.0.1"}, False),
    ({"hostPort": 80}, {"hostPort": 0}, True),  # port <= 0 never conflicts
])
def test_host_port_kat(used, want, fits):
    c = _one_node({}, dict(ports=[dict(want)]))
    c.pods.append(m.Pod(ns="y", name="r", uid="y-r", node="n", phase="Running",
                        containers=[m.Container(req={m.CPU: 100}, ports=[dict(used)])]))
    out = pyoracle.evaluate(c, ["x-t"])
    assert out["tasks"][0]["reasons"] == [[] if fits else [PORTS]]
