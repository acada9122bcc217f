"""Known-answer tests pinning the oracle to the reference's own unit tests.

Each case restates a reference test (file:line) with the same inputs and expected
outputs; together they pin the oracle's arithmetic where the Go reference cannot be
run (no Go toolchain in this image).
"""
import pytest

from oracle import pyoracle
from scheduler_amd import model as m


def R(cpu=0, mem=0, scalars=None, max_task=0):
    return {"cpu": cpu, "memory": mem, "scalars": scalars, "maxTaskNum": max_task}


def norm(r):
    return (r["cpu"], r["memory"], r["scalars"], r["maxTaskNum"])


# --- pkg/scheduler/api/resource_info_test.go -------------------------------
def test_new_resource():  # TestNewResource :27-57
    assert norm(pyoracle.resource_op("NewResource", list={})["result"]) == (0, 0, None, 0)
    lst = {"cpu": 4, "memory": 2000, "scalar.test/scalar1": 1000, "hugepages-test": 2000}
    assert norm(pyoracle.resource_op("NewResource", list=lst)["result"]) == (
        4, 2000, {"hugepages-test": 2000, "scalar.test/scalar1": 1000}, 0)


def test_add_scalar():  # TestResourceAddScalar :59-96
    r = pyoracle.resource_op("AddScalar", l=R(), name="scalar1", quantity=100)["result"]
    assert norm(r) == (0, 0, {"scalar1": 100}, 0)
    r = pyoracle.resource_op("AddScalar", l=R(4000, 8000, {"hugepages-test": 2}), name="scalar2", quantity=200)["result"]
    assert norm(r) == (4000, 8000, {"hugepages-test": 2, "scalar2": 200}, 0)


def test_set_max_resource():  # TestSetMaxResource :98-142
    r = pyoracle.resource_op("SetMaxResource", l=R(), r=R(4000, 2000, {"scalar.test/scalar1": 1, "hugepages-test": 2}))
    assert norm(r["result"]) == (4000, 2000, {"scalar.test/scalar1": 1, "hugepages-test": 2}, 0)
    r = pyoracle.resource_op("SetMaxResource", l=R(4000, 4000, {"scalar.test/scalar1": 1, "hugepages-test": 2}),
                             r=R(4000, 2000, {"scalar.test/scalar1": 4, "hugepages-test": 5}))
    assert norm(r["result"]) == (4000, 4000, {"scalar.test/scalar1": 4, "hugepages-test": 5}, 0)


def test_is_zero():  # TestIsZero :144-181
    assert pyoracle.resource_op("IsZero", l=R(), name="cpu")["result"] is True
    full = R(4000, 4000, {"scalar.test/scalar1": 4, "hugepages-test": 5})
    assert pyoracle.resource_op("IsZero", l=full, name="cpu")["result"] is False
    assert pyoracle.resource_op("IsZero", l=full, name="scalar.test/scalar1")["result"] is True


def test_add_resource():  # TestAddResource :183-243
    cases = [
        (R(), R(4000, 2000, {"scalar.test/scalar1": 1, "hugepages-test": 2}),
         (4000, 2000, {"scalar.test/scalar1": 1, "hugepages-test": 2}, 0)),
        (R(4000, 4000, {"scalar.test/scalar1": 1, "hugepages-test": 2}),
         R(4000, 2000, {"scalar.test/scalar1": 4, "hugepages-test": 5}),
         (8000, 6000, {"scalar.test/scalar1": 5, "hugepages-test": 7}, 0)),
        (R(4000, 4000, {"scalar.test/scalar1": 1}), R(4000, 2000, {"scalar.test/scalar1": 4, "hugepages-test": 5}),
         (8000, 6000, {"scalar.test/scalar1": 5, "hugepages-test": 5}, 0)),
    ]
    for l, r, exp in cases:
        assert norm(pyoracle.resource_op("Add", l=l, r=r)["result"]) == exp


@pytest.mark.parametrize("l,r,exp", [  # TestLessEqual :246-304
    (R(), R(4000, 2000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}), True),
    (R(4000, 4000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}),
     R(2000, 2000, {"scalar.test/scalar1": 4000, "hugepages-test": 5000}), False),
    (R(4, 4000, {"scalar.test/scalar1": 1}), R(), False),
    (R(4000, 4000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}),
     R(8000, 8000, {"scalar.test/scalar1": 4000, "hugepages-test": 5000}), True),
])
def test_less_equal(l, r, exp):
    assert pyoracle.resource_op("LessEqual", l=l, r=r)["result"] is exp


def test_sub_resource():  # TestSubResource :306-350
    r = pyoracle.resource_op("Sub", l=R(4000, 2000, {"scalar.test/scalar1": 1, "hugepages-test": 2}), r=R())
    assert norm(r["result"]) == (4000, 2000, {"scalar.test/scalar1": 1, "hugepages-test": 2}, 0)
    r = pyoracle.resource_op("Sub", l=R(4000, 4000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}),
                             r=R(3000, 2000, {"scalar.test/scalar1": 500, "hugepages-test": 1000}))
    assert norm(r["result"]) == (1000, 2000, {"scalar.test/scalar1": 500, "hugepages-test": 1000}, 0)


def test_sub_underflow_panics():  # util/assert/assert.go:17-40 (panicOnError default true)
    with pytest.raises(pyoracle.OraclePanic):
        pyoracle.resource_op("Sub", l=R(1000, 1000), r=R(2000, 1000))


@pytest.mark.parametrize("l,r,exp", [  # TestLess :352-420
    (R(), R(), False),
    (R(), R(4000, 2000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}), True),
    (R(4000, 4000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}),
     R(8000, 8000, {"scalar.test/scalar1": 4000, "hugepages-test": 5000}), True),
    (R(4000, 4000, {"scalar.test/scalar1": 5000, "hugepages-test": 2000}),
     R(8000, 8000, {"scalar.test/scalar1": 4000, "hugepages-test": 5000}), False),
    (R(9000, 4000, {"scalar.test/scalar1": 1000, "hugepages-test": 2000}),
     R(8000, 8000, {"scalar.test/scalar1": 4000, "hugepages-test": 5000}), False),
])
def test_less(l, r, exp):
    assert pyoracle.resource_op("Less", l=l, r=r)["result"] is exp


def test_tolerance_edges():  # resource_info.go:70-72,253-276: |rr - r| < 10m / 10Mi / 10m
    assert pyoracle.resource_op("LessEqual", l=R(1009, 0), r=R(1000, 0))["result"] is True
    assert pyoracle.resource_op("LessEqual", l=R(1010, 0), r=R(1000, 0))["result"] is False
    mi = 1024 * 1024
    assert pyoracle.resource_op("LessEqual", l=R(0, 10 * mi - 1), r=R(0, 0))["result"] is True
    assert pyoracle.resource_op("LessEqual", l=R(0, 10 * mi), r=R(0, 0))["result"] is False
    assert pyoracle.resource_op("LessEqual", l=R(0, 0, {"a/b": 9}), r=R(0, 0, {}))["result"] is True
    assert pyoracle.resource_op("LessEqual", l=R(0, 0, {"a/b": 0}), r=R(0, 0, None))["result"] is False


# --- pkg/scheduler/api/pod_info_test.go ------------------------------------
def _pod(containers, init=()):
    p = m.Pod(ns="c1", name="p", uid="c1-p", containers=[m.Container(req=c) for c in containers],
              init=[m.Container(req=c) for c in init])
    return p.to_json()


def test_pod_resource_request():  # TestGetPodResourceRequest :26-93 / WithoutInitContainers :95-160
    rl = lambda c, mem: m.canon_resource_list({"cpu": c, "memory": mem})  # api/test_utils.go buildResourceList
    r = pyoracle.resource_op("PodRequest", pod=_pod([rl("1000m", "1G"), rl("2000m", "1G")]))
    assert (r["initreq"]["cpu"], r["initreq"]["memory"]) == (3000, 2e9)
    assert (r["resreq"]["cpu"], r["resreq"]["memory"]) == (3000, 2e9)
    r = pyoracle.resource_op("PodRequest", pod=_pod([rl("1000m", "1G"), rl("2000m", "1G")],
                                                    [rl("2000m", "5G"), rl("2000m", "1G")]))
    assert (r["initreq"]["cpu"], r["initreq"]["memory"]) == (3000, 5e9)
    assert (r["resreq"]["cpu"], r["resreq"]["memory"]) == (3000, 2e9)


# --- pkg/scheduler/api/node_info_test.go -----------------------------------
def test_node_info_add_remove():  # TestNodeInfo_AddPod :35-81, TestNodeInfo_RemovePod :83-137
    rl = lambda c, mem: m.canon_resource_list({"cpu": c, "memory": mem})
    node = m.build_node("n1", rl("8000m", "10G")).to_json()
    pods = [m.Pod(ns="c1", name=f"p{i}", uid=f"c1-p{i}", node="n1", phase="Running",
                  containers=[m.Container(req=rl(f"{i}000m", f"{i}G"))]).to_json() for i in (1, 2, 3)]
    r = pyoracle.resource_op("NodeTasks", node=node, pods=pods[:2])
    assert (r["idle"]["cpu"], r["idle"]["memory"]) == (5000, 7e9)
    assert (r["used"]["cpu"], r["used"]["memory"]) == (3000, 3e9)
    assert r["tasks"] == ["c1/p1", "c1/p2"]
    r = pyoracle.resource_op("NodeTasks", node=node, pods=pods, remove=[pods[1]])
    assert (r["idle"]["cpu"], r["idle"]["memory"]) == (4000, 6e9)
    assert (r["used"]["cpu"], r["used"]["memory"]) == (4000, 4e9)
    assert r["tasks"] == ["c1/p1", "c1/p3"]


# --- pkg/scheduler/actions/allocate/allocate_test.go -----------------------
def _drf_proportion_tiers():  # allocate_test.go:180-195 (only the listed flags are set)
    return [{"plugins": [
        m.plugin("drf", defaults=False, enabledPreemptable=True, enabledJobOrder=True),
        m.plugin("proportion", defaults=False, enabledQueueOrder=True, enabledReclaimable=True),
    ]}]


def allocate_test_cases():
    rl = m.build_resource_list
    c1 = m.Cluster(
        nodes=[m.build_node("n1", rl("2", "4Gi"))],
        pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1"),
              m.build_pod("c1", "p2", "", "Pending", rl("1", "1G"), "pg1")],
        pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="c1")],
        queues=[m.Queue(name="c1", weight=1)], tiers=_drf_proportion_tiers())
    c2 = m.Cluster(
        nodes=[m.build_node("n1", rl("2", "4G"))],
        pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1"),
              m.build_pod("c1", "p2", "", "Pending", rl("1", "1G"), "pg1"),
              m.build_pod("c2", "p1", "", "Pending", rl("1", "1G"), "pg2"),
              m.build_pod("c2", "p2", "", "Pending", rl("1", "1G"), "pg2")],
        pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="c1"), m.PodGroup(ns="c2", name="pg2", queue="c2")],
        queues=[m.Queue(name="c1", weight=1), m.Queue(name="c2", weight=1)], tiers=_drf_proportion_tiers())
    return [("one Job with two Pods on one node", c1, {"c1/p1": "n1", "c1/p2": "n1"}),
            ("two Jobs on one node", c2, {"c2/p1": "n1", "c1/p1": "n1"})]


@pytest.mark.parametrize("name,cluster,expected", allocate_test_cases(), ids=lambda x: x if isinstance(x, str) else "")
def test_allocate_reference_cases(name, cluster, expected):  # TestAllocate :38-212
    out = pyoracle.allocate(cluster)
    assert out["binds"] == expected


# --- pkg/scheduler/util/scheduler_helper_test.go ----------------------------
# TestSelectBestNode :26-63 -- with the lowest-index tie-break the winner must lie in the expected set.
def test_select_best_node_rule():
    # case 1: scores {1: [node1, node2], 2: [node3, node4]} -> node3 (lowest index among the max)
    # case 2: scores {1: [...], 3: [node3], 2: [...]} -> node3
    # Exercised end-to-end: two equal best nodes -> the name-sorted first wins.
    rl = m.build_resource_list
    alloc = dict(rl("4", "8Gi"), pods=10)
    c = m.Cluster(nodes=[m.build_node(n, alloc) for n in ("node4", "node3")],
                  pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1")],
                  pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="q")], queues=[m.Queue(name="q")])
    out = pyoracle.allocate(c)
    assert out["binds"] == {"c1/p1": "node3"}
    # the nil-scalar-map quirk (resource_info.go:264-267): a task carrying nvidia.com/gpu: 0 never fits a
    # node whose allocatable lists no scalar resource.
    for n in c.nodes:
        n.alloc = m.resource_list(cpu="4", memory="8Gi", pods=10)
    out = pyoracle.allocate(c)
    assert out["binds"] == {}
    assert out["fit_errors"]["c1/pg1"]["c1-p1"] == {"node(s) resource fit failed": 2}


# --- hand-derived KATs from the vendored formulas ----------
def _one_node_eval(alloc, existing_req, pod_req):
    node = m.Node(name="n", alloc=alloc, labels={})
    pods = [m.Pod(ns="x", name="e", uid="x-e", node="n", phase="Running", containers=[m.Container(req=existing_req)])]
    pods.append(m.Pod(ns="x", name="t", uid="x-t", group="g", containers=[m.Container(req=pod_req)]))
    c = m.Cluster(nodes=[node], pods=pods, pod_groups=[m.PodGroup(ns="x", name="g", queue="q")],
                  queues=[m.Queue(name="q")],
                  tiers=[{"plugins": [m.plugin("predicates"), m.plugin("nodeorder", {"balancedresource.weight": "0",
                                                                                       "podaffinity.weight": "0"})]}])
    return c


def test_least_requested_kat():
    # LR: alloc 4000m / 10000 B, node nz 1000m / 2000 B, pod nz 1000m / 1000 B => (5 + 7) / 2 = 6
    c = _one_node_eval({"cpu": 4000, "memory": 10000, "pods": 10}, {"cpu": 1000, "memory": 2000},
                       {"cpu": 1000, "memory": 1000})
    out = pyoracle.evaluate(c, ["x-t"])
    assert out["tasks"][0]["score"] == [6]


def test_balanced_resource_kat():
    # BRA: cpu 2000/4000 = 0.5, mem 3000/10000 = 0.3 => int((1 - 0.2) * 10) = 8
    c = _one_node_eval({"cpu": 4000, "memory": 10000, "pods": 10}, {"cpu": 1000, "memory": 2000},
                       {"cpu": 1000, "memory": 1000})
    for p in c.tiers[0]["plugins"]:
        if p["name"] == "nodeorder":
            p["arguments"] = {"leastrequested.weight": "0", "balancedresource.weight": "1", "podaffinity.weight": "0"}
    out = pyoracle.evaluate(c, ["x-t"])
    assert out["tasks"][0]["score"] == [8]


def test_missing_pods_allocatable_rejects_everything():
    # util.BuildNode lists no `pods` => MaxTaskNum = 0 => "node(s) pod number exceeded" (predicates.go:162-166)
    rl = m.build_resource_list
    c = m.Cluster(nodes=[m.build_node("n1", rl("2", "4Gi"))],
                  pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1")],
                  pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="q")], queues=[m.Queue(name="q")])
    out = pyoracle.allocate(c)
    assert out["binds"] == {}
    assert out["fit_errors"] == {"c1/pg1": {"c1-p1": {"node(s) pod number exceeded": 1}}}


def test_scalar_resource_names():  # core/v1/helper/helpers.go:36-104
    for name, exp in [("nvidia.com/gpu", True), ("hugepages-2Mi", True), ("kubernetes.io/foo", True),
                      ("attachable-volumes-aws-ebs", True), ("cpu", False), ("ephemeral-storage", False),
                      ("requests.foo/bar", False), ("foo", False)]:
        assert pyoracle.resource_op("IsScalarResourceName", name=name)["result"] is exp, name


@pytest.mark.parametrize("exprs,labels,valid,exp", [  # labels/selector.go:133-236
    ([{"key": "zone", "operator": "In", "values": ["a", "b"]}], {"zone": "a"}, True, True),
    ([{"key": "zone", "operator": "NotIn", "values": ["a"]}], {}, True, True),
    ([{"key": "zone", "operator": "Exists"}], {"zone": ""}, True, True),
    ([{"key": "zone", "operator": "DoesNotExist"}], {"zone": "x"}, True, False),
    ([{"key": "cores", "operator": "Gt", "values": ["8"]}], {"cores": "16"}, True, True),
    ([{"key": "cores", "operator": "Lt", "values": ["8"]}], {"cores": "x16"}, True, False),
    ([{"key": "cores", "operator": "Gt", "values": ["eight"]}], {"cores": "16"}, False, False),
    ([{"key": "zone", "operator": "In", "values": []}], {"zone": "a"}, False, False),
    ([{"key": "bad key!", "operator": "Exists"}], {}, False, False),
    ([], {"zone": "a"}, True, False),  # NodeSelectorRequirementsAsSelector([]) = Nothing()
])
def test_selector_semantics(exprs, labels, valid, exp):
    r = pyoracle.resource_op("SelectorMatches", exprs=exprs, labels=labels)
    assert r["valid"] is valid and r["result"] is exp


# --- pkg/scheduler/api/job_info_test.go ------------------------------------
def _api_pod(ns, name, node, phase, cpu, mem):  # api/test_utils.go:71-94 (UID "<ns>-<name>")
    return m.Pod(ns=ns, name=name, uid=f"{ns}-{name}", node=node, phase=phase,
                 containers=[m.Container(req=m.canon_resource_list({"cpu": cpu, "memory": mem}))]).to_json()


def _cm(r):
    return (r["cpu"], r["memory"])


def test_job_add_task_info():  # TestAddTaskInfo :35-102
    pods = [_api_pod("c1", "p1", "", "Pending", "1000m", "1G"), _api_pod("c1", "p2", "n1", "Running", "2000m", "2G"),
            _api_pod("c1", "p3", "n1", "Pending", "1000m", "1G"), _api_pod("c1", "p4", "n1", "Pending", "1000m", "1G")]
    r = pyoracle.resource_op("JobTasks", pods=pods)
    assert _cm(r["allocated"]) == (4000, 4e9)
    assert _cm(r["total_request"]) == (5000, 5e9)
    assert r["status_index"] == {"Pending": ["c1-p1"], "Bound": ["c1-p3", "c1-p4"], "Running": ["c1-p2"]}
    assert r["tasks"] == ["c1-p1", "c1-p2", "c1-p3", "c1-p4"]


@pytest.mark.parametrize("ns,pods,rm", [  # TestDeleteTaskInfo :104-200
    ("c1", [("p1", "", "Pending", "1000m", "1G"), ("p2", "n1", "Running", "2000m", "2G"),
            ("p3", "n1", "Running", "3000m", "3G")], "p2"),
    ("c2", [("p1", "", "Pending", "1000m", "1G"), ("p2", "n1", "Pending", "2000m", "2G"),
            ("p3", "n1", "Running", "3000m", "3G")], "p2"),
])
def test_job_delete_task_info(ns, pods, rm):
    ps = {p[0]: _api_pod(ns, *p) for p in pods}
    r = pyoracle.resource_op("JobTasks", pods=list(ps.values()), remove=[ps[rm]])
    assert _cm(r["allocated"]) == (3000, 3e9)
    assert _cm(r["total_request"]) == (4000, 4e9)
    assert r["status_index"] == {"Pending": [f"{ns}-p1"], "Running": [f"{ns}-p3"]}
    assert r["tasks"] == [f"{ns}-p1", f"{ns}-p3"]


# --- pkg/scheduler/cache/cache_test.go -------------------------------------
@pytest.mark.parametrize("pods_first", [False, True])  # TestAddPod :128-188 (node first), TestAddNode :190-259
def test_cache_node_and_job_state(pods_first):
    """The cache's NodeInfo for n1 holds the running pod p2 (Idle 1000m / 9G, Used 1000m / 1G) whichever of
    node and pods arrives first, and the job holds both tasks. The session snapshot is built from the final
    state only (cache/cache.go:584-654), so the arrival order cannot change it."""
    node = m.build_node("n1", m.canon_resource_list({"cpu": "2000m", "memory": "10G"})).to_json()
    p1 = _api_pod("c1", "p1", "", "Pending", "1000m", "1G")
    p2 = _api_pod("c1", "p2", "n1", "Running", "1000m", "1G")
    r = pyoracle.resource_op("NodeTasks", node=node, pods=[p2])
    assert _cm(r["idle"]) == (1000, 9e9) and _cm(r["used"]) == (1000, 1e9) and r["tasks"] == ["c1/p2"]
    j = pyoracle.resource_op("JobTasks", pods=[p2, p1] if pods_first else [p1, p2])
    assert j["tasks"] == ["c1-p1", "c1-p2"]
    assert _cm(j["allocated"]) == (1000, 1e9) and _cm(j["total_request"]) == (2000, 2e9)


def test_cache_pods_without_job_are_not_scheduled():  # TestGetOrCreateJob :261-306 (group-annotated part)
    """A pod that belongs to a job (pi1) becomes a task of a session job; a pod with no job of its own (pi3,
    other scheduler) does not, so allocate never places it. The shadow-PodGroup case (pi2) is out of scope
    (DESIGN.md §8)."""
    rl = m.build_resource_list
    c = m.Cluster(nodes=[m.build_node("n1", dict(rl("2", "4Gi"), pods=10))],
                  pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "j1"),
                        m.build_pod("c3", "p3", "", "Pending", rl("1", "1G"), "")],
                  pod_groups=[m.PodGroup(ns="c1", name="j1", queue="q")], queues=[m.Queue(name="q")])
    out = pyoracle.allocate(c)
    assert out["binds"] == {"c1/p1": "n1"}
    assert out["status"]["c3-p3"] == "Pending"


# --- pkg/scheduler/util_test.go ---------------------------------------------
def test_load_scheduler_conf():  # TestLoadSchedulerConf :27-120
    conf = """
actions: "allocate, backfill"
tiers:
- plugins:
  - name: priority
  - name: gang
  - name: conformance
- plugins:
  - name: drf
  - name: predicates
  - name: proportion
  - name: nodeorder
"""
    actions, tiers = m.load_scheduler_conf(conf)
    assert actions == ["allocate", "backfill"]
    expected = [[m.plugin(n) for n in ("priority", "gang", "conformance")],
                [m.plugin(n) for n in ("drf", "predicates", "proportion", "nodeorder")]]
    assert [t["plugins"] for t in tiers] == expected
    for t in tiers:
        for p in t["plugins"]:
            assert all(p[f] is True for f in m.PLUGIN_FLAGS)
    # the default conf (util.go:30-40) is the tier set the benchmarks and parity clusters use
    assert m.load_scheduler_conf(m.DEFAULT_SCHEDULER_CONF) == (["allocate", "backfill"], m.default_tiers())
    # an explicit false survives the defaults; an unknown action is an error (util.go:62-69)
    _, t2 = m.load_scheduler_conf("actions: allocate\ntiers:\n- plugins:\n  - name: gang\n    enableJobReady: false\n")
    assert t2[0]["plugins"][0]["enabledJobReady"] is False and t2[0]["plugins"][0]["enabledJobOrder"] is True
    with pytest.raises(ValueError):
        m.load_scheduler_conf("actions: allocate, shuffle\n")
