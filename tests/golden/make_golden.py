"""Generate the golden fixtures under tests/golden/ (inputs + expected outputs, JSON).

Two kinds of fixture:
  * ref-*    : the reference's own unit-test vectors, restated as data. The expected values come from the
               reference's test files (file:line in "source"), NOT from the oracle. The Go reference cannot be
               built in this image (no Go toolchain), so these pin the oracle; they are the only outputs of
               the reference itself available here.
  * oracle-* : allocate outcomes of the oracle (oracle/oracle.cpp, the CPU restatement of the reference's
               allocate path) on small seeded clusters covering every predicate / priority / ordering feature
               the device path implements. They freeze the oracle's behaviour (a change to it shows up as a
               fixture diff) and let the GPU tests check the HIP path without running the oracle.

Run from the repo root:  python tests/golden/make_golden.py   (rewrites every fixture; commit the diff)
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

from oracle import pyoracle  # noqa: E402
from scheduler_amd import model as m  # noqa: E402
from scheduler_amd import synth  # noqa: E402

from helpers import _without, affinity_edge_cluster, edge_cluster  # noqa: E402


def _partial_gang(cl, frac):
    for pg in cl.pod_groups:
        pg.min_member = max(1, int(pg.min_member * frac))
    return cl


def _drf_proportion_tiers():  # allocate_test.go:180-195 (only the listed flags are set)
    return [{"plugins": [
        m.plugin("drf", defaults=False, enabledPreemptable=True, enabledJobOrder=True),
        m.plugin("proportion", defaults=False, enabledQueueOrder=True, enabledReclaimable=True),
    ]}]


def reference_cases():
    """(name, source, cluster, expected binds) restated from the reference's tests."""
    rl = m.build_resource_list
    one = m.Cluster(
        nodes=[m.build_node("n1", rl("2", "4Gi"))],
        pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1"),
              m.build_pod("c1", "p2", "", "Pending", rl("1", "1G"), "pg1")],
        pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="c1")],
        queues=[m.Queue(name="c1", weight=1)], tiers=_drf_proportion_tiers())
    two = m.Cluster(
        nodes=[m.build_node("n1", rl("2", "4G"))],
        pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1"),
              m.build_pod("c1", "p2", "", "Pending", rl("1", "1G"), "pg1"),
              m.build_pod("c2", "p1", "", "Pending", rl("1", "1G"), "pg2"),
              m.build_pod("c2", "p2", "", "Pending", rl("1", "1G"), "pg2")],
        pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="c1"), m.PodGroup(ns="c2", name="pg2", queue="c2")],
        queues=[m.Queue(name="c1", weight=1), m.Queue(name="c2", weight=1)], tiers=_drf_proportion_tiers())
    alloc = dict(rl("4", "8Gi"), pods=10)
    best = m.Cluster(nodes=[m.build_node(n, alloc) for n in ("node4", "node3")],
                     pods=[m.build_pod("c1", "p1", "", "Pending", rl("1", "1G"), "pg1")],
                     pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="q")], queues=[m.Queue(name="q")])
    return [
        ("ref-allocate-one-job", "pkg/scheduler/actions/allocate/allocate_test.go:45-86", one,
         {"c1/p1": "n1", "c1/p2": "n1"}),
        ("ref-allocate-two-jobs", "pkg/scheduler/actions/allocate/allocate_test.go:87-145", two,
         {"c2/p1": "n1", "c1/p1": "n1"}),
        # TestSelectBestNode (pkg/scheduler/util/scheduler_helper_test.go:26-63): the winner lies in the highest
        # score's node set; with the canonical lowest-index tie-break (name order) node3 wins.
        ("ref-select-best-node", "pkg/scheduler/util/scheduler_helper_test.go:26-63", best, {"c1/p1": "node3"}),
    ]


def oracle_cases():
    return [
        ("oracle-c1", synth.c1(n_nodes=40, n_jobs=8, tasks_per_job=10, seed=101)),
        ("oracle-c2", synth.c2(n_nodes=60, n_jobs=10, tasks_per_job=12, seed=102)),
        ("oracle-c2-fill", synth.c2(n_nodes=30, n_jobs=8, tasks_per_job=15, seed=103, fill=0.9)),
        ("oracle-c2-nogang", _without(synth.c2(n_nodes=30, n_jobs=6, tasks_per_job=8, seed=104), "gang")),
        ("oracle-c2-halfgang", _partial_gang(synth.c2(n_nodes=30, n_jobs=8, tasks_per_job=10, seed=105), 0.5)),
        ("oracle-c3", synth.c3(n_nodes=60, n_jobs=10, tasks_per_job=8, seed=106, n_zones=3, n_racks=12)),
        ("oracle-c4", synth.c4(n_nodes=40, n_jobs=8, tasks_per_job=6, n_zones=2, n_racks=8, n_pre=40,
                               pre_job_size=10, seed=107)),
        ("oracle-edge-mixed", edge_cluster()),
        ("oracle-aff-edge", affinity_edge_cluster()),
    ]


def outcome(out):
    return {"binds": out["binds"], "events": out["events"], "fit_errors": out["fit_errors"],
            "status": out["status"]}


def write(name, source, cluster, expected):
    doc = {"name": name, "source": source, "generator": "tests/golden/make_golden.py",
           "cluster": cluster.to_json(), "expected": expected}
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(doc, f, separators=(",", ":"), sort_keys=True)
        f.write("\n")


def main():
    for name, source, cl, binds in reference_cases():
        out = pyoracle.allocate(cl)
        assert out["binds"] == binds, (name, out["binds"])  # the oracle agrees with the reference's test
        write(name, source, cl, {"binds": binds})
    for name, cl in oracle_cases():
        write(name, "oracle/oracle.cpp (CPU restatement), seeded generator", cl, outcome(pyoracle.allocate(cl)))
    print("wrote", len(reference_cases()) + len(oracle_cases()), "fixtures to", HERE)


if __name__ == "__main__":
    main()
