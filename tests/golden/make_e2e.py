"""The reference's end-to-end scheduling expectations as fixtures.

The vendored k8s tests were pruned from the reference (Gopkg.toml:87), so the only expectations the
reference itself states for LeastRequested / NodeAffinity / InterPodAffinity / taints / host ports / max pods
are its e2e specs, which need a cluster:
  test/e2e/nodeorder.go:29-72    preferred NodeAffinity (weight 100) -> the pod lands on nodeNames[0]
  test/e2e/nodeorder.go:74-136   preferred pod affinity (weight 100, hostname) -> next to the labelled pod
  test/e2e/nodeorder.go:138-237  LeastRequested: two nodes loaded by pinned jobs -> the third node
  test/e2e/predicates.go:35-82   required NodeAffinity on the metadata.name field -> that node
  test/e2e/predicates.go:84-110  host port 28080, 2 x nodes replicas, minMember = nodes -> nodes bound, rest pending
  test/e2e/predicates.go:112-159 required pod affinity to its own labels (hostname), gang of computeNode's rep
                                 -> every pod on one node
  test/e2e/predicates.go:161-207 every node tainted NoSchedule -> pending; taints removed -> placed
  test/e2e/predicates.go:209-314 max pods: the node filled to its pod capacity by BestEffort pods pinned to
                                 it (backfill), then one more pinned pod -> pending
  test/e2e/predicates.go:316-525 70 % cpu fillers per node, then a job of 50 % of the largest node's cpu ->
                                 pending

Each scenario is restated as data: the cluster hack/run-e2e.sh brings up (kubeadm-dind, NUM_NODES=3: a tainted
master plus kube-node-1..3; node capacity chosen here: 4 cpu, 8Gi, 110 pods, since dind nodes report the host's),
the jobs the spec creates in order (util.go createJob: one PodGroup per job, minMember = sum of task.min, pods
named <job>-<i>), and the outcome the spec asserts after each scheduling cycle. The helpers the specs call
(getAllWorkerNodes, computeNode, clusterNodeNumber: util.go:586-712, 808-821) are evaluated here on the
restated cluster. Quirk kept as written: the memory fillers and the additional memory job of
predicates.go:422-521 request NewMilliQuantity(...) bytes, i.e. a thousandth of the intended memory, and
waitTimeoutPodGroupReady accepts either outcome, so the memory half asserts nothing (recorded as "any").

Run from the repo root:  python tests/golden/make_e2e.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GI = 1024 ** 3
CPU4, MEM8, PODS = 4000, 8 * GI, 110
MASTER_TAINT = {"key": "node-role.kubernetes.io/master", "value": "", "effect": "NoSchedule"}
WORKERS = ["kube-node-1", "kube-node-2", "kube-node-3"]
HOST = "kubernetes.io/hostname"


def nodes():
    out = [{"name": "kube-master", "alloc": {"cpu": CPU4, "memory": MEM8, "pods": PODS}, "taints": [MASTER_TAINT]}]
    out += [{"name": w, "alloc": {"cpu": CPU4, "memory": MEM8, "pods": PODS}, "taints": []} for w in WORKERS]
    return out


def host_in(name):
    return {"nodeAffinity": {"required": [{"matchExpressions": [{"key": HOST, "operator": "In", "values": [name]}]}]}}


def job(name, req, min_, rep, affinity=None, labels=None, hostport=0, pri=0):
    return {"name": name, "req": req, "min": min_, "rep": rep, "affinity": affinity, "labels": labels or {},
            "hostport": hostport, "priority": pri}


ONE, HALF = {"cpu": 1000}, {"cpu": 500}

NODEORDER = [
    {"name": "node-affinity", "source": "test/e2e/nodeorder.go:29-72", "nodes": nodes(), "steps": [
        {"create": job("pa-job", ONE, 1, 1, {"nodeAffinity": {"preferred": [
            {"weight": 100, "preference": {"matchExpressions": [{"key": HOST, "operator": "In",
                                                                  "values": [WORKERS[0]]}]}}]}})},
        {"cycle": [{"job": "pa-job", "bound": 1, "all_on": WORKERS[0]}]}]},
    {"name": "pod-affinity", "source": "test/e2e/nodeorder.go:74-136", "nodes": nodes(), "steps": [
        {"create": job("pa-job1", HALF, 1, 1, labels={"test": "e2e"})},
        {"cycle": [{"job": "pa-job1", "bound": 1}]},
        {"create": job("pa-job2", HALF, 1, 1, {"podAffinity": {"preferred": [
            {"weight": 100, "podAffinityTerm": {"labelSelector": {"matchExpressions": [
                {"key": "test", "operator": "In", "values": ["e2e"]}]}, "topologyKey": HOST}}]}})},
        {"cycle": [{"job": "pa-job2", "bound": 1, "with_job": "pa-job1"}]}]},
    {"name": "least-requested", "source": "test/e2e/nodeorder.go:138-237", "nodes": nodes(), "steps": [
        {"create": job("pa-job", HALF, 3, 3, host_in(WORKERS[0]))},
        {"cycle": [{"job": "pa-job", "bound": 3, "all_on": WORKERS[0]}]},
        {"create": job("pa-job1", HALF, 3, 3, host_in(WORKERS[1]))},
        {"cycle": [{"job": "pa-job1", "bound": 3, "all_on": WORKERS[1]}]},
        {"create": job("pa-test-job", ONE, 1, 1)},
        {"cycle": [{"job": "pa-test-job", "bound": 1, "none_on": [WORKERS[0], WORKERS[1]]}]}]},
]

# computeNode(oneCPU) on the restated cluster: the first untainted node in list (name) order, and how many
# oneCPU slots fit its allocatable (util.go:660-712)
CN_NODE, CN_REP = WORKERS[0], CPU4 // 1000

PREDICATES = [
    {"name": "node-affinity-field", "source": "test/e2e/predicates.go:35-82", "nodes": nodes(), "steps": [
        {"create": job("na-job", ONE, 1, 1, {"nodeAffinity": {"required": [{"matchFields": [
            {"key": "metadata.name", "operator": "In", "values": [CN_NODE]}]}]}})},
        {"cycle": [{"job": "na-job", "bound": 1, "all_on": CN_NODE}]}]},
    {"name": "hostport", "source": "test/e2e/predicates.go:84-110", "nodes": nodes(), "steps": [
        {"create": job("hp-job", ONE, len(WORKERS), 2 * len(WORKERS), hostport=28080)},
        {"cycle": [{"job": "hp-job", "bound": len(WORKERS), "pending": len(WORKERS), "distinct_nodes": True}]}]},
    {"name": "pod-affinity-required", "source": "test/e2e/predicates.go:112-159", "nodes": nodes(), "steps": [
        {"create": job("pa-job", ONE, CN_REP, CN_REP, {"podAffinity": {"required": [
            {"labelSelector": {"matchLabels": {"foo": "bar"}}, "topologyKey": HOST}]}}, labels={"foo": "bar"})},
        {"cycle": [{"job": "pa-job", "bound": CN_REP, "same_node": True}]}]},
    {"name": "taints-tolerations", "source": "test/e2e/predicates.go:161-207", "nodes": nodes(), "steps": [
        {"taint_all": {"key": "test-taint-key", "value": "test-taint-val", "effect": "NoSchedule"}},
        {"create": job("tt-job", ONE, 1, 1)},
        {"cycle": [{"job": "tt-job", "bound": 0}]},
        {"untaint_all": "test-taint-key"},
        {"cycle": [{"job": "tt-job", "bound": 1}]}]},
    {"name": "max-pods", "source": "test/e2e/predicates.go:209-314", "nodes": nodes(), "steps": [
        {"create": job("max-pods", {}, PODS, PODS, host_in(WORKERS[0]))},
        {"cycle": [{"job": "max-pods", "bound": PODS, "all_on": WORKERS[0]}]},
        {"create": job("unscheduled-pod", {}, 1, 1, host_in(WORKERS[0]))},
        {"cycle": [{"job": "unscheduled-pod", "bound": 0}]}]},
    {"name": "resource-limits", "source": "test/e2e/predicates.go:316-525", "nodes": nodes(), "steps":
        [{"create": job(f"cpu-filler-job-{w}", {"cpu": CPU4 * 7 // 10}, 1, 1, host_in(w), pri=1000)} for w in WORKERS]
        + [{"cycle": [{"job": f"cpu-filler-job-{w}", "bound": 1, "all_on": w} for w in WORKERS]}]
        # the memory fillers ask for NewMilliQuantity(mem * 7 / 10): mem * 7 / 10 milli-bytes, rounded up
        + [{"create": job(f"mem-filler-job-{w}", {"memory": -(-(MEM8 * 7 // 10) // 1000)}, 1, 1, host_in(w),
                          pri=1000)} for w in WORKERS]
        + [{"cycle": [{"job": f"mem-filler-job-{w}", "bound": 1, "all_on": w} for w in WORKERS]}]
        + [{"create": job("additional-job-cpu", {"cpu": CPU4 * 5 // 10}, 1, 1, pri=1000)},
           {"cycle": [{"job": "additional-job-cpu", "bound": 0}]},
           {"create": job("additional-job-mem", {"memory": -(-(CPU4 * 5 // 10) // 1000)}, 1, 1, pri=1000)},
           {"cycle": [{"job": "additional-job-mem", "any": True}]}]},
]


def main():
    for name, scen in (("nodeorder", NODEORDER), ("predicates", PREDICATES)):
        meta = {"source": "kube-batch test/e2e (reference); restated by tests/golden/make_e2e.py",
                "cluster": "hack/run-e2e.sh: kubeadm-dind, NUM_NODES=3 (a tainted master + 3 workers); "
                           "capacity 4 cpu / 8Gi / 110 pods chosen here",
                "actions": "allocate, backfill (config/kube-batch-conf.yaml; enqueue / reclaim / preempt are "
                           "outside the hot path and change nothing in these scenarios)",
                "scenarios": scen}
        with open(os.path.join(HERE, f"ref-e2e-{name}.json"), "w") as f:
            json.dump(meta, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
