"""Seeded synthetic clusters for the BASELINE.json configurations.

C1  1k nodes x 5k pods: 100 gang jobs x 50, gang+drf+predicates+nodeorder (the reference's CPU path)
C2  10k homogeneous nodes x 100k pods: 1k gang jobs x 100, resource fit + LeastRequested/Balanced
C3  20k heterogeneous nodes x 200k pods: GPU scalars, taints/tolerations, node selector/affinity
C4  10k nodes x 100k pods with inter-pod (anti)affinity over hostname / zone / rack domains
C5  50k nodes x 1M pods: the C2 shape scaled (the 8-GPU configuration)
C2M the C2 shape with ~2% two-template (PS/worker) jobs and ~2% jobs with inter-pod anti-affinity (a mixed cycle)

Every generator takes explicit sizes so tests can run "parity variants" (<= 1k x 5k) of the
same shapes. There is no network: all data is synthetic.
"""
from __future__ import annotations

import dataclasses

import numpy as np

from . import model as M

GI = 1024 ** 3
SEED = 20250217


class Parts:
    """A generated cluster before its pods exist: nodes, pod groups, queues and pod blocks. A block is (template pod,
    pod names, node indices or None): the pods of one job share everything but their name / uid (ns-name) and node,
    so the cluster (per-pod objects, expand()) and its columns (columns(): numpy per pod, objects per node and per
    job) come from the same draws."""

    def __init__(self):
        self.nodes, self.pod_groups, self.queues, self.blocks = [], [], [], []

    def cluster(self) -> M.Cluster:
        cl = M.Cluster(nodes=self.nodes, pod_groups=self.pod_groups, queues=self.queues)
        for tp, names, where in self.blocks:
            for i, nm in enumerate(names):
                cl.pods.append(dataclasses.replace(
                    tp, name=nm, uid=f"{tp.ns}-{nm}", node="" if where is None else self.nodes[int(where[i])].name,
                    labels=dict(tp.labels), containers=[M.Container(req=dict(c.req)) for c in tp.containers],
                    tolerations=[dict(x) for x in tp.tolerations], node_selector=dict(tp.node_selector)))
        return cl

    def columns(self):
        from . import columns as CL
        blocks = [(tp, [f"{tp.ns}-{nm}" for nm in names], where) for tp, names, where in self.blocks]
        return CL.columns_of_blocks(self.nodes, blocks, self.pod_groups, self.queues, M.Cluster().tiers)


def _block(parts, ns, names, group, req, node_ix=None, **kw):
    tp = M.Pod(ns=ns, name=names[0], uid=f"{ns}-{names[0]}", group=group, containers=[M.Container(req=dict(req))],
               node="" if node_ix is None else parts.nodes[int(node_ix[0])].name, **kw)
    parts.blocks.append((tp, names, node_ix))


def _queue_pg_parts(parts, n_jobs, min_member, queue="default", prefix="job", ns="ns"):
    parts.queues.append(M.Queue(name=queue, weight=1))
    for j in range(n_jobs):
        parts.pod_groups.append(M.PodGroup(ns=ns, name=f"{prefix}{j:05d}", queue=queue, min_member=min_member))


def c1_parts(n_nodes=1000, n_jobs=100, tasks_per_job=50, seed=SEED) -> Parts:
    """C1: 1k nodes {32 cores, 128Gi, 110 pods, hostname/zone/rack labels}; jobs of 50 identical tasks."""
    rng = np.random.default_rng(seed)
    pt = Parts()
    for i in range(n_nodes):
        pt.nodes.append(M.Node(name=f"node-{i:05d}", alloc={M.CPU: 32000, M.MEMORY: 128 * GI, M.PODS: 110},
                               labels={"kubernetes.io/hostname": f"node-{i:05d}", "zone": f"z{i % 10}",
                                       "rack": f"r{i % 100}"}))
    _queue_pg_parts(pt, n_jobs, tasks_per_job)
    cpus, mems = [500, 1000, 2000], [1 * GI, 2 * GI, 4 * GI]
    for j in range(n_jobs):
        req = {M.CPU: int(rng.choice(cpus)), M.MEMORY: int(rng.choice(mems))}
        _block(pt, "ns", [f"job{j:05d}-{t:04d}" for t in range(tasks_per_job)], f"job{j:05d}", req)
    return pt


def c1(n_nodes=1000, n_jobs=100, tasks_per_job=50, seed=SEED) -> M.Cluster:
    return c1_parts(n_nodes, n_jobs, tasks_per_job, seed).cluster()


def c2(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=SEED, fill=None) -> M.Cluster:
    """C2: homogeneous nodes {64 cores, 256Gi, 110 pods}; per-job cpu U{250..4000 step 250}m, mem U{0.5..8}Gi.

    fill=f rescales node capacity so the workload needs ~f of the cpu (f=0.9 exercises no-fit)."""
    rng = np.random.default_rng(seed)
    cpu_cap, mem_cap = 64000, 256 * GI
    cpus = rng.integers(1, 17, n_jobs) * 250
    mems = rng.integers(1, 17, n_jobs) * (GI // 2)
    if fill is not None:
        need = float((cpus * tasks_per_job).sum())
        cpu_cap = max(4000, int(need / fill / n_nodes) // 1000 * 1000)
    pt = Parts()
    for i in range(n_nodes):
        pt.nodes.append(M.Node(name=f"node-{i:05d}", alloc={M.CPU: cpu_cap, M.MEMORY: mem_cap, M.PODS: 110}))
    _queue_pg_parts(pt, n_jobs, tasks_per_job)
    for j in range(n_jobs):
        _block(pt, "ns", [f"job{j:05d}-{t:04d}" for t in range(tasks_per_job)], f"job{j:05d}",
               {M.CPU: int(cpus[j]), M.MEMORY: int(mems[j])})
    return pt.cluster()


def c3_parts(n_nodes=20000, n_jobs=2000, tasks_per_job=100, seed=SEED, n_zones=20, n_racks=400) -> Parts:
    """C3: 4 node classes; 25% GPU nodes (nvidia.com/gpu=8, taint gpu=true:NoSchedule); 5% maint:NoExecute.
    Jobs: 20% request GPUs and tolerate gpu; 30% required zone affinity; 30% preferred terms; 10% nodeSelector."""
    rng = np.random.default_rng(seed)
    classes = [(16000, 64 * GI, "small"), (32000, 128 * GI, "medium"), (64000, 256 * GI, "large"),
               (96000, 512 * GI, "xlarge")]
    pt = Parts()
    for i in range(n_nodes):
        cpu, mem, typ = classes[int(rng.integers(0, 4))]
        alloc = {M.CPU: cpu, M.MEMORY: mem, M.PODS: 110}
        taints = []
        if rng.random() < 0.25:
            alloc[M.GPU_RESOURCE_NAME] = 8000  # milli-units (resource_info.go:89-91)
            taints.append({"key": "gpu", "value": "true", "effect": "NoSchedule"})
        if rng.random() < 0.05:
            taints.append({"key": "maint", "value": "", "effect": "NoExecute"})
        zone = f"zone-{int(rng.integers(0, n_zones)):02d}"
        pt.nodes.append(M.Node(name=f"node-{i:05d}", alloc=alloc, taints=taints,
                               labels={"zone": zone, "rack": f"rack-{int(rng.integers(0, n_racks)):03d}",
                                       "node-type": typ, "kubernetes.io/hostname": f"node-{i:05d}"}))
    _queue_pg_parts(pt, n_jobs, tasks_per_job)
    for j in range(n_jobs):
        req = {M.CPU: int(rng.integers(1, 17)) * 250, M.MEMORY: int(rng.integers(1, 17)) * (GI // 2)}
        tol, sel, aff = [], {}, None
        kind = rng.random()
        if kind < 0.2:
            req[M.GPU_RESOURCE_NAME] = int(rng.integers(1, 9)) * 1000
            tol = [{"key": "gpu", "operator": "Equal", "value": "true", "effect": "NoSchedule"}]
        r2 = rng.random()
        if r2 < 0.3:
            zones = sorted({f"zone-{int(z):02d}" for z in rng.integers(0, n_zones, 3)})
            aff = {"nodeAffinity": {"required": [{"matchExpressions": [
                {"key": "zone", "operator": "In", "values": zones}]}]}}
        elif r2 < 0.6:
            prefs = []
            for _ in range(int(rng.integers(1, 4))):
                prefs.append({"weight": int(rng.integers(1, 101)), "preference": {"matchExpressions": [
                    {"key": "rack", "operator": "In",
                     "values": [f"rack-{int(r):03d}" for r in rng.integers(0, n_racks, 4)]}]}})
            aff = {"nodeAffinity": {"preferred": prefs}}
        elif r2 < 0.7:
            sel = {"node-type": classes[int(rng.integers(0, 4))][2]}
        _block(pt, "ns", [f"job{j:05d}-{t:04d}" for t in range(tasks_per_job)], f"job{j:05d}", req,
               tolerations=[dict(x) for x in tol], node_selector=dict(sel), affinity=aff)
    return pt


def c3(n_nodes=20000, n_jobs=2000, tasks_per_job=100, seed=SEED, n_zones=20, n_racks=400) -> M.Cluster:
    return c3_parts(n_nodes, n_jobs, tasks_per_job, seed, n_zones, n_racks).cluster()


def c4_parts(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=SEED, n_zones=10, n_racks=100, n_pre=None,
             pre_job_size=100) -> Parts:
    """C4: nodes {64 cores, 256Gi, 110 pods} in n_zones zones x n_racks racks (contiguous), plus n_pre
    running pods (default n_nodes) in running gang jobs labelled job=<name>, app=svc|web. Services (app=svc)
    run only in the first 30% of the zones; the first service also carries required anti-affinity
    (hostname) and preferred anti-affinity (zone, w=10) against noisy=true pods.
    Pending jobs: 30% required podAntiAffinity (hostname) to their own job label, 30% preferred
    podAffinity (rack, w=50) to their own job label, 20% required podAffinity (zone) to app=svc, 20% plain;
    10% of the jobs are noisy=true."""
    rng = np.random.default_rng(seed)
    n_pre = n_nodes if n_pre is None else n_pre
    pt = Parts()
    racks_per_zone = max(1, n_racks // n_zones)
    for i in range(n_nodes):
        rack = i * n_racks // n_nodes
        pt.nodes.append(M.Node(name=f"node-{i:05d}", alloc={M.CPU: 64000, M.MEMORY: 256 * GI, M.PODS: 110},
                               labels={"kubernetes.io/hostname": f"node-{i:05d}",
                                       "zone": f"z{min(n_zones - 1, rack // racks_per_zone)}",
                                       "rack": f"r{rack}"}))
    pt.queues.append(M.Queue(name="default", weight=1))
    # running jobs (lister pods)
    n_pre_jobs = max(1, n_pre // pre_job_size)
    svc_nodes = max(1, int(n_nodes * 0.3))
    for j in range(n_pre_jobs):
        name = f"pre{j:04d}"
        svc = j % 5 == 0
        pt.pod_groups.append(M.PodGroup(ns="ns", name=name, queue="default", min_member=pre_job_size,
                                        phase="Running"))
        aff = None
        if j == 0:
            noisy = {"labelSelector": {"matchLabels": {"noisy": "true"}}}
            aff = {"podAntiAffinity": {
                "required": [dict(noisy, topologyKey="kubernetes.io/hostname")],
                "preferred": [{"weight": 10, "podAffinityTerm": dict(noisy, topologyKey="zone")}]}}
        where = np.array([int(rng.integers(0, svc_nodes if svc else n_nodes)) for _ in range(pre_job_size)], np.int64)
        _block(pt, "ns", [f"{name}-{t:04d}" for t in range(pre_job_size)], name, {M.CPU: 1000, M.MEMORY: 2 * GI},
               node_ix=where, phase="Running", labels={"job": name, "app": "svc" if svc else "web"}, affinity=aff)
    # pending jobs
    for j in range(n_jobs):
        name = f"job{j:05d}"
        pt.pod_groups.append(M.PodGroup(ns="ns", name=name, queue="default", min_member=tasks_per_job))
        req = {M.CPU: int(rng.integers(1, 9)) * 250, M.MEMORY: int(rng.integers(1, 9)) * (GI // 2)}
        labels = {"job": name}
        if rng.random() < 0.1:
            labels["noisy"] = "true"
        own = {"labelSelector": {"matchLabels": {"job": name}}}
        kind = rng.random()
        aff = None
        if kind < 0.3:
            aff = {"podAntiAffinity": {"required": [dict(own, topologyKey="kubernetes.io/hostname")]}}
        elif kind < 0.6:
            aff = {"podAffinity": {"preferred": [{"weight": 50, "podAffinityTerm": dict(own, topologyKey="rack")}]}}
        elif kind < 0.8:
            aff = {"podAffinity": {"required": [{"labelSelector": {"matchLabels": {"app": "svc"}},
                                                 "topologyKey": "zone"}]}}
        _block(pt, "ns", [f"{name}-{t:04d}" for t in range(tasks_per_job)], name, req, labels=dict(labels),
               affinity=aff)
    return pt


def c4(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=SEED, n_zones=10, n_racks=100, n_pre=None,
       pre_job_size=100) -> M.Cluster:
    return c4_parts(n_nodes, n_jobs, tasks_per_job, seed, n_zones, n_racks, n_pre, pre_job_size).cluster()


def c2m_parts(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=SEED, frac_multi=0.02, frac_aff=0.02,
              fill=None) -> Parts:
    """C2M: the C2 shape with a mixed job population: C2's nodes (plus a hostname label) and
    per-job requests, where ~frac_multi of the jobs have two pod templates (a PS/worker job: 10% of its tasks are
    'ps' pods with their own request, ordered before the workers -- two runs of two specs in one job) and ~frac_aff
    of the jobs carry required pod anti-affinity to their own pods over hostname (one pod per node: inter-pod
    terms, which the resident engine does not run). The rest are C2 jobs."""
    rng = np.random.default_rng(seed)
    cpu_cap, mem_cap = 64000, 256 * GI
    cpus = rng.integers(1, 17, n_jobs) * 250
    mems = rng.integers(1, 17, n_jobs) * (GI // 2)
    kind = rng.random(n_jobs)
    if fill is not None:  # as c2: node capacity for ~1/fill of the cpu the jobs ask for
        cpu_cap = max(4000, int(float((cpus * tasks_per_job).sum()) / fill / n_nodes) // 1000 * 1000)
    pt = Parts()
    for i in range(n_nodes):
        pt.nodes.append(M.Node(name=f"node-{i:05d}", alloc={M.CPU: cpu_cap, M.MEMORY: mem_cap, M.PODS: 110},
                               labels={"kubernetes.io/hostname": f"node-{i:05d}"}))
    _queue_pg_parts(pt, n_jobs, tasks_per_job)
    n_ps = max(1, tasks_per_job // 10)
    for j in range(n_jobs):
        name = f"job{j:05d}"
        req = {M.CPU: int(cpus[j]), M.MEMORY: int(mems[j])}
        if kind[j] < frac_multi:  # PS / worker: two templates ("-ps-" sorts before "-wk-": ps pods first)
            _block(pt, "ns", [f"{name}-ps-{t:04d}" for t in range(n_ps)], name, {M.CPU: 2000, M.MEMORY: 4 * GI},
                   labels={"job": name, "role": "ps"})
            _block(pt, "ns", [f"{name}-wk-{t:04d}" for t in range(tasks_per_job - n_ps)], name, req,
                   labels={"job": name, "role": "worker"})
        elif kind[j] < frac_multi + frac_aff:  # spread: one pod of the job per node
            _block(pt, "ns", [f"{name}-{t:04d}" for t in range(tasks_per_job)], name, req, labels={"job": name},
                   affinity={"podAntiAffinity": {"required": [
                       {"labelSelector": {"matchLabels": {"job": name}}, "topologyKey": "kubernetes.io/hostname"}]}})
        else:
            _block(pt, "ns", [f"{name}-{t:04d}" for t in range(tasks_per_job)], name, req)
    return pt


def c2m(**kw) -> M.Cluster:
    return c2m_parts(**kw).cluster()


def c2m_columns(**kw):
    return c2m_parts(**kw).columns()


def c1_columns(**kw):
    """synth.c1's columns straight from the generator's draws (no per-pod objects: columns.columns_of_blocks)."""
    return c1_parts(**kw).columns()


def c3_columns(**kw):
    return c3_parts(**kw).columns()


def c4_columns(**kw):
    return c4_parts(**kw).columns()


CONFIGS = {"C1": c1, "C2": c2, "C3": c3, "C4": c4, "C2M": c2m}
COLUMNS = {"C1": c1_columns, "C3": c3_columns, "C4": c4_columns, "C2M": c2m_columns}


class ArraySnapshot:
    """The export.Snapshot arrays of a C2-shaped cluster built directly with numpy (no per-pod objects), for
    the large configurations (C2 at full size, C5: 50k nodes x 1M pods). Same arrays as
    export.Snapshot(c2(...)) -- tests/test_export.py checks that field by field."""

    def __init__(self, **kw):
        self.__dict__.update(kw)


def c2_snapshot(n_nodes=10000, n_jobs=1000, tasks_per_job=100, seed=SEED, fill=None) -> ArraySnapshot:
    """export.Snapshot(c2(n_nodes, n_jobs, tasks_per_job, seed, fill)) without building the cluster."""
    from . import export as E
    rng = np.random.default_rng(seed)  # the same draws, in the same order, as c2()
    cpu_cap, mem_cap = 64000, 256 * GI
    cpus = rng.integers(1, 17, n_jobs) * 250
    mems = rng.integers(1, 17, n_jobs) * (GI // 2)
    if fill is not None:
        need = float((cpus * tasks_per_job).sum())
        cpu_cap = max(4000, int(need / fill / n_nodes) // 1000 * 1000)
    proto = E.Snapshot(c2(n_nodes=1, n_jobs=1, tasks_per_job=1, seed=seed))  # defaults: config, tiers, tables
    n = n_nodes
    z = lambda dt, *s: np.zeros(s, dtype=dt)
    cols = {"idle_cpu": np.full(n, cpu_cap, np.int64), "idle_mem": np.full(n, mem_cap, np.int64),
            "rel_cpu": z(np.int64, n), "rel_mem": z(np.int64, n),
            "alloc_cpu": np.full(n, cpu_cap, np.int64), "alloc_mem": np.full(n, mem_cap, np.int64),
            "nz_cpu": z(np.int64, n), "nz_mem": z(np.int64, n), "idle_sc": z(np.int64, 0, n),
            "rel_sc": z(np.int64, 0, n), "pod_count": z(np.int32, n), "max_pods": np.full(n, 110, np.int32),
            "flags": z(np.uint32, n), "label_val": z(np.int32, 0, n), "label_int": z(np.int64, 0, n),
            "label_int_ok": z(np.uint8, 0, n), "taint_set": z(np.int32, n), "port_used": z(np.uint64, 0, n)}
    # one spec per distinct (cpu, mem), numbered in first-occurrence order (export._specs dedupes by signature)
    pair = cpus.astype(np.int64) * (1 << 40) + mems.astype(np.int64)
    uniq, first, inv = np.unique(pair, return_index=True, return_inverse=True)
    order = np.argsort(first)
    rank = np.empty_like(order)
    rank[order] = np.arange(len(order))
    job_spec = rank[inv].astype(np.int32)
    m = len(uniq)
    spec_arr = np.zeros(m, E.SPEC_DTYPE)
    spec_arr[:] = proto.spec_arr[0]
    j0 = first[order]
    for f, v in (("init_cpu", cpus), ("req_cpu", cpus), ("nz_cpu", cpus), ("init_mem", mems), ("req_mem", mems),
                 ("nz_mem", mems)):
        spec_arr[f] = v[j0]
    nt = n_jobs * tasks_per_job
    task_job = np.repeat(np.arange(n_jobs, dtype=np.int32), tasks_per_job)
    resreq = np.zeros((nt, 2), np.float64)
    resreq[:, 0] = np.repeat(cpus, tasks_per_job)
    resreq[:, 1] = np.repeat(mems, tasks_per_job)
    total = np.array([float(cpu_cap) * n, float(mem_cap) * n])
    return ArraySnapshot(
        n_nodes=n, cols=cols, config=dict(proto.config), scalars=[], n_label=0, n_port=0,
        spec_arr=spec_arr, sc_init=np.zeros(0, np.int64), sc_req=np.zeros(0, np.int64),
        term_arr=proto.term_arr, req_arr=proto.req_arr, val_arr=proto.val_arr, port_arr=proto.port_arr,
        tolerates=proto.tolerates, aff=None, acc_scalars=[],
        session_tasks=range(nt), jobs=range(n_jobs), queues=proto.queues,
        s_task_job=task_job, s_task_spec=job_spec[task_job], s_task_status=np.full(nt, E.ST["Pending"], np.int32),
        s_task_priority=np.ones(nt, np.int32), s_task_ctime=np.zeros(nt, np.int64),
        s_task_uid_rank=np.arange(nt, dtype=np.int32), s_task_resreq=resreq,
        s_task_resreq_mask=np.zeros(nt, np.uint64),
        s_job_queue=np.zeros(n_jobs, np.int32), s_job_priority=np.full(n_jobs, proto.s_job_priority[0], np.int32),
        s_job_min=np.full(n_jobs, tasks_per_job, np.int32), s_job_ctime=np.zeros(n_jobs, np.int64),
        s_job_uid_rank=np.arange(n_jobs, dtype=np.int32), s_job_pg_pending=np.zeros(n_jobs, np.int32),
        s_queue_weight=proto.s_queue_weight, s_queue_ctime=proto.s_queue_ctime,
        s_queue_uid_rank=proto.s_queue_uid_rank, s_total=total, s_total_mask=proto.s_total_mask,
        s_tiers=proto.s_tiers)
