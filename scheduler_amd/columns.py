"""Columnar session export: the session snapshot built from columns in vectorised steps.

The reference opens a session by cloning every node and job (cache.Snapshot, cache/cache.go:584-654), and its
plugins build their node maps and pod lister (GenerateNodeMapAndSlice, NewPodLister: plugins/util/util.go:57-82,
186-198). The Go shim of INTEGRATION.md walks those objects once into flat columns with interned strings; this
module is what happens after that walk, for the whole session at once:

  Columns  -- nodes as columns (allocatable per resource, label value ids per label key, taint-set ids, condition
              flags), pods as columns (template id, pod group, node, task status, creation time, uid), and the
              distinct pod templates (a template: everything in a pod spec the scheduler reads -- requests,
              init containers, ports, selector, tolerations, (anti)affinity, labels, namespace, priority).
  build()  -- the same arrays as export.Snapshot: node rows (Idle / Releasing / Used from the pods on each node,
              NodeInfo.AddTask, api/node_info.go:165-193), the task specs (one SpecTable entry per template),
              the session arrays and the inter-pod affinity tables (affinity.Tables over template groups).

Per-pod work is numpy over the pod columns; Python runs per template and per distinct label value only.
columns_of(cluster) converts a model.Cluster (per pod, for tests); synth.c3_columns / c4_columns build the
bench configurations' columns directly. tests/test_columns.py checks build(columns_of(cl)) == export.Snapshot(cl)
array by array on every parity, affinity and edge cluster.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Tuple

import numpy as np

from . import export as E
from . import model as M

ALLOCATED = (E.ST["Bound"], E.ST["Binding"], E.ST["Running"], E.ST["Allocated"])
TERMINAL = (E.ST["Succeeded"], E.ST["Failed"])
POD_NODE_NONE, POD_NODE_UNKNOWN = -1, -2


@dataclass
class Columns:
    node_name: List[str]
    node_alloc: Dict[str, np.ndarray]           # resource -> int64[N] (0 where absent)
    node_alloc_has: Dict[str, np.ndarray]       # scalar resource -> bool[N]: the key is present (map semantics)
    node_labels: Dict[str, Tuple[np.ndarray, List[str]]]  # key -> (value id int32[N], -1 absent; values)
    node_taint: np.ndarray                      # int32[N] -> taint_sets
    taint_sets: List[List[dict]]
    node_flags: np.ndarray                      # uint32[N]: conditions, unschedulable, pressure (E.NODE_*)
    templates: List[M.Pod]
    pod_tpl: np.ndarray                         # int32[P]
    pod_group: np.ndarray                       # int32[P] -> pod_groups, -1: none
    pod_node: np.ndarray                        # int32[P] -> node, -1: none, -2: a node outside the cluster
    pod_status: np.ndarray                      # int32[P] task status (getTaskStatus, api/helpers.go:35-69)
    pod_ctime: np.ndarray                       # int64[P]
    pod_uid: np.ndarray                         # str[P]
    pod_groups: List[M.PodGroup] = field(default_factory=list)
    queues: List[M.Queue] = field(default_factory=list)
    tiers: list = field(default_factory=list)


def node_flags(node: M.Node) -> int:
    """The kb node flags of conditions, unschedulable and pressure (export.Snapshot._node_table)."""
    f = 0
    for c in node.conditions:  # CheckNodeConditionPredicate (predicates.go:1568-1596)
        typ, st = c.get("type"), c.get("status")
        if typ == "Ready" and st != "True":
            f |= E.NODE_NOT_READY
        elif typ == "OutOfDisk" and st != "False":
            f |= E.NODE_OUT_OF_DISK
        elif typ == "NetworkUnavailable" and st != "False":
            f |= E.NODE_NET_UNAVAIL
    if node.unschedulable:
        f |= E.NODE_UNSCHEDULABLE
    press = {}
    for c in node.conditions:  # schedulercache SetNode keeps the last of each (cache/node_info.go:613-626)
        if c.get("type") in ("MemoryPressure", "DiskPressure", "PIDPressure"):
            press[c["type"]] = c.get("status")
    if press.get("MemoryPressure") == "True":
        f |= E.NODE_MEM_PRESSURE
    if press.get("DiskPressure") == "True":
        f |= E.NODE_DISK_PRESSURE
    if press.get("PIDPressure") == "True":
        f |= E.NODE_PID_PRESSURE
    return f


def template_key(p: M.Pod):
    return repr((p.ns, sorted(p.labels.items()), p.priority, [(c.req, c.ports) for c in p.containers],
                 [(c.req, c.ports) for c in p.init], sorted(p.node_selector.items()), p.tolerations, p.affinity))


def _node_columns(nodes) -> dict:
    """The node half of Columns from per-node objects."""
    n = len(nodes)
    res_names = sorted({k for nd in nodes for k in nd.alloc})
    alloc = {k: np.array([nd.alloc.get(k, 0) for nd in nodes], np.int64) for k in res_names}
    has = {k: np.array([k in nd.alloc for nd in nodes], bool) for k in res_names if E.is_scalar_resource_name(k)}
    labels = {}
    for k in sorted({k for nd in nodes for k in nd.labels}):
        vals, ids = {}, np.full(n, -1, np.int32)
        for i, nd in enumerate(nodes):
            if k in nd.labels:
                ids[i] = vals.setdefault(nd.labels[k], len(vals))
        labels[k] = (ids, list(vals))
    tsets, tix = {}, np.zeros(n, np.int32)
    for i, nd in enumerate(nodes):
        tix[i] = tsets.setdefault(repr(nd.taints), (len(tsets), nd.taints))[0]
    taint_sets = [t for _, t in sorted(tsets.values(), key=lambda x: x[0])]
    return dict(node_name=[nd.name for nd in nodes], node_alloc=alloc, node_alloc_has=has, node_labels=labels,
                node_taint=tix, taint_sets=taint_sets, node_flags=np.array([node_flags(nd) for nd in nodes], np.uint32))


def columns_of_blocks(nodes, blocks, pod_groups, queues, tiers) -> Columns:
    """Columns from per-node objects and pod blocks, without per-pod objects: a block is (template pod, uids,
    node indices or None) -- pods that share one template (the first pod of the block: its spec, status and group),
    in pod order. Templates are deduplicated by template_key in block order, as columns_of does per pod, so
    build(columns_of_blocks(...)) equals build(columns_of(cluster)) for the cluster those pods make up."""
    nc = _node_columns(nodes)
    pg_ix = {(g.ns, g.name): i for i, g in enumerate(pod_groups)}
    tpls, tpl_ix = [], {}
    parts = {"tpl": [], "group": [], "node": [], "status": [], "ctime": [], "uid": []}
    for tp, uids, where in blocks:
        k = template_key(tp)
        t = tpl_ix.get(k)
        if t is None:
            t = tpl_ix[k] = len(tpls)
            tpls.append(tp)
        m = len(uids)
        g = -1
        if tp.group:
            g = pg_ix.get((tp.ns, tp.group), -1) if (tp.ns, tp.group) in pg_ix else -3
        parts["tpl"].append(np.full(m, t, np.int32))
        parts["group"].append(np.full(m, g, np.int32))
        parts["node"].append(np.full(m, -1, np.int32) if where is None else np.asarray(where, np.int32))
        parts["status"].append(np.full(m, E.task_status(tp), np.int32))
        parts["ctime"].append(np.full(m, tp.ctime, np.int64))
        parts["uid"].append(np.asarray(uids))
    cat = {k: (np.concatenate(v) if v else np.zeros(0)) for k, v in parts.items()}
    return Columns(**nc, templates=tpls, pod_tpl=cat["tpl"].astype(np.int32), pod_group=cat["group"].astype(np.int32),
                   pod_node=cat["node"].astype(np.int32), pod_status=cat["status"].astype(np.int32),
                   pod_ctime=cat["ctime"].astype(np.int64), pod_uid=cat["uid"], pod_groups=list(pod_groups),
                   queues=list(queues), tiers=tiers)


def columns_of(cl: M.Cluster) -> Columns:
    """A model.Cluster as columns (per pod and per node: the Go shim's walk, for tests)."""
    nc = _node_columns(cl.nodes)
    name_ix = {nd.name: i for i, nd in enumerate(cl.nodes)}
    pg_ix = {(g.ns, g.name): i for i, g in enumerate(cl.pod_groups)}
    tpls, tpl_ix = [], {}
    P = len(cl.pods)
    pod_tpl, pod_group, pod_node = np.zeros(P, np.int32), np.full(P, -1, np.int32), np.full(P, -1, np.int32)
    pod_status, pod_ctime = np.zeros(P, np.int32), np.zeros(P, np.int64)
    for i, p in enumerate(cl.pods):
        k = template_key(p)
        t = tpl_ix.get(k)
        if t is None:
            t = tpl_ix[k] = len(tpls)
            tpls.append(p)
        pod_tpl[i] = t
        if p.group:
            pod_group[i] = pg_ix.get((p.ns, p.group), -1) if (p.ns, p.group) in pg_ix else -3
        if p.node:
            pod_node[i] = name_ix.get(p.node, POD_NODE_UNKNOWN)
        pod_status[i] = E.task_status(p)
        pod_ctime[i] = p.ctime
    return Columns(**nc, templates=tpls, pod_tpl=pod_tpl, pod_group=pod_group, pod_node=pod_node, pod_status=pod_status, pod_ctime=pod_ctime,
                   pod_uid=np.array([p.uid for p in cl.pods]), pod_groups=list(cl.pod_groups),
                   queues=list(cl.queues), tiers=cl.tiers)


def isum(idx, v, n):
    """Per-bin sums of int64 values, exact: np.bincount accumulates its weights in float64, exact only while every
    partial sum stays below 2^53 (export.Snapshot sums in exact ints); past that, np.add.at in int64."""
    if not len(idx):
        return np.zeros(n, np.int64)
    if v is None:
        return np.bincount(idx, minlength=n).astype(np.int64)
    v = np.asarray(v, np.int64)
    if int(np.abs(v).sum(dtype=np.float64)) < (1 << 52):
        return np.bincount(idx, weights=v, minlength=n).astype(np.int64)
    out = np.zeros(n, np.int64)
    np.add.at(out, idx, v)
    return out


class ColumnarSnapshot:
    """export.Snapshot's arrays from Columns (no per-task dicts: session_tasks / jobs are ranges)."""

    def __init__(self, c: Columns):
        self.c = c
        self._templates()
        self._nodes()
        self._jobs()
        E.Snapshot._config(self)  # the plugin configuration (the exporter's own code, over self.cluster.tiers)
        self._specs()
        self._node_table()
        self.aff = None
        if self.aff_in_play:
            from .affinity import Tables
            self.aff = Tables(self, E.Unsupported).build()
        self._session_arrays()

    # the plugin configuration reads self.cluster.tiers
    @property
    def cluster(self):
        return self

    @property
    def tiers(self):
        return self.c.tiers

    # ---------------- templates: requests, non-zero requests, affinity ----------------
    def _templates(self):
        memo = {}
        self.t_rr, self.t_ir, self.t_nz, self.t_paff, self.t_prio = [], [], [], [], []
        for p in self.c.templates:
            rr = E.Res()
            for ct in p.containers:
                rr.add(E.Res.of_request(ct.req, memo))
            ir = rr.copy()
            for ct in p.init:
                ir.set_max(E.Res.of_request(ct.req, memo))
            nzc = nzm = 0
            for ct in p.containers:
                a, b = E.nonzero(ct.req)
                nzc += a
                nzm += b
            self.t_rr.append(rr)
            self.t_ir.append(ir)
            self.t_nz.append((nzc, nzm))
            self.t_paff.append(E.has_pod_affinity(p))
            self.t_prio.append(p.priority if p.priority is not None else 1)
        T = len(self.c.templates)
        self.t_cpu = np.array([r.cpu for r in self.t_rr], np.int64).reshape(T)
        self.t_mem = np.array([r.mem for r in self.t_rr], np.int64).reshape(T)
        self.t_nzc = np.array([a for a, _ in self.t_nz], np.int64).reshape(T)
        self.t_nzm = np.array([b for _, b in self.t_nz], np.int64).reshape(T)

    # ---------------- nodes: NewNodeInfo + AddTask per pod on the node; keep used <= allocatable ----------------
    def _nodes(self):
        c = self.c
        N = len(c.node_name)
        live = (c.pod_node >= 0) & ~np.isin(c.pod_status, TERMINAL)
        self.live = live
        on = c.pod_node[live]
        tp = c.pod_tpl[live]
        st = c.pod_status[live]
        rel_m = st == E.ST["Releasing"]
        pip_m = st == E.ST["Pipelined"]
        z = np.zeros(N, np.int64)
        a_cpu = c.node_alloc.get(M.CPU, z)
        a_mem = c.node_alloc.get(M.MEMORY, z)
        w = lambda v, m=None: isum(on if m is None else on[m], None if v is None else (v if m is None else v[m]), N)
        cpu, mem = self.t_cpu[tp], self.t_mem[tp]
        idle_cpu = a_cpu - w(cpu, ~pip_m)
        idle_mem = a_mem - w(mem, ~pip_m)
        rel_cpu = w(cpu, rel_m) - w(cpu, pip_m)
        rel_mem = w(mem, rel_m) - w(mem, pip_m)
        used_cpu, used_mem = w(cpu), w(mem)
        # scalar resources (maps: a node's Idle has one when its allocatable lists a scalar)
        sc_names = sorted(set(c.node_alloc_has) | {k for r in self.t_rr for k in (r.sc or {})})
        S = len(sc_names)
        t_sc = np.zeros((max(1, len(self.t_rr)), S), np.int64)
        t_has = np.zeros(max(1, len(self.t_rr)), bool)
        for t, r in enumerate(self.t_rr):
            for k, v in (r.sc or {}).items():
                t_sc[t, sc_names.index(k)] = v
                t_has[t] = True
        a_has = np.zeros(N, bool)
        for k in c.node_alloc_has:
            a_has |= c.node_alloc_has[k]
        idle_sc, rel_sc, used_sc = np.zeros((S, N), np.int64), np.zeros((S, N), np.int64), np.zeros((S, N), np.int64)
        for j, k in enumerate(sc_names):
            v = t_sc[tp, j] if len(tp) else np.zeros(0, np.int64)
            idle_sc[j] = np.where(a_has, c.node_alloc.get(k, z) - w(v, ~pip_m), 0)
            rel_sc[j] = w(v, rel_m)
            used_sc[j] = w(v)
        rel_has = np.zeros(N, bool)
        if len(on):
            rel_has[on[rel_m & t_has[tp]]] = True
        # Resource.Sub asserts InitResreq <= Idle at every AddTask (resource_info.go:145-159): Idle only decreases,
        # so the last state decides; a pod with scalars on a node whose Idle has no map fails there too
        if (idle_cpu <= -E.MIN_CPU).any() or (idle_mem <= -E.MIN_MEM).any() or \
                (len(on) and (t_has[tp] & ~a_has[on]).any()) or (idle_sc[:, a_has] <= -E.MIN_SCALAR).any():
            raise E.AssertPanic("resource is not sufficient to do operation")
        if pip_m.any():
            raise E.Unsupported("Pipelined tasks at session open")  # (getTaskStatus never reports one)
        # Snapshot keeps the nodes whose Used fits their allocatable (LessEqual, used <= alloc)
        keep = (used_cpu - a_cpu < E.MIN_CPU) & (used_mem - a_mem < E.MIN_MEM)
        used_has = np.zeros(N, bool)  # Used gets a map from the first pod with scalars
        if len(on):
            used_has[on[t_has[tp]]] = True
        keep &= ~used_has | a_has  # Used with a map against an allocatable without one: False
        for j, k in enumerate(sc_names):
            ak = c.node_alloc_has.get(k, np.zeros(N, bool))
            keep &= ~used_has | (used_sc[j] - np.where(ak, c.node_alloc.get(k, z), 0) < E.MIN_SCALAR)
        names = np.array(c.node_name)
        order = np.argsort(names, kind="stable")
        kept = order[keep[order]]
        self.kept = kept
        self.n_nodes = n = len(kept)
        self.node_pos = np.full(N, -1, np.int64)
        self.node_pos[kept] = np.arange(n)
        self.node_names_arr = names[kept]
        self.sc_names = sc_names
        pos = self.node_pos[on]
        ok = pos >= 0
        self.cols_base = {
            "idle_cpu": idle_cpu[kept], "idle_mem": idle_mem[kept], "rel_cpu": rel_cpu[kept], "rel_mem": rel_mem[kept],
            "alloc_cpu": a_cpu[kept].astype(np.int64), "alloc_mem": a_mem[kept].astype(np.int64),
            "nz_cpu": isum(pos[ok], self.t_nzc[tp][ok], n),
            "nz_mem": isum(pos[ok], self.t_nzm[tp][ok], n),
            "pod_count": np.bincount(pos[ok], minlength=n).astype(np.int32),
            "max_pods": c.node_alloc.get(M.PODS, z)[kept].astype(np.int32),
            "flags": (c.node_flags[kept] | np.where(a_has[kept], E.NODE_IDLE_HAS_MAP, 0) |
                      np.where(rel_has[kept], E.NODE_REL_HAS_MAP, 0)).astype(np.uint32)}
        self.node_idle_sc = {k: idle_sc[j][kept] for j, k in enumerate(sc_names)}
        self.node_rel_sc = {k: rel_sc[j][kept] for j, k in enumerate(sc_names)}
        self.alloc_total = (int(a_cpu[kept].sum()), int(a_mem[kept].sum()),
                            {k: int(c.node_alloc.get(k, z)[kept][c.node_alloc_has[k][kept]].sum())
                             for k in c.node_alloc_has if c.node_alloc_has[k][kept].any()})
        # existing pods per session node (positions) in pod order, for the host ports and the affinity score
        self.live_pos = pos  # per live pod (-1: its node was dropped)
        self.live_tpl = tp
        self.live_idx = np.nonzero(live)[0]

    # ---------------- jobs and session order ----------------
    def _jobs(self):
        c = self.c
        qnames = {q.name for q in c.queues}
        valid = np.array([g.queue in qnames for g in c.pod_groups] + [False], bool)  # [-1] -> no group
        g = np.where(c.pod_group >= 0, c.pod_group, len(c.pod_groups))
        in_ssn = valid[g]
        pods = np.nonzero(in_ssn)[0]
        juid = [f"{g.ns}/{g.name}" for g in c.pod_groups]
        used = np.unique(c.pod_group[pods]) if len(pods) else np.zeros(0, np.int64)
        used = sorted(used.tolist(), key=lambda i: juid[i])
        jrank = np.full(len(c.pod_groups) + 1, -1, np.int64)
        jrank[used] = np.arange(len(used))
        self.job_groups = used
        self.jobs = range(len(used))
        r = jrank[c.pod_group[pods]]
        order = np.lexsort((pods, r))
        self.ssn_pods = pods[order]  # session task i -> pod index
        self.session_tasks = range(len(self.ssn_pods))
        qn = sorted({c.pod_groups[j].queue for j in used})
        self.queue_names = qn
        qd = {q.name: q for q in c.queues}
        self.queues = [qd[q] for q in qn]
        tp = c.pod_tpl[self.ssn_pods]
        on_kept = self.live_pos >= 0
        self.aff_in_play = bool(np.array(self.t_paff + [False])[tp].any() or
                                np.array(self.t_paff + [False])[self.live_tpl[on_kept]].any())

    # ---------------- task specs: one SpecTable entry per pending template, in first-occurrence order ----------------
    def _specs(self):
        c = self.c
        st = c.pod_status[self.ssn_pods]
        tp = c.pod_tpl[self.ssn_pods]
        pend = st == E.ST["Pending"]
        ptp = tp[pend]
        uniq, first = np.unique(ptp, return_index=True)
        firsts = uniq[np.argsort(first)]
        scal = set()
        for t in firsts:
            scal.update((self.t_ir[t].sc or {}).keys())
            scal.update((self.t_rr[t].sc or {}).keys())
        tab = E.SpecTable(sorted(scal), self.aff_in_play)
        t_spec = np.full(len(c.templates) + 1, -1, np.int32)
        for t in firsts:
            t_spec[t] = tab.add(c.templates[t], self.t_ir[t], self.t_rr[t])
        tab.finish(self)
        self.t_spec = t_spec
        self.s_task_spec = np.where(pend, t_spec[tp], -1).astype(np.int32)

    # ---------------- node SoA ----------------
    def _node_table(self):
        c, n = self.c, self.n_nodes
        S, K, P = len(self.scalars), len(self.label_keys.ids), len(self.port_slots.ids)
        cols = dict(self.cols_base)
        cols["idle_sc"] = np.zeros((S, n), np.int64)
        cols["rel_sc"] = np.zeros((S, n), np.int64)
        for s, name in enumerate(self.scalars):
            if name in self.node_idle_sc:
                cols["idle_sc"][s] = self.node_idle_sc[name]
                cols["rel_sc"][s] = self.node_rel_sc[name]
        cols["label_val"] = np.full((K, n), -1, np.int32)
        cols["label_int"] = np.zeros((K, n), np.int64)
        cols["label_int_ok"] = np.zeros((K, n), np.uint8)
        keycols = []
        for key, k in sorted(self.label_keys.ids.items(), key=lambda kv: kv[1]):
            if key == "\x00metadata.name":
                keycols.append((key, k, list(self.node_names_arr), np.arange(n)))
            elif key in c.node_labels:
                col, strs = c.node_labels[key]
                keycols.append((key, k, strs, col[self.kept]))
        # new values interned in the exporter's order: by node, then by key id
        seen = []
        for key, k, strs, ids in keycols:
            u, first = np.unique(ids, return_index=True)
            seen += [(int(f), k, strs[int(v)]) for v, f in zip(u, first) if v >= 0]
        for _, _, v in sorted(seen, key=lambda x: (x[0], x[1])):
            self.values(v)
        for key, k, strs, ids in keycols:
            present = ids >= 0
            lut = np.array([self.values.ids[v] for v in strs] + [-1], np.int32)
            cols["label_val"][k] = np.where(present, lut[ids], -1)
            if key in self.gtlt_keys:
                iv = [E.parse_int64(v) for v in strs] + [None]
                ok = np.array([x is not None for x in iv], bool)
                vals = np.array([x if x is not None else 0 for x in iv], np.int64)
                cols["label_int"][k] = np.where(present & ok[ids], vals[ids], 0)
                cols["label_int_ok"][k] = (present & ok[ids]).astype(np.uint8)
        # taint sets (NoSchedule / NoExecute taints, sorted) interned in node order as the exporter does
        taint_sets = E._Interner()
        taint_sets(())
        taint_list = [[]]
        canon = []
        for ts in c.taint_sets:
            canon.append(tuple(sorted((t.get("key", ""), t.get("value", ""), t.get("effect", "")) for t in ts
                                      if t.get("effect") in ("NoSchedule", "NoExecute"))))
        tix = c.node_taint[self.kept]
        set_id = np.zeros(len(canon), np.int32)
        u, first = np.unique(tix, return_index=True)
        for ti in u[np.argsort(first)]:  # in order of first appearance over the nodes
            tid = taint_sets(canon[ti])
            if tid == len(taint_list):
                taint_list.append([{"key": a, "value": b, "effect": e} for a, b, e in canon[ti]])
            set_id[ti] = tid
        cols["taint_set"] = set_id[tix] if n else np.zeros(0, np.int32)
        # existing pods' host ports in the slots a spec asks for (HostPortInfo.Add)
        cols["port_used"] = np.zeros((P, n), np.uint64)
        if P:
            ok = self.live_pos >= 0
            for t in np.unique(self.live_tpl[ok]):
                pairs = []
                for ct in c.templates[t].containers:
                    for pt in ct.ports:
                        hp = int(pt.get("hostPort", 0) or 0)
                        s_id = self.port_slots.ids.get((pt.get("protocol") or "TCP", hp)) if hp > 0 else None
                        if s_id is not None:
                            pairs.append((s_id, self.port_ips[s_id].ids.get(pt.get("hostIP") or "0.0.0.0", 63)))
                if pairs:
                    where = self.live_pos[ok & (self.live_tpl == t)]
                    for s_id, ipid in pairs:
                        np.bitwise_or.at(cols["port_used"][s_id], where, np.uint64(1 << ipid))
        self.cols = cols
        if not self.tol_list:
            self.tol_list.append([])
        self.tolerates = np.zeros((len(self.tol_list), len(taint_list)), np.uint8)
        for a, tols in enumerate(self.tol_list):
            for b, taints in enumerate(taint_list):
                self.tolerates[a, b] = all(any(E._tolerates(o, t) for o in tols) for t in taints)
        self.n_label, self.n_port = K, P

    # ---------------- affinity tables' inputs (affinity.Tables.build) ----------------
    def slot_domains(self, keys):
        n = self.n_nodes
        ids = np.zeros((len(keys), n), np.int64)
        present = np.ones(n, bool)
        for j, k in enumerate(keys):
            if k not in self.c.node_labels:
                return np.full(n, -1, np.int32), 0
            col = self.c.node_labels[k][0][self.kept]
            present &= col >= 0
            ids[j] = col
        if not present.any():
            return np.full(n, -1, np.int32), 0
        sub = ids[:, present].T
        _, first, inv = np.unique(sub, axis=0, return_index=True, return_inverse=True)
        rank = np.empty(len(first), np.int64)
        rank[np.argsort(first, kind="stable")] = np.arange(len(first))  # ids in order of first appearance
        dom = np.full(n, -1, np.int32)
        dom[present] = rank[inv.reshape(-1)]
        return dom, len(first)

    def aff_groups(self, unsupported):
        c = self.c
        st = c.pod_status[self.ssn_pods]
        lm = np.isin(st, ALLOCATED)
        lp = self.ssn_pods[lm]
        if len(lp) and ((c.pod_node[lp] < 0) | (self.node_pos[np.maximum(c.pod_node[lp], 0)] < 0)).any():
            raise unsupported("lister pod on a node outside the session (predicates.go: failed to find node)")
        ltp = c.pod_tpl[lp]
        lister = []
        if len(lp):
            uniq, first = np.unique(ltp, return_index=True)
            for t in uniq[np.argsort(first)]:
                m = ltp == t
                lister.append((c.templates[t], self.node_pos[c.pod_node[lp[m]]].tolist(), c.pod_uid[lp[m]].tolist()))
        ok = self.live_pos >= 0
        pos, tp = self.live_pos[ok], self.live_tpl[ok]
        existing = []
        if len(pos):
            o = np.lexsort((self.live_idx[ok], pos))  # node order, then pod order
            tp_o = tp[o]
            uniq, first = np.unique(tp_o, return_index=True)
            for t in uniq[np.argsort(first)]:
                existing.append((c.templates[t], pos[o][tp_o == t].tolist()))
        m = len(self.spec_arr)
        spec_pod = [None] * m
        for t in range(len(c.templates)):
            s = self.t_spec[t]
            if s >= 0 and spec_pod[s] is None:
                spec_pod[s] = c.templates[t]
        return lister, existing, spec_pod

    # ---------------- session arrays (kb_session) ----------------
    def _session_arrays(self):
        c = self.c
        sp = self.ssn_pods
        tp = c.pod_tpl[sp]
        acc = set()
        for t in np.unique(tp):
            acc.update((self.t_rr[t].sc or {}).keys())
        acc.update(self.alloc_total[2].keys())
        self.acc_scalars = sorted(acc)
        if len(self.acc_scalars) > 62:
            raise E.Unsupported("more than 62 accounting scalar resources")
        aslot = {k: i for i, k in enumerate(self.acc_scalars)}
        R = 2 + len(self.acc_scalars)
        T = len(c.templates)
        t_res = np.zeros((max(1, T), R), np.float64)
        t_mask = np.zeros(max(1, T), np.uint64)
        for t, r in enumerate(self.t_rr):
            t_res[t, 0], t_res[t, 1] = r.cpu, r.mem
            mk = 0
            if r.sc is not None:
                mk |= 1 << 63
                for k, q in r.sc.items():
                    t_res[t, 2 + aslot[k]] = q
                    mk |= 1 << aslot[k]
            t_mask[t] = mk
        jrank = np.full(len(c.pod_groups) + 1, -1, np.int64)
        jrank[self.job_groups] = np.arange(len(self.job_groups))
        self.s_task_job = jrank[c.pod_group[sp]].astype(np.int32)
        self.s_task_status = c.pod_status[sp].astype(np.int32)
        self.s_task_priority = np.array(self.t_prio + [1], np.int32)[tp]
        self.s_task_ctime = c.pod_ctime[sp].astype(np.int64)
        uo = np.argsort(c.pod_uid[sp], kind="stable")
        self.s_task_uid_rank = np.empty(len(sp), np.int32)
        self.s_task_uid_rank[uo] = np.arange(len(sp), dtype=np.int32)
        self.s_task_resreq = t_res[tp] if len(sp) else np.zeros((0, R), np.float64)
        self.s_task_resreq_mask = t_mask[tp] if len(sp) else np.zeros(0, np.uint64)
        pgs = [c.pod_groups[j] for j in self.job_groups]
        q_idx = {q: i for i, q in enumerate(self.queue_names)}
        self.s_job_queue = np.array([q_idx[g.queue] for g in pgs], np.int32)
        self.s_job_priority = np.array([g.priority for g in pgs], np.int32)
        self.s_job_min = np.array([g.min_member for g in pgs], np.int32)
        self.s_job_ctime = np.array([g.ctime for g in pgs], np.int64)
        self.s_job_uid_rank = np.arange(len(pgs), dtype=np.int32)
        self.s_job_pg_pending = np.array([1 if g.phase == "Pending" else 0 for g in pgs], np.int32)
        self.s_queue_weight = np.array([q.weight for q in self.queues], np.int32)
        self.s_queue_ctime = np.array([q.ctime for q in self.queues], np.int64)
        self.s_queue_uid_rank = np.arange(len(self.queues), dtype=np.int32)
        tot = np.zeros(R, np.float64)
        tot[0], tot[1] = self.alloc_total[0], self.alloc_total[1]
        mk = 0
        if self.alloc_total[2]:
            mk |= 1 << 63
            for k, q in self.alloc_total[2].items():
                tot[2 + aslot[k]] = q
                mk |= 1 << aslot[k]
        self.s_total, self.s_total_mask = tot, mk
        dt = np.dtype([("tier", "<i4"), ("plugin", "<i4"), ("enable", "<u4"), ("pad", "<i4")])
        self.s_tiers = np.array([(ti, pid, en, 0) for ti, pid, en in self.tier_plugins], dt) \
            if self.tier_plugins else np.zeros(0, dt)

    def node_names(self):
        return list(self.node_names_arr)


def build(c: Columns) -> ColumnarSnapshot:
    return ColumnarSnapshot(c)
