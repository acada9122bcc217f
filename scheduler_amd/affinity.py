"""Inter-pod (anti)affinity tables for the device (rows a6 / a9 of SURVEY.md §8).

The reference evaluates pod (anti)affinity per (task, node) by scanning the pod lister
(vendor/.../predicates/predicates.go:1155-1465, metadata.go:310-526) and, for the score, by looping over
every node for every matching (pod, term) (priorities/interpod_affinity.go:119-241). Both only ever ask
"is there a matching pod in this node's topology domain", so they restate exactly as counts per
topology domain:

* topology slot   : a tuple of label keys; a node's domain id is the interned tuple of its values for
                    those keys (-1 when a key is missing: NodesHaveSameTopologyKey is false then,
                    priorities/util/topologies.go:53-71).
* count table     : counts per domain of one slot (+ a total), of lister pods (allocated-status tasks,
                    plugins/util/util.go:57-130) that
    EXISTING_ANTI - carry a given required anti-affinity term (satisfiesExistingPodsAntiAffinity,
                    predicates.go:1293-1333: the incoming pod fails in every domain with a count > 0
                    when it matches the term's namespaces + selector);
    ANTI          - match all required anti-affinity terms of a spec (predicates.go:1431-1440);
    AFFINITY      - match all required affinity terms of a spec (predicates.go:1414-1430, 1444-1457:
                    no domain match fails unless no lister pod matches anywhere (total = 0) and the
                    pod matches its own terms, metadata.go:498-510).
* IPA histogram   : for spec s and topology key k, H[s,k][v] = sum of the weights every existing pod in
                    domain v contributes to s for terms on key k (incoming soft terms +-w, existing hard
                    affinity +1, existing soft terms +-w; interpod_affinity.go:150-187); a node's count is
                    the sum over k of H[s,k][domain_k(node)], then normalised over all nodes (:221-238).

Commits update the tables: an Allocate adds the task to the lister (PodLister.UpdateTask,
util.go:108-130; Pipelined tasks are not listed), every commit adds the pod to its node for the score
(nodeorder.go:161-172). Those updates are precomputed per spec as increment lists.

Inputs the device path does not express raise `export.Unsupported` (invalid selectors, required terms
with an empty topologyKey, lister pods on nodes outside the session): the reference returns an error for
those per node; here the snapshot is refused, there is no fallback.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

# kbgpu.h
AFF_EXISTING_ANTI, AFF_ANTI, AFF_AFFINITY = 0, 1, 2
AFF_SELF_DYNAMIC = 1 << 0

AFF_TABLE_DTYPE = np.dtype([("slot", "<i4"), ("cnt_off", "<u4")], align=True)
AFF_CHECK_DTYPE = np.dtype([("table", "<i4"), ("kind", "<i4")], align=True)
IPA_HIST_DTYPE = np.dtype([("slot", "<i4"), ("h_off", "<u4")], align=True)
IPA_INCR_DTYPE = np.dtype([("slot", "<i4"), ("h_off", "<u4"), ("weight", "<i4"), ("pad", "<i4")], align=True)
AFF_SPEC_DTYPE = np.dtype([("check_off", "<u4"), ("check_cnt", "<u4"), ("lister_off", "<u4"),
                           ("lister_cnt", "<u4"), ("hist_off", "<u4"), ("hist_cnt", "<u4"),
                           ("incr_off", "<u4"), ("incr_cnt", "<u4"), ("self_match", "<i4"),
                           ("flags", "<u4")], align=True)
assert AFF_SPEC_DTYPE.itemsize == 40 and IPA_INCR_DTYPE.itemsize == 16


# ---- labels.Selector from a metav1.LabelSelector (apimachinery/pkg/apis/meta/v1/helpers.go:34-77) ----
NOTHING = None          # nil selector: matches nothing
EVERYTHING = ()         # empty selector: matches everything


def label_selector(sel, unsupported):
    """Canonical requirement tuple; `unsupported` is raised for selectors the reference rejects
    (LabelSelectorAsSelector returns an error: the predicate fails with an error string per node)."""
    from .export import is_qualified_name, is_valid_label_value
    if sel is None:
        return NOTHING
    ml = sel.get("matchLabels") or {}
    ex = sel.get("matchExpressions") or []
    if not ml and not ex:
        return EVERYTHING
    reqs = []
    for k, v in ml.items():
        if not is_qualified_name(k) or not is_valid_label_value(v):
            raise unsupported(f"invalid label selector {k}={v}")
        reqs.append((k, "In", (v,)))
    for e in ex:
        op, k, vs = e.get("operator"), e.get("key", ""), tuple(e.get("values") or [])
        if op not in ("In", "NotIn", "Exists", "DoesNotExist") or not is_qualified_name(k):
            raise unsupported(f"invalid label selector expression {e}")
        if op in ("In", "NotIn") and not vs or op in ("Exists", "DoesNotExist") and vs:
            raise unsupported(f"invalid label selector expression {e}")
        if not all(is_valid_label_value(v) for v in vs):
            raise unsupported(f"invalid label selector value in {e}")
        reqs.append((k, op, tuple(sorted(set(vs)))))
    return tuple(sorted(reqs))


def selector_matches(reqs, labels) -> bool:  # labels.internalSelector.Matches (selector.go:185-236)
    if reqs is NOTHING:
        return False
    for k, op, vs in reqs:
        has = k in labels
        if op == "In":
            if not has or labels[k] not in vs:
                return False
        elif op == "NotIn":
            if has and labels[k] in vs:
                return False
        elif op == "Exists":
            if not has:
                return False
        elif has:  # DoesNotExist
            return False
    return True


class Term:
    """A PodAffinityTerm resolved against its owner pod (namespaces default to the owner's,
    priorities/util/topologies.go:28-38)."""
    __slots__ = ("ns", "sel", "key")

    def __init__(self, owner_ns, d, unsupported):
        self.ns = frozenset(d.get("namespaces") or [owner_ns])
        self.sel = label_selector(d.get("labelSelector"), unsupported)
        self.key = d.get("topologyKey", "")

    def ident(self):
        return (self.ns, self.sel)

    def matches(self, ns, labels) -> bool:  # PodMatchesTermsNamespaceAndSelector (topologies.go:42-51)
        return ns in self.ns and selector_matches(self.sel, labels)


class PodAff:
    """The pod (anti)affinity of one pod, resolved."""
    __slots__ = ("has_pod", "has_anti", "req_aff", "pref_aff", "req_anti", "pref_anti")

    def __init__(self, pod, unsupported):
        a = pod.affinity or {}
        pa, paa = a.get("podAffinity"), a.get("podAntiAffinity")
        self.has_pod, self.has_anti = pa is not None, paa is not None
        pa, paa = pa or {}, paa or {}
        self.req_aff = [Term(pod.ns, t, unsupported) for t in pa.get("required") or []]
        self.req_anti = [Term(pod.ns, t, unsupported) for t in paa.get("required") or []]
        self.pref_aff = [(int(w.get("weight", 0)), Term(pod.ns, w.get("podAffinityTerm") or {}, unsupported))
                         for w in pa.get("preferred") or []]
        self.pref_anti = [(int(w.get("weight", 0)), Term(pod.ns, w.get("podAffinityTerm") or {}, unsupported))
                          for w in paa.get("preferred") or []]

    def any(self):
        return bool(self.req_aff or self.req_anti or self.pref_aff or self.pref_anti)


def pod_ident(pod):
    return (pod.ns, tuple(sorted(pod.labels.items())))


def _candidates(terms, index, universe):
    """Identities that can match every term: intersect the label index over each term's In requirements."""
    cand = None
    for t in terms:
        if t.sel is NOTHING:
            return set()
        best = None
        for k, op, vs in t.sel:
            if op == "In":
                s = set()
                for v in vs:
                    s |= index.get((k, v), set())
                best = s if best is None or len(s) < len(best) else best
        if best is None:
            continue
        cand = best if cand is None else cand & best
    return set(universe) if cand is None else cand


def _all_match(terms, ns, labels):
    return all(t.matches(ns, labels) for t in terms)


class Tables:
    """Builds the kb_affinity arrays for a Snapshot (export.Snapshot calls `build`)."""

    def __init__(self, snap, unsupported):
        self.snap = snap
        self.U = unsupported
        n = snap.n_nodes
        self.n = n
        self.slot_ids = {}        # key tuple -> slot
        self.slot_doms = []       # [slot] np.int32[n]
        self.slot_D = []
        self.tables = {}          # table key -> id
        self.table_slot = []
        self.table_kind = []

    # ---- topology slots ----
    def slot(self, keys):
        keys = tuple(keys)
        s = self.slot_ids.get(keys)
        if s is not None:
            return s
        s = self.slot_ids[keys] = len(self.slot_doms)
        ids, dom = {}, np.full(self.n, -1, np.int32)
        for i, nd in enumerate(self.snap.nodes):
            labels = nd["node"].labels
            if all(k in labels for k in keys):
                dom[i] = ids.setdefault(tuple(labels[k] for k in keys), len(ids))
        self.slot_doms.append(dom)
        self.slot_D.append(len(ids))
        return s

    def table(self, key, keys, kind):
        t = self.tables.get(key)
        if t is None:
            t = self.tables[key] = len(self.table_slot)
            self.table_slot.append(self.slot(keys))
            self.table_kind.append(kind)
        return t

    def build(self):
        snap, U = self.snap, self.U
        node_index = snap.node_index
        # lister pods: allocated-status session tasks (NewPodLister, util.go:57-82)
        from .export import allocated_status
        lister = [t for t in snap.session_tasks if allocated_status(t["status"])]
        for t in lister:
            if t["pod"].node not in node_index:
                raise U("lister pod on a node outside the session (predicates.go: failed to find node)")
        # existing pods per session node (schedulercache NodeInfo pods, for the score)
        existing = [(t, i) for i, nd in enumerate(snap.nodes) for t in nd["tasks"]]
        pending_specs = {}
        for t in snap.session_tasks:
            if "spec" in t and t["status"] == 1:
                pending_specs.setdefault(t["spec"], t["pod"])
        m = len(snap.spec_arr)
        spec_pod = [pending_specs[s] for s in range(m)]
        aff_cache = {}

        def paff(pod):
            k = id(pod)
            a = aff_cache.get(k)
            if a is None:
                a = aff_cache[k] = PodAff(pod, U)
            return a

        for a in (paff(p) for p in spec_pod):
            for t in a.req_aff + a.req_anti:
                if not t.key:
                    raise U("required pod (anti)affinity term with an empty topologyKey")

        # ---- predicate tables ----
        checks = [[] for _ in range(m)]
        lister_incr = [[] for _ in range(m)]
        self_match = [0] * m
        e_classes = {}  # (ns, sel, key) -> table id
        for t in lister:
            for term in paff(t["pod"]).req_anti:
                if term.key:
                    e_classes.setdefault((term.ns, term.sel, term.key), None)
        for s in range(m):
            for term in paff(spec_pod[s]).req_anti:
                if term.key:
                    e_classes.setdefault((term.ns, term.sel, term.key), None)
        for ck in list(e_classes):
            e_classes[ck] = self.table(("E",) + ck, (ck[2],), AFF_EXISTING_ANTI)
        # which specs match each existing-anti class (the incoming pod is matched against the term)
        spec_ids = [pod_ident(p) for p in spec_pod]
        for (ns, sel, key), tid in e_classes.items():
            term = Term.__new__(Term)
            term.ns, term.sel, term.key = ns, sel, key
            for s in range(m):
                if term.matches(spec_pod[s].ns, spec_pod[s].labels):
                    checks[s].append((tid, AFF_EXISTING_ANTI))
        for s in range(m):
            a = paff(spec_pod[s])
            if a.req_anti:
                tid = self.table(("B", tuple(t.ident() for t in a.req_anti), tuple(t.key for t in a.req_anti)),
                                 tuple(t.key for t in a.req_anti), AFF_ANTI)
                checks[s].append((tid, AFF_ANTI))
            if a.has_pod and a.req_aff:
                tid = self.table(("C", tuple(t.ident() for t in a.req_aff), tuple(t.key for t in a.req_aff)),
                                 tuple(t.key for t in a.req_aff), AFF_AFFINITY)
                checks[s].append((tid, AFF_AFFINITY))
                self_match[s] = int(_all_match(a.req_aff, spec_pod[s].ns, spec_pod[s].labels))
        # B/C tables: which identities (lister or pending) match all their terms
        bc = {}  # table id -> list of terms
        for s in range(m):
            a = paff(spec_pod[s])
            if a.req_anti:
                bc[self.tables[("B", tuple(t.ident() for t in a.req_anti), tuple(t.key for t in a.req_anti))]] = \
                    a.req_anti
            if a.has_pod and a.req_aff:
                bc[self.tables[("C", tuple(t.ident() for t in a.req_aff), tuple(t.key for t in a.req_aff))]] = \
                    a.req_aff
        # identities of lister pods (with their nodes) and of pending specs
        lid = defaultdict(list)
        for t in lister:
            lid[pod_ident(t["pod"])].append(node_index[t["pod"].node])
        index = defaultdict(set)
        for ident in set(lid) | set(spec_ids):
            for k, v in ident[1]:
                index[(k, v)].add(ident)
        n_tab = len(self.table_slot)
        cnt_off = np.zeros(n_tab, np.int64)
        off = 0
        for tid in range(n_tab):
            cnt_off[tid] = off
            off += max(1, self.slot_D[self.table_slot[tid]])
        counters = np.zeros(off, np.int64)
        totals = np.zeros(n_tab, np.int64)

        def add_nodes(tid, nodes):
            dom = self.slot_doms[self.table_slot[tid]][np.asarray(nodes, np.int64)]
            ok = dom >= 0
            np.add.at(counters, cnt_off[tid] + dom[ok], 1)
            totals[tid] += len(nodes)

        for t in lister:  # existing-anti classes carried by lister pods
            for term in paff(t["pod"]).req_anti:
                if term.key:
                    add_nodes(e_classes[(term.ns, term.sel, term.key)], [node_index[t["pod"].node]])
        spec_by_ident = defaultdict(list)
        for s, ident in enumerate(spec_ids):
            spec_by_ident[ident].append(s)
        for tid, terms in bc.items():
            for ident in _candidates(terms, index, set(lid) | set(spec_ids)):
                ns, labels = ident[0], dict(ident[1])
                if not _all_match(terms, ns, labels):
                    continue
                if ident in lid:
                    add_nodes(tid, lid[ident])
                for s in spec_by_ident.get(ident, []):
                    lister_incr[s].append(tid)
        for s in range(m):
            for term in paff(spec_pod[s]).req_anti:
                if term.key:
                    lister_incr[s].append(e_classes[(term.ns, term.sel, term.key)])
            lister_incr[s] = sorted(set(lister_incr[s]))

        # ---- InterPodAffinity histograms ----
        # identities for the score carry the pod's own terms too
        def sid(pod):
            return (pod.ns, tuple(sorted(pod.labels.items())), repr((pod.affinity or {}).get("podAffinity")),
                    repr((pod.affinity or {}).get("podAntiAffinity")))
        e_nodes = defaultdict(list)
        e_pod = {}
        for t, i in existing:
            k = sid(t["pod"])
            e_nodes[k].append(i)
            e_pod.setdefault(k, t["pod"])
        spec_sid = [sid(p) for p in spec_pod]
        for s, k in enumerate(spec_sid):
            e_pod.setdefault(k, spec_pod[s])
        all_e = list(e_pod)
        e_index = defaultdict(set)
        for k in all_e:
            for lk, lv in k[1]:
                e_index[(lk, lv)].add(k)
        s_index = defaultdict(set)
        for s, p in enumerate(spec_pod):
            for lk, lv in p.labels.items():
                s_index[(lk, lv)].add(s)
        W = defaultdict(lambda: defaultdict(int))  # (s, e) -> {key: weight}
        for s in range(m):
            a = paff(spec_pod[s])
            terms = ([(w, t) for w, t in a.pref_aff] if a.has_pod else []) + \
                    ([(-w, t) for w, t in a.pref_anti] if a.has_anti else [])
            for w, term in terms:
                if not term.key or w == 0:
                    continue
                for k in _candidates([term], e_index, all_e):
                    if term.matches(k[0], dict(k[1])):
                        W[(s, k)][term.key] += w
        for k in all_e:
            a = paff(e_pod[k])
            terms = []
            if a.has_pod:
                terms += [(1, t) for t in a.req_aff] + [(w, t) for w, t in a.pref_aff]
            if a.has_anti:
                terms += [(-w, t) for w, t in a.pref_anti]
            for w, term in terms:
                if not term.key or w == 0:
                    continue
                for s in _candidates([term], s_index, range(m)):
                    if term.matches(spec_pod[s].ns, spec_pod[s].labels):
                        W[(s, k)][term.key] += w
        hist_keys = defaultdict(set)
        for (s, k), kw in W.items():
            for key, w in kw.items():
                if w:
                    hist_keys[s].add(key)
        hists = [[] for _ in range(m)]
        h_off = {}
        hoff = 0
        for s in range(m):
            for key in sorted(hist_keys[s]):
                sl = self.slot((key,))
                h_off[(s, key)] = hoff
                hists[s].append((sl, hoff))
                hoff += max(1, self.slot_D[sl])
        H = np.zeros(hoff, np.int64)
        incr = [[] for _ in range(m)]
        sid_specs = defaultdict(list)
        for s, k in enumerate(spec_sid):
            sid_specs[k].append(s)
        for (s, k), kw in W.items():
            for key, w in kw.items():
                if not w:
                    continue
                sl = self.slot((key,))
                if k in e_nodes:
                    dom = self.slot_doms[sl][np.asarray(e_nodes[k], np.int64)]
                    ok = dom >= 0
                    np.add.at(H, h_off[(s, key)] + dom[ok], w)
                for sigma in sid_specs.get(k, []):
                    incr[sigma].append((sl, h_off[(s, key)], w))

        # ---- flags and packing ----
        own_h = [set(o for _, o in hists[s]) for s in range(m)]
        flags = [0] * m
        for s in range(m):
            mine = set(t for t, _ in checks[s])
            if mine & set(lister_incr[s]) or any(o in own_h[s] for _, o, _ in incr[s]):
                flags[s] |= AFF_SELF_DYNAMIC
        lim = (1 << 31) - 1
        if counters.size and np.abs(counters).max() > lim or H.size and np.abs(H).max() > lim or \
                totals.size and totals.max() > lim:
            raise U("affinity counts exceed int32")
        self.topo_dom = np.stack(self.slot_doms).astype(np.int32) if self.slot_doms else np.zeros((0, self.n), np.int32)
        self.table_arr = np.array([(self.table_slot[t], cnt_off[t]) for t in range(n_tab)], AFF_TABLE_DTYPE) \
            if n_tab else np.zeros(0, AFF_TABLE_DTYPE)
        self.counters = counters.astype(np.int32)
        self.totals = totals.astype(np.int32)
        spec_rows, chk, lst, hst, inc = [], [], [], [], []
        for s in range(m):
            spec_rows.append((len(chk), len(checks[s]), len(lst), len(lister_incr[s]), len(hst), len(hists[s]),
                              len(inc), len(incr[s]), self_match[s], flags[s]))
            chk += checks[s]
            lst += lister_incr[s]
            hst += hists[s]
            inc += [(sl, o, w, 0) for sl, o, w in incr[s]]
        self.spec_arr = np.array(spec_rows, AFF_SPEC_DTYPE) if spec_rows else np.zeros(0, AFF_SPEC_DTYPE)
        self.check_arr = np.array(chk, AFF_CHECK_DTYPE) if chk else np.zeros(0, AFF_CHECK_DTYPE)
        self.lister_arr = np.array(lst, np.int32)
        self.hist_arr = np.array(hst, IPA_HIST_DTYPE) if hst else np.zeros(0, IPA_HIST_DTYPE)
        self.h = H.astype(np.int32)
        self.incr_arr = np.array(inc, IPA_INCR_DTYPE) if inc else np.zeros(0, IPA_INCR_DTYPE)
        self.n_self_dynamic = sum(1 for f in flags if f & AFF_SELF_DYNAMIC)
        return self
