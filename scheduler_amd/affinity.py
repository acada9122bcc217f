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

Where the reference's predicate returns a plain error instead of a failure reason, the node fails with
that error's string (FitErrors.SetNodeError, api/unschedule_info.go:40-54). Those cases are tables too,
checked with KB_AFF_ERROR (the device reports KB_R_HOST_ERROR; `host_error_string` below gives the string):
    XB            - lister pods carrying a required anti-affinity term with an invalid selector
                    (satisfiesExistingPodsAntiAffinity errors for every node, predicates.go:1302-1313);
    ALL           - every lister pod: a pod whose own required affinity has an invalid selector errors as
                    soon as the lister has a pod (podMatchesPodAffinityTerms, :1189-1214, 1401-1413), and
                    its invalid required anti-affinity fails every node (:1431-1440);
    C / B prefix  - a required term with an empty topologyKey errors (affinity) or fails (anti-affinity)
                    where every earlier term's topology is shared (:1205-1212): the table's slot is the key
                    tuple before the first empty key.
An invalid selector among the terms CalculateInterPodAffinityPriority meets makes the batch score error,
and SelectBestNode then panics (KB_SPEC_IPA_ERROR). Still refused (export.Unsupported): lister pods on
nodes outside the session, and a pending pod with invalid score terms whose own evaluation may not error.
"""
from __future__ import annotations

from collections import defaultdict

import numpy as np

# kbgpu.h
AFF_EXISTING_ANTI, AFF_ANTI, AFF_AFFINITY, AFF_ERROR = 0, 1, 2, 3
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


class Invalid(str):
    """LabelSelectorAsSelector's error (the text the reference puts into its error strings)."""


EMPTY_TOPOLOGY_KEY = "empty topologyKey is not allowed except for PreferredDuringScheduling pod anti-affinity"
_SEL_OPS = {"In": "in", "NotIn": "notin", "Exists": "exists", "DoesNotExist": "!"}


def label_selector(sel, unsupported=None):
    """Canonical requirement tuple, or Invalid(error text) for a selector the reference rejects.
    matchLabels go in key order (a Go map: random there when several pairs are invalid)."""
    from .export import go_quote, new_requirement_error
    if sel is None:
        return NOTHING
    ml = sel.get("matchLabels") or {}
    ex = sel.get("matchExpressions") or []
    if not ml and not ex:
        return EVERYTHING
    reqs = []
    for k in sorted(ml):
        err = new_requirement_error(k, "=", [ml[k]])
        if err:
            return Invalid(err)
        reqs.append((k, "In", (ml[k],)))
    for e in ex:
        op, k, vs = e.get("operator"), e.get("key", ""), tuple(e.get("values") or [])
        if op not in _SEL_OPS:
            return Invalid(f"{go_quote(str(op))} is not a valid pod selector operator")
        err = new_requirement_error(k, _SEL_OPS[op], vs)
        if err:
            return Invalid(err)
        reqs.append((k, op, tuple(sorted(set(vs)))))
    return tuple(sorted(reqs))


def selector_matches(reqs, labels) -> bool:  # labels.internalSelector.Matches (selector.go:185-236)
    if reqs is NOTHING or isinstance(reqs, Invalid):
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

    def __init__(self, owner_ns, d, unsupported=None):
        self.ns = frozenset(d.get("namespaces") or [owner_ns])
        self.sel = label_selector(d.get("labelSelector"))
        self.key = d.get("topologyKey", "")

    @property
    def invalid(self):
        return isinstance(self.sel, Invalid)

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
        dom, d = self.snap.slot_domains(keys)
        self.slot_doms.append(dom)
        self.slot_D.append(d)
        return s

    def table(self, key, keys, kind):
        t = self.tables.get(key)
        if t is None:
            t = self.tables[key] = len(self.table_slot)
            self.table_slot.append(self.slot(keys))
            self.table_kind.append(kind)
        return t

    def build(self):
        """The snapshot supplies its pods grouped (a group: pods with one spec template -- namespace, labels,
        (anti)affinity -- and their session nodes): snap.aff_groups() -> (lister, existing, spec_pod) with
        lister  : [(pod, nodes, uids)] the allocated-status session tasks (NewPodLister, util.go:57-82),
        existing: [(pod, nodes)] the pods on session nodes (schedulercache NodeInfo pods, for the score),
        spec_pod: the first pending pod of every spec; and snap.slot_domains(keys) -> (domain id per node, D)."""
        snap, U = self.snap, self.U
        from .export import has_pod_affinity
        lister, existing, spec_pod = snap.aff_groups(U)
        m = len(spec_pod)
        aff_cache = {}

        def paff(pod):
            k = id(pod)
            a = aff_cache.get(k)
            if a is None:
                a = aff_cache[k] = PodAff(pod, U)
            return a

        def first_invalid(terms):
            return next((t.sel for t in terms if t.invalid), None)

        def prefix(terms):  # the key tuple before the first empty topologyKey (all keys when none is empty)
            keys = tuple(t.key for t in terms)
            return keys[:keys.index("")] if "" in keys else keys

        # ---- predicate tables ----
        checks = [[] for _ in range(m)]
        lister_incr = [[] for _ in range(m)]
        self_match = [0] * m
        # XB: lister pods with an invalid required anti-affinity selector; every spec checks it first
        # (satisfiesExistingPodsAntiAffinity errors before it looks at any term, predicates.go:1302-1313)
        self.xb_pods = sorted((u, first_invalid(paff(pod).req_anti)) for pod, _, uids in lister
                              if first_invalid(paff(pod).req_anti) for u in uids)
        xb_spec = ((s, first_invalid(paff(spec_pod[s]).req_anti)) for s in range(m))
        self.xb_spec = {s: inv for s, inv in xb_spec if inv}
        if self.xb_pods or self.xb_spec:
            xb = self.table(("XB",), (), AFF_ERROR)
            for s in range(m):
                checks[s].append((xb, AFF_ERROR))
            for s in self.xb_spec:
                lister_incr[s].append(xb)
        e_classes = {}  # (ns, sel, key) -> table id
        for pod, _, _ in lister:
            for term in paff(pod).req_anti:
                if term.key and not term.invalid:
                    e_classes.setdefault((term.ns, term.sel, term.key), None)
        for s in range(m):
            for term in paff(spec_pod[s]).req_anti:
                if term.key and not term.invalid:
                    e_classes.setdefault((term.ns, term.sel, term.key), None)
        for ck in list(e_classes):
            e_classes[ck] = self.table(("E",) + ck, (ck[2],), AFF_EXISTING_ANTI)
        # which specs match each existing-anti class (the incoming pod is matched against the term)
        spec_ids = [pod_ident(p) for p in spec_pod]
        spec_lab = defaultdict(set)  # (label key, value) -> specs: candidates of a term's In requirements
        for s, p in enumerate(spec_pod):
            for lk, lv in p.labels.items():
                spec_lab[(lk, lv)].add(s)
        for (ns, sel, key), tid in e_classes.items():
            term = Term.__new__(Term)
            term.ns, term.sel, term.key = ns, sel, key
            for s in sorted(_candidates([term], spec_lab, range(m))):
                if term.matches(spec_pod[s].ns, spec_pod[s].labels):
                    checks[s].append((tid, AFF_EXISTING_ANTI))
        # the pod's own terms (satisfiesPodsAffinityAntiAffinity, :1401-1457): an affinity error comes from
        # the first target pod, before any anti-affinity failure; anti failures come before the affinity
        # rule that is decided after the loop
        self.own_err = {}
        bc = {}  # table id -> terms whose properties a lister pod must match
        all_t = None

        def table_all():
            nonlocal all_t
            if all_t is None:
                all_t = self.table(("ALL",), (), AFF_ANTI)
            return all_t
        for s in range(m):
            a = paff(spec_pod[s])
            aff_chk = []
            if a.has_pod and a.req_aff:
                inv = first_invalid(a.req_aff)
                if inv is not None:  # getAffinityTermProperties errors once the lister has a pod
                    self.own_err[s] = str(inv)
                    checks[s].append((table_all(), AFF_ERROR))
                    aff_chk = [(table_all(), AFF_AFFINITY)]
                else:
                    keys = prefix(a.req_aff)
                    tid = self.table(("C", tuple(t.ident() for t in a.req_aff), keys), keys, AFF_AFFINITY)
                    bc[tid] = a.req_aff
                    if len(keys) < len(a.req_aff):  # an empty topologyKey reached: error
                        self.own_err[s] = EMPTY_TOPOLOGY_KEY
                        checks[s].append((tid, AFF_ERROR))
                    aff_chk = [(tid, AFF_AFFINITY)]
                self_match[s] = int(_all_match(a.req_aff, spec_pod[s].ns, spec_pod[s].labels))
            if a.req_anti:
                if first_invalid(a.req_anti) is not None:  # any lister pod fails every node
                    checks[s].append((table_all(), AFF_ANTI))
                else:
                    keys = prefix(a.req_anti)
                    tid = self.table(("B", tuple(t.ident() for t in a.req_anti), keys), keys, AFF_ANTI)
                    bc[tid] = a.req_anti
                    checks[s].append((tid, AFF_ANTI))
            checks[s] += aff_chk
        # identities of lister pods (with their nodes) and of pending specs
        lid = defaultdict(list)
        for pod, nodes, _ in lister:
            lid[pod_ident(pod)].extend(nodes)
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

        for pod, nodes, _ in lister:  # existing-anti classes carried by lister pods
            for term in paff(pod).req_anti:
                if term.key and not term.invalid:
                    add_nodes(e_classes[(term.ns, term.sel, term.key)], nodes)
        if self.xb_pods:
            add_nodes(self.tables[("XB",)], [i for pod, nodes, _ in lister if first_invalid(paff(pod).req_anti)
                                            for i in nodes])
        if all_t is not None:
            add_nodes(all_t, [i for _, nodes, _ in lister for i in nodes])
            for s in range(m):
                lister_incr[s].append(all_t)
        spec_by_ident = defaultdict(list)
        for s, ident in enumerate(spec_ids):
            spec_by_ident[ident].append(s)
        universe = set(lid) | set(spec_ids)  # (once: every table's candidates come out of it)
        for tid, terms in bc.items():
            for ident in _candidates(terms, index, universe):
                ns, labels = ident[0], dict(ident[1])
                if not _all_match(terms, ns, labels):
                    continue
                if ident in lid:
                    add_nodes(tid, lid[ident])
                for s in spec_by_ident.get(ident, []):
                    lister_incr[s].append(tid)
        for s in range(m):
            for term in paff(spec_pod[s]).req_anti:
                if term.key and not term.invalid:
                    lister_incr[s].append(e_classes[(term.ns, term.sel, term.key)])
            lister_incr[s] = sorted(set(lister_incr[s]))

        # ---- InterPodAffinity histograms ----
        # identities for the score carry the pod's own terms too
        def sid(pod):
            return (pod.ns, tuple(sorted(pod.labels.items())), repr((pod.affinity or {}).get("podAffinity")),
                    repr((pod.affinity or {}).get("podAntiAffinity")))
        e_nodes = defaultdict(list)
        e_pod = {}
        for pod, nodes in existing:
            k = sid(pod)
            e_nodes[k].extend(nodes)
            e_pod.setdefault(k, pod)
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
        # CalculateInterPodAffinityPriority errors when processTerm meets an invalid selector
        # (interpod_affinity.go:86-93): the incoming pod's preferred terms against every pod it considers,
        # and the considered pods' own score terms (:150-187)
        def own_score_terms(a):  # the terms a pod contributes as an existing pod
            return (a.req_aff + [t for _, t in a.pref_aff] if a.has_pod else []) + \
                   ([t for _, t in a.pref_anti] if a.has_anti else [])

        def incoming_terms(a):
            return ([t for _, t in a.pref_aff] if a.has_pod else []) + ([t for _, t in a.pref_anti] if a.has_anti else [])
        bad_e = [first_invalid(own_score_terms(paff(e_pod[k]))) is not None for k in all_e]
        any_e = bool(all_e and any(k in e_nodes for k in all_e))
        any_e_aff = any(k in e_nodes and has_pod_affinity(e_pod[k]) for k in all_e)
        bad_e_present = any(b and k in e_nodes for b, k in zip(bad_e, all_e))
        self.ipa_error = [False] * m
        for s in range(m):
            a = paff(spec_pod[s])
            considered = any_e if (a.has_pod or a.has_anti) else any_e_aff
            own = first_invalid(incoming_terms(a)) is not None
            self.ipa_error[s] = bool(snap.config["nodeorder_enabled"]) and (bad_e_present or (considered and own))
        if snap.config["nodeorder_enabled"]:
            for s in range(m):  # a pod with invalid score terms that can commit would make later scores error
                a = paff(spec_pod[s])
                if first_invalid(own_score_terms(a)) is None or self.ipa_error[s]:
                    continue
                if snap.config["predicates_enabled"] and a.has_pod and first_invalid(a.req_aff) is not None:
                    continue  # fails every node's predicate: never commits
                raise U("a pending pod with invalid inter-pod affinity score terms may commit")
        W = defaultdict(lambda: defaultdict(int))  # (s, e) -> {key: weight}
        for s in range(m):
            a = paff(spec_pod[s])
            terms = ([(w, t) for w, t in a.pref_aff] if a.has_pod else []) + \
                    ([(-w, t) for w, t in a.pref_anti] if a.has_anti else [])
            for w, term in terms:
                if not term.key or w == 0 or term.invalid:
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
                if not term.key or w == 0 or term.invalid:
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
        # what pod_deltas needs to place a pod outside the pending specs into these tables
        self._paff, self._bc, self._e_classes, self._all_t, self._spec_pod, self._h_off = \
            paff, bc, e_classes, all_t, spec_pod, h_off
        self._incoming_bad = any(first_invalid(incoming_terms(paff(p))) is not None for p in spec_pod)
        self._nodeorder = bool(snap.config["nodeorder_enabled"])
        from .export import SPEC_IPA_ERROR
        for s in range(m):
            if self.ipa_error[s]:
                snap.spec_arr["flags"][s] |= SPEC_IPA_ERROR
        return self

    def pod_deltas(self, pod, node, lister=0, existing=0):
        """kb_apply_affinity entries (node, table, slot, h_off, weight) for a pod that is not one of the session's
        pending specs, on session node `node`: `lister` = +1 / -1 when it joins / leaves the predicate lister (an
        allocated-status session task, util.go:57-130), `existing` = +1 / -1 when it is bound to / removed from the
        node (the InterPodAffinity priority's NodeInfo pods, interpod_affinity.go:150-187). The entries are the
        counts build() would have made with the pod there. Unsupported when the pod would need a table or a
        histogram the pending specs do not have, or would change the error paths (invalid selectors)."""
        U = self.U
        a = PodAff(pod, U)  # (build's cache is keyed by object id: only for pods it keeps alive)
        out = []
        if lister:
            if any(t.invalid for t in a.req_anti):
                raise U("a lister pod with an invalid anti-affinity selector changes the error strings")
            for term in a.req_anti:
                if not term.key:
                    continue
                tid = self._e_classes.get((term.ns, term.sel, term.key))
                if tid is None:
                    if any(term.matches(p.ns, p.labels) for p in self._spec_pod):
                        raise U("the pod's required anti-affinity term is a class no table holds")
                    continue  # no pending spec matches the term: no check reads it
                out.append((node, tid, -1, 0, lister))
            if self._all_t is not None:
                out.append((node, self._all_t, -1, 0, lister))
            for tid, terms in self._bc.items():
                if _all_match(terms, pod.ns, pod.labels):
                    out.append((node, tid, -1, 0, lister))
        if existing and self._nodeorder:
            own = (a.req_aff + [t for _, t in a.pref_aff] if a.has_pod else []) + \
                  ([t for _, t in a.pref_anti] if a.has_anti else [])
            if any(t.invalid for t in own) or self._incoming_bad:
                raise U("invalid inter-pod affinity score terms: the batch score error depends on the pods present")
            mine = ([(1, t) for t in a.req_aff] + list(a.pref_aff) if a.has_pod else []) + \
                   ([(-w, t) for w, t in a.pref_anti] if a.has_anti else [])
            for s, sp in enumerate(self._spec_pod):
                b = self._paff(sp)
                W = defaultdict(int)
                theirs = (list(b.pref_aff) if b.has_pod else []) + ([(-w, t) for w, t in b.pref_anti] if b.has_anti else [])
                for w, term in theirs:  # the incoming spec's terms against this pod
                    if term.key and w and term.matches(pod.ns, pod.labels):
                        W[term.key] += w
                for w, term in mine:  # this pod's own terms against the spec's pod
                    if term.key and w and term.matches(sp.ns, sp.labels):
                        W[term.key] += w
                for key, w in sorted(W.items()):
                    if not w:
                        continue
                    h = self._h_off.get((s, key))
                    if h is None:
                        raise U("the pod's score terms need a histogram the spec does not have")
                    out.append((node, -1, self.slot_ids[(key,)], h, w * existing))
        return out

    def host_error_string(self, pod, spec, node_name, allocated_before):
        """The FitErrors string of a node the device failed with KB_R_HOST_ERROR at the affinity stage: the
        error the reference's predicate returns there (FitErrors.SetNodeError, unschedule_info.go:40-54).
        `allocated_before`: (uid, spec) of the cycle's Allocate commits before the failing task (the lister's
        additions). XB errors first (predicates.go:1302-1313; the first such lister pod in UID order -- a Go
        map walk, so random there when several differ), else the pod's own required affinity (:1401-1413)."""
        pn = f"{pod.ns}/{pod.name}"  # podName (predicates.go:721-723)
        xb = list(self.xb_pods) + [(u, self.xb_spec[sp]) for u, sp in allocated_before if sp in self.xb_spec]
        if xb:
            return f"Failed to get all terms that pod {pn} matches, err: {min(xb)[1]}"
        if spec not in self.own_err:  # (host_reason_strings asks only for specs with an error source)
            raise self.U(f"spec {spec} has no inter-pod affinity error to report")
        return f"Cannot schedule pod {pn} onto node {node_name}, because of PodAffinity, err: {self.own_err[spec]}"
