"""Snapshot exporter: cluster objects -> the C-ABI arrays of include/kbgpu.h.

This is the host-side half of the drop-in boundary: what a Go
shim would do with `ssn.Nodes` / `ssn.Jobs` at session open. It restates
cache.Snapshot (pkg/scheduler/cache/cache.go:584-654), NodeInfo.AddTask
(api/node_info.go:165-193), NewTaskInfo (api/job_info.go:69-95) and the
plugins' session-open state (plugins/util/util.go:57-82,186-198), then interns
every string the device needs (scalar names, label keys/values, taint and
toleration sets, host ports) into integer ids.

The device never sees a string; node index = position in name order.
"""
from __future__ import annotations

import functools
import re

import numpy as np

from . import model as M

# ---- C struct layouts (include/kbgpu.h) ------------------------------------
SPEC_DTYPE = np.dtype([
    ("init_cpu", "<i8"), ("init_mem", "<i8"), ("req_cpu", "<i8"), ("req_mem", "<i8"),
    ("nz_cpu", "<i8"), ("nz_mem", "<i8"), ("init_sc_mask", "<u8"), ("req_sc_mask", "<u8"),
    ("flags", "<u4"), ("tol_set", "<i4"), ("sc_off", "<u4"), ("sel_term", "<u4"),
    ("req_term_off", "<u4"), ("req_term_cnt", "<u4"), ("pref_term_off", "<u4"), ("pref_term_cnt", "<u4"),
    ("port_off", "<u4"), ("port_cnt", "<u4"), ("aff_class", "<i4"), ("pad", "<i4")], align=True)
REQ_DTYPE = np.dtype([("key", "<i4"), ("op", "<i4"), ("val_off", "<u4"), ("val_cnt", "<u4"), ("ival", "<i8")],
                     align=True)
TERM_DTYPE = np.dtype([("req_off", "<u4"), ("req_cnt", "<u4"), ("weight", "<i4"), ("pad", "<i4")], align=True)
PORT_DTYPE = np.dtype([("slot", "<i4"), ("ip", "<i4")], align=True)
assert SPEC_DTYPE.itemsize == 112 and REQ_DTYPE.itemsize == 24 and TERM_DTYPE.itemsize == 16

# flags / enums (kbgpu.h)
NODE_IDLE_HAS_MAP, NODE_REL_HAS_MAP = 1 << 0, 1 << 1
NODE_NOT_READY, NODE_OUT_OF_DISK, NODE_NET_UNAVAIL, NODE_UNSCHEDULABLE = 1 << 2, 1 << 3, 1 << 4, 1 << 5
NODE_MEM_PRESSURE, NODE_DISK_PRESSURE, NODE_PID_PRESSURE = 1 << 9, 1 << 10, 1 << 11
SPEC_INIT_HAS_MAP, SPEC_REQ_HAS_MAP, SPEC_BEST_EFFORT = 1 << 0, 1 << 1, 1 << 2
SPEC_HAS_SELECTOR, SPEC_HAS_REQUIRED, SPEC_NA_ERROR, SPEC_POD_AFFINITY = 1 << 3, 1 << 4, 1 << 5, 1 << 6
SPEC_IPA_ERROR = 1 << 7
OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE, OP_GT, OP_LT, OP_TRUE, OP_FALSE = range(8)

ST = {"Pending": 1 << 0, "Allocated": 1 << 1, "Pipelined": 1 << 2, "Binding": 1 << 3, "Bound": 1 << 4,
      "Running": 1 << 5, "Releasing": 1 << 6, "Succeeded": 1 << 7, "Failed": 1 << 8, "Unknown": 1 << 9}
ST_NAME = {v: k for k, v in ST.items()}
PLUGIN_IDS = {"priority": 0, "gang": 1, "drf": 2, "proportion": 3, "predicates": 4, "nodeorder": 5,
              "conformance": 6}
EN_BITS = {"enabledJobOrder": 0, "enabledJobReady": 1, "enabledJobPipelined": 2, "enabledTaskOrder": 3,
           "enabledPreemptable": 4, "enabledReclaimable": 5, "enabledQueueOrder": 6, "enabledPredicate": 7,
           "enabledNodeOrder": 8}

REASONS = [  # bit i of a reason mask (kbgpu.h KB_R_*)
    "node(s) resource fit failed", "node(s) pod number exceeded", "node(s) were not ready",
    "node(s) were out of disk space", "node(s) had unavailable network", "node(s) were unschedulable",
    "node(s) didn't match node selector", "node(s) didn't have free ports for the requested pod ports",
    "node(s) had taints that the pod didn't tolerate", "node(s) had memory pressure", "node(s) had disk pressure",
    "node(s) had pid pressure", "node(s) didn't match pod affinity/anti-affinity",
    "node(s) didn't satisfy existing pods anti-affinity rules", "node(s) didn't match pod affinity rules",
    "node(s) didn't match pod anti-affinity rules",
    None]  # KB_R_HOST_ERROR: the string is the host's (a plain error of the reference's predicate, or an overlay's)


class Unsupported(RuntimeError):
    """The snapshot uses a feature the device path does not express (fails loudly, never falls back)."""


class AssertPanic(RuntimeError):
    """util/assert.Assertf would panic in the reference (resource underflow)."""


# ---- k8s validation (apimachinery/pkg/util/validation/validation.go:42-144) ----
def _alnum(c):
    return c.isascii() and c.isalnum()


def _qname_fmt(s):
    return bool(s) and _alnum(s[0]) and _alnum(s[-1]) and all(_alnum(c) or c in "-_." for c in s)


@functools.lru_cache(maxsize=1 << 16)
def is_qualified_name(v: str) -> bool:
    return not qualified_name_errors(v)


@functools.lru_cache(maxsize=1 << 16)
def is_valid_label_value(v: str) -> bool:
    return not label_value_errors(v)


# the error texts (validation.go:38-106, 342-372): the reference puts them into FitErrors strings
_QNAME_FMT = "([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]"
_QNAME_MSG = ("must consist of alphanumeric characters, '-', '_' or '.', and must start and end with an "
              "alphanumeric character")
_DNS1123_FMT = "[a-z0-9]([-a-z0-9]*[a-z0-9])?(\\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*"
_DNS1123_MSG = ("a DNS-1123 subdomain must consist of lower case alphanumeric characters, '-' or '.', and must "
                "start and end with an alphanumeric character")
_LABEL_FMT = "(" + _QNAME_FMT + ")?"
_LABEL_MSG = ("a valid label must be an empty string or consist of alphanumeric characters, '-', '_' or '.', and "
              "must start and end with an alphanumeric character")


def _regex_error(msg, fmt, *examples):  # RegexError (validation.go:347-362), double spaces included
    if not examples:
        return msg + " (regex used for validation is '" + fmt + "')"
    msg += " (e.g. "
    for i, e in enumerate(examples):
        msg += (" or " if i else "") + "'" + e + "', "
    return msg + "regex used for validation is '" + fmt + "')"


_DNS1123_RE = re.compile(r"[a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*")


def qualified_name_errors(v: str):  # IsQualifiedName (validation.go:42-71)
    errs = []
    parts = v.split("/")
    if len(parts) == 1:
        name = parts[0]
    elif len(parts) == 2:
        prefix, name = parts
        if not prefix:
            errs.append("prefix part must be non-empty")
        else:  # IsDNS1123Subdomain (validation.go:135-144), each message prefixed
            if len(prefix) > 253:
                errs.append("prefix part must be no more than 253 characters")
            if not _DNS1123_RE.fullmatch(prefix):
                errs.append("prefix part " + _regex_error(_DNS1123_MSG, _DNS1123_FMT, "example.com"))
    else:
        return ["a qualified name " + _regex_error(_QNAME_MSG, _QNAME_FMT, "MyName", "my.name", "123-abc") +
                " with an optional DNS subdomain prefix and '/' (e.g. 'example.com/MyName')"]
    if not name:
        errs.append("name part must be non-empty")
    elif len(name) > 63:
        errs.append("name part must be no more than 63 characters")
    if not _qname_fmt(name):
        errs.append("name part " + _regex_error(_QNAME_MSG, _QNAME_FMT, "MyName", "my.name", "123-abc"))
    return errs


def label_value_errors(v: str):  # IsValidLabelValue (validation.go:97-106)
    errs = []
    if len(v) > 63:
        errs.append("must be no more than 63 characters")
    if not (v == "" or _qname_fmt(v)):
        errs.append(_regex_error(_LABEL_MSG, _LABEL_FMT, "MyValue", "my_value", "12345"))
    return errs


def go_quote(s: str) -> str:
    """fmt %q of a printable ASCII string (strconv.Quote)."""
    return '"' + s.replace("\\", "\\\\").replace('"', '\\"') + '"'


def new_requirement_error(key: str, op: str, vals) -> str | None:
    """labels.NewRequirement's error text (apimachinery/pkg/labels/selector.go:133-170), or None; op is the
    selection operator ("=" for matchLabels pairs, "in", "notin", "exists", "!")."""
    e = qualified_name_errors(key)
    if e:
        return f"invalid label key {go_quote(key)}: " + "; ".join(e)
    if op in ("in", "notin") and not vals:
        return "for 'in', 'notin' operators, values set can't be empty"
    if op == "=" and len(vals) != 1:
        return "exact-match compatibility requires one single value"
    if op in ("exists", "!") and vals:
        return "values set must be empty for exists and does not exist"
    for v in vals:
        e = label_value_errors(v)
        if e:
            return f"invalid label value: {go_quote(v)}: " + "; ".join(e)
    return None


@functools.lru_cache(maxsize=4096)
def is_scalar_resource_name(n: str) -> bool:  # core/v1/helper/helpers.go:36-104
    prefixed_native = "kubernetes.io/" in n
    native = "/" not in n or prefixed_native
    extended = (not native) and not n.startswith("requests.") and is_qualified_name("requests." + n)
    return extended or n.startswith("hugepages-") or prefixed_native or n.startswith("attachable-volumes-")


def parse_int64(s: str):
    """strconv.ParseInt(s, 10, 64); None on failure."""
    if not s:
        return None
    body = s[1:] if s[0] in "+-" else s
    if not body or not body.isascii() or not body.isdigit():
        return None
    v = int(s)
    if v < -(1 << 63) or v > (1 << 63) - 1:
        return None
    return v


# ---- api.Resource (api/resource_info.go) with nil-map presence -------------
MIN_CPU, MIN_MEM, MIN_SCALAR = 10, 10 * 1024 * 1024, 10


class Res:
    __slots__ = ("cpu", "mem", "sc", "max_task")

    def __init__(self, cpu=0, mem=0, sc=None, max_task=0):
        self.cpu, self.mem, self.sc, self.max_task = cpu, mem, sc, max_task

    @classmethod
    def from_list(cls, rl):  # NewResource (:75-93)
        r = cls()
        for k, q in rl.items():
            if k == M.CPU:
                r.cpu += q
            elif k == M.MEMORY:
                r.mem += q
            elif k == M.PODS:
                r.max_task += q
            elif is_scalar_resource_name(k):
                if r.sc is None:
                    r.sc = {}
                r.sc[k] = r.sc.get(k, 0) + q
        return r

    def copy(self):
        return Res(self.cpu, self.mem, None if self.sc is None else dict(self.sc), self.max_task)

    @classmethod
    def of_request(cls, rl, memo):
        """from_list for a request that is only read (container requests): one Res per distinct request in
        `memo` (a session-open dict), so pods built from one template parse their quantities once."""
        key = tuple(rl.items())
        r = memo.get(key)
        if r is None:
            r = memo[key] = cls.from_list(rl)
        return r

    def add(self, rr):  # Add (:131-143)
        self.cpu += rr.cpu
        self.mem += rr.mem
        for k, v in (rr.sc or {}).items():
            if self.sc is None:
                self.sc = {}
            self.sc[k] = self.sc.get(k, 0) + v
        return self

    def sub(self, rr):  # Sub (:145-159)
        if not rr.less_equal(self):
            raise AssertPanic("resource is not sufficient to do operation")
        self.cpu -= rr.cpu
        self.mem -= rr.mem
        for k, v in (rr.sc or {}).items():
            if self.sc is None:
                return self
            self.sc[k] = self.sc.get(k, 0) - v
        return self

    def set_max(self, rr):  # SetMaxResource (:162-190)
        self.cpu = max(self.cpu, rr.cpu)
        self.mem = max(self.mem, rr.mem)
        for k, v in (rr.sc or {}).items():
            if self.sc is None:
                self.sc = dict(rr.sc)
                return
            if v > self.sc.get(k, 0):
                self.sc[k] = v

    def less_equal(self, rr):  # LessEqual (:253-276), integral form r - rr < tol
        if not (self.cpu - rr.cpu < MIN_CPU and self.mem - rr.mem < MIN_MEM):
            return False
        if self.sc is None:
            return True
        for k, v in self.sc.items():
            if rr.sc is None:
                return False
            if not (v - rr.sc.get(k, 0) < MIN_SCALAR):
                return False
        return True

    def is_empty(self):  # IsEmpty (:96-108)
        if not (self.cpu < MIN_CPU and self.mem < MIN_MEM):
            return False
        return all(v < MIN_SCALAR for v in (self.sc or {}).values())


def task_status(p: M.Pod) -> int:  # getTaskStatus (api/helpers.go:35-69)
    if p.phase == "Running":
        return ST["Releasing"] if p.deleting else ST["Running"]
    if p.phase == "Pending":
        if p.deleting:
            return ST["Releasing"]
        return ST["Pending"] if not p.node else ST["Bound"]
    return {"Succeeded": ST["Succeeded"], "Failed": ST["Failed"]}.get(p.phase, ST["Unknown"])


def allocated_status(s: int) -> bool:  # api/helpers.go:72-79
    return s in (ST["Bound"], ST["Binding"], ST["Running"], ST["Allocated"])


def nonzero(req):  # GetNonzeroRequests (priorities/util/non_zero.go:31-52)
    return req.get(M.CPU, 100), req.get(M.MEMORY, 200 * 1024 * 1024)


def has_pod_affinity(p: M.Pod) -> bool:
    a = p.affinity or {}
    return bool(a.get("podAffinity") is not None or a.get("podAntiAffinity") is not None)


def _tolerates(tol, taint) -> bool:  # Toleration.ToleratesTaint (api/core/v1/toleration.go:37-56)
    if tol.get("effect") and tol.get("effect") != taint.get("effect"):
        return False
    if tol.get("key") and tol.get("key") != taint.get("key"):
        return False
    op = tol.get("operator", "")
    if op in ("", "Equal"):
        return tol.get("value", "") == taint.get("value", "")
    return op == "Exists"


class _Interner:
    def __init__(self):
        self.ids = {}

    def __call__(self, key):
        i = self.ids.get(key)
        if i is None:
            i = self.ids[key] = len(self.ids)
        return i


class SpecTable:
    """Pending pods deduplicated into task specs (kb_spec rows) with their compiled selector / affinity terms,
    toleration sets and host ports, in first-occurrence order. Export.Snapshot feeds it every pending task;
    the columnar exporter (columns.py) feeds it one pod per distinct template (pods of one template share
    every field the signature reads)."""

    def __init__(self, scalars, aff_in_play):
        self.scalars = list(scalars)
        if len(self.scalars) > 64:
            raise Unsupported("more than 64 scalar resources")
        self.slot = {n: i for i, n in enumerate(self.scalars)}
        self.aff_in_play = aff_in_play
        self.label_keys = _Interner()
        self.values = _Interner()
        self.gtlt_keys = set()
        self.port_slots = _Interner()
        self.port_ips = {}  # slot -> Interner of ips (0.0.0.0 first)
        self.tol_sets = _Interner()
        self.tol_list = []
        self.terms, self.reqs, self.vals, self.ports = [], [], [], []
        self.specs, self.sc_init, self.sc_req = [], [], []
        self.sig_index = {}
        self.reprs = {}  # repr of a pod's affinity sub-dicts, by object (pods of one template share them)

    def rp(self, x):
        k = id(x)
        v = self.reprs.get(k)
        if v is None:
            v = self.reprs[k] = (x, repr(x))  # keeps x alive: its id is not reused during the export
        return v[1]

    def req_rows(self, exprs, allow_gtlt=True):
        """NodeSelectorRequirementsAsSelector (helpers.go:222-254) -> requirement rows, None if invalid."""
        rows = []
        for e in exprs:
            op = {"In": OP_IN, "NotIn": OP_NOTIN, "Exists": OP_EXISTS, "DoesNotExist": OP_DNE,
                  "Gt": OP_GT, "Lt": OP_LT}.get(e.get("operator"))
            key, vs = e.get("key", ""), list(e.get("values") or [])
            if op is None or not is_qualified_name(key):
                return None
            if op in (OP_IN, OP_NOTIN) and not vs:
                return None
            if op in (OP_EXISTS, OP_DNE) and vs:
                return None
            ival = 0
            if op in (OP_GT, OP_LT):
                if len(vs) != 1 or parse_int64(vs[0]) is None:
                    return None
                ival = parse_int64(vs[0])
                self.gtlt_keys.add(key)
            if not all(is_valid_label_value(v) for v in vs):
                return None
            rows.append((self.label_keys(key), op, tuple(self.values(v) for v in vs) if op < OP_EXISTS else (),
                         ival))
        return rows

    def add_term(self, rows, weight=0):
        off = len(self.reqs)
        for key, op, vv, ival in rows:
            self.reqs.append((key, op, len(self.vals), len(vv), ival))
            self.vals.extend(vv)
        self.terms.append((off, len(rows), weight, 0))
        return len(self.terms) - 1

    def add(self, p, ir, rr) -> int:
        """The spec id of a pending pod with InitResreq ir and Resreq rr (a new spec for a new signature)."""
        nzc = nzm = 0
        for c in p.containers:
            a, b = nonzero(c.req)
            nzc += a
            nzm += b
        aff = p.affinity or {}
        nodeaff = aff.get("nodeAffinity") if p.affinity is not None else None
        tols = tuple(sorted((d.get("key", ""), d.get("operator", ""), d.get("value", ""), d.get("effect", ""))
                            for d in p.tolerations))
        port_list = []
        for c in p.containers:
            for pt in c.ports:
                hp = int(pt.get("hostPort", 0) or 0)
                if hp <= 0:
                    continue
                port_list.append(((pt.get("protocol") or "TCP"), hp, pt.get("hostIP") or "0.0.0.0"))
        best_effort = not any(M.CPU in c.req or M.MEMORY in c.req for c in list(p.containers) + list(p.init))
        sig = (ir.cpu, ir.mem, tuple(sorted((ir.sc or {}).items())) if ir.sc is not None else None,
               rr.cpu, rr.mem, tuple(sorted((rr.sc or {}).items())) if rr.sc is not None else None,
               nzc, nzm, tuple(sorted(p.node_selector.items())), self.rp(nodeaff), tols, tuple(port_list),
               best_effort)
        if self.aff_in_play:  # selectors and terms see the pod's namespace, labels and own terms
            sig = sig + (p.ns, tuple(sorted(p.labels.items())), self.rp(aff.get("podAffinity")),
                         self.rp(aff.get("podAntiAffinity")))
        if sig in self.sig_index:
            return self.sig_index[sig]
        slot = self.slot
        flags = 0
        if ir.sc is not None:
            flags |= SPEC_INIT_HAS_MAP
        if rr.sc is not None:
            flags |= SPEC_REQ_HAS_MAP
        if best_effort:
            flags |= SPEC_BEST_EFFORT
        if self.aff_in_play:
            flags |= SPEC_POD_AFFINITY
        imask = sum(1 << slot[k] for k in (ir.sc or {}))
        rmask = sum(1 << slot[k] for k in (rr.sc or {}))
        si = [0] * len(self.scalars)
        sr = [0] * len(self.scalars)
        for k, v in (ir.sc or {}).items():
            si[slot[k]] = v
        for k, v in (rr.sc or {}).items():
            sr[slot[k]] = v
        # nodeSelector: SelectorFromSet, any invalid pair => Everything (labels/selector.go:849-866)
        sel_term = 0
        if p.node_selector:
            ok = all(is_qualified_name(k) and is_valid_label_value(v) for k, v in p.node_selector.items())
            if ok:
                sel_term = self.add_term([(self.label_keys(k), OP_IN, (self.values(v),), 0)
                                          for k, v in sorted(p.node_selector.items())])
                flags |= SPEC_HAS_SELECTOR
        # required node affinity (MatchNodeSelectorTerms, helpers.go:302-333)
        req_off, req_cnt = len(self.terms), 0
        if nodeaff is not None and nodeaff.get("required") is not None:
            flags |= SPEC_HAS_REQUIRED
            built = []
            for term in nodeaff["required"]:
                exprs = term.get("matchExpressions") or []
                fields = term.get("matchFields") or []
                if not exprs and not fields:
                    built.append([])  # empty term: matches nothing
                    continue
                rows = []
                if exprs:
                    r = self.req_rows(exprs)
                    rows.extend(r if r is not None else [(0, OP_FALSE, (), 0)])
                if fields:  # NodeSelectorRequirementsAsFieldSelector over {metadata.name: node.Name}
                    for e in fields:
                        op, vs = e.get("operator"), list(e.get("values") or [])
                        if op not in ("In", "NotIn") or len(vs) != 1:
                            rows = [(0, OP_FALSE, (), 0)]
                            break
                        if e.get("key") == "metadata.name":
                            rows.append((self.label_keys("\x00metadata.name"), OP_IN if op == "In" else OP_NOTIN,
                                         (self.values(vs[0]),), 0))
                        else:
                            truth = (vs[0] == "") if op == "In" else (vs[0] != "")
                            rows.append((0, OP_TRUE if truth else OP_FALSE, (), 0))
                built.append(rows)
            req_off = len(self.terms)
            for rows in built:
                self.add_term(rows)
            req_cnt = len(built)
        # preferred node affinity (node_affinity.go:47-67)
        pref_rows = []
        if nodeaff is not None:
            for pt in nodeaff.get("preferred") or []:
                w = int(pt.get("weight", 0))
                if w == 0:
                    continue
                exprs = (pt.get("preference") or {}).get("matchExpressions") or []
                rows = self.req_rows(exprs) if exprs else []
                if rows is None:
                    flags |= SPEC_NA_ERROR
                    pref_rows = []
                    break
                pref_rows.append((rows, w))
        pref_off = len(self.terms)
        for rows, w in pref_rows:
            self.add_term(rows, w)
        # tolerations
        tol_id = self.tol_sets(tols)
        if tol_id == len(self.tol_list):
            self.tol_list.append([{"key": a, "operator": b, "value": c, "effect": d} for a, b, c, d in tols])
        # ports
        port_off = len(self.ports)
        for proto, hp, ip in port_list:
            s_id = self.port_slots((proto, hp))
            ipi = self.port_ips.setdefault(s_id, _Interner())
            if not ipi.ids:
                ipi("0.0.0.0")
            self.ports.append((s_id, ipi(ip)))
        specs = self.specs
        specs.append((ir.cpu, ir.mem, rr.cpu, rr.mem, nzc, nzm, imask, rmask, flags, tol_id,
                      len(self.sc_init) * len(self.scalars), sel_term, req_off, req_cnt, pref_off, len(pref_rows),
                      port_off, len(self.ports) - port_off, len(specs) if self.aff_in_play else -1, 0))
        self.sc_init.extend(si)
        self.sc_req.extend(sr)
        self.sig_index[sig] = len(specs) - 1
        return len(specs) - 1

    def finish(self, snap):
        """The spec arrays and interners onto the snapshot."""
        for s_id, ipi in self.port_ips.items():
            if len(ipi.ids) > 63:
                raise Unsupported("more than 62 host IPs for one (protocol, port)")
        snap.scalars = self.scalars
        for k in ("label_keys", "values", "gtlt_keys", "port_slots", "port_ips", "tol_sets", "tol_list"):
            setattr(snap, k, getattr(self, k))
        snap.spec_arr = np.array(self.specs, dtype=SPEC_DTYPE) if self.specs else np.zeros(0, SPEC_DTYPE)
        snap.sc_init = np.array(self.sc_init, dtype=np.int64)
        snap.sc_req = np.array(self.sc_req, dtype=np.int64)
        snap.term_arr = np.array(self.terms, dtype=TERM_DTYPE) if self.terms else np.zeros(0, TERM_DTYPE)
        snap.req_arr = np.array(self.reqs, dtype=REQ_DTYPE) if self.reqs else np.zeros(0, REQ_DTYPE)
        snap.val_arr = np.array(self.vals, dtype=np.int32)
        snap.port_arr = np.array(self.ports, dtype=PORT_DTYPE) if self.ports else np.zeros(0, PORT_DTYPE)


class Snapshot:
    """Session-open view of a Cluster, exported as kb_nodes / kb_specs / kb_session arrays."""

    def __init__(self, cluster: M.Cluster):
        self.cluster = cluster
        self._snapshot()
        self._config()
        self._specs()
        self._node_table()
        self.aff = None
        if self.aff_in_play:
            from .affinity import Tables
            self.aff = Tables(self, Unsupported).build()
        self._session_arrays()

    # ---------------- cache.Snapshot + session open ----------------
    def _snapshot(self):
        cl = self.cluster
        names = sorted(n.name for n in cl.nodes)
        by_name = {n.name: n for n in cl.nodes}
        node_pods = {n: [] for n in names}
        # tasks
        self.tasks = []
        memo = {}
        for p in cl.pods:
            resreq = Res()
            for c in p.containers:
                resreq.add(Res.of_request(c.req, memo))
            initreq = resreq.copy()
            for c in p.init:
                initreq.set_max(Res.of_request(c.req, memo))
            t = {"pod": p, "uid": p.uid, "status": task_status(p), "resreq": resreq, "initreq": initreq,
                 "priority": p.priority if p.priority is not None else 1,
                 "job": f"{p.ns}/{p.group}" if p.group else ""}
            self.tasks.append(t)
            if p.node and p.node in node_pods and t["status"] not in (ST["Succeeded"], ST["Failed"]):
                node_pods[p.node].append(t)
        # nodes: NewNodeInfo + AddTask; Snapshot keeps Ready ones (used <= allocatable)
        self.nodes = []
        for nm in names:
            nd = by_name[nm]
            alloc = Res.from_list(nd.alloc)
            idle, rel, used = Res.from_list(nd.alloc), Res(), Res()
            for t in node_pods[nm]:
                st = t["status"]
                if st == ST["Releasing"]:
                    rel.add(t["resreq"])
                    idle.sub(t["resreq"])
                elif st == ST["Pipelined"]:
                    rel.sub(t["resreq"])
                else:
                    idle.sub(t["resreq"])
                used.add(t["resreq"])
            if not used.less_equal(Res.from_list(nd.alloc)):
                continue
            self.nodes.append({"node": nd, "alloc": alloc, "idle": idle, "rel": rel, "tasks": node_pods[nm]})
        self.node_index = {n["node"].name: i for i, n in enumerate(self.nodes)}
        # jobs (PodGroup + existing queue)
        queues = {q.name: q for q in cl.queues}
        pgs = {f"{g.ns}/{g.name}": g for g in cl.pod_groups}
        jobs = {}
        for t in self.tasks:
            if t["job"] and t["job"] in pgs and pgs[t["job"]].queue in queues:
                jobs.setdefault(t["job"], []).append(t)
        self.job_uids = sorted(jobs)
        self.jobs = [{"uid": u, "pg": pgs[u], "tasks": jobs[u]} for u in self.job_uids]
        used_q = sorted({pgs[u].queue for u in self.job_uids})
        self.queue_names = used_q
        self.queues = [queues[q] for q in used_q]
        self.session_tasks = [t for j in self.jobs for t in j["tasks"]]
        for i, t in enumerate(self.session_tasks):
            t["sidx"] = i
        # k8s NodeInfo state (GenerateNodeMapAndSlice): pods = the node's tasks
        for n in self.nodes:
            nz_c = nz_m = 0
            for t in n["tasks"]:
                for c in t["pod"].containers:
                    a, b = nonzero(c.req)
                    nz_c += a
                    nz_m += b
            n["nz"] = (nz_c, nz_m)
        # pod (anti)affinity anywhere the predicate or the score can see it: build the affinity tables
        self.aff_in_play = any(has_pod_affinity(t["pod"]) for t in self.session_tasks) or \
            any(has_pod_affinity(t["pod"]) for nd in self.nodes for t in nd["tasks"])

    # ---------------- plugin configuration ----------------
    def _config(self):
        tiers = self.cluster.tiers
        self.tier_plugins = []
        opts = {}
        for ti, tier in enumerate(tiers):
            for p in tier.get("plugins", []):
                pid = PLUGIN_IDS.get(p["name"], 7)
                en = 0
                for f, b in EN_BITS.items():
                    if p.get(f):
                        en |= 1 << b
                self.tier_plugins.append((ti, pid, en))
                opts.setdefault(p["name"], p)

        def enabled(name, flag):
            return any(p["name"] == name and p.get(flag) for t in tiers for p in t.get("plugins", []))

        def get_int(args, key, dflt):  # Arguments.GetInt (framework/arguments.go:26-44)
            v = (args or {}).get(key)
            if v is None or v == "":
                return dflt
            x = parse_int64(str(v))
            return dflt if x is None else x

        def get_bool(args, key, dflt):
            v = (args or {}).get(key)
            if v is None or v == "":
                return dflt
            v = str(v)
            if v in ("1", "t", "T", "TRUE", "true", "True"):
                return True
            if v in ("0", "f", "F", "FALSE", "false", "False"):
                return False
            return dflt

        pa = opts.get("predicates", {}).get("arguments", {})
        na = opts.get("nodeorder", {}).get("arguments", {})
        self.config = {
            "predicates_enabled": int(enabled("predicates", "enabledPredicate")),
            "nodeorder_enabled": int(enabled("nodeorder", "enabledNodeOrder")),
            "mem_pressure": int(get_bool(pa, "predicate.MemoryPressureEnable", False)),
            "disk_pressure": int(get_bool(pa, "predicate.DiskPressureEnable", False)),
            "pid_pressure": int(get_bool(pa, "predicate.PIDPressureEnable", False)),
            "w_lr": get_int(na, "leastrequested.weight", 1), "w_bra": get_int(na, "balancedresource.weight", 1),
            "w_na": get_int(na, "nodeaffinity.weight", 1), "w_pa": get_int(na, "podaffinity.weight", 1),
        }

    # ---------------- task specs ----------------
    def _specs(self):
        pending = [t for t in self.session_tasks if t["status"] == ST["Pending"]]
        scal = set()
        for t in pending:
            scal.update((t["initreq"].sc or {}).keys())
            scal.update((t["resreq"].sc or {}).keys())
        tab = SpecTable(sorted(scal), self.aff_in_play)
        for t in pending:
            t["spec"] = tab.add(t["pod"], t["initreq"], t["resreq"])
        tab.finish(self)

    # ---------------- node SoA ----------------
    def _node_table(self):
        n = len(self.nodes)
        S, K, P = len(self.scalars), len(self.label_keys.ids), len(self.port_slots.ids)
        self.n_nodes = n
        z64 = lambda *s: np.zeros(s, dtype=np.int64)
        cols = {k: z64(n) for k in ("idle_cpu", "idle_mem", "rel_cpu", "rel_mem", "alloc_cpu", "alloc_mem",
                                    "nz_cpu", "nz_mem")}
        cols["idle_sc"], cols["rel_sc"] = z64(S, n), z64(S, n)
        cols["pod_count"] = np.zeros(n, np.int32)
        cols["max_pods"] = np.zeros(n, np.int32)
        cols["flags"] = np.zeros(n, np.uint32)
        cols["label_val"] = np.full((K, n), -1, np.int32)
        cols["label_int"] = z64(K, n)
        cols["label_int_ok"] = np.zeros((K, n), np.uint8)
        cols["taint_set"] = np.zeros(n, np.int32)
        cols["port_used"] = np.zeros((P, n), np.uint64)
        taint_sets = _Interner()
        taint_sets(())
        taint_list = [[]]
        keys = sorted(self.label_keys.ids.items(), key=lambda kv: kv[1])
        for i, nd in enumerate(self.nodes):
            node = nd["node"]
            cols["idle_cpu"][i], cols["idle_mem"][i] = nd["idle"].cpu, nd["idle"].mem
            cols["rel_cpu"][i], cols["rel_mem"][i] = nd["rel"].cpu, nd["rel"].mem
            for s, name in enumerate(self.scalars):
                cols["idle_sc"][s, i] = (nd["idle"].sc or {}).get(name, 0)
                cols["rel_sc"][s, i] = (nd["rel"].sc or {}).get(name, 0)
            cols["alloc_cpu"][i] = node.alloc.get(M.CPU, 0)      # schedulercache NewResource: cpu MilliValue
            cols["alloc_mem"][i] = node.alloc.get(M.MEMORY, 0)   # memory Value
            cols["nz_cpu"][i], cols["nz_mem"][i] = nd["nz"]
            cols["pod_count"][i] = len(nd["tasks"])
            cols["max_pods"][i] = nd["alloc"].max_task
            f = 0
            if nd["idle"].sc is not None:
                f |= NODE_IDLE_HAS_MAP
            if nd["rel"].sc is not None:
                f |= NODE_REL_HAS_MAP
            for c in node.conditions:  # CheckNodeConditionPredicate (predicates.go:1568-1596)
                typ, st = c.get("type"), c.get("status")
                if typ == "Ready" and st != "True":
                    f |= NODE_NOT_READY
                elif typ == "OutOfDisk" and st != "False":
                    f |= NODE_OUT_OF_DISK
                elif typ == "NetworkUnavailable" and st != "False":
                    f |= NODE_NET_UNAVAIL
            if node.unschedulable:
                f |= NODE_UNSCHEDULABLE
            press = {}
            for c in node.conditions:  # schedulercache SetNode keeps the last of each (cache/node_info.go:613-626)
                if c.get("type") in ("MemoryPressure", "DiskPressure", "PIDPressure"):
                    press[c["type"]] = c.get("status")
            if press.get("MemoryPressure") == "True":
                f |= NODE_MEM_PRESSURE
            if press.get("DiskPressure") == "True":
                f |= NODE_DISK_PRESSURE
            if press.get("PIDPressure") == "True":
                f |= NODE_PID_PRESSURE
            cols["flags"][i] = f
            for key, k in keys:
                v = node.name if key == "\x00metadata.name" else node.labels.get(key)
                if v is None:
                    continue
                cols["label_val"][k, i] = self.values(v)
                iv = parse_int64(v) if key in self.gtlt_keys else None
                if iv is not None:
                    cols["label_int"][k, i] = iv
                    cols["label_int_ok"][k, i] = 1
            ts = tuple(sorted((t.get("key", ""), t.get("value", ""), t.get("effect", "")) for t in node.taints
                              if t.get("effect") in ("NoSchedule", "NoExecute")))
            tid = taint_sets(ts)
            if tid == len(taint_list):
                taint_list.append([{"key": a, "value": b, "effect": c} for a, b, c in ts])
            cols["taint_set"][i] = tid
            for t in nd["tasks"]:  # existing pods' host ports (HostPortInfo.Add)
                for c in t["pod"].containers:
                    for pt in c.ports:
                        hp = int(pt.get("hostPort", 0) or 0)
                        if hp <= 0:
                            continue
                        key = (pt.get("protocol") or "TCP", hp)
                        s_id = self.port_slots.ids.get(key)
                        if s_id is None:
                            continue
                        ip = pt.get("hostIP") or "0.0.0.0"
                        ipid = self.port_ips[s_id].ids.get(ip, 63)
                        cols["port_used"][s_id, i] |= np.uint64(1 << ipid)
        self.cols = cols
        if not self.tol_list:
            self.tol_list.append([])
        self.tolerates = np.zeros((len(self.tol_list), len(taint_list)), np.uint8)
        for a, tols in enumerate(self.tol_list):
            for b, taints in enumerate(taint_list):
                self.tolerates[a, b] = all(any(_tolerates(o, t) for o in tols) for t in taints)
        self.n_label, self.n_port = K, P

    # ---------------- session arrays (kb_session) ----------------
    def _session_arrays(self):
        acc = set()
        for t in self.session_tasks:
            acc.update((t["resreq"].sc or {}).keys())
        total = Res()
        for nd in self.nodes:
            total.add(nd["alloc"])
        acc.update((total.sc or {}).keys())
        self.acc_scalars = sorted(acc)
        if len(self.acc_scalars) > 62:
            raise Unsupported("more than 62 accounting scalar resources")
        aslot = {n: i for i, n in enumerate(self.acc_scalars)}
        R = 2 + len(self.acc_scalars)

        def pack(r):
            v = np.zeros(R, np.float64)
            v[0], v[1] = r.cpu, r.mem
            mask = 0
            if r.sc is not None:
                mask |= 1 << 63
                for k, q in r.sc.items():
                    v[2 + aslot[k]] = q
                    mask |= 1 << aslot[k]
            return v, mask

        ts = self.session_tasks
        nt = len(ts)
        job_idx = {j["uid"]: i for i, j in enumerate(self.jobs)}
        q_idx = {q: i for i, q in enumerate(self.queue_names)}
        uid_rank = {u: i for i, u in enumerate(sorted(t["uid"] for t in ts))}
        self.s_task_job = np.array([job_idx[t["job"]] for t in ts], np.int32)
        self.s_task_spec = np.array([t.get("spec", -1) if t["status"] == ST["Pending"] else -1 for t in ts], np.int32)
        self.s_task_status = np.array([t["status"] for t in ts], np.int32)
        self.s_task_priority = np.array([t["priority"] for t in ts], np.int32)
        self.s_task_ctime = np.array([t["pod"].ctime for t in ts], np.int64)
        self.s_task_uid_rank = np.array([uid_rank[t["uid"]] for t in ts], np.int32)
        res = np.zeros((nt, R), np.float64)
        masks = np.zeros(nt, np.uint64)
        for i, t in enumerate(ts):
            res[i], masks[i] = pack(t["resreq"])
        self.s_task_resreq, self.s_task_resreq_mask = res, masks
        js = self.jobs
        self.s_job_queue = np.array([q_idx[j["pg"].queue] for j in js], np.int32)
        self.s_job_priority = np.array([j["pg"].priority for j in js], np.int32)
        self.s_job_min = np.array([j["pg"].min_member for j in js], np.int32)
        self.s_job_ctime = np.array([j["pg"].ctime for j in js], np.int64)
        self.s_job_uid_rank = np.arange(len(js), dtype=np.int32)  # jobs are already in UID order
        self.s_job_pg_pending = np.array([1 if j["pg"].phase == "Pending" else 0 for j in js], np.int32)
        self.s_queue_weight = np.array([q.weight for q in self.queues], np.int32)
        self.s_queue_ctime = np.array([q.ctime for q in self.queues], np.int64)
        self.s_queue_uid_rank = np.arange(len(self.queues), dtype=np.int32)
        self.s_total, tm = pack(total)
        self.s_total_mask = tm
        self.s_tiers = np.array([(ti, pid, en, 0) for ti, pid, en in self.tier_plugins],
                                dtype=np.dtype([("tier", "<i4"), ("plugin", "<i4"), ("enable", "<u4"),
                                                ("pad", "<i4")])) if self.tier_plugins else \
            np.zeros(0, dtype=np.dtype([("tier", "<i4"), ("plugin", "<i4"), ("enable", "<u4"), ("pad", "<i4")]))

    # ---------------- inputs of the affinity tables (affinity.Tables.build) ----------------
    def slot_domains(self, keys):
        """Topology domain of every session node for the key tuple (-1: a key missing) and the domain count."""
        ids, dom = {}, np.full(self.n_nodes, -1, np.int32)
        for i, nd in enumerate(self.nodes):
            labels = nd["node"].labels
            if all(k in labels for k in keys):
                dom[i] = ids.setdefault(tuple(labels[k] for k in keys), len(ids))
        return dom, len(ids)

    def aff_groups(self, unsupported):
        """Lister pods, existing pods and every spec's pending pod, one pod per group here."""
        lister = []
        for t in self.session_tasks:
            if allocated_status(t["status"]):
                if t["pod"].node not in self.node_index:
                    raise unsupported("lister pod on a node outside the session (predicates.go: failed to find node)")
                lister.append((t["pod"], [self.node_index[t["pod"].node]], [t["uid"]]))
        existing = [(t["pod"], [i]) for i, nd in enumerate(self.nodes) for t in nd["tasks"]]
        pending = {}
        for t in self.session_tasks:
            if "spec" in t and t["status"] == ST["Pending"]:
                pending.setdefault(t["spec"], t["pod"])
        return lister, existing, [pending[s] for s in range(len(self.spec_arr))]

    # ---------------- helpers ----------------
    def node_names(self):
        return [n["node"].name for n in self.nodes]

    def pending_spec(self, uid: str) -> int:
        for t in self.session_tasks:
            if t["uid"] == uid:
                return t["spec"]
        raise KeyError(uid)


# ---- kb_apply rows: commits made outside the device ----------------------------------------------------
def pod_delta(snap: Snapshot, pod: M.Pod, node: int, remove: bool = False, spec: int = -1, kind: int = 1):
    """The kb_row_delta of NodeInfo.AddTask (or RemoveTask) of `pod` on session node `node` (api/node_info.go:
    165-221) plus the plugins' schedulercache AddPod / RemovePod (cache/node_info.go:498-630): Idle /
    Releasing by the pod's status, pod count, non-zero requests, host ports. The node's resource maps are the
    session-open ones (a caller that commits in between keeps its own). Returns (row dict, scalar deltas,
    ports): the scalar deltas are [idle per slot..., releasing per slot...] or None."""
    st = task_status(pod)
    rr = Res()
    for c in pod.containers:
        rr.add(Res.from_list(c.req))
    idle, rel = snap.nodes[node]["idle"].copy(), snap.nodes[node]["rel"].copy()
    i0, r0 = idle.copy(), rel.copy()
    if not remove:
        if st == ST["Releasing"]:
            rel.add(rr)
            idle.sub(rr)
        elif st == ST["Pipelined"]:
            rel.sub(rr)
        else:
            idle.sub(rr)
    else:
        if st == ST["Releasing"]:
            rel.sub(rr)
            idle.add(rr)
        elif st == ST["Pipelined"]:
            rel.add(rr)
        else:
            idle.add(rr)
    sign = -1 if remove else 1
    nzc = nzm = 0
    for c in pod.containers:
        a, b = nonzero(c.req)
        nzc += a
        nzm += b
    flags_set = (NODE_IDLE_HAS_MAP if i0.sc is None and idle.sc is not None else 0) | \
        (NODE_REL_HAS_MAP if r0.sc is None and rel.sc is not None else 0)
    sc = None
    if snap.scalars and (idle.sc is not None or rel.sc is not None):
        sc = [(idle.sc or {}).get(k, 0) - (i0.sc or {}).get(k, 0) for k in snap.scalars] + \
             [(rel.sc or {}).get(k, 0) - (r0.sc or {}).get(k, 0) for k in snap.scalars]
    ports = []
    for c in pod.containers:  # HostPortInfo.Add / Remove, only the (protocol, port) slots a spec asks for
        for pt in c.ports:
            hp = int(pt.get("hostPort", 0) or 0)
            s_id = snap.port_slots.ids.get((pt.get("protocol") or "TCP", hp)) if hp > 0 else None
            if s_id is not None:
                ports.append((s_id, snap.port_ips[s_id].ids.get(pt.get("hostIP") or "0.0.0.0", 63)))
    row = {"node": node, "pods": sign, "idle_cpu": idle.cpu - i0.cpu, "idle_mem": idle.mem - i0.mem,
           "rel_cpu": rel.cpu - r0.cpu, "rel_mem": rel.mem - r0.mem, "nz_cpu": sign * nzc, "nz_mem": sign * nzm,
           "flags_set": flags_set, "flags_clear": 0, "spec": spec, "kind": kind}
    return row, sc, ports


def row_deltas(rows):
    """Pack pod_delta results into kb_apply's arrays (deltas, scalar deltas, ports)."""
    from .runtime import ROW_DELTA_DTYPE
    d = np.zeros(len(rows), ROW_DELTA_DTYPE)
    sc, ports = [], []
    for i, (row, s, p) in enumerate(rows):
        for k, v in row.items():
            d[i][k] = v
        d[i]["sc_off"] = 0xffffffff if s is None else len(sc)
        sc += s or []
        d[i]["port_off"], d[i]["port_cnt"] = len(ports), len(p)
        ports += p
    return d, np.array(sc, np.int64), np.array(ports, PORT_DTYPE) if ports else np.zeros(0, PORT_DTYPE)
