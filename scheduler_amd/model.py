"""Cluster object model for the allocate hot path (host side, no GPU).

Plain-data restatement of the k8s / kube-batch objects the allocate path reads:
v1.Node, v1.Pod, v1alpha1.PodGroup, v1alpha1.Queue and the scheduler tier
configuration. The builders mirror the reference's fixture helpers
(`pkg/scheduler/util/test_utils.go:34-92`) so tests read like the reference's
own tests.

Quantities are parsed once here into the canonical integer units the reference
converts them to (`pkg/scheduler/api/resource_info.go:75-93`): cpu and scalar
resources in milli-units (`Quantity.MilliValue`), memory and pods in units
(`Quantity.Value`). Both the oracle (C++) and the device exporter consume these
integers.
"""
from __future__ import annotations

import copy
import json
import re
from dataclasses import dataclass, field
from fractions import Fraction
from typing import Dict, List, Optional

# --------------------------------------------------------------------------
# resource.Quantity parsing (k8s.io/apimachinery/pkg/api/resource/quantity.go)
# --------------------------------------------------------------------------
_BIN = {"Ki": 2 ** 10, "Mi": 2 ** 20, "Gi": 2 ** 30, "Ti": 2 ** 40, "Pi": 2 ** 50, "Ei": 2 ** 60}
_DEC = {"n": Fraction(1, 10 ** 9), "u": Fraction(1, 10 ** 6), "m": Fraction(1, 1000), "": Fraction(1),
        "k": Fraction(10 ** 3), "M": Fraction(10 ** 6), "G": Fraction(10 ** 9), "T": Fraction(10 ** 12),
        "P": Fraction(10 ** 15), "E": Fraction(10 ** 18)}
_QRE = re.compile(r"^([+-]?)(\d*)(?:\.(\d*))?(.*)$")


def parse_quantity(s) -> Fraction:
    """Exact value of a k8s quantity string ("500m", "1G", "4Gi", "1e3", 2)."""
    if isinstance(s, (int, Fraction)):
        return Fraction(s)
    s = str(s).strip()
    m = _QRE.match(s)
    if not m or (m.group(2) == "" and not m.group(3)):
        raise ValueError(f"invalid quantity {s!r}")
    sign, ip, fp, suf = m.group(1), m.group(2) or "0", m.group(3) or "", m.group(4)
    v = Fraction(int(ip)) + (Fraction(int(fp), 10 ** len(fp)) if fp else 0)
    if suf in _BIN:
        v *= _BIN[suf]
    elif suf in _DEC:
        v *= _DEC[suf]
    elif suf[:1] in ("e", "E"):
        v *= Fraction(10) ** int(suf[1:])
    else:
        raise ValueError(f"invalid quantity suffix {s!r}")
    return -v if sign == "-" else v


def _ceil(f: Fraction) -> int:
    return -((-f.numerator) // f.denominator)


def milli_value(q) -> int:
    """Quantity.MilliValue(): ceil(q * 1000)."""
    return _ceil(parse_quantity(q) * 1000)


def value(q) -> int:
    """Quantity.Value(): ceil(q)."""
    return _ceil(parse_quantity(q))


CPU, MEMORY, PODS, EPHEMERAL = "cpu", "memory", "pods", "ephemeral-storage"
GPU_RESOURCE_NAME = "nvidia.com/gpu"  # api/resource_info.go:40


def canon_resource_list(rl: Dict[str, object]) -> Dict[str, int]:
    """Convert a v1.ResourceList to canonical integers (milli for cpu/scalars)."""
    out = {}
    for k, q in rl.items():
        if k in (MEMORY, PODS, EPHEMERAL):
            out[k] = value(q)
        else:
            out[k] = milli_value(q)
    return out


# --------------------------------------------------------------------------
# Objects
# --------------------------------------------------------------------------
@dataclass
class Node:
    name: str
    alloc: Dict[str, int]
    cap: Optional[Dict[str, int]] = None
    labels: Dict[str, str] = field(default_factory=dict)
    taints: List[dict] = field(default_factory=list)  # {"key","value","effect"}
    unschedulable: bool = False
    conditions: List[dict] = field(default_factory=list)  # {"type","status"}

    def to_json(self):
        return {"name": self.name, "alloc": self.alloc, "cap": self.cap if self.cap is not None else self.alloc,
                "labels": self.labels, "taints": self.taints, "unschedulable": self.unschedulable,
                "conditions": self.conditions}


@dataclass
class Container:
    req: Dict[str, int] = field(default_factory=dict)
    ports: List[dict] = field(default_factory=list)  # {"hostPort","hostIP","protocol"}

    def to_json(self):
        return {"req": self.req, "ports": self.ports}


@dataclass
class Pod:
    ns: str
    name: str
    uid: str
    node: str = ""
    phase: str = "Pending"
    deleting: bool = False
    group: str = ""
    priority: Optional[int] = None
    ctime: int = 0
    labels: Dict[str, str] = field(default_factory=dict)
    containers: List[Container] = field(default_factory=list)
    init: List[Container] = field(default_factory=list)
    node_selector: Dict[str, str] = field(default_factory=dict)
    tolerations: List[dict] = field(default_factory=list)
    affinity: Optional[dict] = None

    def to_json(self):
        return {"ns": self.ns, "name": self.name, "uid": self.uid, "node": self.node, "phase": self.phase,
                "deleting": self.deleting, "group": self.group, "priority": self.priority, "ctime": self.ctime,
                "labels": self.labels, "containers": [c.to_json() for c in self.containers],
                "init": [c.to_json() for c in self.init], "nodeSelector": self.node_selector,
                "tolerations": self.tolerations, "affinity": self.affinity}


@dataclass
class PodGroup:
    ns: str
    name: str
    queue: str
    min_member: int = 0
    phase: str = ""
    ctime: int = 0
    priority: int = 0  # resolved priority-class value (cache/cache.go:608-617)

    def to_json(self):
        return {"ns": self.ns, "name": self.name, "queue": self.queue, "minMember": self.min_member,
                "phase": self.phase, "ctime": self.ctime, "priority": self.priority}


@dataclass
class Queue:
    name: str
    weight: int = 1
    ctime: int = 0

    def to_json(self):
        return {"name": self.name, "weight": self.weight, "ctime": self.ctime}


PLUGIN_FLAGS = ("enabledJobOrder", "enabledJobReady", "enabledJobPipelined", "enabledTaskOrder",
                "enabledPreemptable", "enabledReclaimable", "enabledQueueOrder", "enabledPredicate",
                "enabledNodeOrder")


def plugin(name: str, arguments: Optional[Dict[str, str]] = None, defaults: bool = True, **flags):
    """A conf.PluginOption (conf/scheduler_conf.go:37-56). With defaults=True every unset flag
    becomes true, as plugins.ApplyPluginConfDefaults does (plugins/defaults.go:22-52)."""
    p = {"name": name, "arguments": dict(arguments or {})}
    for f in PLUGIN_FLAGS:
        p[f] = flags.get(f, True if defaults else None)
    return p


def default_tiers(nodeorder_args=None, predicate_args=None):
    """The default scheduler conf (pkg/scheduler/util.go:31-42) with defaults applied."""
    return [
        {"plugins": [plugin("priority"), plugin("gang")]},
        {"plugins": [plugin("drf"), plugin("predicates", predicate_args), plugin("proportion"),
                     plugin("nodeorder", nodeorder_args)]},
    ]


# pkg/scheduler/util.go:30-40 (defaultSchedulerConf)
DEFAULT_SCHEDULER_CONF = """
actions: "allocate, backfill"
tiers:
- plugins:
  - name: priority
  - name: gang
- plugins:
  - name: drf
  - name: predicates
  - name: proportion
  - name: nodeorder
"""
ACTIONS = ("reclaim", "allocate", "backfill", "preempt", "enqueue")  # actions/factory.go:29-35
# conf.PluginOption yaml tags (conf/scheduler_conf.go:33-56) -> the flag names used in tier dicts
_YAML_FLAGS = {"enable" + f[len("enabled"):]: f for f in PLUGIN_FLAGS}


def load_scheduler_conf(text: str):
    """loadSchedulerConf (pkg/scheduler/util.go:44-73): parse the YAML conf, apply the plugin defaults to
    every unset enable flag (plugins/defaults.go:22-52) and resolve the comma-separated action list.
    Returns (action names, tiers); an unknown action raises ValueError as the reference returns an error."""
    import yaml
    doc = yaml.safe_load(text) or {}
    tiers = []
    for t in doc.get("tiers") or []:
        plugins = []
        for p in t.get("plugins") or []:
            flags = {_YAML_FLAGS[k]: bool(v) for k, v in p.items() if k in _YAML_FLAGS and v is not None}
            args = {str(k): str(v) for k, v in (p.get("arguments") or {}).items()}
            plugins.append(plugin(p.get("name", ""), args, defaults=True, **flags))
        tiers.append({"plugins": plugins})
    actions = []
    for name in str(doc.get("actions", "")).split(","):
        name = name.strip()
        if name not in ACTIONS:
            raise ValueError(f"failed to found Action {name}, ignore it")
        actions.append(name)
    return actions, tiers


@dataclass
class Cluster:
    """The scheduler cache contents one allocate cycle snapshots."""
    nodes: List[Node] = field(default_factory=list)
    pods: List[Pod] = field(default_factory=list)
    pod_groups: List[PodGroup] = field(default_factory=list)
    queues: List[Queue] = field(default_factory=list)
    tiers: List[dict] = field(default_factory=default_tiers)

    def to_json(self):
        return {"nodes": [n.to_json() for n in self.nodes], "pods": [p.to_json() for p in self.pods],
                "podGroups": [g.to_json() for g in self.pod_groups], "queues": [q.to_json() for q in self.queues],
                "tiers": self.tiers}

    def dumps(self) -> str:
        return json.dumps(self.to_json(), separators=(",", ":"))

    @staticmethod
    def from_json(d) -> "Cluster":
        """Inverse of to_json (fixtures under tests/golden/)."""
        def ctr(c):
            return Container(req=dict(c["req"]), ports=list(c["ports"]))
        nodes = [Node(name=n["name"], alloc=dict(n["alloc"]), cap=dict(n["cap"]), labels=dict(n["labels"]),
                      taints=list(n["taints"]), unschedulable=n["unschedulable"], conditions=list(n["conditions"]))
                 for n in d["nodes"]]
        pods = [Pod(ns=p["ns"], name=p["name"], uid=p["uid"], node=p["node"], phase=p["phase"],
                    deleting=p["deleting"], group=p["group"], priority=p["priority"], ctime=p["ctime"],
                    labels=dict(p["labels"]), containers=[ctr(c) for c in p["containers"]],
                    init=[ctr(c) for c in p["init"]], node_selector=dict(p["nodeSelector"]),
                    tolerations=list(p["tolerations"]), affinity=p["affinity"]) for p in d["pods"]]
        groups = [PodGroup(ns=g["ns"], name=g["name"], queue=g["queue"], min_member=g["minMember"], phase=g["phase"],
                           ctime=g["ctime"], priority=g["priority"]) for g in d["podGroups"]]
        queues = [Queue(name=q["name"], weight=q["weight"], ctime=q["ctime"]) for q in d["queues"]]
        return Cluster(nodes=nodes, pods=pods, pod_groups=groups, queues=queues, tiers=d["tiers"])

    def copy(self) -> "Cluster":
        return copy.deepcopy(self)


# --------------------------------------------------------------------------
# Builders (pkg/scheduler/util/test_utils.go)
# --------------------------------------------------------------------------
def build_resource_list(cpu, memory, **scalars) -> Dict[str, int]:
    """util.BuildResourceList (test_utils.go:34-40): always carries nvidia.com/gpu: 0."""
    rl = {CPU: cpu, MEMORY: memory, GPU_RESOURCE_NAME: "0"}
    for k, v in scalars.items():
        rl[k.replace("__", "/").replace("_", ".")] = v
    return canon_resource_list(rl)


def build_resource_list_with_gpu(cpu, memory, gpu) -> Dict[str, int]:
    return canon_resource_list({CPU: cpu, MEMORY: memory, GPU_RESOURCE_NAME: gpu})


def resource_list(**kw) -> Dict[str, int]:
    """Arbitrary v1.ResourceList: resource_list(cpu="2", memory="4Gi", pods=110, **{"nvidia.com/gpu": 8})."""
    return canon_resource_list(kw)


def build_node(name, alloc, labels=None, **kw) -> Node:
    """util.BuildNode (test_utils.go:52-63). Note: no `pods` allocatable unless alloc carries it."""
    return Node(name=name, alloc=dict(alloc), cap=dict(alloc), labels=dict(labels or {}), **kw)


def build_pod(ns, name, nodename, phase, req, group_name, labels=None, selector=None, **kw) -> Pod:
    """util.BuildPod (test_utils.go:66-92): UID = "<ns>-<name>", one container."""
    return Pod(ns=ns, name=name, uid=f"{ns}-{name}", node=nodename, phase=phase, group=group_name,
               labels=dict(labels or {}), node_selector=dict(selector or {}),
               containers=[Container(req=dict(req))], **kw)
