"""ctypes loader for the oracle (CPU restatement of the reference's allocate path).

TEST INFRASTRUCTURE: imported only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker or the CPU baseline -- never by the
product package `scheduler_amd`.
"""
from __future__ import annotations

import ctypes
import json
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH) or (
            os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(os.path.join(_HERE, f))
                                              for f in ("oracle.cpp", "json.h"))):
        subprocess.check_call(["make", "-s", "-C", _HERE], stdout=subprocess.DEVNULL)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        build()
        lib = ctypes.CDLL(_LIB_PATH)
        lib.oracle_call.restype = ctypes.c_void_p
        lib.oracle_call.argtypes = [ctypes.c_char_p]
        lib.oracle_free.argtypes = [ctypes.c_void_p]
        _lib = lib
    return _lib


class OraclePanic(RuntimeError):
    """The reference would panic (util/assert or SelectBestNode on an empty map)."""


def call(req: dict) -> dict:
    lib = _load()
    ptr = lib.oracle_call(json.dumps(req, separators=(",", ":")).encode())
    try:
        out = json.loads(ctypes.string_at(ptr).decode())
    finally:
        lib.oracle_free(ptr)
    if "panic" in out:
        raise OraclePanic(out["panic"])
    if "exception" in out:
        raise RuntimeError(out["exception"])
    return out


def allocate(cluster, workers: int = 1, literal_affinity: bool = False, max_tasks: int = -1) -> dict:
    """Run allocateAction.Execute on the cluster snapshot (actions/allocate/allocate.go:42-193)."""
    req = cluster.to_json() if hasattr(cluster, "to_json") else dict(cluster)
    req = dict(req)
    req["op"] = "allocate"
    req["options"] = {"workers": workers, "literal_affinity": literal_affinity, "max_tasks": max_tasks}
    return call(req)


def allocate_backfill(cluster, literal_affinity: bool = False) -> dict:
    """allocate then backfill (the default action list, util.go:32; actions/backfill/backfill.go:40-90)."""
    req = dict(cluster.to_json())
    req["op"] = "allocate_backfill"
    req["options"] = {"workers": 1, "literal_affinity": literal_affinity, "max_tasks": -1}
    return call(req)


def evaluate(cluster, task_uids, literal_affinity: bool = False) -> dict:
    """Per-(task, node) predicate reasons and total score at session-open state."""
    req = dict(cluster.to_json())
    req["op"] = "eval"
    req["eval_tasks"] = list(task_uids)
    req["options"] = {"workers": 1, "literal_affinity": literal_affinity}
    return call(req)


def sort_nodes(cluster, task_uids, literal_affinity: bool = False) -> dict:
    """preempt's sweep per task: PredicateNodes(PredicateFn) -> PrioritizeNodes -> SortNodes order
    (actions/preempt/preempt.go:187-195) at session-open state."""
    req = dict(cluster.to_json())
    req["op"] = "sort_nodes"
    req["eval_tasks"] = list(task_uids)
    req["options"] = {"workers": 1, "literal_affinity": literal_affinity}
    return call(req)


def resource_op(op: str, **kw) -> dict:
    req = {"op": op}
    req.update(kw)
    return call(req)
