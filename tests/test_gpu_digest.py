"""Full-size parity: the HIP path against the oracle's frozen outcome on BASELINE.json's configurations at
full size (tests/golden/digest-<cfg>.{npz,json}, written by tests/golden/make_digests.py from the oracle).

The GPU run rebuilds the same seeded cluster, runs one allocate cycle through the C-ABI and compares the
whole placement sequence (task, node, kind per event), every job's failing task, the sha256 of those arrays
and the FitErrors of the failed jobs. No oracle runs on the GPU box.
"""
import json
import os

import numpy as np
import pytest

from scheduler_amd import export as E
from scheduler_amd import runtime, synth

from helpers import digest_arrays

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DIGESTS = sorted(f[len("digest-"):-len(".json")] for f in os.listdir(HERE) if f.startswith("digest-")
                 and f.endswith(".json"))


def _load(cfg):
    with open(os.path.join(HERE, f"digest-{cfg}.json")) as f:
        meta = json.load(f)
    arr = np.load(os.path.join(HERE, f"digest-{cfg}.npz"), allow_pickle=False)
    return meta, {k: arr[k] for k in arr.files}


FULL = [c for c in DIGESTS if _load(c)[0].get("max_tasks", -1) < 0]  # whole cycles (prefixes: test_gpu_shard)
# BASELINE.json configs[4] (C5): the C2 shape at 50k nodes x 1M pods (tests/golden/make_digests.py SHAPES); one GPU
# runs it whole on the split fed engine with range selectors
ARRAY_SHAPES = {"C5": dict(n_nodes=50000, n_jobs=10000, tasks_per_job=100, seed=synth.SEED)}


def test_digests_are_consistent():
    """CPU: every committed digest's arrays hash to its recorded sha256."""
    assert DIGESTS, "no full-size digests committed"
    for cfg in DIGESTS:
        meta, a = _load(cfg)
        assert digest_arrays(a["event_task"], a["event_node"], a["event_kind"], a["job_fail"]) == meta["sha256"]
        assert len(a["event_task"]) == meta["events"]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", FULL)
def test_full_size_matches_oracle_digest(cfg):
    meta, want = _load(cfg)
    if cfg in ARRAY_SHAPES:  # 1M pods: the numpy session builder (equal to the exporter: test_export.py)
        snap = synth.c2_snapshot(**ARRAY_SHAPES[cfg])
    else:
        snap = E.Snapshot(synth.CONFIGS[cfg]())
    assert (snap.n_nodes, len(snap.session_tasks)) == (meta["nodes"], meta["pods"])
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
    finally:
        ctx.close()
    k = int(out["n_events"])
    et = out["event_task"][:k].astype(np.int32)
    en = out["task_node"][et].astype(np.int32)
    ek = np.where(out["task_status"][et] == E.ST["Pipelined"], 2, 1).astype(np.int8)
    jf = out["job_fail_task"][:len(snap.jobs)].astype(np.int32)
    assert k == meta["events"]
    assert np.array_equal(et, want["event_task"])
    assert np.array_equal(en, want["event_node"])
    assert np.array_equal(ek, want["event_kind"])
    assert np.array_equal(jf, want["job_fail"])
    assert digest_arrays(et, en, ek, jf) == meta["sha256"]
    if cfg not in ARRAY_SHAPES:
        assert runtime.result_dict(snap, out)["fit_errors"] == meta["fit_errors"]
    else:
        assert not meta["fit_errors"] and (jf < 0).all()
