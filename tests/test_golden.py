"""Golden fixtures (tests/golden/*.json, written by tests/golden/make_golden.py).

ref-*    : the reference's own unit-test vectors as data (expected binds from its test files): the oracle
           and the HIP path must both reproduce them.
oracle-* : the oracle's allocate outcomes on small seeded clusters: the oracle must still reproduce them
           (CPU), and the HIP path must match them through the C-ABI (GPU), bit for bit.
"""
import glob
import json
import os

import pytest

from oracle import pyoracle
from scheduler_amd import model as m

GOLDEN = sorted(p for p in glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json"))
                if not os.path.basename(p).startswith(("digest-", "ref-e2e-")))  # own formats: test_gpu_digest.py,
# test_e2e_ref.py
IDS = [os.path.basename(p)[:-5] for p in GOLDEN]


def _load(path):
    with open(path) as f:
        doc = json.load(f)
    return doc, m.Cluster.from_json(doc["cluster"])


def _check(doc, out):
    exp = doc["expected"]
    assert out["binds"] == exp["binds"]
    if "events" in exp:
        assert out["events"] == exp["events"]
        assert out["fit_errors"] == exp["fit_errors"]
        for uid, st in out["status"].items():  # as tests/test_gpu_parity.py: pods outside any job are not reported
            assert exp["status"][uid] == st, uid


def test_fixture_set_present():
    names = set(IDS)
    assert {"ref-allocate-one-job", "ref-allocate-two-jobs", "ref-select-best-node"} <= names
    assert sum(n.startswith("oracle-") for n in names) >= 8


@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_fixture_round_trip(path):
    doc, cl = _load(path)
    assert cl.to_json() == doc["cluster"]


@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_oracle_reproduces_golden(path):
    doc, cl = _load(path)
    _check(doc, pyoracle.allocate(cl))


@pytest.mark.gpu
@pytest.mark.parametrize("path", GOLDEN, ids=IDS)
def test_device_matches_golden(path):
    from scheduler_amd import runtime
    doc, cl = _load(path)
    _check(doc, runtime.allocate(cl))
