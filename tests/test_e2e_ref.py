"""The reference's e2e expectations (test/e2e/nodeorder.go:29-237, test/e2e/predicates.go:35-525), restated as
fixtures (tests/golden/ref-e2e-*.json): they pin LeastRequested, NodeAffinity, InterPodAffinity, taints, host
ports, max pods and resource fit to outcomes the reference itself states. CPU: the oracle meets every
assertion. GPU: the HIP path meets them too, with the oracle's binds cycle by cycle."""
import pytest

from oracle import pyoracle
from scheduler_amd import runtime

import e2e_scenarios as E2E

SCENARIOS = [(f"{f}/{s['name']}", s) for f in ("nodeorder", "predicates") for s in E2E.load(f)]


@pytest.mark.parametrize("name,scenario", SCENARIOS, ids=[n for n, _ in SCENARIOS])
def test_oracle_meets_reference_e2e(name, scenario):
    E2E.run(scenario, pyoracle.allocate_backfill)


@pytest.mark.gpu
@pytest.mark.parametrize("name,scenario", SCENARIOS, ids=[n for n, _ in SCENARIOS])
def test_gpu_meets_reference_e2e(name, scenario):
    want = E2E.run(scenario, pyoracle.allocate_backfill)
    got = E2E.run(scenario, runtime.allocate_backfill)
    assert got == want
