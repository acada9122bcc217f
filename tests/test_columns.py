"""The columnar exporter (scheduler_amd/columns.py) against the per-pod exporter: the same
arrays, field by field, on every parity, affinity, error and edge cluster, and the same refusals."""
import numpy as np
import pytest

from scheduler_amd import columns as COL
from scheduler_amd import export as E
from scheduler_amd import synth

from helpers import (affinity_clusters, affinity_error_clusters, backfill_cluster, ipa_error_clusters,
                     parity_clusters)

FIELDS = ("n_nodes", "config", "scalars", "n_label", "n_port", "spec_arr", "sc_init", "sc_req", "term_arr", "req_arr",
          "val_arr", "port_arr", "tolerates", "acc_scalars", "s_task_job", "s_task_spec", "s_task_status",
          "s_task_priority", "s_task_ctime", "s_task_uid_rank", "s_task_resreq", "s_task_resreq_mask", "s_job_queue",
          "s_job_priority", "s_job_min", "s_job_ctime", "s_job_uid_rank", "s_job_pg_pending", "s_queue_weight",
          "s_queue_ctime", "s_queue_uid_rank", "s_total", "s_total_mask", "s_tiers")
AFF = ("topo_dom", "table_arr", "totals", "counters", "spec_arr", "check_arr", "lister_arr", "hist_arr", "h",
       "own_err", "xb_pods", "xb_spec", "ipa_error")


def _eq(a, b, what):
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        a, b = np.asarray(a), np.asarray(b)
        assert a.shape == b.shape and a.dtype == b.dtype, (what, a.shape, b.shape, a.dtype, b.dtype)
        assert np.array_equal(a, b), what
    else:
        assert a == b, what


def assert_same_snapshot(ref, got):
    for f in FIELDS:
        _eq(getattr(ref, f), getattr(got, f), f)
    assert set(ref.cols) == set(got.cols)
    for k in ref.cols:
        _eq(ref.cols[k], got.cols[k], f"cols[{k}]")
    assert ref.node_names() == got.node_names()
    assert (ref.aff is None) == (got.aff is None)
    if ref.aff is not None:
        for f in AFF:
            _eq(getattr(ref.aff, f), getattr(got.aff, f), f"aff.{f}")
        # increments: one list per spec, order-free (the device applies them with atomics)
        for s, row in enumerate(ref.aff.spec_arr):
            a = sorted(map(tuple, ref.aff.incr_arr[row["incr_off"]:row["incr_off"] + row["incr_cnt"]].tolist()))
            b = sorted(map(tuple, got.aff.incr_arr[row["incr_off"]:row["incr_off"] + row["incr_cnt"]].tolist()))
            assert a == b, ("incr", s)


CLUSTERS = parity_clusters() + affinity_clusters() + affinity_error_clusters() + ipa_error_clusters() + [
    ("backfill", backfill_cluster()),
    ("C3-small", synth.c3(n_nodes=400, n_jobs=30, tasks_per_job=12, seed=9, n_zones=5, n_racks=40)),
    ("C4-small", synth.c4(n_nodes=300, n_jobs=30, tasks_per_job=10, n_zones=5, n_racks=25, n_pre=300,
                          pre_job_size=20, seed=23)),
]


@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_columnar_equals_exporter(name, cluster):
    try:
        ref = E.Snapshot(cluster)
    except (E.Unsupported, E.AssertPanic) as e:
        with pytest.raises(type(e)):
            COL.build(COL.columns_of(cluster))
        return
    assert_same_snapshot(ref, COL.build(COL.columns_of(cluster)))


@pytest.mark.gpu
@pytest.mark.parametrize("name,cluster", CLUSTERS[-2:] + affinity_clusters()[:2],
                         ids=[c[0] for c in CLUSTERS[-2:] + affinity_clusters()[:2]])
def test_columnar_snapshot_allocates_like_the_exporter(name, cluster):
    """The device cycle over the columnar snapshot: the same placements as over the exporter's."""
    from scheduler_amd import runtime
    outs = []
    for snap in (E.Snapshot(cluster), COL.build(COL.columns_of(cluster))):
        ctx = runtime.Context(0)
        try:
            ctx.upload(snap)
            outs.append(ctx.allocate(snap))
        finally:
            ctx.close()
    a, b = outs
    k = int(a["n_events"])
    assert k == int(b["n_events"]) and k > 0
    for f in ("task_node", "task_status", "job_fail_task", "job_reason_hist"):
        assert np.array_equal(a[f], b[f]), f
    assert np.array_equal(a["event_task"][:k], b["event_task"][:k])


GEN_COLUMNS = [
    ("C1", dict(n_nodes=150, n_jobs=12, tasks_per_job=9, seed=5)),
    ("C3", dict(n_nodes=400, n_jobs=30, tasks_per_job=12, seed=9, n_zones=5, n_racks=40)),
    ("C4", dict(n_nodes=300, n_jobs=30, tasks_per_job=10, n_zones=5, n_racks=25, n_pre=300, pre_job_size=20, seed=23)),
]


@pytest.mark.parametrize("name,kw", GEN_COLUMNS, ids=[g[0] for g in GEN_COLUMNS])
def test_generator_columns_equal_the_walk(name, kw):
    """synth.c1/c3/c4_columns build the bench configurations' columns from the generator's draws, per node and per
    job (bench.py's session open for C1 / C3 / C4: no per-pod walk): the snapshot equals the exporter's on the same
    cluster, array by array."""
    gen = {"C1": synth.c1, "C3": synth.c3, "C4": synth.c4}[name]
    ref = E.Snapshot(gen(**kw))
    got = COL.build(synth.COLUMNS[name](**kw))
    assert_same_snapshot(ref, got)


def test_isum_exact_past_float53():
    """Per-node sums of int64 requests stay exact where float64 bincount would round."""
    idx = np.array([0, 0, 1, 0])
    v = np.array([(1 << 53) + 1, 2, 5, -3], np.int64)
    assert COL.isum(idx, v, 2).tolist() == [(1 << 53), 5]
    assert COL.isum(np.array([1, 1]), np.array([3, 4], np.int64), 3).tolist() == [0, 7, 0]
    assert COL.isum(np.zeros(0, np.int64), None, 2).tolist() == [0, 0]
