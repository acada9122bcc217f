"""GPU parity: the HIP path (through the C-ABI) against the oracle on the same seeded snapshots.

Bar: bit-exact. Masks (first-fail reason sets) and scores for every (spec, node) pair, and identical
allocate outcomes (placement sequence, binds, statuses, FitErrors histograms) under the lowest-index
tie-break applied to both.
"""
import copy

import numpy as np
import pytest

from oracle import pyoracle
from scheduler_amd import export as E
from scheduler_amd import model as m
from scheduler_amd import runtime, synth

from helpers import affinity_clusters, parity_clusters, plain_edge_cluster
from test_oracle_kat import allocate_test_cases

pytestmark = pytest.mark.gpu

CLUSTERS = parity_clusters() + affinity_clusters()


def _compare(ref, got):
    assert got["nodes"] == ref["nodes"]
    assert got["events"] == ref["events"]
    assert got["binds"] == ref["binds"]
    assert got["fit_errors"] == ref["fit_errors"]
    for uid, st in got["status"].items():
        assert ref["status"][uid] == st, uid


@pytest.mark.parametrize("path", list(runtime.PATHS))
@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_allocate_parity(name, cluster, path):
    """Every device path: the top-T selection, precomputed per-node key trajectories with a one-wave
    argmax loop, and the per-commit re-key loop."""
    ref = pyoracle.allocate(cluster)
    got = runtime.allocate(cluster, path=path)
    _compare(ref, got)
    assert len(got["events"]) > 0


@pytest.mark.parametrize("name,cluster,expected", allocate_test_cases(), ids=lambda x: x if isinstance(x, str) else "")
def test_reference_allocate_cases(name, cluster, expected):  # actions/allocate/allocate_test.go:38-212
    assert runtime.allocate(cluster)["binds"] == expected


@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_eval_masks_and_scores(name, cluster):
    snap = E.Snapshot(cluster)
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t["uid"]
    spec_ids = sorted(reps)
    ref = pyoracle.evaluate(cluster, [reps[s] for s in spec_ids])
    assert ref["nodes"] == snap.node_names()
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        reasons, scores = ctx.eval(spec_ids)
    finally:
        ctx.close()
    for i, s in enumerate(spec_ids):
        rt = ref["tasks"][i]
        for n in range(snap.n_nodes):
            want = sorted(rt["reasons"][n])
            got = sorted(E.REASONS[b] for b in range(16) if (int(reasons[i, n]) >> b) & 1)
            assert got == want, (s, n, got, want)
        assert list(scores[i]) == rt["score"], s


@pytest.mark.parametrize("name,cluster", CLUSTERS, ids=[c[0] for c in CLUSTERS])
def test_eval32_equals_eval(name, cluster):
    """kb_eval32 (int32 scores, 8 B per pair) returns kb_eval's reasons and scores wherever they fit."""
    snap = E.Snapshot(cluster)
    ids = list(range(len(snap.spec_arr)))
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        r64, s64 = ctx.eval(ids)
        try:
            r32, s32 = ctx.eval32(ids)
        except runtime.KbError as e:  # only for scores beyond int32 (IPA batch errors)
            assert e.code == runtime.KB_E_UNSUPPORTED and (np.abs(s64) >= 2 ** 31).any()
            return
    finally:
        ctx.close()
    assert np.array_equal(r32, r64)
    assert np.array_equal(s32.astype(np.int64), s64)


def _plain_spec(snap):
    a = snap.spec_arr
    bad = (E.SPEC_HAS_SELECTOR | E.SPEC_HAS_REQUIRED | E.SPEC_INIT_HAS_MAP | E.SPEC_NA_ERROR | E.SPEC_POD_AFFINITY |
           E.SPEC_IPA_ERROR)
    return ((a["flags"] & bad) == 0) & (a["pref_term_cnt"] == 0) & (a["port_cnt"] == 0) & (a["aff_class"] < 0) & \
        (snap.tolerates.shape[1] == 1)


@pytest.mark.parametrize("extra", [0, 1, 2, 3])
def test_eval_plain_matches_oracle(extra):
    """kb_eval's row-only kernel (plain specs: resource fit, pod count, conditions, memory / disk / PID pressure,
    BestEffort, LeastRequested + Balanced) against the oracle on every (spec, node) pair. `extra` copies of the first
    nodes make every residue of N mod 4: N % 4 == 0 takes the four-nodes-per-lane kernel (eval_plain4_kernel), the
    others the one-node-per-lane kernel."""
    cl = plain_edge_cluster()
    for k in range(extra):
        nd = copy.deepcopy(cl.nodes[k])
        nd.name += f"-x{k}"
        cl.nodes.append(nd)
    snap = E.Snapshot(cl)
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t["uid"]
    spec_ids = sorted(reps)
    assert _plain_spec(snap)[spec_ids].all() and (snap.spec_arr["flags"][spec_ids] & E.SPEC_BEST_EFFORT).any()
    ref = pyoracle.evaluate(cl, [reps[s] for s in spec_ids])
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        reasons, scores = ctx.eval(spec_ids)
        r32, s32 = ctx.eval32(spec_ids)
    finally:
        ctx.close()
    for i, s in enumerate(spec_ids):
        rt = ref["tasks"][i]
        for n in range(snap.n_nodes):
            got = sorted(E.REASONS[b] for b in range(16) if (int(reasons[i, n]) >> b) & 1)
            assert got == sorted(rt["reasons"][n]), (s, n)
        assert list(scores[i]) == rt["score"], s
    assert np.array_equal(r32, reasons) and np.array_equal(s32.astype(np.int64), scores)


@pytest.mark.parametrize("name,cfg", [("plain-edge", None), ("C2-2000", None), ("C2-2002", None), ("C1-parity", None),
                                      ("plain-edge", {"nodeorder_enabled": 0}),
                                      ("plain-edge", {"predicates_enabled": 0})])
def test_eval_plain_equals_general(name, cfg):
    """The row-only kernel returns the general eval_kernel's arrays (option no_eval_plain) on plain batches, also with
    the nodeorder or predicates plugin off (the score table all 0; no post reasons)."""
    cl = {"plain-edge": plain_edge_cluster, "C2-2000": lambda: synth.c2(n_nodes=2000, n_jobs=64, tasks_per_job=1,
                                                                        seed=9),
          "C2-2002": lambda: synth.c2(n_nodes=2002, n_jobs=64, tasks_per_job=1, seed=9),
          "C1-parity": lambda: synth.c1(n_nodes=120, n_jobs=24, tasks_per_job=25, seed=1)}[name]()
    snap = E.Snapshot(cl)
    if cfg:
        snap.config.update(cfg)
    ids = [int(s) for s in np.nonzero(_plain_spec(snap))[0]]
    assert ids
    out = []
    for general in (False, True):
        ctx = runtime.Context(0, options={"no_eval_plain": general})
        try:
            ctx.upload(snap)
            out.append(ctx.eval(ids) + ctx.eval32(ids))
        finally:
            ctx.close()
    for a, b in zip(out[0], out[1]):
        assert np.array_equal(a, b)


def test_full_size_c2_properties():
    """BASELINE configs[1] at full size (10k x 100k): size-independent invariants, determinism, and
    identical placements from the two device paths."""
    cl = synth.c2()
    snap = E.Snapshot(cl)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out1 = ctx.allocate(snap)
        after = ctx.read_nodes(snap.n_nodes)
        ctx.restore()
        out2 = ctx.allocate(snap)
    finally:
        ctx.close()
    others = []
    for path in ("engine", "trajectory", "rekey"):
        ctx = runtime.Context(0, path=path)
        try:
            ctx.upload(snap)
            others.append(ctx.allocate(snap))
        finally:
            ctx.close()
    assert np.array_equal(out1["task_node"], out2["task_node"])          # deterministic
    assert np.array_equal(out1["event_task"], out2["event_task"])
    for out3 in others:                                                  # every device path agrees
        assert np.array_equal(out1["task_node"], out3["task_node"])
        assert np.array_equal(out1["event_task"], out3["event_task"])
    placed = out1["task_node"][: len(snap.session_tasks)] >= 0
    assert placed.sum() == out1["n_events"] > 0.9 * len(snap.session_tasks)
    # conservation: idle = allocatable - sum(resreq of tasks placed there)  (NodeInfo.AddTask)
    cpu = np.full(snap.n_nodes, snap.cols["idle_cpu"][0])
    mem = np.full(snap.n_nodes, snap.cols["idle_mem"][0])
    cnt = np.zeros(snap.n_nodes, np.int64)
    for t, node in enumerate(out1["task_node"][: len(snap.session_tasks)]):
        if node >= 0:
            r = snap.session_tasks[t]["resreq"]
            cpu[node] -= r.cpu
            mem[node] -= r.mem
            cnt[node] += 1
    assert np.array_equal(after["idle_cpu"], cpu) and np.array_equal(after["idle_mem"], mem)
    assert np.array_equal(after["pod_count"], cnt) and (cnt <= 110).all()
    assert (cpu > -10).all() and (mem > -10 * 1024 * 1024).all()  # LessEqual tolerance (resource_info.go:70-72)
    # gang: every job is either fully placed (minMember = all tasks) or left with a fit error
    jobs = np.asarray(snap.s_task_job)
    for j in range(len(snap.jobs)):
        k = placed[jobs == j].sum()
        assert k == (jobs == j).sum() or out1["job_fail_task"][j] >= 0


def test_affinity_restore_reopens_tables():
    """kb_restore_nodes also restores the affinity tables: two cycles from one upload agree."""
    cl = affinity_clusters()[0][1]
    snap = E.Snapshot(cl)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        a = ctx.allocate(snap)
        ctx.restore()
        b = ctx.allocate(snap)
    finally:
        ctx.close()
    assert np.array_equal(a["task_node"], b["task_node"]) and np.array_equal(a["event_task"], b["event_task"])


def test_c4_full_size_properties():
    """BASELINE configs[3] (C4, 10k x 100k) at full size: hard inter-pod constraints hold in the result
    (no two pods of a hostname-anti-affinity job share a node; svc-affinity pods land in svc zones) and
    both device paths agree."""
    cl = synth.c4()
    snap = E.Snapshot(cl)
    outs = []
    for path in runtime.PATHS:
        ctx = runtime.Context(0, path=path)
        try:
            ctx.upload(snap)
            outs.append(ctx.allocate(snap))
        finally:
            ctx.close()
    for o in outs[1:]:
        assert np.array_equal(outs[0]["task_node"], o["task_node"])
    tn = outs[0]["task_node"][: len(snap.session_tasks)]
    assert (tn >= 0).sum() > 0.5 * len(snap.session_tasks)
    names = snap.node_names()
    svc_zones = {cl_node.labels["zone"] for p in cl.pods if p.labels.get("app") == "svc"
                 for cl_node in [next(n for n in cl.nodes if n.name == p.node)]}
    by_job = {}
    for t, node in zip(snap.session_tasks, tn):
        if node < 0 or t["status"] != E.ST["Pending"]:
            continue
        by_job.setdefault(t["pod"].group, []).append(node)
        aff = t["pod"].affinity or {}
        if "podAffinity" in aff and aff["podAffinity"].get("required"):
            zone = next(n for n in cl.nodes if n.name == names[node]).labels["zone"]
            assert zone in svc_zones
    for t in snap.session_tasks:
        aff = t["pod"].affinity or {}
        if t["status"] == E.ST["Pending"] and "podAntiAffinity" in aff:
            nodes = by_job.get(t["pod"].group, [])
            assert len(nodes) == len(set(nodes)), t["pod"].group


def test_engine_idle_exit_and_relaunch():
    """The placement engine exits by itself after 1 s without a command; the next kb_place_job relaunches
    it and the session goes on with the same results as the launch-per-job path."""
    import time
    cl = synth.c2(n_nodes=300, n_jobs=20, tasks_per_job=20, seed=9)
    snap = E.Snapshot(cl)
    outs = []
    for path in ("engine", "select"):
        ctx = runtime.Context(0, path=path)
        try:
            ctx.upload(snap)
            first = ctx.allocate(snap)
            time.sleep(1.5)  # engine idles out
            spec = int(snap.s_task_spec[0])
            nodes, kinds, res = ctx.place_job([spec] * 7, ready_num=0, min_available=7, gang_ready=1)
            outs.append((first, nodes, kinds, res.stop, res.n_placed))
        finally:
            ctx.close()
    (a, na, ka, sa, pa), (b, nb, kb, sb, pb) = outs
    assert np.array_equal(a["task_node"], b["task_node"]) and np.array_equal(a["event_task"], b["event_task"])
    assert np.array_equal(na, nb) and np.array_equal(ka, kb) and (sa, pa) == (sb, pb)


def _partial_gang(cl, frac):
    for pg in cl.pod_groups:
        pg.min_member = max(1, int(pg.min_member * frac))
    return cl


def _few_candidates():
    """40 nodes with room for exactly one task each and a 60-task gang job: the selection sees K = 40
    candidates, more than the all-pairs rank takes and fewer than the segment's T = 60 tasks (threshold
    path with K < T), then the no-fit stop."""
    rl = m.build_resource_list
    cl = m.Cluster(nodes=[m.build_node(f"n{i:02d}", dict(rl("1", "4Gi"), pods=110)) for i in range(40)],
                   pods=[m.build_pod("c1", f"p{i:02d}", "", "Pending", rl("600m", "1Gi"), "pg1") for i in range(60)]
                   + [m.build_pod("c2", f"q{i:02d}", "", "Pending", rl("300m", "512Mi"), "pg2") for i in range(30)],
                   pod_groups=[m.PodGroup(ns="c1", name="pg1", queue="q", min_member=60),
                               m.PodGroup(ns="c2", name="pg2", queue="q", min_member=30)],
                   queues=[m.Queue(name="q")])
    return cl


PIPE_CLUSTERS = CLUSTERS + [
    ("few-candidates", _few_candidates()),
    # minMember below the job size: jobs stop READY mid-way and are pushed back (the speculated next job
    # is often the same job), and ready jobs compete with unready ones in the gang order
    ("C2-halfgang", _partial_gang(synth.c2(n_nodes=120, n_jobs=30, tasks_per_job=20, seed=31), 0.5)),
    ("C1-thirdgang", _partial_gang(synth.c1(n_nodes=100, n_jobs=20, tasks_per_job=24, seed=32), 0.34)),
    # two-template jobs (two units per pop on the engine) and anti-affinity jobs (off the engine) among C2 jobs
    ("C2M-mixed", synth.c2m(n_nodes=300, n_jobs=30, tasks_per_job=12, seed=33, frac_multi=0.3, frac_aff=0.2)),
]


@pytest.mark.parametrize("mode", ["fed", "launch", "serial"])
@pytest.mark.parametrize("name,cluster", PIPE_CLUSTERS, ids=[c[0] for c in PIPE_CLUSTERS])
def test_driver_pipeline_parity(name, cluster, mode):
    """kb_allocate's driver issues job k+1 before job k's result is read, guarded on job k's predicted
    outcome (a failed guard turns job k+1 into no-ops and the driver re-issues the real next job), with
    job k+1's level-0 sweep overlapping job k. fed: one resident selection workgroup fed by the sweeps
    (cycles whose jobs are single selection runs); launch: a place kernel per job; serial: one
    kb_place_job round trip per job. All match the oracle."""
    opts = {"launch": {"no_fed": True}, "serial": {"no_pipeline": True}}.get(mode, {})
    ref = pyoracle.allocate(cluster)
    got = runtime.allocate(cluster, options=opts)
    _compare(ref, got)


AFF_VARIANTS = {"default": {}, "aff-reg": {"no_cap1": True, "no_cls": True},
                "aff-global": {"no_cap1": True, "no_cls": True, "no_aff_reg": True}}


@pytest.mark.parametrize("variant", sorted(AFF_VARIANTS))
@pytest.mark.parametrize("name,cluster", affinity_clusters(), ids=[c[0] for c in affinity_clusters()])
def test_affinity_loop_variants(name, cluster, variant):
    """Specs whose own commits move their inter-pod affinity inputs. default: cap-1 specs (required
    anti-affinity to their own pods over hostname) as selection runs and histogram-only specs on the class
    loop (cls_place_kernel), the rest on the register-resident loop; aff-reg: every such spec on the
    register-resident loop (aff_reg_kernel); aff-global: the global-memory loop (aff_place_kernel). All
    match the oracle."""
    ref = pyoracle.allocate(cluster)
    ctx_stats = {}
    got = runtime.allocate(cluster, stats_out=ctx_stats, options=AFF_VARIANTS[variant])
    _compare(ref, got)
    if name.startswith("self-aff") or name == "C4-parity":
        # the clusters built for them do reach the new paths (or, with them off, none of them)
        on = variant == "default"
        assert (ctx_stats["cap1_runs"] > 0) == on and (ctx_stats["cls_runs"] > 0) == on, ctx_stats


def test_fed_engine_survives_a_host_stall():
    """The resident engine exits after its idle bound without a command. A host stall longer than that in
    the middle of a cycle (a GC pause, descheduling) must not fail the cycle: the job the host waits for, and
    the rest of the cycle, finish on the launch path with the oracle's placements."""
    cl = synth.c2(n_nodes=300, n_jobs=20, tasks_per_job=20, seed=9)
    ref = pyoracle.allocate(cl)
    snap = E.Snapshot(cl)
    ctx = runtime.Context(0, options={"fed_idle_ms": 40, "test_stall_job": 3, "test_stall_ms": 400})
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        st = ctx.stats()
    finally:
        ctx.close()
    assert st["fed_abandon"] == 1
    _compare(ref, runtime.result_dict(snap, out))


SPLIT_CLUSTERS = [
    ("C2-3000", synth.c2(n_nodes=3000, n_jobs=60, tasks_per_job=40, seed=41)),
    # jobs stop READY and come back (the speculated next job is often the same job)
    ("C2-halfgang-2500", _partial_gang(synth.c2(n_nodes=2500, n_jobs=50, tasks_per_job=30, seed=42), 0.5)),
    # capacity for ~75% of the work: no-fit jobs (the histogram over every node's rebuilt key)
    ("C2-nofit-2100", synth.c2(n_nodes=2100, n_jobs=70, tasks_per_job=60, seed=43, fill=1.3)),
    # node classes, taints, GPUs, node affinity; jobs of up to 100 tasks (one segment)
    ("C3-2500", synth.c3(n_nodes=2500, n_jobs=40, tasks_per_job=100, seed=44)),
]


SPLIT_MODES = {
    "split": {},
    "split-kernel-sweeps": {"fed_kernel_sweeps": True},
    # the placer computes every e-sequence level itself (no level records from the sweepers)
    "split-no-levels": {"fed_no_levels": True},
    "one-workgroup": {"no_fed_split": True},
    # a one-XCC census (a one-XCC device or partition): the resident sweepers share the placer's XCC
    "split-one-xcc": {"test_one_xcc": True},
    # the speculative chain two and three units deep (kb_opts.fed_depth; the default is the driver's choice)
    "split-depth2": {"fed_depth": 2},
    "split-depth3": {"fed_depth": 3},
}


@pytest.mark.parametrize("mode", list(SPLIT_MODES))
@pytest.mark.parametrize("name,cluster", SPLIT_CLUSTERS, ids=[c[0] for c in SPLIT_CLUSTERS])
def test_fed_split_engine_parity(name, cluster, mode):
    """The split fed engine (n > 2048, every job one segment): a second workgroup selects each job's
    candidate nodes one job ahead, leaving out the nodes the job before may commit to, which the placer
    re-keys and merges in. Same placements, statuses and FitErrors as the oracle, and as the one-workgroup
    engine (option no_fed_split). The split engine's sweeps come from its resident sweepers (commands through a
    pinned ring) -- off the placer's XCC, or on it when the census finds one XCC only -- or per job from sweep
    kernels (option fed_kernel_sweeps); the driver keeps two to four units in flight (fed_depth)."""
    split = mode != "one-workgroup"
    ref = pyoracle.allocate(cluster)
    snap = E.Snapshot(cluster)
    ctx = runtime.Context(0, options=SPLIT_MODES[mode])
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        st = ctx.stats()
    finally:
        ctx.close()
    assert st["fed_cycles"] == 1 and st["fed_split"] == (1 if split else 0)
    assert st["fed_abandon"] == 0, st
    if mode in ("split", "split-one-xcc", "split-depth2", "split-depth3", "split-no-levels"):
        assert st["fed_last_sweepers"] > 0, st
    if mode == "split-kernel-sweeps":
        assert st["fed_last_sweepers"] == 0, st
    if mode.startswith("split-depth"):
        assert st["fed_last_depth"] == int(mode[-1]), st
    got = runtime.result_dict(snap, out)
    _compare(ref, got)
    assert len(got["events"]) > 0


def test_fed_split_engine_takes_long_jobs_as_units():
    """A job of more than one segment (150 tasks) goes to the split engine as units of at most one segment (the
    driver runs the job's next unit in the same pop when a unit places all its tasks without the job becoming
    ready): the cycle stays on the split engine, with the oracle's placements."""
    cl = synth.c2(n_nodes=2200, n_jobs=8, tasks_per_job=150, seed=45)
    ref = pyoracle.allocate(cl)
    snap = E.Snapshot(cl)
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        st = ctx.stats()
    finally:
        ctx.close()
    assert st["fed_cycles"] == 1 and st["fed_split"] == 1 and st["off_engine_units"] == 0, st
    _compare(ref, runtime.result_dict(snap, out))


MIXED_CLUSTERS = [
    # the split engine (n > 2048) with two-template jobs and anti-affinity jobs among C2 jobs
    ("C2M-split", synth.c2m(n_nodes=2500, n_jobs=60, tasks_per_job=30, seed=61, frac_multi=0.15, frac_aff=0.15)),
    # the one-workgroup engine, half gangs (jobs stop READY and come back mid-way through their units)
    ("C2M-small-halfgang", _partial_gang(synth.c2m(n_nodes=600, n_jobs=40, tasks_per_job=20, seed=62,
                                                   frac_multi=0.2, frac_aff=0.2), 0.5)),
    # two-template jobs only: every unit on the engine, one launch for the cycle
    ("C2M-multi-only", synth.c2m(n_nodes=2300, n_jobs=40, tasks_per_job=40, seed=63, frac_multi=0.5, frac_aff=0.0)),
    # capacity for ~80% of the work: NO_FIT units on both paths
    ("C2M-nofit", synth.c2m(n_nodes=2100, n_jobs=50, tasks_per_job=60, seed=64, frac_multi=0.2, frac_aff=0.1,
                            fill=1.3)),
]


@pytest.mark.parametrize("aff_path", ["engine", "pause"])
@pytest.mark.parametrize("name,cluster", MIXED_CLUSTERS, ids=[c[0] for c in MIXED_CLUSTERS])
def test_mixed_cycle_matches_oracle(name, cluster, aff_path):
    """A cycle mixing plain units with inter-pod-affinity units (cap-1: required anti-affinity to the job's own pods
    over hostname). On the split engine they are engine units by default (aff_path "engine": the resident sweepers fold
    the terms into the static cache, the placer commits the tables before its publish). With option
    fed_no_aff, and on the one-workgroup engine, the driver pauses the engine for them (nothing in flight), runs them
    on the launch path beside the idle engine, and hands the engine its next unit flagged fresh. A two-template job
    is two units of one pop. Placements, statuses and FitErrors equal the oracle's."""
    ref = pyoracle.allocate(cluster)
    st = {}
    got = runtime.allocate(cluster, stats_out=st, options={"fed_no_aff": aff_path == "pause"})
    _compare(ref, got)
    assert st["fed_cycles"] == 1, st
    split = st["fed_split"] >= 1
    if name == "C2M-multi-only":
        assert st["off_engine_units"] == 0 and st["fed_aff_units"] == 0, st
    elif aff_path == "engine" and split:  # every affinity unit on the engine: no pause
        assert st["off_engine_units"] == 0 and st["fed_pauses"] == 0 and st["fed_aff_units"] > 0, st
    else:  # the affinity units ran while the engine was paused (one launch for the whole cycle)
        assert st["off_engine_units"] > 0 and st["fed_pauses"] > 0 and st["fed_aff_units"] == 0, st


def _ratio_cluster(seed=77, n_nodes=3000, n_specs=48):
    """Random capacities and loads, so LeastRequested / BalancedResource see many distinct quotients (and
    some exactly on an integer boundary, like 2000/4000 vs 3000/10000)."""
    rng = np.random.default_rng(seed)
    GI = 1024 ** 3
    cl = m.Cluster()
    for i in range(n_nodes):
        cpu = int(rng.choice([4000, 10000, 8000, int(rng.integers(1000, 200000))]))
        mem = int(rng.choice([10000, 16 * GI, int(rng.integers(1, 1 << 40))]))
        cl.nodes.append(m.Node(name=f"n{i:05d}", alloc={m.CPU: cpu, m.MEMORY: mem, m.PODS: 110}))
        for k in range(int(rng.integers(0, 3))):
            cl.pods.append(m.Pod(ns="x", name=f"r{i}-{k}", uid=f"x-r{i}-{k}", node=f"n{i:05d}", phase="Running",
                                 containers=[m.Container(req={m.CPU: int(rng.integers(0, cpu // 3 + 1)),
                                                              m.MEMORY: int(rng.integers(0, mem // 3 + 1))})]))
    cl.queues.append(m.Queue(name="q"))
    for j in range(n_specs):
        cl.pod_groups.append(m.PodGroup(ns="t", name=f"g{j}", queue="q", min_member=1))
        req = {m.CPU: int(rng.choice([1000, 3000, int(rng.integers(1, 20000))])),
               m.MEMORY: int(rng.choice([1000, 2000, int(rng.integers(1, 1 << 34))]))}
        cl.pods.append(m.Pod(ns="t", name=f"p{j}", uid=f"t-p{j}", group=f"g{j}", containers=[m.Container(req=req)]))
    return cl


def test_eval_scores_random_ratios():
    """kb_eval's reciprocal fast paths for LeastRequested / BalancedResource (exact by construction, with
    the IEEE divisions near integer boundaries) against the oracle on ~70k (spec, node) pairs."""
    cl = _ratio_cluster()
    snap = E.Snapshot(cl)
    reps = {}
    for t in snap.session_tasks:
        if t["status"] == E.ST["Pending"] and t["spec"] not in reps:
            reps[t["spec"]] = t["uid"]
    spec_ids = sorted(reps)
    ref = pyoracle.evaluate(cl, [reps[s] for s in spec_ids])
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        reasons, scores = ctx.eval(spec_ids)
    finally:
        ctx.close()
    for i, s in enumerate(spec_ids):
        assert list(scores[i]) == ref["tasks"][i]["score"], s


def test_allocate_reused_result_buffers():
    """Context.allocate(snap, out=previous): the same arrays as a fresh call, cycle after cycle (restore between)."""
    snap = E.Snapshot(synth.c2(n_nodes=200, n_jobs=40, tasks_per_job=30, seed=2, fill=0.9))
    ctx = runtime.Context(0)
    try:
        ctx.upload(snap)
        fresh = ctx.allocate(snap)
        prev = None
        for _ in range(3):
            ctx.restore()
            prev = ctx.allocate(snap, out=prev)
            for k in ("task_node", "task_status", "job_fail_task", "job_reason_hist", "event_task"):
                assert np.array_equal(prev[k], fresh[k]), k
            assert prev["n_events"] == fresh["n_events"]
    finally:
        ctx.close()


@pytest.mark.parametrize("kind", ["disjoint", "shared", "tail"])
def test_affinity_sweep_overlap(kind):
    """The launch path overlaps job k+1's level-0 sweep with job k's place kernel (second stream) only when no job
    still in flight writes an affinity table that sweep reads: the previous job's own commits (aff_sweep_indep),
    and a table commit the job two back queued after its publish (the 64-bit re-key loop's aff_commit_kernel),
    which the host may have read past before that kernel ran. disjoint: the sweeps overlap; shared / tail: they
    stay in order. Oracle parity in every case."""
    from helpers import overlap_cluster
    cl = overlap_cluster(kind)
    ref = pyoracle.allocate(cl)
    st = {}
    got = runtime.allocate(cl, stats_out=st)
    _compare(ref, got)
    assert st["fed_cycles"] == 0, st  # (affinity jobs: the per-job launch path)
    if kind == "disjoint":
        assert st["sweep_overlap"] > 0 and st["overlap_refused_tables"] == 0, st
    else:
        assert st["overlap_refused_tables"] > 0, st


def _fed_aff_cluster(seed=91, n_nodes=2200, n_jobs=48, tasks=24):
    """The split engine's affinity units and their limits, with every kind of inter-pod input:
    own-job hostname anti-affinity (cap-1, independent units), a team anti-affinity shared by several jobs (a unit's
    sweep reads the table an earlier unit's commits write: it waits for the chain to drain), required zone affinity
    to running services (static checks), noisy pods that a running pod's preferred anti-affinity scores (a static
    histogram: min / max prepared before the launch), and preferred rack affinity to another pending job's pods (a
    histogram the cycle's commits write: those units stay on the launch path, the engine pauses)."""
    rng = np.random.default_rng(seed)
    GI = 1024 ** 3
    cl = m.Cluster()
    for i in range(n_nodes):
        rack = i * 40 // n_nodes
        cl.nodes.append(m.Node(name=f"n{i:05d}", alloc={m.CPU: 16000, m.MEMORY: 64 * GI, m.PODS: 110},
                               labels={"kubernetes.io/hostname": f"n{i:05d}", "zone": f"z{rack // 8}",
                                       "rack": f"r{rack}"}))
    cl.queues.append(m.Queue(name="q"))
    noisy_sel = {"labelSelector": {"matchLabels": {"noisy": "true"}}}
    for k in range(30):  # running services in the first two zones; one carries the noisy terms
        aff = None
        if k == 0:
            aff = {"podAntiAffinity": {"preferred": [{"weight": 10, "podAffinityTerm": dict(noisy_sel,
                                                                                            topologyKey="zone")}]}}
        node = int(rng.integers(0, n_nodes // 5 * 2))
        cl.pods.append(m.Pod(ns="s", name=f"svc{k}", uid=f"s-svc{k}", node=f"n{node:05d}", phase="Running",
                             labels={"app": "svc"}, affinity=aff,
                             containers=[m.Container(req={m.CPU: 500, m.MEMORY: GI})]))
    for j in range(n_jobs):
        name = f"j{j:03d}"
        cl.pod_groups.append(m.PodGroup(ns="t", name=name, queue="q", min_member=tasks // 2))
        req = {m.CPU: int(rng.integers(1, 5)) * 250, m.MEMORY: int(rng.integers(1, 5)) * GI // 2}
        labels = {"job": name}
        kind = j % 6
        aff = None
        if kind == 0:
            aff = {"podAntiAffinity": {"required": [{"labelSelector": {"matchLabels": {"job": name}},
                                                     "topologyKey": "kubernetes.io/hostname"}]}}
        elif kind == 1:
            labels["team"] = "blue"
            aff = {"podAntiAffinity": {"required": [{"labelSelector": {"matchLabels": {"team": "blue"}},
                                                     "topologyKey": "kubernetes.io/hostname"}]}}
        elif kind == 2:
            aff = {"podAffinity": {"required": [{"labelSelector": {"matchLabels": {"app": "svc"}},
                                                 "topologyKey": "zone"}]}}
        elif kind == 3:
            labels["noisy"] = "true"
        elif kind == 4:
            labels["team"] = "green"
            aff = {"podAffinity": {"preferred": [{"weight": 30, "podAffinityTerm": {
                "labelSelector": {"matchLabels": {"team": "red"}}, "topologyKey": "rack"}}]}}
        else:
            labels["team"] = "red"
        for t in range(tasks):
            cl.pods.append(m.Pod(ns="t", name=f"{name}-{t:03d}", uid=f"t-{name}-{t:03d}", group=name,
                                 labels=dict(labels), affinity=aff, containers=[m.Container(req=dict(req))]))
    return cl


def test_fed_affinity_units_match_oracle():
    """Affinity units on the resident engine against the oracle: placements, statuses and FitErrors equal, the
    independent ones in flight together, the team units waiting for the chain, the green units (their histograms
    move with the red jobs' commits) on the launch path while the engine pauses; and the same with the engine's
    affinity units off (option fed_no_aff: every unit of this cycle has inter-pod inputs, so it runs without the
    engine)."""
    cl = _fed_aff_cluster()
    ref = pyoracle.allocate(cl)
    st = {}
    got = runtime.allocate(cl, stats_out=st)
    _compare(ref, got)
    assert st["fed_cycles"] == 1 and st["fed_split"] == 1, st
    assert st["fed_aff_units"] > 0 and st["fed_aff_waits"] > 0, st
    assert st["off_engine_units"] > 0 and st["fed_pauses"] > 0, st
    st2 = {}
    got2 = runtime.allocate(cl, stats_out=st2, options={"fed_no_aff": True})
    _compare(ref, got2)
    # (every unit of this cycle has inter-pod inputs: without them the engine has nothing, the cycle is launch path)
    assert st2["fed_aff_units"] == 0 and st2["fed_cycles"] == 0, st2
