"""ctypes binding of libkbgpu.so (include/kbgpu.h) and the high-level allocate call.

The product path: cluster snapshot -> export.Snapshot -> kb_upload_* ->
kb_allocate (host ordering plugins + per-job device placement) -> binds.
There is no CPU fallback: if the HIP library or a GPU is missing this raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from . import export as E

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KBGPU_LIB", os.path.join(_HERE, "libkbgpu.so"))

KB_NUM_REASONS = 17
KB_R_HOST_ERROR = 16
KB_OK, KB_E_INVALID, KB_E_HIP, KB_E_UNSUPPORTED, KB_E_NOMEM, KB_E_PANIC, KB_E_STATE = 0, -1, -2, -3, -4, -5, -6
KB_STOP_DONE, KB_STOP_NO_FIT, KB_STOP_READY = 0, 1, 2
KB_PLACE_ALLOCATE, KB_PLACE_PIPELINE = 1, 2

P = C.c_void_p


class kb_nodes(C.Structure):
    _fields_ = [("n", C.c_uint32), ("n_scalar", C.c_uint32), ("n_label", C.c_uint32), ("n_port", C.c_uint32)] + [
        (f, P) for f in ("idle_cpu", "idle_mem", "rel_cpu", "rel_mem", "idle_sc", "rel_sc", "alloc_cpu", "alloc_mem",
                         "nz_cpu", "nz_mem", "pod_count", "max_pods", "flags", "label_val", "label_int",
                         "label_int_ok", "taint_set", "port_used")]


class kb_specs(C.Structure):
    _fields_ = [("m", C.c_uint32), ("specs", P), ("sc_init", P), ("sc_req", P), ("n_terms", C.c_uint32),
                ("terms", P), ("n_reqs", C.c_uint32), ("reqs", P), ("n_vals", C.c_uint32), ("vals", P),
                ("n_ports", C.c_uint32), ("ports", P), ("n_tol_sets", C.c_uint32), ("n_taint_sets", C.c_uint32),
                ("tolerates", P)]


class kb_affinity(C.Structure):
    _fields_ = [("n_slots", C.c_uint32), ("topo_dom", P), ("n_tables", C.c_uint32), ("tables", P), ("totals", P),
                ("n_counters", C.c_uint32), ("counters", P), ("m", C.c_uint32), ("specs", P),
                ("n_checks", C.c_uint32), ("checks", P), ("n_lister", C.c_uint32), ("lister", P),
                ("n_hists", C.c_uint32), ("hists", P), ("n_h", C.c_uint32), ("h", P), ("n_incr", C.c_uint32),
                ("incr", P)]


class kb_config(C.Structure):
    _fields_ = [(f, C.c_int32) for f in ("predicates_enabled", "nodeorder_enabled", "mem_pressure", "disk_pressure",
                                          "pid_pressure", "w_lr", "w_bra", "w_na", "w_pa")]


class kb_shard(C.Structure):
    _fields_ = [("n_total", C.c_uint32), ("node_begin", C.c_uint32), ("rank", C.c_int32), ("world", C.c_int32)]


# kb_allgather_fn: int (*)(void* user, const void* send, void* recv, size_t bytes)
ALLGATHER_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t)
# kb_nofit_fn: void (*)(void* user, int32_t job, int32_t task, uint32_t n_events, const uint32_t* reasons, uint32_t n)
NOFIT_FN = C.CFUNCTYPE(None, C.c_void_p, C.c_int32, C.c_int32, C.c_uint32, C.POINTER(C.c_uint32), C.c_uint32)

# kb_row_delta (kb_apply)
ROW_DELTA_DTYPE = np.dtype([("node", "<i4"), ("pods", "<i4"), ("idle_cpu", "<i8"), ("idle_mem", "<i8"),
                            ("rel_cpu", "<i8"), ("rel_mem", "<i8"), ("nz_cpu", "<i8"), ("nz_mem", "<i8"),
                            ("flags_set", "<u4"), ("flags_clear", "<u4"), ("spec", "<i4"), ("kind", "<i4"),
                            ("sc_off", "<u4"), ("port_off", "<u4"), ("port_cnt", "<u4"), ("pad", "<i4")], align=True)
assert ROW_DELTA_DTYPE.itemsize == 88
# kb_aff_delta (kb_apply_affinity)
AFF_DELTA_DTYPE = np.dtype([("node", "<i4"), ("table", "<i4"), ("slot", "<i4"), ("h_off", "<u4"), ("weight", "<i4"),
                            ("pad", "<i4")])
assert AFF_DELTA_DTYPE.itemsize == 24


def aff_delta_array(entries):
    """Pack (node, table, slot, h_off, weight) entries (affinity.Tables.pod_deltas) into kb_aff_delta records."""
    d = np.zeros(len(entries), AFF_DELTA_DTYPE)
    for i, (node, table, slot, h_off, weight) in enumerate(entries):
        d[i] = (node, table, slot, h_off, weight, 0)
    return d


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous block of canonical nodes held by `rank` (the first n_total % world ranks get one more)."""
    q, r = divmod(n_total, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


class kb_opts(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32), ("timing_every", C.c_uint32), ("fed_idle_ms", C.c_int32),
                ("eval_spb", C.c_int32), ("test_stall_ms", C.c_int32), ("test_stall_job", C.c_int64),
                ("shard_epoch0", C.c_uint32), ("fed_xcc", C.c_int32), ("fed_depth", C.c_int32)]


class kb_job_req(C.Structure):
    _fields_ = [("task_specs", P), ("n_tasks", C.c_uint32), ("ready_num", C.c_int32), ("min_available", C.c_int32),
                ("gang_ready", C.c_int32)]


class kb_job_result(C.Structure):
    _fields_ = [("n_placed", C.c_uint32), ("stop", C.c_int32), ("fail_task", C.c_int32), ("pad", C.c_int32),
                ("reason_hist", C.c_uint32 * KB_NUM_REASONS)]


class kb_session(C.Structure):
    _fields_ = [("n_rscalar", C.c_uint32), ("n_tasks", C.c_uint32)] + [
        (f, P) for f in ("task_job", "task_spec", "task_status", "task_priority", "task_ctime", "task_uid_rank",
                         "task_resreq", "task_resreq_mask")] + [
        ("n_jobs", C.c_uint32)] + [(f, P) for f in ("job_queue", "job_priority", "job_min_available", "job_ctime",
                                                    "job_uid_rank", "job_pg_pending")] + [
        ("n_queues", C.c_uint32)] + [(f, P) for f in ("queue_weight", "queue_ctime", "queue_uid_rank")] + [
        ("total_alloc", P), ("total_alloc_mask", C.c_uint64), ("n_tier_plugins", C.c_uint32), ("tier_plugins", P)]


class kb_cycle_result(C.Structure):
    _fields_ = [("task_node", P), ("task_status", P), ("job_fail_task", P), ("job_reason_hist", P),
                ("event_task", P), ("n_events", C.c_uint32), ("pad", C.c_int32), ("elapsed_ms", C.c_double),
                ("device_ms", C.c_double)]


class kb_stats(C.Structure):
    _fields_ = [("launches", C.c_uint64 * 15), ("kernel_ms", C.c_double * 15), ("pairs", C.c_uint64 * 15),
                ("job_calls", C.c_uint64), ("device_ms", C.c_double), ("diag", C.c_uint64 * 8),
                ("fed_abandon", C.c_uint64), ("fed_cycles", C.c_uint64), ("fed_split", C.c_uint64),
                ("cap1_runs", C.c_uint64), ("cls_runs", C.c_uint64),
                ("fed_sharded", C.c_uint64), ("shard_rezero", C.c_uint64), ("shard_xchg", C.c_uint64),
                ("shard_wait_ticks", C.c_uint64), ("fed_clock_ticks", C.c_uint64), ("fed_real_ticks", C.c_uint64),
                ("sweep_overlap", C.c_uint64), ("overlap_refused_tables", C.c_uint64),
                ("shard_phase_ticks", C.c_uint64 * 6), ("peer_checks", C.c_uint64), ("fed_wg_place", C.c_uint64 * 2),
                ("off_engine_units", C.c_uint64), ("fed_pauses", C.c_uint64),
                ("fed_mispredicts", C.c_uint64), ("fed_skipped", C.c_uint64), ("fed_units", C.c_uint64),
                ("nofit_predicted", C.c_uint64), ("fed_last_depth", C.c_int32), ("fed_last_sweepers", C.c_int32),
                ("fed_aff_units", C.c_uint64), ("fed_aff_waits", C.c_uint64)]


KB_OPT_TIMING = 1
KB_OPT_NO_TRAJECTORY = 2
KB_OPT_NO_SELECT = 4
KB_OPT_ENGINE = 8
# path selection / measurement switches (kb_opts.flags, include/kbgpu.h KB_OPT_*): the default is the production
# path; tests and the profiler name the others through Context(options=...)
OPTION_FLAGS = {"no_fed": 1 << 4, "no_fed_split": 1 << 5, "no_pipeline": 1 << 6, "no_aff_reg": 1 << 7,
                "no_cap1": 1 << 8, "no_cls": 1 << 9, "no_eval_plain": 1 << 10, "fed_shared_queues": 1 << 11,
                "fed_plain_launch": 1 << 12, "shard_self_inbox": 1 << 13, "fed_diag": 1 << 14,
                "fed_coop_launch": 1 << 15, "test_peer_badtag": 1 << 16, "fed_kernel_sweeps": 1 << 17,
                "test_one_xcc": 1 << 18, "fed_no_levels": 1 << 19, "fed_no_aff": 1 << 20}
OPTION_VALUES = ("fed_idle_ms", "eval_spb", "test_stall_job", "test_stall_ms", "shard_epoch0", "fed_xcc", "fed_depth")
KERNELS = ("sweep_keys_kernel", "place_loop_kernel", "eval_kernel", "traj_sweep_kernel", "traj_place_kernel",
           "aff_place_kernel", "ipa_minmax_kernel", "sel_place_kernel", "engine_kernel", "sel_sweep_kernel",
           "shard_propose_kernel", "shard_exchange", "shard_commit_kernel", "fed_engine_kernel", "cls_place_kernel")
# device paths for a run of same-spec tasks (kb_place_job picks the first one that applies):
#   select     - per-job launches of the level-0 sweep + the top-T selection kernel (default)
#   engine     - the same selection served by one persistent workgroup (no launches; single-CU sweep)
#   trajectory - precomputed per-node key trajectories + a one-wave argmax loop (traj_place_kernel)
#   rekey      - 64-bit keys, per-commit re-key + one-wave argmax loop (place_loop_kernel)
PATHS = {"select": 0, "engine": KB_OPT_ENGINE, "trajectory": KB_OPT_NO_SELECT,
         "rekey": KB_OPT_NO_SELECT | KB_OPT_NO_TRAJECTORY}

ABI_VERSION = 16  # include/kbgpu.h KBGPU_ABI_VERSION

EXPORTS = ["kb_abi_version", "kb_create", "kb_destroy", "kb_last_error", "kb_set_config", "kb_upload_nodes",
           "kb_upload_specs", "kb_place_job", "kb_eval", "kb_eval32", "kb_read_nodes", "kb_allocate", "kb_restore_nodes",
           "kb_get_stats", "kb_upload_affinity", "kb_set_shard", "kb_comm_unique_id", "kb_set_shard_rccl",
           "kb_set_shard_peer",
           "kb_set_host_overlay", "kb_apply", "kb_apply_affinity", "kb_set_nofit_hook", "kb_sort_nodes", "kb_predicate_nodes"]

_lib = None


class KbError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"kbgpu error {code}: {msg}")
        self.code = code


def load_library(path: str = LIB_PATH):
    """Load libkbgpu.so (fails loudly when it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: run `make -C scheduler_amd/csrc` (or __graft_entry__.build())")
    lib = C.CDLL(path)
    lib.kb_abi_version.restype = C.c_int
    if lib.kb_abi_version() != ABI_VERSION:
        raise KbError(KB_E_INVALID, f"libkbgpu ABI {lib.kb_abi_version()} != binding ABI {ABI_VERSION}")
    lib.kb_create.restype = P
    lib.kb_create.argtypes = [C.POINTER(kb_opts)]
    lib.kb_destroy.argtypes = [P]
    lib.kb_last_error.restype = C.c_char_p
    lib.kb_last_error.argtypes = [P]
    lib.kb_set_config.argtypes = [P, C.POINTER(kb_config)]
    lib.kb_upload_nodes.argtypes = [P, C.POINTER(kb_nodes)]
    lib.kb_upload_specs.argtypes = [P, C.POINTER(kb_specs)]
    lib.kb_upload_affinity.argtypes = [P, C.POINTER(kb_affinity)]
    lib.kb_place_job.argtypes = [P, C.POINTER(kb_job_req), P, P, C.POINTER(kb_job_result)]
    lib.kb_eval.argtypes = [P, P, C.c_uint32, P, P]
    lib.kb_eval32.argtypes = [P, P, C.c_uint32, P, P]
    lib.kb_read_nodes.argtypes = [P] + [P] * 7
    lib.kb_allocate.argtypes = [P, C.POINTER(kb_session), C.POINTER(kb_cycle_result)]
    lib.kb_restore_nodes.argtypes = [P]
    lib.kb_get_stats.argtypes = [P, C.POINTER(kb_stats), C.c_int]
    lib.kb_set_shard.argtypes = [P, C.POINTER(kb_shard), ALLGATHER_FN, P]
    lib.kb_comm_unique_id.argtypes = [P]
    lib.kb_set_shard_rccl.argtypes = [P, C.POINTER(kb_shard), P]
    lib.kb_set_shard_peer.argtypes = [P, C.POINTER(kb_shard), ALLGATHER_FN, P]
    lib.kb_set_host_overlay.argtypes = [P, C.c_int32, P, P]
    lib.kb_apply.argtypes = [P, P, C.c_uint32, P, C.c_uint32, P, C.c_uint32]
    lib.kb_apply_affinity.argtypes = [P, P, C.c_uint32]
    lib.kb_set_nofit_hook.argtypes = [P, NOFIT_FN, P]
    lib.kb_sort_nodes.argtypes = [P, C.c_int32, P, P, C.POINTER(C.c_uint32)]
    lib.kb_predicate_nodes.argtypes = [P, C.c_int32, P, C.POINTER(C.c_uint32), P]
    _lib = lib
    return lib


SESSION_ARRAYS = ("s_task_job", "s_task_spec", "s_task_status", "s_task_priority", "s_task_ctime", "s_task_uid_rank",
                  "s_task_resreq", "s_task_resreq_mask", "s_job_queue", "s_job_priority", "s_job_min", "s_job_ctime",
                  "s_job_uid_rank", "s_job_pg_pending", "s_queue_weight", "s_queue_ctime", "s_queue_uid_rank",
                  "s_total", "s_tiers")


def _ptr(a):
    return a.ctypes.data_as(P) if a is not None and a.size else None


def make_opts(device: int = 0, timing: bool = False, path: str = "select", timing_every: int = 1,
              options: dict | None = None) -> kb_opts:
    """kb_opts for kb_create. `options`: names of OPTION_FLAGS (true: set) and OPTION_VALUES (ints); an unknown
    name raises (a misspelt switch must not silently leave the production path on)."""
    options = dict(options or {})
    flags = (KB_OPT_TIMING if timing else 0) | PATHS[path]
    vals = {"fed_idle_ms": 0, "eval_spb": 0, "test_stall_job": -1, "test_stall_ms": 0, "shard_epoch0": 0,
            "fed_xcc": 0, "fed_depth": 0}
    for k, v in options.items():
        if k in OPTION_FLAGS:
            flags |= OPTION_FLAGS[k] if v else 0
        elif k in vals:
            vals[k] = int(v)
        else:
            raise KbError(KB_E_INVALID, f"unknown context option {k!r}")
    return kb_opts(device, flags, timing_every, vals["fed_idle_ms"], vals["eval_spb"], vals["test_stall_ms"],
                   vals["test_stall_job"], vals["shard_epoch0"], vals["fed_xcc"], vals["fed_depth"])


def parse_options(text: str | None) -> dict:
    """`name,name=value,...` (bench.py / scripts --opt) -> a Context options dict."""
    out = {}
    for part in (text or "").split(","):
        part = part.strip()
        if not part or part == "none":
            continue
        k, _, v = part.partition("=")
        out[k.strip()] = int(v) if v else True
    return out


class Context:
    """One device-resident session snapshot (kb_ctx). `options`: make_opts's switches (tests, profiling)."""

    def __init__(self, device: int = 0, timing: bool = False, path: str = "select", timing_every: int = 1,
                 options: dict | None = None):
        self.lib = load_library()
        self._keep = []
        self.overlay_reason = {}
        self.overlay_fail = {}
        opts = make_opts(device, timing, path, timing_every, options)
        self.ctx = self.lib.kb_create(C.byref(opts))
        if not self.ctx:
            raise KbError(KB_E_HIP, "kb_create failed")
        err = self.lib.kb_last_error(self.ctx)
        if err:  # no HIP device: there is no CPU fallback
            self.lib.kb_destroy(self.ctx)
            self.ctx = None
            raise KbError(KB_E_HIP, err.decode())

    def close(self):
        if self.ctx:
            self.lib.kb_destroy(self.ctx)
            self.ctx = None
        self.forget_session()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != KB_OK:
            raise KbError(rc, self.lib.kb_last_error(self.ctx).decode())

    def set_shard(self, rank: int, world: int, n_total: int, allgather=None, rccl_id: bytes = None,
                  peer: bool = False):
        """Node sharding (kb_set_shard / kb_set_shard_rccl / kb_set_shard_peer): this context holds
        shard_range(n_total, rank, world). `allgather(send: bytes) -> bytes` (all ranks' records, rank order) for the
        host-staged exchange, or the RCCL id from comm_unique_id() (the same bytes on every rank) for the RCCL
        exchange. peer=True (with allgather): the node-sharded fed engine's device exchange (inboxes mapped across
        the ranks' GPUs; allgather carries their IPC handles once, then the jobs the engine does not run)."""
        begin, end = shard_range(n_total, rank, world)
        sh = kb_shard(n_total, begin, rank, world)
        self.rows = (begin, end)
        if rccl_id is not None:
            buf = (C.c_uint8 * 128).from_buffer_copy(rccl_id)
            self._check(self.lib.kb_set_shard_rccl(self.ctx, C.byref(sh), C.cast(buf, P)))
            return

        def cb(user, send, recv, nbytes):
            try:
                out = allgather(C.string_at(send, nbytes))
                if len(out) != world * nbytes:
                    return -1
                C.memmove(recv, out, len(out))
                return 0
            except Exception:  # an error must not unwind through the C frames
                return -1
        self._ag_cb = ALLGATHER_FN(cb)  # kept alive as long as the context
        fn = self.lib.kb_set_shard_peer if peer else self.lib.kb_set_shard
        self._check(fn(self.ctx, C.byref(sh), self._ag_cb, None))

    def upload(self, snap: E.Snapshot):
        cfg = kb_config(**snap.config)
        self._check(self.lib.kb_set_config(self.ctx, C.byref(cfg)))
        lo, hi = getattr(self, "rows", (0, snap.n_nodes))  # node sharding: only this rank's rows
        self.n_nodes = hi - lo
        c = snap.cols
        keep = {k: np.ascontiguousarray(v[..., lo:hi]) for k, v in c.items()}
        self._keep = [keep]
        nodes = kb_nodes(hi - lo, len(snap.scalars), snap.n_label, snap.n_port,
                         *[_ptr(keep[f]) for f in ("idle_cpu", "idle_mem", "rel_cpu", "rel_mem", "idle_sc", "rel_sc",
                                                   "alloc_cpu", "alloc_mem", "nz_cpu", "nz_mem", "pod_count",
                                                   "max_pods", "flags", "label_val", "label_int", "label_int_ok",
                                                   "taint_set", "port_used")])
        self._check(self.lib.kb_upload_nodes(self.ctx, C.byref(nodes)))
        tol = np.ascontiguousarray(snap.tolerates)
        specs = kb_specs(len(snap.spec_arr), _ptr(snap.spec_arr), _ptr(snap.sc_init), _ptr(snap.sc_req),
                         len(snap.term_arr), _ptr(snap.term_arr), len(snap.req_arr), _ptr(snap.req_arr),
                         len(snap.val_arr), _ptr(snap.val_arr), len(snap.port_arr), _ptr(snap.port_arr),
                         tol.shape[0], tol.shape[1], _ptr(tol))
        self._check(self.lib.kb_upload_specs(self.ctx, C.byref(specs)))
        if snap.aff is not None:
            # (node-sharded: every rank holds the whole topo_dom and the replicated count tables)
            a = snap.aff
            arrs = [np.ascontiguousarray(x) for x in (a.topo_dom, a.table_arr, a.totals, a.counters, a.spec_arr,
                                                      a.check_arr, a.lister_arr, a.hist_arr, a.h, a.incr_arr)]
            self._keep.append(arrs)
            td, tb, tot, cnt, sp, ck, ls, hs, h, inc = arrs
            aff = kb_affinity(td.shape[0], _ptr(td), len(tb), _ptr(tb), _ptr(tot), len(cnt), _ptr(cnt), len(sp),
                              _ptr(sp), len(ck), _ptr(ck), len(ls), _ptr(ls), len(hs), _ptr(hs), len(h), _ptr(h),
                              len(inc), _ptr(inc))
            self._check(self.lib.kb_upload_affinity(self.ctx, C.byref(aff)))

    def restore(self):
        self._check(self.lib.kb_restore_nodes(self.ctx))

    # ---- per-node Go fallback (kb_set_host_overlay / kb_apply / kb_set_nofit_hook) ----
    def set_host_overlay(self, spec: int, fail=None, score=None, reason=None):
        """A plugin predicate / node-order fn the device does not express, evaluated per node on the host:
        fail[i] rejects node i (KB_R_HOST_ERROR), score[i] is added to its order score. `reason` is the
        plugin's FitErrors string for a rejected node: a str or a callable(node name) -> str (result_dict puts
        it into the job's histogram). No arrays: clear the overlay."""
        n = self.n_nodes
        f = None if fail is None else np.ascontiguousarray(np.asarray(fail, dtype=np.uint8).reshape(n))
        sc = None if score is None else np.ascontiguousarray(np.asarray(score, dtype=np.int64).reshape(n))
        self._check(self.lib.kb_set_host_overlay(self.ctx, int(spec), _ptr(f), _ptr(sc)))
        if f is None and sc is None:
            self.overlay_reason.pop(int(spec), None)
            self.overlay_fail.pop(int(spec), None)
        else:
            self.overlay_reason[int(spec)] = reason
            self.overlay_fail[int(spec)] = None if f is None else f.copy()

    def apply(self, deltas, sc=None, ports=None):
        """kb_apply: rows changed by commits made outside the device (ROW_DELTA_DTYPE records; see
        export.pod_delta for one pod's AddTask + AddPod)."""
        d = np.ascontiguousarray(np.asarray(deltas, dtype=ROW_DELTA_DTYPE))
        sc = np.ascontiguousarray(np.asarray(sc if sc is not None else [], dtype=np.int64))
        pt = np.ascontiguousarray(np.asarray(ports if ports is not None else [], dtype=E.PORT_DTYPE))
        self._check(self.lib.kb_apply(self.ctx, _ptr(d), len(d), _ptr(sc), len(sc), _ptr(pt), len(pt)))

    def apply_affinity(self, deltas):
        """kb_apply_affinity: inter-pod affinity table / histogram entries of pods outside the session's pending
        specs (AFF_DELTA_DTYPE records; affinity.Tables.pod_deltas derives them)."""
        d = np.ascontiguousarray(np.asarray(deltas, dtype=AFF_DELTA_DTYPE))
        self._check(self.lib.kb_apply_affinity(self.ctx, _ptr(d), len(d)))

    def _hook(self):
        """Collect the per-node reason masks kb_allocate hands over at a NO_FIT with host-evaluated stages."""
        if getattr(self, "_nofit_cb", None) is not None:
            return

        def cb(user, job, task, n_events, reasons, n):
            try:
                self._nofit[int(job)] = (int(task), int(n_events), np.ctypeslib.as_array(reasons, shape=(n,)).copy())
            except Exception:  # an error must not unwind through the C frames
                self._nofit_err = True
        self._nofit = {}
        self._nofit_cb = NOFIT_FN(cb)  # kept alive as long as the context
        self._check(self.lib.kb_set_nofit_hook(self.ctx, self._nofit_cb, None))

    def stats(self, reset=False):
        st = kb_stats()
        self._check(self.lib.kb_get_stats(self.ctx, C.byref(st), int(reset)))
        return {"launches": list(st.launches), "kernel_ms": list(st.kernel_ms), "pairs": list(st.pairs),
                "job_calls": st.job_calls, "device_ms": st.device_ms, "diag": list(st.diag),
                "fed_abandon": st.fed_abandon, "fed_cycles": st.fed_cycles, "fed_split": st.fed_split,
                "cap1_runs": st.cap1_runs, "cls_runs": st.cls_runs,
                "fed_sharded": st.fed_sharded, "shard_rezero": st.shard_rezero, "shard_xchg": st.shard_xchg,
                "shard_wait_ticks": st.shard_wait_ticks, "fed_clock_ticks": st.fed_clock_ticks,
                "fed_real_ticks": st.fed_real_ticks, "sweep_overlap": st.sweep_overlap,
                "overlap_refused_tables": st.overlap_refused_tables,
                "shard_phase_ticks": list(st.shard_phase_ticks), "peer_checks": st.peer_checks,
                "off_engine_units": st.off_engine_units, "fed_wg_place": list(st.fed_wg_place),
                "fed_pauses": st.fed_pauses, "fed_mispredicts": st.fed_mispredicts, "fed_skipped": st.fed_skipped,
                "fed_units": st.fed_units, "nofit_predicted": st.nofit_predicted,
                "fed_last_depth": st.fed_last_depth,
                "fed_last_sweepers": st.fed_last_sweepers, "fed_aff_units": st.fed_aff_units,
                "fed_aff_waits": st.fed_aff_waits}

    def eval(self, spec_ids):
        ids = np.ascontiguousarray(np.asarray(spec_ids, dtype=np.int32))
        n = self.n_nodes
        reasons = np.zeros((len(ids), n), np.uint32)
        scores = np.zeros((len(ids), n), np.int64)
        self._check(self.lib.kb_eval(self.ctx, _ptr(ids), len(ids), _ptr(reasons), _ptr(scores)))
        return reasons, scores

    def eval32(self, spec_ids):
        """kb_eval32: the same with 32-bit scores (KbError KB_E_UNSUPPORTED when a spec's scores do not fit)."""
        ids = np.ascontiguousarray(np.asarray(spec_ids, dtype=np.int32))
        n = self.n_nodes
        reasons = np.zeros((len(ids), n), np.uint32)
        scores = np.zeros((len(ids), n), np.int32)
        self._check(self.lib.kb_eval32(self.ctx, _ptr(ids), len(ids), _ptr(reasons), _ptr(scores)))
        return reasons, scores

    def sort_nodes(self, spec: int):
        """kb_sort_nodes: preempt's PredicateNodes -> PrioritizeNodes -> SortNodes for one spec (preempt.go:
        187-195). Returns (node indices best first, their scores)."""
        order = np.zeros(max(self.n_nodes, 1), np.int32)
        scores = np.zeros(max(self.n_nodes, 1), np.int64)
        k = C.c_uint32(0)
        self._check(self.lib.kb_sort_nodes(self.ctx, int(spec), _ptr(order), _ptr(scores), C.byref(k)))
        return order[:k.value].copy(), scores[:k.value].copy()

    def predicate_nodes(self, spec: int):
        """kb_predicate_nodes: util.PredicateNodes with Session.PredicateFn (the set reclaim walks,
        reclaim.go:122-126). Returns (feasible node indices in node order, FitErrors reason histogram)."""
        nodes = np.zeros(max(self.n_nodes, 1), np.int32)
        hist = np.zeros(KB_NUM_REASONS, np.uint32)
        k = C.c_uint32(0)
        self._check(self.lib.kb_predicate_nodes(self.ctx, int(spec), _ptr(nodes), C.byref(k), _ptr(hist)))
        return nodes[:k.value].copy(), hist

    def read_nodes(self, n):
        cols = [np.zeros(n, np.int64) for _ in range(4)] + [np.zeros(n, np.int32)] + [np.zeros(n, np.int64)
                                                                                       for _ in range(2)]
        self._check(self.lib.kb_read_nodes(self.ctx, *[_ptr(a) for a in cols]))
        return dict(zip(("idle_cpu", "idle_mem", "rel_cpu", "rel_mem", "pod_count", "nz_cpu", "nz_mem"), cols))

    def place_job(self, spec_ids, ready_num=0, min_available=0, gang_ready=1):
        ids = np.ascontiguousarray(np.asarray(spec_ids, dtype=np.int32))
        nodes = np.zeros(max(len(ids), 1), np.int32)
        kinds = np.zeros(max(len(ids), 1), np.int32)
        req = kb_job_req(_ptr(ids), len(ids), ready_num, min_available, gang_ready)
        res = kb_job_result()
        self._check(self.lib.kb_place_job(self.ctx, C.byref(req), _ptr(nodes), _ptr(kinds), C.byref(res)))
        k = res.n_placed
        return nodes[:k].copy(), kinds[:k].copy(), res

    def allocate(self, snap: E.Snapshot, out: dict | None = None):
        """kb_allocate: allocateAction.Execute over the uploaded snapshot. `out`: the result dict of an earlier
        call on a session of the same size, whose arrays this cycle overwrites (a serving loop's reused result
        buffers: no fresh pages per cycle); by default new arrays."""
        nt, nj = len(snap.session_tasks), len(snap.jobs)
        # The cached kb_session points into the snapshot's arrays: in-place edits of them are seen by the next call,
        # a reassigned attribute or a changed scalar (counts, the total's scalar mask) rebuilds it. task_resreq is
        # the one array the struct may hold a copy of (when the snapshot's is not C-contiguous): editing such an
        # array in place needs forget_session().
        key = ((id(snap), nt, nj, len(snap.acc_scalars), len(snap.queues), len(snap.s_tiers), int(snap.s_total_mask))
               + tuple(id(getattr(snap, a)) for a in SESSION_ARRAYS))
        cached = getattr(self, "_ssn_cache", None)
        if cached is not None and cached[0] == key:  # the session arrays' struct, built once per snapshot and arrays
            ssn = cached[1]
        else:
            ssn = self._session_struct(snap, nt, nj)
            self._ssn_cache = (key, ssn, self._ssn_keep)
        if out is not None and len(out["task_node"]) == max(nt, 1) and len(out["job_fail_task"]) == max(nj, 1):
            out = {k: out[k] for k in ("task_node", "task_status", "job_fail_task", "job_reason_hist", "event_task")}
        else:
            out = {"task_node": np.zeros(max(nt, 1), np.int32), "task_status": np.zeros(max(nt, 1), np.int32),
                   "job_fail_task": np.zeros(max(nj, 1), np.int32),
                   "job_reason_hist": np.zeros((max(nj, 1), KB_NUM_REASONS), np.uint32),
                   "event_task": np.zeros(max(nt, 1), np.int32)}
        res = kb_cycle_result(*[_ptr(out[k]) for k in ("task_node", "task_status", "job_fail_task", "job_reason_hist",
                                                       "event_task")], 0, 0, 0.0, 0.0)
        self._hook()
        self._nofit = {}
        self._nofit_err = False
        self._check(self.lib.kb_allocate(self.ctx, C.byref(ssn), C.byref(res)))
        if self._nofit_err:
            raise KbError(KB_E_INVALID, "NO_FIT hook failed")
        out["nofit"] = dict(self._nofit)
        out["overlay_reason"] = dict(self.overlay_reason)
        out["overlay_fail"] = dict(self.overlay_fail)
        out["event_task"][res.n_events:] = 0  # (kb_allocate writes the first n_events entries; a reused array's tail)
        out["n_events"] = res.n_events
        out["elapsed_ms"] = res.elapsed_ms
        out["device_ms"] = res.device_ms
        return out

    def forget_session(self):
        """Drop the cached kb_session (and the snapshot it keeps alive): the next allocate() rebuilds it."""
        self._ssn_cache = None
        self._ssn_keep = None

    def _session_struct(self, snap, nt, nj):
        """kb_session over the snapshot's session arrays (kept alive with the struct in self._ssn_cache)."""
        arrs = dict(
            task_job=snap.s_task_job, task_spec=snap.s_task_spec, task_status=snap.s_task_status,
            task_priority=snap.s_task_priority, task_ctime=snap.s_task_ctime, task_uid_rank=snap.s_task_uid_rank,
            task_resreq=np.ascontiguousarray(snap.s_task_resreq), task_resreq_mask=snap.s_task_resreq_mask,
            job_queue=snap.s_job_queue, job_priority=snap.s_job_priority, job_min_available=snap.s_job_min,
            job_ctime=snap.s_job_ctime, job_uid_rank=snap.s_job_uid_rank, job_pg_pending=snap.s_job_pg_pending,
            queue_weight=snap.s_queue_weight, queue_ctime=snap.s_queue_ctime, queue_uid_rank=snap.s_queue_uid_rank,
            total_alloc=snap.s_total, tier_plugins=snap.s_tiers)
        ssn = kb_session(
            len(snap.acc_scalars), nt, *[_ptr(arrs[k]) for k in ("task_job", "task_spec", "task_status",
                                                               "task_priority", "task_ctime", "task_uid_rank",
                                                               "task_resreq", "task_resreq_mask")],
            nj, *[_ptr(arrs[k]) for k in ("job_queue", "job_priority", "job_min_available", "job_ctime",
                                         "job_uid_rank", "job_pg_pending")],
            len(snap.queues), *[_ptr(arrs[k]) for k in ("queue_weight", "queue_ctime", "queue_uid_rank")],
            _ptr(arrs["total_alloc"]), snap.s_total_mask, len(snap.s_tiers), _ptr(arrs["tier_plugins"]))
        self._ssn_keep = (snap, arrs)  # (the struct points into these)
        return ssn

    def backfill(self, snap: E.Snapshot, out: dict) -> dict:
        """backfillAction.Execute (actions/backfill/backfill.go:40-90) on the session kb_allocate left in `out`.

        Jobs and their Pending tasks go in UID order (the maps of backfill.go:45, :54). A task whose InitResreq
        is empty takes the first node, in the canonical node order, that passes Session.PredicateFn (:62-71).
        On the device that is kb_place_job with the node order switched off -- every score is then equal and
        the selection keeps the lowest feasible index -- and the job's JobReady stop out of reach, so one call
        places a whole run of same-spec tasks (each pick is still the lowest feasible index after the previous
        commit). A task that fits nowhere records the device's FitErrors histogram (:84-86); the rest of its
        run sees the same table and fails the same way. Commits are Session.Allocate, each followed by the
        JobReady dispatch (session.go:286-294). Updates `out` in place and returns it with
        "backfill_fit" = {job index: {task index: reason histogram}}.

        The device's predicate also applies allocate's resource check (InitResreq <= Idle or Releasing), which
        backfill.go does not: an empty request passes it unless a node's Idle is below the tolerance or the
        scalar-map rule bites (a zero scalar request against a node without scalars, resource_info.go:264-267),
        where the reference's own Resource.Sub would then assert. Such a divergence raises KbError."""
        cfg = dict(snap.config)
        tiers = [(int(p), int(en)) for _, p, en in snap.tier_plugins]
        has_gang = any(p == E.PLUGIN_IDS["gang"] for p, _ in tiers)
        gang_ready = any(p == E.PLUGIN_IDS["gang"] and en >> E.EN_BITS["enabledJobReady"] & 1 for p, en in tiers)
        st, node = out["task_status"], out["task_node"]
        ts = snap.session_tasks
        by_job = {}
        for t in np.argsort(snap.s_task_uid_rank, kind="stable"):
            by_job.setdefault(int(snap.s_task_job[t]), []).append(int(t))
        alloc_st = E.ST["Bound"] | E.ST["Binding"] | E.ST["Running"] | E.ST["Allocated"]
        valid_st = alloc_st | E.ST["Succeeded"] | E.ST["Pipelined"] | E.ST["Pending"]
        fit = {}
        n_ev = int(out["n_events"])
        never = 1 << 30  # JobReady never stops a backfill run on the device; the host replays it per task
        self._check(self.lib.kb_set_config(self.ctx, C.byref(kb_config(**dict(cfg, nodeorder_enabled=0)))))
        try:
            for j in np.argsort(snap.s_job_uid_rank, kind="stable"):
                j = int(j)
                if snap.s_job_pg_pending[j]:
                    continue
                tasks = by_job.get(j, [])
                if has_gang and sum(1 for t in tasks if st[t] & valid_st) < snap.s_job_min[j]:
                    continue  # JobValid (gang.go:48-69)
                be = []
                for t in tasks:
                    if st[t] != E.ST["Pending"]:
                        continue
                    r = ts[t]["initreq"]
                    if r.cpu < 10 and r.mem < 10 * 1024 * 1024 and all(q < 10 for q in (r.sc or {}).values()):
                        be.append(t)  # Resource.IsEmpty (resource_info.go:96-108); others are left alone
                ready = sum(1 for u in tasks if st[u] & (alloc_st | E.ST["Succeeded"]))
                allocated = [u for u in tasks if st[u] == E.ST["Allocated"]]
                k = 0
                while k < len(be):
                    spec = int(snap.s_task_spec[be[k]])
                    e = k
                    while e < len(be) and int(snap.s_task_spec[be[e]]) == spec:
                        e += 1
                    placed, kinds, res = self.place_job([spec] * (e - k), 0, never, 1)
                    if (kinds != KB_PLACE_ALLOCATE).any() or (len(placed) < e - k and res.reason_hist[0]):
                        raise KbError(KB_E_UNSUPPORTED, "backfill: the device's resource check diverges from "
                                                        "backfill.go's PredicateFn-only test (DESIGN.md §7b)")
                    for i, w in enumerate(placed):
                        t = be[k + i]
                        st[t], node[t] = E.ST["Allocated"], int(w)
                        out["event_task"][n_ev] = t
                        n_ev += 1
                        ready += 1
                        allocated.append(t)
                        if not gang_ready or ready >= snap.s_job_min[j]:  # dispatch (session.go:286-294)
                            for u in allocated:
                                st[u] = E.ST["Binding"]
                            allocated = []
                    if len(placed) < e - k:  # the run's failed task and the rest of the run
                        hist = {E.REASONS[b]: int(c) for b, c in enumerate(res.reason_hist)
                                if c and b != KB_R_HOST_ERROR}
                        reasons = None
                        if res.reason_hist[KB_R_HOST_ERROR]:
                            # host-evaluated failures (overlay plugins, affinity errors): the reference records
                            # each node's own error (fe.SetNodeError, backfill.go:84-86). Every node's mask at
                            # this state (the run's commits applied), mapped per task as allocate's NO_FIT hook
                            # does (the strings name the pod)
                            reasons = self.eval([spec])[0][0]
                        for t in be[k + len(placed):e]:
                            h = dict(hist)
                            if reasons is not None:
                                view = dict(out, nofit={j: (t, n_ev, reasons)}, overlay_fail=dict(self.overlay_fail),
                                            overlay_reason=dict(self.overlay_reason))
                                for key, c in host_reason_strings(snap, view, j, t).items():
                                    h[key] = h.get(key, 0) + c
                            fit.setdefault(j, {})[t] = h
                    k = e
        finally:
            self._check(self.lib.kb_set_config(self.ctx, C.byref(kb_config(**cfg))))
        out["n_events"] = n_ev
        out["backfill_fit"] = fit
        return out


def comm_unique_id() -> bytes:
    """RCCL unique id for kb_set_shard_rccl (made on one rank, broadcast to the others)."""
    lib = load_library()
    buf = (C.c_uint8 * 128)()
    rc = lib.kb_comm_unique_id(C.cast(buf, P))
    if rc != KB_OK:
        raise KbError(rc, "ncclGetUniqueId failed")
    return bytes(buf)


def result_dict(snap: E.Snapshot, out: dict) -> dict:
    """Map kb_allocate's arrays back to names, in the oracle's output format."""
    names = snap.node_names()
    ts = snap.session_tasks
    events = []
    for i in range(out["n_events"]):
        t = ts[out["event_task"][i]]
        st = out["task_status"][out["event_task"][i]]
        kind = "pipeline" if st == E.ST["Pipelined"] else "allocate"
        events.append({"task": t["uid"], "node": names[out["task_node"][out["event_task"][i]]], "kind": kind})
    binds = {}
    status = {}
    for i, t in enumerate(ts):
        st = int(out["task_status"][i])
        status[t["uid"]] = E.ST_NAME[st]
        if st == E.ST["Binding"]:
            binds[f"{t['pod'].ns}/{t['pod'].name}"] = names[out["task_node"][i]]
    fit = {}
    for j, job in enumerate(snap.jobs):
        ft = int(out["job_fail_task"][j])
        if ft >= 0:
            hist = {E.REASONS[b]: int(c) for b, c in enumerate(out["job_reason_hist"][j]) if c and b != KB_R_HOST_ERROR}
            if out["job_reason_hist"][j][KB_R_HOST_ERROR]:
                for k, c in host_reason_strings(snap, out, j, ft).items():
                    hist[k] = hist.get(k, 0) + c
            fit[job["uid"]] = {ts[ft]["uid"]: hist}
    return {"events": events, "binds": binds, "fit_errors": fit, "status": status, "nodes": names,
            "elapsed_ms": out["elapsed_ms"], "device_ms": out["device_ms"]}


def host_reason_strings(snap: E.Snapshot, out: dict, job: int, task: int) -> dict:
    """The strings of the KB_R_HOST_ERROR bucket of a failed job: per node that failed there, the error the
    reference's affinity predicate returns (affinity.Tables.host_error_string) or the overlay plugin's reason
    (FitErrors.SetNodeError, api/unschedule_info.go:40-54)."""
    names = snap.node_names()
    t = snap.session_tasks[task]
    spec = int(t["spec"])
    if job not in out.get("nofit", {}):
        raise KbError(KB_E_STATE, f"job {job}: host-evaluated reasons without the NO_FIT hook's node masks")
    _, n_events, reasons = out["nofit"][job]
    before = []
    for i in range(n_events):
        u = int(out["event_task"][i])
        if out["task_status"][u] != E.ST["Pipelined"]:
            before.append((snap.session_tasks[u]["uid"], int(snap.session_tasks[u]["spec"])))
    # the inter-pod predicate errors at every node that reaches it when the spec's own terms are invalid or an
    # invalid lister pod exists by now (at session open, or one of the cycle's commits before this task)
    aff_err = snap.aff is not None and (spec in snap.aff.own_err or bool(snap.aff.xb_pods) or
                                        any(sp in snap.aff.xb_spec for _, sp in before))
    ov = out.get("overlay_reason", {}).get(spec)
    ov_fail = out.get("overlay_fail", {}).get(spec)
    hist = {}
    for i in np.nonzero((reasons >> KB_R_HOST_ERROR) & 1)[0]:
        # per node, in chain order: the inter-pod predicate's error, else the overlay plugin's verdict (the
        # overlay is the chain's last stage)
        if aff_err:
            s = snap.aff.host_error_string(t["pod"], spec, names[i], before)
        elif ov is not None and (ov_fail is None or ov_fail[i]):
            s = ov(names[i]) if callable(ov) else str(ov)
        else:
            raise KbError(KB_E_STATE, f"job {job}: node {names[i]} failed a host-evaluated stage that neither the "
                                      f"overlay nor the affinity tables account for")
        hist[s] = hist.get(s, 0) + 1
    return hist


def allocate(cluster, device: int = 0, path: str = "select", stats_out: dict | None = None,
             options: dict | None = None) -> dict:
    """One allocate cycle of `cluster` on the GPU; returns binds / events / fit errors like the oracle
    (stats_out: filled with the context's kb_get_stats counters; options: Context's)."""
    snap = E.Snapshot(cluster)
    ctx = Context(device, path=path, options=options)
    try:
        ctx.upload(snap)
        out = ctx.allocate(snap)
        if stats_out is not None:
            stats_out.update(ctx.stats())
        return result_dict(snap, out)
    finally:
        ctx.close()


def allocate_backfill(cluster, device: int = 0, path: str = "select", options: dict | None = None) -> dict:
    """The default action list, allocate then backfill (util.go:32), on the GPU. Returns what allocate() does
    plus "backfill_fit_errors" in the oracle's format."""
    snap = E.Snapshot(cluster)
    ctx = Context(device, path=path, options=options)
    try:
        ctx.upload(snap)
        out = ctx.backfill(snap, ctx.allocate(snap))
        d = result_dict(snap, out)
        ts = snap.session_tasks
        d["backfill_fit_errors"] = {
            snap.jobs[j]["uid"]: {ts[t]["uid"]: dict(h) for t, h in tf.items()} for j, tf in out["backfill_fit"].items()}
        return d
    finally:
        ctx.close()
