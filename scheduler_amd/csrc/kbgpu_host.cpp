// Host side of the device layer: context, HBM residency of the node table and
// spec tables, per-job placement batches, parity evaluation.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <map>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "kbgpu_ctx.h"

// hipMemset on device memory runs on the null stream and may return before it is done; the library's kernels run on
// non-blocking streams, which do not wait for the null stream. So every zeroing waits for itself: a context whose
// buffers come from memory an earlier context of the process freed must not start a kernel on the old contents
// (round 4: the fed engine's counters and command ring, recycled, let a node-sharded engine read a stale command).
static hipError_t memset_sync(void* p, int v, size_t n) {
  const hipError_t e = hipMemset(p, v, n);
  return e != hipSuccess ? e : hipStreamSynchronize(nullptr);
}

using namespace kbgpu;

namespace {

int fail(kb_ctx* c, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (c) {
    c->err = buf;
    c->prev_listed = false;
  }
  return code;
}

#define HIP_OK(ctx, expr)                                                                      \
  do {                                                                                         \
    hipError_t e_ = (expr);                                                                    \
    if (e_ != hipSuccess) return fail(ctx, KB_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

template <class T>
int upload(kb_ctx* c, std::vector<void*>& owned, T** dst, const T* src, size_t count, bool required = true) {
  *dst = nullptr;
  size_t bytes = std::max<size_t>(count, 1) * sizeof(T);
  void* p = nullptr;
  HIP_OK(c, hipMalloc(&p, bytes));
  owned.push_back(p);
  if (count && src) {
    HIP_OK(c, hipMemcpy(p, src, count * sizeof(T), hipMemcpyHostToDevice));
  } else {
    if (count && required) return fail(c, KB_E_INVALID, "missing array of %zu elements", count);
    HIP_OK(c, memset_sync(p, 0, bytes));
  }
  *dst = (T*)p;
  return KB_OK;
}

void free_all(std::vector<void*>& v) {
  for (void* p : v) (void)hipFree(p);
  v.clear();
}

void drop_overlay(kb_ctx* c) {
  free_all(c->ov_mem);
  c->ov_slot.clear();
  c->ov_fail.clear();
  c->ov_score.clear();
  c->ov_absmax.clear();
  c->ov_any_fail.clear();
  c->P.ov_slot = nullptr;
  c->P.ov_fail = nullptr;
  c->P.ov_score = nullptr;
}

void drop_affinity(kb_ctx* c) {
  free_all(c->aff_mem);
  c->aff_pristine.clear();
  c->aff_ok = false;
  c->P.A = kbgpu::DevAff{};
  c->spec_dyn.clear();
  c->spec_hist.clear();
  c->spec_incr.clear();
  c->spec_aff_err.clear();
  c->mm_eval = nullptr;
  c->mm_eval_cap = 0;
  c->d_mm_ids = nullptr;
  c->mm_ids_cap = 0;
  c->mm_spec_ok.clear();
  c->spec_cap1.clear();
  c->spec_cls.clear();
  c->cls_coff.clear();
  c->cls_mem.clear();
}

// Which self-dependent specs (KB_AFF_SELF_DYNAMIC) leave the per-task re-sweep loops:
//  * cap-1 (kSpecCap1 on the device copy of the spec): every self-dependent entry is a required
//    anti-affinity check (EXISTING_ANTI / ANTI) of a table the spec's own Allocates join, over a slot whose
//    domains are single nodes, and no histogram moves. A commit then changes one thing: that node fails the
//    check for the rest of the run. The run is a selection run (traj_key64's cap).
//  * class loop (spec_cls = its finest moving slot F): every check is static (the spec's commits join none
//    of its tables) and at least one of its InterPodAffinity histograms moves. Every entry's domain is a
//    function of the node's F-domain, so the nodes of one F-domain share their counts all run long, and a
//    task ranks the F-domains' best nodes instead of every node (cls_place_kernel).
void classify_self_dynamic(kb_ctx* c, const kb_affinity* a, const std::vector<int64_t>& D,
                           std::vector<kb_spec>& specs) {
  const size_t n = c->sharded ? (size_t)c->shard.n_total : (size_t)c->N.n;  // rows of topo_dom
  c->spec_cap1.assign(a->m, 0);
  c->spec_cls.assign(a->m, -1);
  for (auto& sp : specs) sp.flags &= ~(kbgpu::kSpecCap1 | kbgpu::kSpecCapAnti);
  std::vector<signed char> single(a->n_slots, -1);  // slot: every node has its own domain
  auto single_node = [&](int32_t sl) {
    if (single[sl] < 0) {
      bool ok = D[sl] == (int64_t)n;
      std::vector<char> seen(ok ? n : 0, 0);
      for (size_t i = 0; ok && i < n; ++i) {
        const int32_t d = a->topo_dom[sl * n + i];
        ok = d >= 0 && !seen[d];
        if (ok) seen[d] = 1;
      }
      single[sl] = ok;
    }
    return single[sl] == 1;
  };
  std::map<std::pair<int32_t, int32_t>, bool> nests;  // (F, S): dom_S is a function of dom_F
  auto nested = [&](int32_t F, int32_t S) {
    auto it = nests.find({F, S});
    if (it != nests.end()) return it->second;
    std::vector<int32_t> map_(D[F] + 1, -2);  // index dom_F + 1
    bool ok = true;
    for (size_t i = 0; ok && i < n; ++i) {
      int32_t& m = map_[a->topo_dom[F * n + i] + 1];
      const int32_t s = a->topo_dom[S * n + i];
      if (m == -2) m = s;
      ok = m == s;
    }
    nests[{F, S}] = ok;
    return ok;
  };
  for (uint32_t s = 0; s < a->m; ++s) {
    const int32_t ac = specs[s].aff_class;
    if (ac < 0 || !(a->specs[ac].flags & KB_AFF_SELF_DYNAMIC)) continue;
    const kb_aff_spec& e = a->specs[ac];
    auto joins = [&](int32_t table) {
      for (uint32_t i = 0; i < e.lister_cnt; ++i)
        if (a->lister[e.lister_off + i] == table) return true;
      return false;
    };
    auto moves = [&](uint32_t h_off) {
      for (uint32_t i = 0; i < e.incr_cnt; ++i)
        if (a->incr[e.incr_off + i].h_off == h_off) return true;
      return false;
    };
    int dyn_checks = 0, first_kind = -1;
    bool cap_ok = true;
    for (uint32_t i = 0; i < e.check_cnt; ++i) {
      const kb_aff_check& ck = a->checks[e.check_off + i];
      if (!joins(ck.table)) continue;
      ++dyn_checks;
      if (first_kind < 0) first_kind = ck.kind;
      cap_ok = cap_ok && (ck.kind == KB_AFF_EXISTING_ANTI || ck.kind == KB_AFF_ANTI) &&
               single_node(a->tables[ck.table].slot);
    }
    int32_t F = -1;
    for (uint32_t i = 0; i < e.hist_cnt; ++i) {
      const kb_ipa_hist& h = a->hists[e.hist_off + i];
      if (moves(h.h_off) && (F < 0 || D[h.slot] > D[F])) F = h.slot;
    }
    if (dyn_checks && cap_ok && F < 0) {
      c->spec_cap1[s] = 1;
      specs[s].flags |= kbgpu::kSpecCap1 | (first_kind == KB_AFF_ANTI ? kbgpu::kSpecCapAnti : 0u);
    } else if (!dyn_checks && F >= 0 && e.hist_cnt <= (uint32_t)kbgpu::kClsE) {
      bool ok = true;
      for (uint32_t i = 0; ok && i < e.hist_cnt; ++i) ok = nested(F, a->hists[e.hist_off + i].slot);
      if (ok) c->spec_cls[s] = F;
    }
  }
}

}  // namespace

hipEvent_t kb_ctx::ev_get() {
  if (!ev_pool.empty()) {
    hipEvent_t e = ev_pool.back();
    ev_pool.pop_back();
    return e;
  }
  hipEvent_t e;
  (void)hipEventCreate(&e);
  return e;
}
void kb_ctx::ev_begin(hipEvent_t* a, hipStream_t s) {
  *a = nullptr;
  if (!timing_now) return;
  *a = ev_get();
  (void)hipEventRecord(*a, s ? s : stream);
}
void kb_ctx::ev_end(hipEvent_t a, int kind, uint64_t pairs, hipStream_t s) {
  if (!timing || !a) return;
  hipEvent_t b = ev_get();
  (void)hipEventRecord(b, s ? s : stream);
  pending.push_back({a, b, kind, pairs});
}
// Fold finished event pairs into the stats, oldest first. `all`: wait for the stream first; otherwise
// stop at the first pair still in flight (it is collected by a later call, off the job's critical path).
// Pairs of kind < 0 (a skipped speculative job) are recycled without counting.
size_t kb_ctx::ev_collect(bool all, size_t limit) {
  if (all && !pending.empty()) (void)hipStreamSynchronize(stream);
  size_t k = 0;
  for (; k < pending.size() && k < limit; ++k) {
    Pending& p = pending[k];
    if (!all && hipEventQuery(p.b) != hipSuccess) break;
    float ms = 0;
    if (p.kind >= 0 && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      stats.kernel_ms[p.kind] += ms;
      stats.launches[p.kind] += 1;
      stats.pairs[p.kind] += p.pairs;
    }
    ev_pool.push_back(p.a);
    ev_pool.push_back(p.b);
  }
  pending.erase(pending.begin(), pending.begin() + k);
  for (auto& sl : slot) {
    sl.ev_b = sl.ev_b > k ? sl.ev_b - k : 0;
    sl.ev_e = sl.ev_e > k ? sl.ev_e - k : 0;
  }
  return k;
}

extern "C" {

int kb_abi_version(void) { return KBGPU_ABI_VERSION; }

kb_ctx* kb_create(const kb_opts* opts) {
  kb_ctx* c = new kb_ctx();
  c->device = opts ? opts->device : 0;
  c->timing = opts && (opts->flags & KB_OPT_TIMING);
  c->timing_every = opts && opts->timing_every > 1 ? opts->timing_every : 1;
  const uint32_t fl = opts ? opts->flags : 0u;
  c->use_aff_reg = !(fl & KB_OPT_NO_AFF_REG);
  c->use_cap1 = !(fl & KB_OPT_NO_CAP1);
  c->use_cls = !(fl & KB_OPT_NO_CLS);
  c->use_fed = !(fl & KB_OPT_NO_FED);
  c->use_eval_plain = !(fl & KB_OPT_NO_EVAL_PLAIN);
  c->use_fed_split = !(fl & KB_OPT_NO_FED_SPLIT);
  c->use_pipeline = !(fl & KB_OPT_NO_PIPELINE);
  c->fed_dedicated = !(fl & KB_OPT_FED_SHARED_QUEUES);
  c->fed_coop = c->fed_dedicated && (fl & KB_OPT_FED_COOP_LAUNCH) && !(fl & KB_OPT_FED_PLAIN_LAUNCH);
  c->shard_self_inbox = (fl & KB_OPT_SHARD_SELF_INBOX) != 0;
  c->test_peer_badtag = (fl & KB_OPT_TEST_PEER_BADTAG) != 0;
  c->fed_kernel_sweeps = (fl & KB_OPT_FED_KERNEL_SWEEPS) != 0;
  c->test_one_xcc = (fl & KB_OPT_TEST_ONE_XCC) != 0;
  c->no_lvl = (fl & KB_OPT_FED_NO_LEVELS) != 0;
  c->use_fed_aff = !(fl & KB_OPT_FED_NO_AFF);
  c->fed_diag = (fl & KB_OPT_FED_DIAG) != 0;
  c->issue_trace = getenv("KB_HOST_TRACE") != nullptr;
  if (opts && opts->fed_idle_ms > 0) c->fed_idle = (uint64_t)opts->fed_idle_ms * 100000ull;
  if (opts && opts->eval_spb > 0) c->eval_spb = opts->eval_spb;
  if (opts) c->shard_epoch0 = opts->shard_epoch0;
  // kb_opts.fed_xcc (ABI 15): 0 the library's default (kbgpu_ctx.h), k + 1 XCC k, < 0 the dispatcher's placement
  if (opts && opts->fed_xcc > 0) c->fed_xcc = opts->fed_xcc - 1;
  if (opts && opts->fed_xcc < 0) c->fed_xcc = -1;
  if (opts && opts->fed_depth >= 2) c->fed_depth = std::min(opts->fed_depth, (int)kJobSlots);
  if (opts && opts->test_stall_job >= 0) {
    c->test_stall_job = opts->test_stall_job;
    if (opts->test_stall_ms > 0) c->test_stall_ms = opts->test_stall_ms;
  }
  c->timing_now = c->timing;
  c->use_traj = !(opts && (opts->flags & KB_OPT_NO_TRAJECTORY));
  c->use_sel = !(opts && (opts->flags & KB_OPT_NO_SELECT));
  c->use_engine = opts && (opts->flags & KB_OPT_ENGINE);
  if (hipSetDevice(c->device) != hipSuccess) {
    c->err = "hipSetDevice failed";
    c->broken = true;
    return c;
  }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    c->err = "hipStreamCreate failed";
    c->broken = true;
    return c;
  }
  if (hipStreamCreateWithFlags(&c->eng_stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->eng_dep, hipEventDisableTiming) != hipSuccess) {
    c->err = "hipStreamCreate (engine) failed";
    c->broken = true;
    return c;
  }
  {  // grids sized per device (eval_plain_kernel's resident round)
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, c->device) == hipSuccess && cu > 0)
      c->cus = cu;
  }
  c->eval_bpc32 = kbgpu::eval_plain_blocks_per_cu(true);
  c->eval_bpc64 = kbgpu::eval_plain_blocks_per_cu(false);
  if (int e = kbgpu::configure_kernels()) {
    c->err = std::string("hipFuncSetAttribute(dynamic LDS): ") + hipGetErrorString((hipError_t)e);
    c->broken = true;
    return c;
  }
  c->cfg = DevCfg{1, 1, 0, 0, 0, 1, 1, 1, 1};
  return c;
}

void kb_destroy(kb_ctx* c) {
  if (!c) return;
  if (!c->broken) {
    (void)hipSetDevice(c->device);
    (void)kb_engine_stop(c);
  }
  free_all(c->node_mem);
  free_all(c->spec_mem);
  free_all(c->aff_mem);
  free_all(c->work_mem);
  free_all(c->ov_mem);
  if (c->h_job) (void)hipHostFree(c->h_job);
  for (int s = 0; s < kJobSlots; ++s)
    if (c->h_jobx[s]) (void)hipHostFree(c->h_jobx[s]);
  for (int s = 0; s < kJobSlots; ++s) {
    if (c->sel_keys[s]) (void)hipFree(c->sel_keys[s]);
    if (c->sel_stat[s]) (void)hipFree(c->sel_stat[s]);
    if (c->sel_lvl[s]) (void)hipFree(c->sel_lvl[s]);
    if (c->commits[s]) (void)hipFree(c->commits[s]);
  }
  if (c->stream_b) (void)hipStreamDestroy(c->stream_b);
  if (c->stream_alt) (void)hipStreamDestroy(c->stream_alt);
  if (c->sweep_ctr) (void)hipFree(c->sweep_ctr);
  if (c->fed_ring) (void)hipFree(c->fed_ring);
  if (c->fed_ctr) (void)hipFree(c->fed_ctr);
  if (c->fed_exit) (void)hipFree(c->fed_exit);
  if (c->fed_xchg) (void)hipFree(c->fed_xchg);
  if (c->h_fed_ctrs) (void)hipHostFree(c->h_fed_ctrs);
  if (c->fed_hring) (void)hipHostFree(c->fed_hring);
  if (c->h_eval) (void)hipHostFree(c->h_eval);
  (void)hipFree(c->eval_ids);
  (void)hipFree(c->eval_r);
  (void)hipFree(c->eval_s);
  if (c->h_cmd) (void)hipHostFree(c->h_cmd);
  if (c->h_rec) (void)hipHostFree(c->h_rec);
  if (c->d_rec) (void)hipFree(c->d_rec);
  if (c->d_rec_all) (void)hipFree(c->d_rec_all);
  if (c->comm) (void)ncclCommDestroy((ncclComm_t)c->comm);
  for (int w = 0; w < kShardMaxWorld; ++w)
    if (c->peer_inbox[w] && c->peer_inbox[w] != c->inbox) (void)hipIpcCloseMemHandle(c->peer_inbox[w]);
  if (c->inbox) (void)hipFree(c->inbox);
  if (c->eng_dep) (void)hipEventDestroy(c->eng_dep);
  if (c->eng_stream) (void)hipStreamDestroy(c->eng_stream);
  for (auto& p : c->pending) {
    c->ev_pool.push_back(p.a);
    c->ev_pool.push_back(p.b);
  }
  for (hipEvent_t e : c->ev_pool) (void)hipEventDestroy(e);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

const char* kb_last_error(const kb_ctx* c) { return c ? c->err.c_str() : "null context"; }

int kb_set_config(kb_ctx* c, const kb_config* cfg) {
  if (c) c->prev_listed = false;
  if (!c || !cfg) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  c->cfg = DevCfg{cfg->predicates_enabled, cfg->nodeorder_enabled, cfg->mem_pressure, cfg->disk_pressure,
                  cfg->pid_pressure, cfg->w_lr, cfg->w_bra, cfg->w_na, cfg->w_pa};
  kb_update_traj_ok(c);
  return kb_check_score_range(c);
}

int kb_upload_nodes(kb_ctx* c, const kb_nodes* in) {
  if (c) c->prev_listed = false;
  if (!c || !in) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (in->n == 0 || in->n >= kMaxNodes) return fail(c, KB_E_INVALID, "node count %u out of range", in->n);
  if (in->n_scalar > 64) return fail(c, KB_E_UNSUPPORTED, "more than 64 scalar resource slots");
  HIP_OK(c, hipSetDevice(c->device));
  free_all(c->node_mem);
  free_all(c->work_mem);
  drop_affinity(c);
  drop_overlay(c);
  c->nodes_ok = false;
  DevNodes& N = c->N;
  const size_t n = in->n;
  N.n = (int32_t)in->n;
  N.base = 0;
  if (c->sharded) {
    if ((uint64_t)c->shard.node_begin + in->n > c->shard.n_total)
      return fail(c, KB_E_INVALID, "shard rows [%u, %u) exceed n_total %u", c->shard.node_begin,
                  c->shard.node_begin + in->n, c->shard.n_total);
    N.base = (int32_t)c->shard.node_begin;
  }
  N.S = (int32_t)in->n_scalar;
  N.K = (int32_t)in->n_label;
  N.P = (int32_t)in->n_port;
  int rc;
#define UP(field, cnt)                                                                   \
  if ((rc = upload(c, c->node_mem, &N.field, in->field, (cnt))) != KB_OK) return rc;
  UP(idle_cpu, n) UP(idle_mem, n) UP(rel_cpu, n) UP(rel_mem, n);
  UP(idle_sc, n * N.S) UP(rel_sc, n * N.S);
  UP(alloc_cpu, n) UP(alloc_mem, n) UP(nz_cpu, n) UP(nz_mem, n);
  UP(pod_count, n) UP(max_pods, n) UP(flags, n);
  UP(label_val, n * N.K) UP(label_int, n * N.K) UP(label_int_ok, n * N.K);
  UP(taint_set, n) UP(port_used, n * N.P);
#undef UP
  // pristine copies of the columns commits mutate
  c->pristine.clear();
  auto keep = [&](void* col, size_t bytes) -> int {
    void* q;
    HIP_OK(c, hipMalloc(&q, std::max<size_t>(bytes, 1)));
    c->node_mem.push_back(q);
    HIP_OK(c, hipMemcpy(q, col, bytes, hipMemcpyDeviceToDevice));
    c->pristine.push_back({col, q, bytes});
    return KB_OK;
  };
  if ((rc = keep(N.idle_cpu, n * 8)) || (rc = keep(N.idle_mem, n * 8)) || (rc = keep(N.rel_cpu, n * 8)) ||
      (rc = keep(N.rel_mem, n * 8)) || (rc = keep(N.idle_sc, n * N.S * 8)) || (rc = keep(N.rel_sc, n * N.S * 8)) ||
      (rc = keep(N.nz_cpu, n * 8)) || (rc = keep(N.nz_mem, n * 8)) || (rc = keep(N.pod_count, n * 4)) ||
      (rc = keep(N.port_used, n * N.P * 8)))
    return rc;
  // work buffers: keys, chunk maxima, job state + placement pairs
  void* p;
  HIP_OK(c, hipMalloc(&p, n * sizeof(uint64_t)));
  c->work_mem.push_back(p);
  c->keys = (uint64_t*)p;
  HIP_OK(c, hipMalloc(&p, ((n + 63) / 64 + 2) * sizeof(uint64_t)));
  c->work_mem.push_back(p);
  c->cmax = (uint64_t*)p;
  HIP_OK(c, hipMalloc(&p, n * sizeof(uint64_t)));
  c->work_mem.push_back(p);
  c->stat = (uint64_t*)p;
  HIP_OK(c, hipMalloc(&p, (size_t)kClsLevels * n * sizeof(uint64_t)));  // class loop scratch
  c->work_mem.push_back(p);
  c->cls_lvl = (uint64_t*)p;
  HIP_OK(c, hipMalloc(&p, n * sizeof(int32_t)));
  c->work_mem.push_back(p);
  c->cls_amax = (int32_t*)p;
  HIP_OK(c, hipMalloc(&p, kClsMaxK * sizeof(uint64_t)));
  c->work_mem.push_back(p);
  c->cls_cbest = (uint64_t*)p;
  HIP_OK(c, memset_sync(p, 0, kClsMaxK * sizeof(uint64_t)));
  c->idx_bits = 1;  // key index field: global node indices when sharded
  const unsigned long long n_keys = c->sharded ? c->shard.n_total : n;
  while ((1ull << c->idx_bits) < n_keys) ++c->idx_bits;
  int pbc;
  c->traj_full = traj_lds_bytes((int)n, 64, &pbc) > 0;
  c->sel_ok = sel_lds_bytes((int)n) >= 0;
  if (c->traj_full || c->sel_ok) {  // trajectory levels, or level 0 only (the selection path's keys)
    const size_t levels = c->traj_full ? (size_t)kTrajMaxJ + 1 : 1;
    HIP_OK(c, hipMalloc(&p, levels * n * sizeof(uint32_t)));
    c->work_mem.push_back(p);
    c->traj = (uint32_t*)p;
    HIP_OK(c, hipMalloc(&p, ((n + 63) / 64 + 4) * sizeof(uint32_t)));
    c->work_mem.push_back(p);
    c->cmax32 = (uint32_t*)p;
    HIP_OK(c, hipMalloc(&p, n * sizeof(uint32_t)));
    c->work_mem.push_back(p);
    c->amax = (uint32_t*)p;
  } else {
    c->traj = nullptr;
  }
  c->nodes_ok = true;
  kb_update_traj_ok(c);  // key widths depend on the node count
  return KB_OK;
}

int kb_upload_specs(kb_ctx* c, const kb_specs* in) {
  if (c) c->prev_listed = false;
  if (!c || !in) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (!c->nodes_ok) return fail(c, KB_E_STATE, "upload nodes before specs");
  HIP_OK(c, hipSetDevice(c->device));
  free_all(c->spec_mem);
  c->specs_ok = false;
  drop_affinity(c);
  drop_overlay(c);
  if (in->n_tol_sets == 0 || in->n_taint_sets == 0) return fail(c, KB_E_INVALID, "empty toleration/taint tables");
  // host-side validation of every index the kernels will follow (no out-of-bounds device access)
  const uint32_t S = (uint32_t)c->N.S;
  for (uint32_t i = 0; i < in->m; ++i) {
    const kb_spec& s = in->specs[i];
    if (s.tol_set < 0 || (uint32_t)s.tol_set >= in->n_tol_sets) return fail(c, KB_E_INVALID, "spec %u tol_set", i);
    if ((s.flags & KB_SPEC_HAS_SELECTOR) && s.sel_term >= in->n_terms) return fail(c, KB_E_INVALID, "spec %u sel", i);
    if ((uint64_t)s.req_term_off + s.req_term_cnt > in->n_terms) return fail(c, KB_E_INVALID, "spec %u req", i);
    if ((uint64_t)s.pref_term_off + s.pref_term_cnt > in->n_terms) return fail(c, KB_E_INVALID, "spec %u pref", i);
    if ((uint64_t)s.port_off + s.port_cnt > in->n_ports) return fail(c, KB_E_INVALID, "spec %u ports", i);
    if (S < 64 && ((s.init_sc_mask | s.req_sc_mask) >> S)) return fail(c, KB_E_INVALID, "spec %u scalar mask", i);
  }
  for (uint32_t i = 0; i < in->n_terms; ++i)
    if ((uint64_t)in->terms[i].req_off + in->terms[i].req_cnt > in->n_reqs)
      return fail(c, KB_E_INVALID, "term %u", i);
  for (uint32_t i = 0; i < in->n_reqs; ++i) {
    const kb_req& r = in->reqs[i];
    if (r.op < KB_OP_IN || r.op > KB_OP_FALSE) return fail(c, KB_E_INVALID, "req %u op", i);
    if (r.op < KB_OP_TRUE && (r.key < 0 || r.key >= c->N.K)) return fail(c, KB_E_INVALID, "req %u key", i);
    if ((uint64_t)r.val_off + r.val_cnt > in->n_vals) return fail(c, KB_E_INVALID, "req %u vals", i);
  }
  for (uint32_t i = 0; i < in->n_ports; ++i)
    if (in->ports[i].slot < 0 || in->ports[i].slot >= c->N.P || in->ports[i].ip < 0 || in->ports[i].ip > 63)
      return fail(c, KB_E_INVALID, "port %u", i);
  std::vector<int32_t> ts(c->N.n);
  HIP_OK(c, hipMemcpy(ts.data(), c->N.taint_set, ts.size() * 4, hipMemcpyDeviceToHost));
  for (int32_t t : ts)
    if (t < 0 || (uint32_t)t >= in->n_taint_sets) return fail(c, KB_E_INVALID, "node taint_set %d out of range", t);

  DevSpecs& P = c->P;
  int rc;
  if ((rc = upload(c, c->spec_mem, &P.specs, in->specs, in->m))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.sc_init, in->sc_init, (size_t)in->m * S))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.sc_req, in->sc_req, (size_t)in->m * S))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.terms, in->terms, in->n_terms))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.reqs, in->reqs, in->n_reqs))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.vals, in->vals, in->n_vals))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.ports, in->ports, in->n_ports))) return rc;
  if ((rc = upload(c, c->spec_mem, &P.tolerates, in->tolerates, (size_t)in->n_tol_sets * in->n_taint_sets))) return rc;
  P.n_taint_sets = (int32_t)in->n_taint_sets;
  P.m = (int32_t)in->m;
  c->max_pref_weight = 0;
  c->spec_pref_weight.assign(in->m, 0);
  c->spec_needs_aff.assign(in->m, 0);
  c->spec_ipa_err.assign(in->m, 0);
  c->ov_absmax.assign(in->m, 0);
  for (uint32_t i = 0; i < in->m; ++i) c->spec_ipa_err[i] = (in->specs[i].flags & KB_SPEC_IPA_ERROR) != 0;
  c->spec_plain.assign(in->m, 0);
  for (uint32_t i = 0; i < in->m; ++i) {
    const kb_spec& s = in->specs[i];
    const uint32_t not_plain = KB_SPEC_HAS_SELECTOR | KB_SPEC_HAS_REQUIRED | KB_SPEC_INIT_HAS_MAP | KB_SPEC_NA_ERROR |
                               KB_SPEC_IPA_ERROR | KB_SPEC_POD_AFFINITY;
    const int64_t lim = 1ll << 49;  // (the row-only kernel's f64 loop: requests below 2^49)
    c->spec_plain[i] = !(s.flags & not_plain) && s.pref_term_cnt == 0 && s.port_cnt == 0 && s.aff_class < 0 &&
                       in->n_taint_sets == 1 && in->tolerates[(size_t)s.tol_set] != 0 && s.init_cpu >= 0 &&
                       s.init_cpu < lim && s.init_mem >= 0 && s.init_mem < lim && s.nz_cpu >= 0 && s.nz_cpu < lim &&
                       s.nz_mem >= 0 && s.nz_mem < lim;
  }
  c->spec_aff_class0.assign(in->m, -1);
  c->spec_rowcols.assign(in->m, 0);
  for (uint32_t i = 0; i < in->m; ++i) {
    const kb_spec& q = in->specs[i];
    c->spec_rowcols[i] = (q.flags & (KB_SPEC_INIT_HAS_MAP | KB_SPEC_REQ_HAS_MAP)) || q.init_sc_mask || q.req_sc_mask ||
                         q.port_cnt;
  }
  for (uint32_t i = 0; i < in->m; ++i) {
    c->spec_needs_aff[i] = (in->specs[i].flags & KB_SPEC_POD_AFFINITY) || in->specs[i].aff_class >= 0;
    c->spec_aff_class0[i] = in->specs[i].aff_class;
  }
  for (uint32_t i = 0; i < in->m; ++i) {
    int64_t sum = 0;
    for (uint32_t j = 0; j < in->specs[i].pref_term_cnt; ++j)
      sum += std::llabs((long long)in->terms[in->specs[i].pref_term_off + j].weight);
    c->max_pref_weight = std::max(c->max_pref_weight, sum);
    c->spec_pref_weight[i] = sum;
  }
  // Feasibility classes (the driver's NO_FIT prediction, kbgpu_allocate.cpp): two specs share a class when everything
  // PredicateFn reads of them other than InitResreq is equal -- flags, tolerations, the selector and required node
  // affinity terms (by content), host ports. Within a class feasibility is monotone in InitResreq
  // (resource_info.go:253-276: LessEqual per resource), and within an allocate cycle every node's Idle, Releasing,
  // pod count and used ports only move toward failure, so a spec that found no node stays without one, and so does
  // every spec of its class whose request is at least as large in every resource. A class's parents are the classes
  // of the same signature with its nodeSelector and / or its required node affinity dropped (predicates.go:
  // PodMatchNodeSelector ANDs both): a parent's feasible nodes are a superset, so a dead parent spec kills too.
  {
    std::unordered_map<std::string, int32_t> ids;
    c->spec_fclass.assign(in->m, -1);
    c->spec_fparent.assign((size_t)in->m * 3, -1);
    c->spec_init.assign((size_t)in->m * (2 + S), 0);
    c->spec_init_mask.assign(in->m, 0);
    std::string k;
    auto put = [&k](const void* p, size_t b) { k.append((const char*)p, b); };
    auto put_term = [&](uint32_t t) {
      const kb_term& tm = in->terms[t];
      put(&tm.req_cnt, 4);
      for (uint32_t q = 0; q < tm.req_cnt; ++q) {
        const kb_req& r = in->reqs[tm.req_off + q];
        put(&r.key, 4), put(&r.op, 4), put(&r.val_cnt, 4), put(&r.ival, 8);
        put(in->vals + r.val_off, 4 * (size_t)r.val_cnt);
      }
    };
    // the signature with the selector (drop & 1) and / or the required terms (drop & 2) left out
    auto sig = [&](const kb_spec& q, int drop) {
      k.clear();
      uint32_t fl = q.flags;
      if (drop & 1) fl &= ~KB_SPEC_HAS_SELECTOR;
      if (drop & 2) fl &= ~KB_SPEC_HAS_REQUIRED;
      put(&fl, 4), put(&q.tol_set, 4);
      if (fl & KB_SPEC_HAS_SELECTOR) put_term(q.sel_term);
      const uint32_t nreq = (fl & KB_SPEC_HAS_REQUIRED) ? q.req_term_cnt : 0u;
      put(&nreq, 4);
      for (uint32_t t = 0; t < nreq; ++t) put_term(q.req_term_off + t);
      put(&q.port_cnt, 4);
      put(in->ports + q.port_off, sizeof(kb_port) * (size_t)q.port_cnt);
      return k;
    };
    auto eligible = [](const kb_spec& q) {
      return !((q.flags & (KB_SPEC_POD_AFFINITY | KB_SPEC_IPA_ERROR)) || q.aff_class >= 0);
    };
    for (uint32_t i = 0; i < in->m; ++i) {
      const kb_spec& q = in->specs[i];
      int64_t* v = c->spec_init.data() + (size_t)i * (2 + S);
      v[0] = q.init_cpu, v[1] = q.init_mem;
      for (uint32_t r = 0; r < S; ++r) v[2 + r] = in->sc_init[(size_t)i * S + r];
      c->spec_init_mask[i] = q.init_sc_mask;
      if (!eligible(q)) continue;
      c->spec_fclass[i] = ids.emplace(sig(q, 0), (int32_t)ids.size()).first->second;
    }
    for (uint32_t i = 0; i < in->m; ++i) {
      const kb_spec& q = in->specs[i];
      if (!eligible(q)) continue;
      for (int drop = 1; drop <= 3; ++drop) {
        if (((drop & 1) && !(q.flags & KB_SPEC_HAS_SELECTOR)) || ((drop & 2) && !(q.flags & KB_SPEC_HAS_REQUIRED)))
          continue;  // (the same signature)
        const auto it = ids.find(sig(q, drop));
        if (it != ids.end()) c->spec_fparent[(size_t)i * 3 + (drop - 1)] = it->second;
      }
    }
    c->n_fclass = (int32_t)ids.size();
  }
  kb_update_traj_ok(c);
  c->specs_ok = true;
  return kb_check_score_range(c);
}

int kb_upload_affinity(kb_ctx* c, const kb_affinity* a) {
  if (c) c->prev_listed = false;
  if (!c || !a) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs before affinity");
  HIP_OK(c, hipSetDevice(c->device));
  drop_affinity(c);
  // node-sharded: topo_dom holds every node of the cluster (a commit on another rank's row moves the
  // replicated count tables at that node's domains); the device sees it from this rank's first row
  const size_t n = c->sharded ? (size_t)c->shard.n_total : (size_t)c->N.n;
  if (a->m != (uint32_t)c->P.m) return fail(c, KB_E_INVALID, "affinity specs %u != specs %d", a->m, c->P.m);
  // every index the kernels follow is checked here (no out-of-bounds device access)
  std::vector<int64_t> D(a->n_slots, 0);  // domains per slot
  for (uint32_t sl = 0; sl < a->n_slots; ++sl)
    for (size_t i = 0; i < n; ++i) {
      const int32_t d = a->topo_dom[sl * n + i];
      if (d < -1) return fail(c, KB_E_INVALID, "topo_dom[%u][%zu] = %d", sl, i, d);
      D[sl] = std::max<int64_t>(D[sl], (int64_t)d + 1);
    }
  auto slot_ok = [&](int32_t sl) { return sl >= 0 && (uint32_t)sl < a->n_slots; };
  for (uint32_t t = 0; t < a->n_tables; ++t) {
    const kb_aff_table& tb = a->tables[t];
    if (!slot_ok(tb.slot) || (int64_t)tb.cnt_off + D[tb.slot] > (int64_t)a->n_counters)
      return fail(c, KB_E_INVALID, "affinity table %u", t);
  }
  for (uint32_t i = 0; i < a->n_checks; ++i)
    if (a->checks[i].table < 0 || (uint32_t)a->checks[i].table >= a->n_tables || a->checks[i].kind < 0 ||
        a->checks[i].kind > KB_AFF_ERROR)
      return fail(c, KB_E_INVALID, "affinity check %u", i);
  for (uint32_t i = 0; i < a->n_lister; ++i)
    if (a->lister[i] < 0 || (uint32_t)a->lister[i] >= a->n_tables) return fail(c, KB_E_INVALID, "lister %u", i);
  for (uint32_t i = 0; i < a->n_hists; ++i)
    if (!slot_ok(a->hists[i].slot) || (int64_t)a->hists[i].h_off + D[a->hists[i].slot] > (int64_t)a->n_h)
      return fail(c, KB_E_INVALID, "ipa hist %u", i);
  for (uint32_t i = 0; i < a->n_incr; ++i)
    if (!slot_ok(a->incr[i].slot) || (int64_t)a->incr[i].h_off + D[a->incr[i].slot] > (int64_t)a->n_h)
      return fail(c, KB_E_INVALID, "ipa incr %u", i);
  for (uint32_t s = 0; s < a->m; ++s) {
    const kb_aff_spec& e = a->specs[s];
    if ((uint64_t)e.check_off + e.check_cnt > a->n_checks || (uint64_t)e.lister_off + e.lister_cnt > a->n_lister ||
        (uint64_t)e.hist_off + e.hist_cnt > a->n_hists || (uint64_t)e.incr_off + e.incr_cnt > a->n_incr)
      return fail(c, KB_E_INVALID, "affinity spec %u offsets", s);
  }
  std::vector<kb_spec> specs(a->m);
  if (a->m) HIP_OK(c, hipMemcpy(specs.data(), c->P.specs, a->m * sizeof(kb_spec), hipMemcpyDeviceToHost));
  for (uint32_t s = 0; s < a->m; ++s) {  // as kb_upload_specs had them (an earlier upload may have marked some inert)
    specs[s].aff_class = c->spec_aff_class0[s];
    c->spec_needs_aff[s] = (specs[s].flags & KB_SPEC_POD_AFFINITY) || specs[s].aff_class >= 0;
  }
  c->spec_dyn.assign(a->m, 0);
  c->spec_hist.assign(a->m, 0);
  c->spec_incr.assign(a->m, 0);
  c->spec_aff_reg.assign(a->m, 0);
  c->spec_aff_err.assign(a->m, 0);
  c->aff_rd.assign(a->m, {});
  c->aff_wr.assign(a->m, {});
  for (uint32_t s = 0; s < a->m; ++s) {
    const int32_t ac = specs[s].aff_class;
    if (ac < -1 || ac >= (int32_t)a->m) return fail(c, KB_E_INVALID, "spec %u aff_class %d", s, ac);
    if (ac >= 0) {
      // what a sweep of this spec reads (check tables, its histograms) and what its commits write (lister tables,
      // histogram increments): histograms as h_off | 1 << 31
      const kb_aff_spec& x = a->specs[ac];
      auto& rd = c->aff_rd[s];
      auto& wr = c->aff_wr[s];
      for (uint32_t i = 0; i < x.check_cnt; ++i) rd.push_back((uint32_t)a->checks[x.check_off + i].table);
      for (uint32_t i = 0; i < x.hist_cnt; ++i) rd.push_back(a->hists[x.hist_off + i].h_off | 1u << 31);
      for (uint32_t i = 0; i < x.lister_cnt; ++i) wr.push_back((uint32_t)a->lister[x.lister_off + i]);
      for (uint32_t i = 0; i < x.incr_cnt; ++i) wr.push_back(a->incr[x.incr_off + i].h_off | 1u << 31);
      std::sort(rd.begin(), rd.end());
      std::sort(wr.begin(), wr.end());
      for (uint32_t i = 0; i < a->specs[ac].check_cnt; ++i)
        if (a->checks[a->specs[ac].check_off + i].kind == KB_AFF_ERROR) c->spec_aff_err[s] = 1;
      c->spec_dyn[s] = (a->specs[ac].flags & KB_AFF_SELF_DYNAMIC) != 0;
      c->spec_hist[s] = a->specs[ac].hist_cnt > 0;
      c->spec_incr[s] = a->specs[ac].lister_cnt > 0 || a->specs[ac].incr_cnt > 0;
      const kb_aff_spec& e = a->specs[ac];
      bool ok = e.check_cnt + e.hist_cnt <= 4 && e.lister_cnt + e.incr_cnt <= 8;  // kAffRegE, kAffRegU; 16-bit domains
      for (uint32_t i = 0; ok && i < e.check_cnt; ++i) ok = D[a->tables[a->checks[e.check_off + i].table].slot] < 0xffff;
      for (uint32_t i = 0; ok && i < e.hist_cnt; ++i) ok = D[a->hists[e.hist_off + i].slot] < 0xffff;
      c->spec_aff_reg[s] = ok && e.check_cnt + e.hist_cnt > 0 ? (char)(e.check_cnt + e.hist_cnt) : 0;  // entries (0: not eligible)
    }
  }
  c->aff_slot_D = D;
  c->aff_n_tables = a->n_tables;
  c->aff_n_h = a->n_h;
  classify_self_dynamic(c, a, D, specs);
  // member lists of every class slot: class k = domain k, class D = the nodes without a domain
  c->cls_coff.assign(a->n_slots, nullptr);
  c->cls_mem.assign(a->n_slots, nullptr);
  for (uint32_t s = 0; s < a->m; ++s) {
    const int32_t F = c->spec_cls[s];
    if (F < 0 || c->cls_coff[F] || n >= 65536 || c->sharded) continue;
    const size_t K = (size_t)D[F] + 1;
    std::vector<uint32_t> off(K + 1, 0);
    std::vector<uint16_t> mem((n + 7) / 8 * 8, 0);  // padded: the kernel reads it in 16-byte loads
    auto cls_of = [&](size_t i) { const int32_t d = a->topo_dom[F * n + i]; return d >= 0 ? (size_t)d : K - 1; };
    for (size_t i = 0; i < n; ++i) ++off[cls_of(i) + 1];
    for (size_t k = 0; k < K; ++k) off[k + 1] += off[k];
    std::vector<uint32_t> cur(off.begin(), off.end() - 1);
    for (size_t i = 0; i < n; ++i) mem[cur[cls_of(i)]++] = (uint16_t)i;
    int rc_;
    if ((rc_ = upload(c, c->aff_mem, &c->cls_coff[F], off.data(), K + 1))) return rc_;
    if ((rc_ = upload(c, c->aff_mem, &c->cls_mem[F], mem.data(), mem.size()))) return rc_;
  }
  // A spec whose affinity entry is empty -- no checks, no InterPodAffinity histograms, no table its commits write,
  // no batch score error -- is one the affinity stages leave alone: every node passes InterPodAffinityMatches, its
  // InterPodAffinity counts are all 0 (score 0, interpod_affinity.go:219-241), and its commits move nothing. It
  // gets KB_SPEC_POD_AFFINITY only because some other pod of the session has terms (the exporter's aff_in_play).
  // Such specs run as plain ones (aff_class -1 on the device): the resident engine takes them (a mixed cycle's
  // C2 jobs beside its affinity jobs).
  for (uint32_t s = 0; s < a->m; ++s) {
    const int32_t ac = specs[s].aff_class;
    if (ac < 0 || c->spec_ipa_err[s]) continue;
    const kb_aff_spec& e = a->specs[ac];
    if (e.check_cnt || e.hist_cnt || e.lister_cnt || e.incr_cnt || (e.flags & KB_AFF_SELF_DYNAMIC)) continue;
    specs[s].aff_class = -1;
    c->spec_needs_aff[s] = 0;
    c->aff_rd[s].clear();
    c->aff_wr[s].clear();
  }
  if (a->m) HIP_OK(c, hipMemcpy(c->P.specs, specs.data(), a->m * sizeof(kb_spec), hipMemcpyHostToDevice));
  DevAff& A = c->P.A;
  int rc;
  if ((rc = upload(c, c->aff_mem, &A.topo_dom, a->topo_dom, (size_t)a->n_slots * n))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.tables, a->tables, a->n_tables))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.totals, a->totals, a->n_tables))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.counters, a->counters, a->n_counters))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.specs, a->specs, a->m))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.checks, a->checks, a->n_checks))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.lister, a->lister, a->n_lister))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.hists, a->hists, a->n_hists))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.h, a->h, a->n_h))) return rc;
  if ((rc = upload(c, c->aff_mem, &A.incr, a->incr, a->n_incr))) return rc;
  int64_t* mm = nullptr;
  if ((rc = upload(c, c->aff_mem, &mm, (const int64_t*)nullptr, 2, false))) return rc;
  A.mm = mm;
  int64_t* mm_spec = nullptr;  // (the fed engine's: kb_fed_ipa_prepare)
  if ((rc = upload(c, c->aff_mem, &mm_spec, (const int64_t*)nullptr, 2 * (size_t)std::max<uint32_t>(a->m, 1), false)))
    return rc;
  A.mm_spec = mm_spec;
  c->mm_spec_ok.assign(a->m, 0);
  if ((rc = upload(c, c->aff_mem, &c->d_mm_ids, (const int32_t*)nullptr, std::max<uint32_t>(a->m, 1), false))) return rc;
  c->mm_ids_cap = a->m;
  A.n = (int32_t)n;
  if (c->sharded) A.topo_dom += c->N.base;  // (aff_mem keeps the allocation's own pointer)
  // pristine copies of the mutable tables (kb_restore_nodes re-opens the session)
  auto keep = [&](void* col, size_t bytes) -> int {
    void* q;
    HIP_OK(c, hipMalloc(&q, std::max<size_t>(bytes, 1)));
    c->aff_mem.push_back(q);
    HIP_OK(c, hipMemcpy(q, col, bytes, hipMemcpyDeviceToDevice));
    c->aff_pristine.push_back({col, q, bytes});
    return KB_OK;
  };
  if ((rc = keep(A.totals, a->n_tables * 4)) || (rc = keep(A.counters, a->n_counters * 4)) ||
      (rc = keep(A.h, a->n_h * 4)))
    return rc;
  A.enabled = 1;
  c->aff_ok = true;
  return KB_OK;
}

// Which specs can use the 32-bit trajectory keys: |score| bound below 2^(30 - idx_bits).
void kb_update_traj_ok(kb_ctx* c) {
  const DevCfg& C = c->cfg;
  const long double bias32 = (long double)(1ll << (30 - c->idx_bits));
  c->spec_traj_ok.assign(c->spec_pref_weight.size(), 0);
  for (size_t i = 0; i < c->spec_pref_weight.size(); ++i) {
    const int64_t ov = i < c->ov_absmax.size() ? c->ov_absmax[i] : 0;
    long double bound = 10.0L * std::llabs((long long)C.w_lr) + 10.0L * std::llabs((long long)C.w_bra) +
                        (long double)c->spec_pref_weight[i] * std::llabs((long long)C.w_na) + (long double)ov +
                        10.0L * std::llabs((long long)C.w_pa);
    // a batch-score error (KB_SPEC_IPA_ERROR) scores far below any 32-bit key
    c->spec_traj_ok[i] = bound < bias32 - 1 && !(i < c->spec_ipa_err.size() && c->spec_ipa_err[i]);
  }
}

int kb_check_score_range(kb_ctx* c) {
  // |score| must stay inside the key's 39-bit biased field, and |NodeAffinity x weight + overlay score|
  // inside the static cache's signed 27-bit field.
  const DevCfg& C = c->cfg;
  for (size_t i = 0; i < c->spec_pref_weight.size(); ++i) {
    const int64_t ov = i < c->ov_absmax.size() ? c->ov_absmax[i] : 0;
    const long double na = (long double)c->spec_pref_weight[i] * std::llabs((long long)C.w_na) + (long double)ov;
    const long double bound = 10.0L * std::llabs((long long)C.w_lr) + 10.0L * std::llabs((long long)C.w_bra) + na +
                              10.0L * std::llabs((long long)C.w_pa);
    if (bound >= (long double)(kScoreBias / 2)) return fail(c, KB_E_UNSUPPORTED, "score range exceeds 2^37");
    if (na >= (long double)(1 << 26))
      return fail(c, KB_E_UNSUPPORTED, "spec %zu: NodeAffinity x weight + overlay score exceeds 2^26", i);
  }
  return KB_OK;
}

// Wait for the last place launch of a job: spin on the sequence number it writes to pinned host memory
// (cheaper than a stream synchronisation's wake-up), checking the stream now and then so a failed launch
// is reported instead of waited on. Kernel timing events are then complete or nearly so.
static int wait_seq(kb_ctx* c, const JobState* hs, uint32_t want) {
  auto t0 = std::chrono::steady_clock::now();
  for (uint64_t spin = 0;; ++spin) {
    if (__atomic_load_n(&hs->seq, __ATOMIC_ACQUIRE) == want) break;
    if ((spin & 4095) == 4095) {
      hipError_t q = hipStreamQuery(c->stream);
      if (q == hipSuccess) {
        if (__atomic_load_n(&hs->seq, __ATOMIC_ACQUIRE) == want) break;
        if (c->fed) {  // the resident engine left: idle exit (a host stall longer than the idle bound)?
          int32_t idle = 0;
          if (hipMemcpy(&idle, c->fed_exit, sizeof(idle), hipMemcpyDeviceToHost) == hipSuccess && idle)
          {
            c->fed_exit_code = idle;  // 1 idle; 2 / 3: a selector / placer hand-off word never came (a bug)
            return fail(c, kFedIdleExit, "fed engine exited (code %d) before command %u", idle, want);
          }
        }
        return fail(c, KB_E_HIP, "place kernel finished without reporting (seq %u, want %u)", hs->seq, want);
      }
      if (q != hipErrorNotReady) return fail(c, KB_E_HIP, "place kernel failed: %s", hipGetErrorString(q));
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        return fail(c, KB_E_HIP, "place kernel did not finish within 120 s");
    }
  }
  return KB_OK;
}
static int wait_seq(kb_ctx* c) { return wait_seq(c, (const JobState*)c->h_job, c->seq); }

static int ensure_job_buffers(kb_ctx* c, uint32_t n_tasks) {
  if (!c->d_job) {
    void* p;
    HIP_OK(c, hipMalloc(&p, sizeof(JobState)));
    c->work_mem.push_back(p);
    c->d_job = (char*)p;
  }
  if (n_tasks <= c->job_cap && c->h_job) return KB_OK;
  uint32_t cap = std::max<uint32_t>(n_tasks, 1024);
  size_t bytes = sizeof(JobState) + (size_t)cap * 2 * sizeof(int32_t);
  if (c->h_job) (void)hipHostFree(c->h_job);
  c->h_job = nullptr;
  // pinned, device-mapped: the place kernel writes placements and the job state straight to host memory
  HIP_OK(c, hipHostMalloc((void**)&c->h_job, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_OK(c, hipHostGetDevicePointer((void**)&c->h_job_dev, c->h_job, 0));
  memset(c->h_job, 0, bytes);
  ((JobState*)c->h_job)->seq = c->seq;
  c->job_cap = cap;
  return KB_OK;
}

// ---- persistent placement engine (kbgpu_device.hip engine_kernel) ----
constexpr uint64_t kEngineIdleTicks = 100000000ull;  // 1 s of s_memrealtime (100 MHz) without a command

int kb_engine_stop(kb_ctx* c) {
  if (!c || !c->eng_running) return KB_OK;
  EngineCmd* cm = (EngineCmd*)c->h_cmd;
  cm->op = KB_ENG_EXIT;
  __atomic_store_n(&cm->seq, ++c->seq, __ATOMIC_RELEASE);
  c->eng_running = false;
  const hipError_t e = hipStreamSynchronize(c->eng_stream);  // bounded: EXIT or the idle timeout ends it
  if (e != hipSuccess) return fail(c, KB_E_HIP, "placement engine: %s", hipGetErrorString(e));
  return KB_OK;
}

// Launch the engine so that it serves commands from seq0 on, after everything queued on c->stream.
static int engine_launch(kb_ctx* c, uint32_t seq0) {
  HIP_OK(c, hipEventRecord(c->eng_dep, c->stream));
  HIP_OK(c, hipStreamWaitEvent(c->eng_stream, c->eng_dep, 0));
  launch_engine(c->N, c->P, c->cfg, c->idx_bits, c->stat, (const EngineCmd*)c->h_cmd_dev, (JobState*)c->d_job,
                (JobState*)c->h_job_dev, (int32_t*)(c->h_job_dev + sizeof(JobState)), seq0, kEngineIdleTicks,
                c->eng_stream);
  HIP_OK(c, hipGetLastError());
  c->eng_running = true;
  return KB_OK;
}

// Every task of the job goes through the selection path: 32-bit keys, no inter-pod affinity, LDS fit.
static bool engine_ok(const kb_ctx* c, const kb_job_req* job) {
  if (!c->use_engine || !c->use_sel || !c->sel_ok) return false;
  for (uint32_t i = 0; i < job->n_tasks; ++i) {
    const int s = job->task_specs[i];
    if (!c->spec_traj_ok[s] || c->spec_needs_aff[s]) return false;
  }
  return true;
}

static int engine_place_job(kb_ctx* c, const kb_job_req* job, int32_t* placed_node, int32_t* placed_kind,
                            kb_job_result* result) {
  uint32_t n_runs = 0;
  for (uint32_t t = 0; t < job->n_tasks; ++t)
    if (t == 0 || job->task_specs[t] != job->task_specs[t - 1]) ++n_runs;
  // buffers the engine holds pointers to: grow them only while it is stopped
  if (n_runs > c->cmd_cap || job->n_tasks > c->job_cap || !c->h_job) {
    if (int rc = kb_engine_stop(c)) return rc;
    if (int rc = ensure_job_buffers(c, job->n_tasks)) return rc;
    if (n_runs > c->cmd_cap || !c->h_cmd) {
      const uint32_t cap = std::max<uint32_t>(n_runs, 256);
      if (c->h_cmd) (void)hipHostFree(c->h_cmd);
      c->h_cmd = nullptr;
      HIP_OK(c, hipHostMalloc((void**)&c->h_cmd, sizeof(EngineCmd) + (size_t)cap * sizeof(EngineRun),
                              hipHostMallocMapped | hipHostMallocCoherent));
      HIP_OK(c, hipHostGetDevicePointer((void**)&c->h_cmd_dev, c->h_cmd, 0));
      memset(c->h_cmd, 0, sizeof(EngineCmd));
      ((EngineCmd*)c->h_cmd)->seq = c->seq;
      c->cmd_cap = cap;
    }
  }
  auto t0 = std::chrono::steady_clock::now();
  EngineCmd* cm = (EngineCmd*)c->h_cmd;
  EngineRun* runs = (EngineRun*)(cm + 1);
  uint32_t r = 0;
  for (uint32_t t = 0; t < job->n_tasks;) {
    uint32_t e = t + 1;
    while (e < job->n_tasks && job->task_specs[e] == job->task_specs[t]) ++e;
    runs[r++] = EngineRun{job->task_specs[t], (int32_t)t, (int32_t)(e - t), 0};
    t = e;
  }
  // an engine that exited (idle timeout) is relaunched below
  if (c->eng_running) {
    const hipError_t q = hipStreamQuery(c->eng_stream);
    if (q == hipSuccess) c->eng_running = false;
    else if (q != hipErrorNotReady) {
      c->eng_running = false;
      return fail(c, KB_E_HIP, "placement engine failed: %s", hipGetErrorString(q));
    }
  }
  cm->op = KB_ENG_RUN;
  cm->n_runs = (int32_t)n_runs;
  cm->ready0 = job->ready_num;
  cm->minav0 = job->min_available;
  cm->gang0 = job->gang_ready;
  const uint32_t want = ++c->seq;
  __atomic_store_n(&cm->seq, want, __ATOMIC_RELEASE);
  if (!c->eng_running)
    if (int rc = engine_launch(c, want)) return rc;
  const JobState* hs = (const JobState*)c->h_job;
  for (uint64_t spin = 0;; ++spin) {
    if (__atomic_load_n(&hs->seq, __ATOMIC_ACQUIRE) == want) break;
    if ((spin & 1023) == 1023) {
      if (__atomic_load_n(&hs->exit_seq, __ATOMIC_ACQUIRE) == want) {  // it timed out just before our post
        (void)hipStreamSynchronize(c->eng_stream);
        c->eng_running = false;
        if (int rc = engine_launch(c, want)) return rc;
        continue;
      }
      const hipError_t q = hipStreamQuery(c->eng_stream);
      if (q == hipSuccess && __atomic_load_n(&hs->seq, __ATOMIC_ACQUIRE) != want &&
          __atomic_load_n(&hs->exit_seq, __ATOMIC_ACQUIRE) != want) {
        c->eng_running = false;
        return fail(c, KB_E_HIP, "placement engine exited without serving command %u", want);
      }
      if (q != hipSuccess && q != hipErrorNotReady) {
        c->eng_running = false;
        return fail(c, KB_E_HIP, "placement engine failed: %s", hipGetErrorString(q));
      }
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(120))
        return fail(c, KB_E_HIP, "placement engine did not answer command %u within 120 s", want);
    }
  }
  const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  c->device_ms += wall;
  c->stats.device_ms += wall;
  c->stats.job_calls += 1;
  for (int k = 0; k < 8; ++k) c->stats.diag[k] += hs->diag[k];
  const uint64_t tasks = (uint64_t)hs->n_placed + (hs->stop == KB_STOP_NO_FIT ? 1 : 0);
  c->stats.launches[KB_KERNEL_ENGINE] += 1;
  c->stats.kernel_ms[KB_KERNEL_ENGINE] += (double)(hs->t_done - hs->t_recv) * 1e-5;  // 100 MHz ticks
  c->stats.pairs[KB_KERNEL_ENGINE] += tasks * (uint64_t)c->N.n;
  const int32_t* ho = (const int32_t*)(c->h_job + sizeof(JobState));
  result->n_placed = (uint32_t)hs->n_placed;
  result->stop = hs->stop;
  result->fail_task = hs->fail_task;
  if (hs->stop == KB_STOP_NO_FIT)
    for (int b = 0; b < KB_NUM_REASONS; ++b) result->reason_hist[b] = hs->hist[b];
  for (int i = 0; i < hs->n_placed; ++i) {
    if (placed_node) placed_node[i] = ho[2 * i];
    if (placed_kind) placed_kind[i] = ho[2 * i + 1];
  }
  if (hs->panic) return fail(c, KB_E_PANIC, "SelectBestNode: no node scored above -1 (task %d)", hs->fail_task);
  return KB_OK;
}

// ---- node sharding across GPUs ----
static int shard_common(kb_ctx* c, const kb_shard* sh) {
  if (!c || !sh) return KB_E_INVALID;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (sh->world < 1 || sh->world > 16 || sh->rank < 0 || sh->rank >= sh->world || sh->n_total == 0 ||
      sh->n_total >= kMaxNodes || sh->node_begin >= sh->n_total)
    return fail(c, KB_E_INVALID, "bad shard (rank %d of %d, begin %u of %u)", sh->rank, sh->world, sh->node_begin,
                sh->n_total);
  if (c->nodes_ok) return fail(c, KB_E_STATE, "kb_set_shard comes before kb_upload_nodes");
  HIP_OK(c, hipSetDevice(c->device));
  if (!c->d_rec) {
    HIP_OK(c, hipMalloc((void**)&c->d_rec, sizeof(ShardRec)));
    HIP_OK(c, memset_sync(c->d_rec, 0, sizeof(ShardRec)));
  }
  if (c->d_rec_all) (void)hipFree(c->d_rec_all);
  c->d_rec_all = nullptr;
  HIP_OK(c, hipMalloc((void**)&c->d_rec_all, sizeof(ShardRec) * (size_t)sh->world));
  HIP_OK(c, memset_sync(c->d_rec_all, 0, sizeof(ShardRec) * (size_t)sh->world));
  c->shard = *sh;
  c->sharded = true;
  c->peer = false;  // (kb_set_shard_peer sets it after this)
  return KB_OK;
}

int kb_set_shard(kb_ctx* c, const kb_shard* sh, kb_allgather_fn fn, void* user) {
  if (!c) return KB_E_INVALID;
  if (!fn) return fail(c, KB_E_INVALID, "kb_set_shard needs an all-gather function");
  if (int rc = shard_common(c, sh)) return rc;
  if (c->h_rec) (void)hipHostFree(c->h_rec);
  c->h_rec = nullptr;
  HIP_OK(c, hipHostMalloc((void**)&c->h_rec, sizeof(ShardRec) * (size_t)(1 + sh->world), hipHostMallocDefault));
  c->ag_fn = fn;
  c->ag_user = user;
  return KB_OK;
}

// The node-sharded fed engine's exchange: this rank's inbox in its GPU's memory (uncached: peers write it over
// xGMI and the engine polls it), its IPC handle all-gathered through fn, the peers' inboxes opened. fn stays the
// host-staged exchange of jobs the engine does not run.
// The next epoch no node-sharded context of this process has used (every rank's contexts advance it alike).
static std::atomic<uint32_t> g_peer_epoch_next{0};
static void note_peer_epoch(uint32_t next) {
  uint32_t cur = g_peer_epoch_next.load();
  while (next > cur && !g_peer_epoch_next.compare_exchange_weak(cur, next)) {
  }
}

// The pre-flight round trip (include/kbgpu.h, kb_set_shard_peer). Inbox words [0, W): rank w's hello; [W, 2W): rank
// w's answer. A word is 0x5EED << 48 | kind << 40 | (sender << 8 | receiver) << 16 | this setup's nonce, so a word
// of an earlier setup in recycled memory never reads as current. Ends with every inbox zeroed and the ranks met.
static int shard_peer_preflight(kb_ctx* c, const kb_shard* sh, kb_allgather_fn fn, void* user, uint32_t start) {
  const int W = sh->world, me = sh->rank;
  uint64_t* own = (uint64_t*)c->inbox;
  uint64_t* got = nullptr;
  HIP_OK(c, hipMalloc((void**)&got, 2 * kShardMaxWorld * sizeof(uint64_t)));
  struct Free {
    uint64_t* p;
    ~Free() { (void)hipFree(p); }
  } free_got{got};
  const uint16_t nonce = (uint16_t)(0x9e37u * (start + 1u));  // (start: the same on every rank)
  const auto word = [&](int kind, int from, int to) {
    return (0x5EEDull << 48) | ((uint64_t)kind << 40) | ((uint64_t)((from << 8) | to) << 16) | nonce;
  };
  struct Outcome {
    int32_t ok, from, to, kind;
    uint64_t seen;
  };
  Outcome mine{1, -1, -1, 0, 0};
  std::vector<uint64_t> h(2 * (size_t)W);
  const auto meet = [&](const char* when) -> int {
    uint32_t tok = 1;
    std::vector<uint32_t> all((size_t)W);
    if (int rc = fn(user, &tok, all.data(), sizeof(tok)))
      return fail(c, KB_E_HIP, "all-gather callback failed (%d) %s", rc, when);
    return KB_OK;
  };
  const auto check = [&](int kind) -> int {  // this rank's inbox words of `kind`: every peer's, with its tag
    launch_peer_get(own, 2 * W, got, c->stream);
    HIP_OK(c, hipGetLastError());
    HIP_OK(c, hipMemcpyAsync(h.data(), got, 2 * W * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream));
    HIP_OK(c, hipStreamSynchronize(c->stream));
    for (int w = 0; w < W && mine.ok; ++w) {
      if (w == me) continue;
      const uint64_t x = h[(size_t)kind * W + w];
      if (x != word(kind, w, me)) mine = Outcome{0, w, me, kind, x};
      else c->stats.peer_checks++;
    }
    return KB_OK;
  };
  // 1. hello: this rank's word into every peer's inbox, over the path the engine's records take
  for (int w = 0; w < W; ++w)
    if (w != me)
      launch_peer_put((uint64_t*)c->peer_inbox[w] + me, word(0, me, w) ^ (c->test_peer_badtag ? 1ull << 47 : 0ull),
                      c->stream);
  HIP_OK(c, hipGetLastError());
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (int rc = meet("after the pre-flight hello")) return rc;
  if (int rc = check(0)) return rc;
  // 2. answer every peer whose hello arrived intact
  for (int w = 0; w < W && mine.ok; ++w)
    if (w != me) launch_peer_put((uint64_t*)c->peer_inbox[w] + W + me, word(1, me, w), c->stream);
  HIP_OK(c, hipGetLastError());
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (int rc = meet("after the pre-flight answers")) return rc;
  if (mine.ok)
    if (int rc = check(1)) return rc;
  // 3. every rank's outcome, so that all of them fail alike (a rank that saw nothing wrong names the first pair that
  //    failed elsewhere)
  std::vector<Outcome> all((size_t)W);
  if (int rc = fn(user, &mine, all.data(), sizeof(Outcome)))
    return fail(c, KB_E_HIP, "all-gather callback failed (%d) exchanging the pre-flight outcomes", rc);
  HIP_OK(c, memset_sync(c->inbox, 0, shard_inbox_bytes()));
  HIP_OK(c, hipDeviceSynchronize());
  if (int rc = meet("after the pre-flight")) return rc;  // no rank starts a cycle before every inbox is clean
  for (int w = 0; w < W; ++w)
    if (!all[w].ok) {
      const Outcome& o = all[w];
      return fail(c, KB_E_STATE,
                  "node-sharded pre-flight: rank %d read %s from rank %d as %016llx, wanted %016llx (the %s path "
                  "between these ranks' GPUs does not deliver the engine's words)", o.to,
                  o.kind ? "the answer" : "the hello", o.from, (unsigned long long)o.seen,
                  (unsigned long long)word(o.kind, o.from, o.to), o.kind ? "answer" : "hello");
    }
  return KB_OK;
}

int kb_set_shard_peer(kb_ctx* c, const kb_shard* sh, kb_allgather_fn fn, void* user) {
  if (int rc = kb_set_shard(c, sh, fn, user)) return rc;
  const size_t bytes = shard_inbox_bytes();
  if (!c->inbox) {
    if (hipExtMallocWithFlags(&c->inbox, bytes, hipDeviceMallocUncached) != hipSuccess) {
      (void)hipGetLastError();
      HIP_OK(c, hipMalloc(&c->inbox, bytes));
    }
  }
  HIP_OK(c, memset_sync(c->inbox, 0, bytes));
  HIP_OK(c, hipDeviceSynchronize());
  for (int w = 0; w < kShardMaxWorld; ++w) {
    if (c->peer_inbox[w] && c->peer_inbox[w] != c->inbox) (void)hipIpcCloseMemHandle(c->peer_inbox[w]);
    c->peer_inbox[w] = nullptr;
  }
  const int W = sh->world;
  // with the handle, each rank's next unused epoch in this process: the context starts past every rank's, so the
  // words an earlier context of these processes left in recycled inbox memory never carry a current tag
  struct PeerHello {
    hipIpcMemHandle_t h;
    uint32_t epoch, pad;
    char bus[32];  // the rank's GPU (PCI bus id): peers on another GPU are checked for peer access
  };
  std::vector<PeerHello> h((size_t)W + 1);
  memset(h.data(), 0, h.size() * sizeof(PeerHello));
  h[0].epoch = g_peer_epoch_next.load();
  uint32_t start = h[0].epoch;
  if (W > 1) {
    HIP_OK(c, hipIpcGetMemHandle(&h[0].h, c->inbox));
    HIP_OK(c, hipDeviceGetPCIBusId(h[0].bus, (int)sizeof(h[0].bus) - 1, c->device));
    if (int rc = fn(user, &h[0], &h[1], sizeof(PeerHello)))
      return fail(c, KB_E_HIP, "all-gather callback failed (%d) exchanging the inbox handles", rc);
    for (int w = 0; w < W; ++w) start = std::max(start, h[1 + w].epoch);
  }
  // Each rank opens every peer's inbox; a failure is recorded, not returned at once: every rank's outcome is
  // all-gathered below, so that every rank fails alike and names the same pair (a rank returning alone would leave
  // the others blocked in the next all-gather)
  struct OpenOutcome {
    int32_t ok, peer, code, pad;  // code: 1 the peer's GPU is not visible, 2 no peer path, 3 the IPC open failed
  };
  OpenOutcome mine{1, -1, 0, 0};
  for (int w = 0; w < W; ++w) {
    if (w == sh->rank) {
      c->peer_inbox[w] = c->inbox;
      continue;
    }
    if (!mine.ok) continue;
    if (strncmp(h[1 + w].bus, h[0].bus, sizeof(h[0].bus)) != 0) {  // another GPU: the xGMI path must be open
      int ord = -1, can = 0;
      if (hipDeviceGetByPCIBusId(&ord, h[1 + w].bus) != hipSuccess || ord < 0) {
        (void)hipGetLastError();
        mine = OpenOutcome{0, w, 1, 0};
        continue;
      }
      if (hipDeviceCanAccessPeer(&can, c->device, ord) != hipSuccess || !can) {
        (void)hipGetLastError();
        mine = OpenOutcome{0, w, 2, 0};
        continue;
      }
    }
    void* p = nullptr;
    if (hipIpcOpenMemHandle(&p, h[1 + w].h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
      (void)hipGetLastError();
      mine = OpenOutcome{0, w, 3, 0};
      continue;
    }
    c->peer_inbox[w] = p;
  }
  if (W > 1) {
    std::vector<OpenOutcome> all((size_t)W);
    if (int rc = fn(user, &mine, all.data(), sizeof(OpenOutcome)))
      return fail(c, KB_E_HIP, "all-gather callback failed (%d) exchanging the inbox opens", rc);
    for (int w = 0; w < W; ++w)
      if (!all[w].ok) {
        const int q = all[w].peer;
        const char* why = all[w].code == 1   ? "does not see the GPU of"
                          : all[w].code == 2 ? "has no peer path to the GPU of"
                                             : "could not open (hipIpcOpenMemHandle) the inbox of";
        return fail(c, KB_E_HIP, "node-sharded setup: rank %d (GPU %s) %s rank %d (GPU %s)", w,
                    w == sh->rank ? h[0].bus : h[1 + w].bus, why, q, q == sh->rank ? h[0].bus : h[1 + q].bus);
      }
  }
  if (W > 1)
    if (int rc = shard_peer_preflight(c, sh, fn, user, start)) return rc;
  c->peer = true;
  c->shard_epoch = c->shard_epoch0 ? c->shard_epoch0 : start;  // (an explicit start: the epoch-wrap tests)
  note_peer_epoch(c->shard_epoch + 1);
  return KB_OK;
}

// The inbox words carry kShardEpochBits of the cycle epoch (shard_tag): a word a cycle left behind -- a longer
// record, a no-fit histogram written only on NO_FIT -- would read as current again 2^kShardEpochBits cycles later in
// the same cycle half. So at every epoch that is a multiple of the wrap every rank zeroes its own inbox between two
// host barriers (the all-gather callback): the first passes once every rank's previous cycle has ended (no peer
// writes in flight), the second once every inbox is clean (no rank starts the cycle before).
static int shard_inbox_rezero(kb_ctx* c) {
  const int W = c->shard.world;
  std::vector<uint32_t> tok((size_t)W + 1, 0u);
  tok[0] = c->shard_epoch + 1;
  if (int rc = c->ag_fn(c->ag_user, tok.data(), tok.data() + 1, sizeof(uint32_t)))
    return fail(c, KB_E_HIP, "all-gather callback failed (%d) before the inbox re-zeroing", rc);
  for (int w = 0; w < W; ++w)
    if (tok[1 + w] != tok[0])
      return fail(c, KB_E_STATE, "node-sharded engine: rank %d is at epoch %u, this rank at %u", w, tok[1 + w], tok[0]);
  HIP_OK(c, memset_sync(c->inbox, 0, shard_inbox_bytes()));
  HIP_OK(c, hipDeviceSynchronize());
  if (int rc = c->ag_fn(c->ag_user, tok.data(), tok.data() + 1, sizeof(uint32_t)))
    return fail(c, KB_E_HIP, "all-gather callback failed (%d) after the inbox re-zeroing", rc);
  c->stats.shard_rezero++;
  return KB_OK;
}

int kb_comm_unique_id(uint8_t id[KB_COMM_ID_BYTES]) {
  if (!id) return KB_E_INVALID;
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return KB_E_HIP;
  memcpy(id, &u, sizeof(u) < KB_COMM_ID_BYTES ? sizeof(u) : KB_COMM_ID_BYTES);
  return KB_OK;
}

int kb_set_shard_rccl(kb_ctx* c, const kb_shard* sh, const uint8_t id[KB_COMM_ID_BYTES]) {
  if (!c) return KB_E_INVALID;
  if (!id) return fail(c, KB_E_INVALID, "missing RCCL id");
  if (int rc = shard_common(c, sh)) return rc;
  ncclUniqueId u;
  memcpy(&u, id, sizeof(u));
  ncclComm_t comm;
  const ncclResult_t r = ncclCommInitRank(&comm, sh->world, u, sh->rank);
  if (r != ncclSuccess) return fail(c, KB_E_HIP, "ncclCommInitRank: %s", ncclGetErrorString(r));
  if (c->comm) (void)ncclCommDestroy((ncclComm_t)c->comm);
  c->comm = comm;
  c->ag_fn = nullptr;
  return KB_OK;
}

// One job on a node-sharded table: per run segment, sweep + local proposal, one all-gather, merge + commit.
// Node-sharded job: per run segment, the sweep and this rank's proposal, the all-gather (RCCL on the library
// stream, or host-staged through the callback), the global merge + commit. Issued into job slot `si` like
// place_issue (`g` guards a speculative job's first segment: every rank sees the same previous job, so every
// rank skips alike, and the all-gather still runs); the host-staged exchange waits for the proposal here.
// This run's InterPodAffinity normalisation over the whole cluster (interpod_affinity.go:221-238: min / max
// count over every node): each rank's over its own rows, then min of the minima and max of the maxima.
static int shard_ipa_minmax(kb_ctx* c, int spec, const JobState* js) {
  int64_t* mm = c->P.A.mm;
  launch_ipa_minmax(c->N, c->P, nullptr, spec, 1, mm, js, c->stream);
  if (c->comm) {
    ncclResult_t r = ncclAllReduce(mm, mm, 1, ncclInt64, ncclMin, (ncclComm_t)c->comm, c->stream);
    if (r == ncclSuccess) r = ncclAllReduce(mm + 1, mm + 1, 1, ncclInt64, ncclMax, (ncclComm_t)c->comm, c->stream);
    if (r != ncclSuccess) return fail(c, KB_E_HIP, "ncclAllReduce: %s", ncclGetErrorString(r));
    return KB_OK;
  }
  const int W = c->shard.world;
  std::vector<int64_t> h(2 * (size_t)(W + 1));
  HIP_OK(c, hipMemcpyAsync(h.data(), mm, 16, hipMemcpyDeviceToHost, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (int rc = c->ag_fn(c->ag_user, h.data(), h.data() + 2, 16))
    return fail(c, KB_E_HIP, "all-gather callback failed (%d)", rc);
  int64_t mn = h[2], mx = h[3];
  for (int w = 1; w < W; ++w) {
    mn = std::min(mn, h[2 + 2 * w]);
    mx = std::max(mx, h[3 + 2 * w]);
  }
  h[0] = mn;
  h[1] = mx;
  HIP_OK(c, hipMemcpyAsync(mm, h.data(), 16, hipMemcpyHostToDevice, c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream));  // (h is pageable and local)
  return KB_OK;
}

static int shard_issue(kb_ctx* c, const kb_job_req* job, int si, const SpecGuard& g) {
  if (!c->sel_ok || !c->traj) return fail(c, KB_E_UNSUPPORTED, "sharded table does not fit the selection path");
  for (uint32_t i = 0; i < job->n_tasks; ++i) {
    const int s = job->task_specs[i];
    if (!c->spec_traj_ok[s]) return fail(c, KB_E_UNSUPPORTED, "spec %d needs a path that does not run sharded", s);
    if (c->spec_needs_aff[s] && (!c->aff_ok || c->spec_aff_err[s]))
      return fail(c, KB_E_UNSUPPORTED, "spec %d: inter-pod affinity error paths do not run sharded", s);
  }
  kb_ctx::JobSlot& S = c->slot[si];
  S.t_issue = std::chrono::steady_clock::now();
  S.ev_b = c->pending.size();
  c->timing_now = c->timing && (c->issue_count++ % c->timing_every == 0);
  memset(((JobState*)S.h)->diag, 0, sizeof(((JobState*)S.h)->diag));
  JobState* js = (JobState*)S.d;
  JobState* hjs_dev = (JobState*)S.hdev;
  int32_t* hout_dev = (int32_t*)(S.hdev + sizeof(JobState));
  const size_t rb = sizeof(ShardRec);
  bool listed = false;
  for (uint32_t t = 0; t < job->n_tasks;) {
    uint32_t e = t + 1;
    while (e < job->n_tasks && job->task_specs[e] == job->task_specs[t]) ++e;
    const int spec = job->task_specs[t];
    // inter-pod affinity: the count tables and histograms are replicated on every rank and every rank applies
    // every commit's increments (global node ids, whole-cluster topo_dom). A spec whose inputs stay put during
    // its run (or a cap-1 spec, whose key sequence stays closed-form) runs in segments as above, after a
    // whole-cluster min / max; a spec whose own commits move its inputs runs one task per segment.
    const bool aff = c->spec_needs_aff[spec];
    const bool per_task = aff && c->spec_dyn[spec] && !c->cap1(spec);
    const uint32_t seg_max = per_task ? 1u : (uint32_t)kShardSegMax;
    // a job of one single-segment run lists the rows it commits; when the previous job (the other slot) did,
    // this job's sweep runs on stream_b beside that job's kernels and the proposal re-keys those rows (as the
    // one-GPU selection path does, place_issue)
    const bool one_run = !aff && t == 0 && e == job->n_tasks && e - t <= (uint32_t)kShardSegMax;
    const bool ov = one_run && c->stream_b && c->prev_listed && c->prev_slot == (si ^ 1);
    uint32_t* kt = one_run ? c->sel_keys[si] : c->traj;
    uint64_t* st = one_run ? c->sel_stat[si] : c->stat;
    for (uint32_t seg = t; seg < e; seg += seg_max) {
      const int T = (int)std::min<uint32_t>(seg_max, e - seg);
      const int first = seg == 0;
      const SpecGuard gr = first ? g : SpecGuard{nullptr, 0, 0, 0};
      hipEvent_t ea;
      if (aff && c->spec_hist[spec]) {
        c->ev_begin(&ea);
        if (int rc = shard_ipa_minmax(c, spec, first ? nullptr : js)) return rc;
        c->ev_end(ea, KB_KERNEL_IPA_MINMAX, (uint64_t)c->N.n);
      }
      if (ov) {
        c->ev_begin(&ea, c->stream_b);
        launch_sel_sweep(c->N, c->P, c->cfg, spec, c->idx_bits, kt, st, nullptr, false, c->stream_b,
                         SpecGuard{nullptr, 0, 0, 0}, c->sweep_ctr + si);
        c->ev_end(ea, KB_KERNEL_SEL_SWEEP, (uint64_t)c->N.n, c->stream_b);
        c->sweep_target[si] += (uint32_t)((c->N.n + 63) / 64);
        c->n_overlap++;
        c->stats.sweep_overlap++;
      } else {
        c->ev_begin(&ea);
        launch_sel_sweep(c->N, c->P, c->cfg, spec, c->idx_bits, kt, st, first ? nullptr : js, aff, c->stream, gr);
        c->ev_end(ea, KB_KERNEL_SEL_SWEEP, (uint64_t)c->N.n);
      }
      // the segment's identity, compared across ranks after the exchange (ShardRec::tag)
      const uint32_t gh = gr.prev ? (uint32_t)(0x40000000u ^ ((uint32_t)gr.stop * 0x9e3779b1u) ^
                                               ((uint32_t)gr.placed * 0x85ebca77u) ^ ((uint32_t)gr.ready * 0xc2b2ae3du))
                                  : 0u;
      const uint32_t tag[4] = {c->seq + 1, (uint32_t)spec, (seg << 16) | (uint32_t)T, gh & 0x7fffffffu};
      c->ev_begin(&ea);
      launch_shard_propose(c->N, c->P, c->cfg, spec, T, c->idx_bits, kt, st, js, first, c->d_rec, gr,
                           ov ? c->commits[si ^ 1] : nullptr, ov ? (const JobState*)c->slot[si ^ 1].d : nullptr,
                           ov ? c->sweep_ctr + si : nullptr, c->sweep_target[si], hjs_dev, c->stream, tag);
      c->ev_end(ea, KB_KERNEL_SHARD_PROPOSE, 0);
      c->ev_begin(&ea);
      if (c->comm) {
        const ncclResult_t r = ncclAllGather(c->d_rec, c->d_rec_all, rb, ncclUint8, (ncclComm_t)c->comm, c->stream);
        if (r != ncclSuccess) return fail(c, KB_E_HIP, "ncclAllGather: %s", ncclGetErrorString(r));
      } else {  // host-staged: every rank calls the exchange for every segment, stopped or not
        HIP_OK(c, hipMemcpyAsync(c->h_rec, c->d_rec, rb, hipMemcpyDeviceToHost, c->stream));
        HIP_OK(c, hipStreamSynchronize(c->stream));
        if (int rc = c->ag_fn(c->ag_user, c->h_rec, c->h_rec + 1, rb))
          return fail(c, KB_E_HIP, "all-gather callback failed (%d)", rc);
        HIP_OK(c, hipMemcpyAsync(c->d_rec_all, c->h_rec + 1, rb * (size_t)c->shard.world, hipMemcpyHostToDevice,
                                 c->stream));
      }
      c->ev_end(ea, KB_KERNEL_SHARD_EXCHANGE, 0);
      c->ev_begin(&ea);
      launch_shard_commit(c->N, c->P, c->cfg, spec, (int)seg, T, c->idx_bits, c->d_rec_all, c->shard.world, js,
                          first, job->ready_num, job->min_available, job->gang_ready, hout_dev, hjs_dev, ++c->seq, gr,
                          one_run ? c->commits[si] : nullptr, c->stream);
      c->ev_end(ea, KB_KERNEL_SHARD_COMMIT, 0);
      if (aff && c->spec_incr[spec])  // every rank: the segment's placements (global ids) into the tables
        launch_aff_commit(c->P, spec, (int)seg, T, js, hout_dev, c->N.base, c->stream);
    }
    listed = one_run;
    t = e;
  }
  HIP_OK(c, hipGetLastError());
  c->prev_listed = listed;
  c->prev_slot = si;
  S.seq = c->seq;
  S.ev_e = c->pending.size();
  S.busy = true;
  S.issue_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - S.t_issue).count();
  return KB_OK;
}

static int validate_job(kb_ctx* c, const kb_job_req* job) {
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs first");
  for (uint32_t i = 0; i < job->n_tasks; ++i) {
    if (job->task_specs[i] < 0 || job->task_specs[i] >= c->P.m)
      return fail(c, KB_E_INVALID, "task %u spec %d out of range", i, job->task_specs[i]);
    if (c->spec_needs_aff[job->task_specs[i]] && !c->aff_ok)
      return fail(c, KB_E_UNSUPPORTED, "spec %d has pod (anti)affinity: upload the affinity tables first",
                  job->task_specs[i]);
  }
  return KB_OK;
}

// Per-slot selection buffers (level-0 keys, static cache, commit list), the sweep stream and its events.
static int ensure_sel_bufs(kb_ctx* c) {
  if (c->sel_n != c->N.n) {
    for (int s = 0; s < kJobSlots; ++s) {
      if (c->sel_keys[s]) (void)hipFree(c->sel_keys[s]);
      if (c->sel_stat[s]) (void)hipFree(c->sel_stat[s]);
      if (c->sel_lvl[s]) (void)hipFree(c->sel_lvl[s]);
      c->sel_keys[s] = nullptr;
      c->sel_stat[s] = nullptr;
      c->sel_lvl[s] = nullptr;
    }
    c->sel_n = -1;
    const size_t n = (size_t)std::max(c->N.n, 1);
    for (int s = 0; s < kJobSlots; ++s) {
      HIP_OK(c, hipMalloc((void**)&c->sel_keys[s], n * 4));
      HIP_OK(c, hipMalloc((void**)&c->sel_stat[s], n * 8));
    }
    c->sel_n = c->N.n;
    c->prev_listed = false;
  }
  if (c->commits_cap < c->job_cap) {
    for (int s = 0; s < kJobSlots; ++s) {
      if (c->commits[s]) (void)hipFree(c->commits[s]);
      c->commits[s] = nullptr;
    }
    c->commits_cap = 0;
    for (int s = 0; s < kJobSlots; ++s) HIP_OK(c, hipMalloc((void**)&c->commits[s], (size_t)c->job_cap * 4));
    c->commits_cap = c->job_cap;
    c->prev_listed = false;
  }
  if (!c->stream_b) {
    HIP_OK(c, hipMalloc((void**)&c->sweep_ctr, 2 * sizeof(uint32_t)));
    HIP_OK(c, memset_sync(c->sweep_ctr, 0, 2 * sizeof(uint32_t)));
    c->sweep_target[0] = c->sweep_target[1] = 0;
    if (c->fed_dedicated) {  // a hardware queue of its own (kb_ctx::fed_dedicated): a mask of every CU
      hipDeviceProp_t prop;
      HIP_OK(c, hipGetDeviceProperties(&prop, c->device));
      const int cus = std::max(prop.multiProcessorCount, 1);
      std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
      if (cus % 32) mask.back() = (1u << (cus % 32)) - 1;
      HIP_OK(c, hipExtStreamCreateWithCUMask(&c->stream_b, (uint32_t)mask.size(), mask.data()));
    } else {
      HIP_OK(c, hipStreamCreateWithFlags(&c->stream_b, hipStreamNonBlocking));
    }
  }
  return KB_OK;
}

// Every job slot with room for n_tasks placements (slot 0 = d_job / h_job; all: slots 1.. as well).
static int ensure_slots(kb_ctx* c, uint32_t n_tasks, bool all) {
  if (int rc = ensure_job_buffers(c, n_tasks)) return rc;
  if (int rc = ensure_sel_bufs(c)) return rc;
  c->slot[0].d = c->d_job;
  c->slot[0].h = c->h_job;
  c->slot[0].hdev = c->h_job_dev;
  if (!all) return KB_OK;
  for (int s = 1; s < kJobSlots; ++s) {
    if (!c->d_jobx[s]) {
      void* p;
      HIP_OK(c, hipMalloc(&p, sizeof(JobState)));
      HIP_OK(c, memset_sync(p, 0, sizeof(JobState)));
      c->work_mem.push_back(p);
      c->d_jobx[s] = (char*)p;
    }
    if (!c->h_jobx[s] || c->jobx_cap[s] < c->job_cap) {
      if (c->h_jobx[s]) (void)hipHostFree(c->h_jobx[s]);
      c->h_jobx[s] = nullptr;
      const size_t bytes = sizeof(JobState) + (size_t)c->job_cap * 2 * sizeof(int32_t);
      HIP_OK(c, hipHostMalloc((void**)&c->h_jobx[s], bytes, hipHostMallocMapped | hipHostMallocCoherent));
      HIP_OK(c, hipHostGetDevicePointer((void**)&c->slot[s].hdev, c->h_jobx[s], 0));
      memset(c->h_jobx[s], 0, bytes);
      ((JobState*)c->h_jobx[s])->seq = c->seq;
      c->jobx_cap[s] = c->job_cap;
    }
    c->slot[s].d = c->d_jobx[s];
    c->slot[s].h = c->h_jobx[s];
  }
  return KB_OK;
}

// the smallest capacity over the pipelined driver's slots
static uint32_t slots_cap(const kb_ctx* c) {
  uint32_t cap = c->job_cap;
  for (int s = 1; s < kJobSlots; ++s) cap = std::min(cap, c->jobx_cap[s]);
  return cap;
}

// The commits of a run of spec a leave every input of a sweep of spec b as it was (the affinity tables b's checks
// and histograms read are not among those a's commits write), so b's sweep may overlap a's place kernel.
static bool aff_sweep_indep(const kb_ctx* c, int a, int b) {
  if (a < 0 || b < 0 || (size_t)a >= c->aff_wr.size() || (size_t)b >= c->aff_rd.size()) return a < 0;
  const auto& w = c->aff_wr[a];
  const auto& r = c->aff_rd[b];
  size_t i = 0, j = 0;
  while (i < w.size() && j < r.size()) {
    if (w[i] == r[j]) return false;
    if (w[i] < r[j]) ++i;
    else ++j;
  }
  return true;
}

// A self-dependent spec the class loop takes (classify_self_dynamic; its LDS plan fits).
static bool cls_run_ok(const kb_ctx* c, int spec) {
  const int F = c->cls_slot(spec);
  return F >= 0 && c->aff_ok && !c->spec_ipa_err[spec] && (size_t)F < c->cls_coff.size() && c->cls_coff[F] &&
         cls_fits(c->N.n, (int)c->aff_slot_D[F] + 1);
}

// Launch every run of the job into slot `si`. The path per run: block-wide re-sweep (self-dependent
// affinity), selection, trajectory, or rekey. `g` (first run only) guards a speculative job.
static int place_issue(kb_ctx* c, const kb_job_req* job, int si, const SpecGuard& g) {
  kb_ctx::JobSlot& S = c->slot[si];
  S.t_issue = std::chrono::steady_clock::now();
  S.ev_b = c->pending.size();
  c->timing_now = c->timing && (c->issue_count++ % c->timing_every == 0);
  JobState* js = (JobState*)S.d;
  JobState* hjs_dev = (JobState*)S.hdev;
  memset(((JobState*)S.h)->diag, 0, sizeof(((JobState*)S.h)->diag));
  int32_t* hout_dev = (int32_t*)(S.hdev + sizeof(JobState));
  bool listed = false;
  int run_spec = -1;
  // the job two back (this slot's last one) may have left an affinity-table commit queued behind its publish
  const int tail_spec = S.aff_tail_spec;
  S.aff_tail_spec = -1;
  uint32_t t = 0;
  while (t < job->n_tasks) {
    uint32_t e = t + 1;
    while (e < job->n_tasks && job->task_specs[e] == job->task_specs[t]) ++e;
    const int spec = job->task_specs[t];
    const int first = t == 0;
    hipEvent_t ea;
    int pbc;
    const int run = (int)(e - t);
    const bool aff = c->aff_ok && c->spec_needs_aff[spec];
    const bool key32 = c->spec_traj_ok[spec] && c->traj != nullptr;
    const bool sel_fits = c->use_sel && key32 && c->sel_ok;
    // self-dependent specs: cap-1 ones run as selection runs, the rest take a per-task loop
    const bool dyn = aff && c->spec_dyn[spec] && !(sel_fits && c->cap1(spec));
    const bool sel = !dyn && sel_fits;
    const bool traj = !sel && !dyn && c->use_traj && key32 && c->traj_full && traj_lds_bytes(c->N.n, run, &pbc) > 0;
    const bool cls = dyn && cls_run_ok(c, spec);
    // the selection kernel applies the run's affinity table commits itself when its placements fit LDS
    const bool sel_pl = sel && aff && c->spec_incr[spec] && sel_aff_pl_fits(c->N.n, (int)run);
    if (first && g.prev && !sel && !cls)
      return fail(c, KB_E_INVALID, "guarded job takes neither the selection path nor the class loop");
    const SpecGuard gr = first ? g : SpecGuard{nullptr, 0, 0, 0};
    if (!dyn && c->aff_ok && c->spec_hist[spec]) {  // this run's InterPodAffinity normalisation
      c->ev_begin(&ea);
      launch_ipa_minmax(c->N, c->P, nullptr, spec, 1, c->P.A.mm, first ? nullptr : js, c->stream);
      c->ev_end(ea, KB_KERNEL_IPA_MINMAX, (uint64_t)c->N.n);
    }
    if (cls) {
      const int cls_F = c->cls_slot(spec);
      c->ev_begin(&ea);
      launch_cls_place(c->N, c->P, c->cfg, spec, cls_F, (int)c->aff_slot_D[cls_F] + 1, (int)t, run, c->keys, c->stat,
                       c->cls_lvl, c->cls_amax, c->cls_coff[cls_F], c->cls_mem[cls_F], c->cls_cbest, js, first,
                       job->ready_num, job->min_available, job->gang_ready, hout_dev, hjs_dev, ++c->seq, gr,
                       c->stream);
      c->ev_end(ea, KB_KERNEL_CLS_PLACE, 0);
      c->stats.cls_runs++;
    } else if (dyn) {
      c->ev_begin(&ea);
      if (c->use_aff_reg && c->spec_aff_reg[spec] && aff_reg_fits(c->N.n, c->spec_aff_reg[spec]) &&
          !((size_t)spec < c->ov_slot.size() && c->ov_slot[spec] >= 0))
        launch_aff_reg(c->N, c->P, c->cfg, spec, c->spec_aff_reg[spec], (int)t, run, c->stat, js, first, job->ready_num,
                       job->min_available, job->gang_ready, hout_dev, hjs_dev, ++c->seq, c->stream);
      else
        launch_aff_place(c->N, c->P, c->cfg, spec, (int)t, run, c->keys, c->stat, js, first, job->ready_num,
                         job->min_available, job->gang_ready, hout_dev, hjs_dev, ++c->seq, c->stream);
      c->ev_end(ea, KB_KERNEL_AFF_PLACE, 0);
    } else if (sel) {  // level-0 keys of every node, then the run as one top-T selection
      if (aff && c->spec_dyn[spec]) c->stats.cap1_runs++;
      uint32_t* kt = c->sel_keys[si];
      uint64_t* st = c->sel_stat[si];
      // A job that is one run (without InterPodAffinity histograms -- their normalisation is a pass of its own
      // before the sweep -- and applying its own table commits before it publishes) lists the rows it commits. When the previous job (the other slot) did, and its
      // commits leave this spec's affinity inputs alone (aff_sweep_indep: the tables its checks and histograms
      // read), this run's level-0 sweep goes to stream_b right after the job before that one, overlapping the
      // previous job's place kernel, and the place kernel re-keys that job's rows.
      const bool one_run = !(aff && (c->spec_hist[spec] || (c->spec_incr[spec] && !sel_pl))) && t == 0 &&
                           e == job->n_tasks;
      // With affinity the sweep reads count tables and histograms: neither the previous job's commits (listed, so
      // applied before it published) nor an aff_commit_kernel the job two back queued after its publish may write
      // what this sweep reads (the latter runs on `stream`, which the overlapped sweep does not wait for).
      const bool ov_ok = one_run && c->stream_b && c->prev_listed && c->prev_slot == (si ^ 1);
      const bool ov = ov_ok && (!aff || (aff_sweep_indep(c, c->prev_run_spec, spec) &&
                                         aff_sweep_indep(c, tail_spec, spec)));
      if (ov_ok && !ov) c->stats.overlap_refused_tables++;
      if (ov) {
        c->ev_begin(&ea, c->stream_b);
        launch_sel_sweep(c->N, c->P, c->cfg, spec, c->idx_bits, kt, st, nullptr, aff, c->stream_b,
                         SpecGuard{nullptr, 0, 0, 0}, c->sweep_ctr + si);
        c->ev_end(ea, KB_KERNEL_SEL_SWEEP, (uint64_t)c->N.n, c->stream_b);
        c->sweep_target[si] += (uint32_t)((c->N.n + 63) / 64);
        c->n_overlap++;
        c->stats.sweep_overlap++;
      } else {
        c->ev_begin(&ea);
        launch_sel_sweep(c->N, c->P, c->cfg, spec, c->idx_bits, kt, st, first ? nullptr : js, aff, c->stream, gr);
        c->ev_end(ea, KB_KERNEL_SEL_SWEEP, (uint64_t)c->N.n);
      }
      c->ev_begin(&ea);
      launch_sel_place(c->N, c->P, c->cfg, spec, (int)t, run, c->idx_bits, kt, st, js, first, job->ready_num,
                       job->min_available, job->gang_ready, hout_dev, hjs_dev, ++c->seq, c->stream, gr,
                       one_run ? c->commits[si] : nullptr, ov ? c->commits[si ^ 1] : nullptr,
                       ov ? (const JobState*)c->slot[si ^ 1].d : nullptr, ov ? c->sweep_ctr + si : nullptr,
                       c->sweep_target[si], sel_pl ? 1 : 0);
      c->ev_end(ea, KB_KERNEL_SEL_PLACE, 0);
      listed = one_run;
      run_spec = spec;
    } else if (traj) {
      const int J = std::min(run, kTrajDefaultJ);
      c->ev_begin(&ea);
      launch_traj_sweep(c->N, c->P, c->cfg, spec, J, c->idx_bits, c->traj, c->cmax32, c->amax, c->stat,
                        first ? nullptr : js, aff, c->stream);
      c->ev_end(ea, KB_KERNEL_TRAJ_SWEEP, (uint64_t)c->N.n);
      c->ev_begin(&ea);
      launch_traj_place(c->N, c->P, c->cfg, spec, (int)t, run, J, c->idx_bits, c->traj, c->cmax32, c->amax,
                        c->stat, js, first, job->ready_num, job->min_available, job->gang_ready, hout_dev, hjs_dev,
                        ++c->seq, c->stream);
      c->ev_end(ea, KB_KERNEL_TRAJ_PLACE, 0);
    } else {
      c->ev_begin(&ea);
      launch_sweep_keys(c->N, c->P, c->cfg, spec, c->keys, c->cmax, c->stat, first ? nullptr : js, aff, c->stream);
      c->ev_end(ea, KB_KERNEL_SWEEP, (uint64_t)c->N.n);
      c->ev_begin(&ea);
      launch_place_loop(c->N, c->P, c->cfg, spec, (int)t, run, c->keys, c->cmax, c->stat, js, first,
                        job->ready_num, job->min_available, job->gang_ready, hout_dev, hjs_dev, ++c->seq,
                        c->stream);
      c->ev_end(ea, KB_KERNEL_PLACE, 0);  // pairs filled in from the placements below
    }
    // this run's commits update the affinity tables (the class loop and the per-task loops apply them themselves,
    // and so does the selection kernel when sel_pl)
    if (aff && !dyn && !sel_pl && c->spec_incr[spec]) {
      launch_aff_commit(c->P, spec, (int)t, run, js, hout_dev, 0, c->stream);
      S.aff_tail_spec = spec;  // (a later run's place kernel, in stream order after it, clears the hazard)
    } else {
      S.aff_tail_spec = -1;
    }
    t = e;
  }
  HIP_OK(c, hipGetLastError());
  c->prev_listed = listed;
  c->prev_run_spec = listed ? run_spec : -1;
  c->prev_slot = si;
  S.seq = c->seq;
  S.ev_e = c->pending.size();
  S.busy = true;
  S.issue_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - S.t_issue).count();
  return KB_OK;
}

static int place_finish(kb_ctx* c, int si, int32_t* placed_node, int32_t* placed_kind, kb_job_result* result,
                        bool skipped) {
  kb_ctx::JobSlot& S = c->slot[si];
  if (!S.busy) return fail(c, KB_E_STATE, "job slot %d has nothing in flight", si);
  S.busy = false;
  const JobState* hs = (const JobState*)S.h;
  const auto t_wait = std::chrono::steady_clock::now();
  if (int rc = wait_seq(c, hs, S.seq)) return rc;
  if (c->fed && c->fed_diag) {
    c->dg_fin0.push_back((t_wait - c->dg_t0).count());
    c->dg_fin1.push_back((std::chrono::steady_clock::now() - c->dg_t0).count());
  }
  // host time spent in the device path for this job: issuing it plus waiting for it (jobs overlap when
  // pipelined, so issue-to-finish walls would count the overlap twice)
  const double wall =
      S.issue_ms + std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_wait).count();
  if (c->issue_trace && c->fed)
    fprintf(stderr, "kb_finish rank=%d seq=%u slot=%d skipped=%d placed=%d stop=%d ready=%d stopped=%d\n",
            c->sharded ? c->shard.rank : 0, S.seq, si, skipped ? 1 : 0, hs->n_placed, hs->stop, hs->ready_num,
            hs->stopped);
  if (hs->stall == 2)
    return fail(c, KB_E_STATE, "node-sharded ranks exchanged different segments (their drivers diverged)");
  if (hs->stall)
    return fail(c, KB_E_HIP, "place kernel gave up waiting for its overlapped level-0 sweep");
  if (skipped) {  // a speculative job whose guard failed: nothing ran, nothing to count
    for (size_t k = S.ev_b; k < S.ev_e && k < c->pending.size(); ++k) c->pending[k].kind = -1;
    return KB_OK;
  }
  c->device_ms += wall;
  c->stats.device_ms += wall;
  c->stats.job_calls += 1;
  for (int k = 0; k < 8; ++k) c->stats.diag[k] += hs->diag[k];
  if (c->fed) c->fed_tasks += (uint64_t)hs->n_placed + (hs->stop == KB_STOP_NO_FIT ? 1 : 0);
  if (c->timing) {
    // a place launch covers (tasks it placed or tried) x n pairs; attribute them to the job's launches
    uint64_t tasks = (uint64_t)hs->n_placed + (hs->stop == KB_STOP_NO_FIT ? 1 : 0);
    for (size_t k = S.ev_b; k < S.ev_e && k < c->pending.size(); ++k) {
      auto& p = c->pending[k];
      if (p.kind == KB_KERNEL_PLACE || p.kind == KB_KERNEL_TRAJ_PLACE || p.kind == KB_KERNEL_AFF_PLACE ||
          p.kind == KB_KERNEL_SEL_PLACE || p.kind == KB_KERNEL_CLS_PLACE || p.kind == KB_KERNEL_SHARD_PROPOSE) {
        p.pairs = tasks * (uint64_t)c->N.n;
        tasks = 0;
      }
    }
    c->ev_collect(false, S.ev_e);  // never a later job's pairs, whose counts are not known yet
  }
  const int32_t* ho = (const int32_t*)(S.h + sizeof(JobState));
  result->n_placed = (uint32_t)hs->n_placed;
  result->stop = hs->stop;
  result->fail_task = hs->fail_task;
  if (hs->stop == KB_STOP_NO_FIT)
    for (int b = 0; b < KB_NUM_REASONS; ++b) result->reason_hist[b] = hs->hist[b];
  for (int i = 0; i < hs->n_placed; ++i) {
    if (placed_node) placed_node[i] = ho[2 * i];
    if (placed_kind) placed_kind[i] = ho[2 * i + 1];
  }
  if (hs->panic) return fail(c, KB_E_PANIC, "SelectBestNode: no node scored above -1 (task %d)", hs->fail_task);
  return KB_OK;
}

int kb_place_job(kb_ctx* c, const kb_job_req* job, int32_t* placed_node, int32_t* placed_kind,
                 kb_job_result* result) {
  if (!c || !job || !result) return KB_E_INVALID;
  memset(result, 0, sizeof(*result));
  result->fail_task = -1;
  if (int rc = validate_job(c, job)) return rc;
  if (job->n_tasks == 0) return KB_OK;
  c->prev_listed = false;
  if (c->sharded) {
    if (c->any_busy()) return fail(c, KB_E_STATE, "a pipelined job is still in flight");
    if (int rc = ensure_slots(c, job->n_tasks, false)) return rc;
    if (int rc = shard_issue(c, job, 0, SpecGuard{nullptr, 0, 0, 0})) return rc;
    return place_finish(c, 0, placed_node, placed_kind, result, false);
  }
  if (engine_ok(c, job)) return engine_place_job(c, job, placed_node, placed_kind, result);
  if (int rc = kb_engine_stop(c)) return rc;
  if (c->any_busy()) return fail(c, KB_E_STATE, "a pipelined job is still in flight");
  if (int rc = ensure_slots(c, job->n_tasks, false)) return rc;
  if (int rc = place_issue(c, job, 0, SpecGuard{nullptr, 0, 0, 0})) return rc;
  return place_finish(c, 0, placed_node, placed_kind, result, false);
}

// Sharded contexts pipeline with the RCCL exchange only (a host-staged exchange waits for the proposal).
// (kb_set_shard_peer: the fed engine's cycles only; kb_allocate's driver drops pipelining for the others)
int kb_job_pipeline_ok(kb_ctx* c) {
  return c && (!c->sharded || c->comm || c->peer) && !c->use_engine && !c->broken;
}

int kb_job_guardable(kb_ctx* c, const kb_job_req* job) {
  if (c->fed) return job->n_tasks > 0 && kb_spec_fed_ok(c, job->task_specs[0]);  // the engine's own guard
  if (!c->use_sel || !c->sel_ok || !c->traj || job->n_tasks == 0) return 0;
  const int s0 = job->task_specs[0];
  if (s0 < 0 || s0 >= c->P.m || !c->spec_traj_ok[s0]) return 0;
  if (c->aff_ok && c->spec_needs_aff[s0] && c->spec_dyn[s0] && !c->cap1(s0) && !cls_run_ok(c, s0)) return 0;
  if (c->sharded && c->spec_needs_aff[s0]) return 0;  // sharded affinity runs issue serially
  return 1;
}

int kb_job_reserve(kb_ctx* c, uint32_t max_tasks) {
  if (!c) return KB_E_INVALID;
  if (c->any_busy()) return fail(c, KB_E_STATE, "a pipelined job is still in flight");
  return ensure_slots(c, std::max<uint32_t>(max_tasks, 1), true);
}

// A spec with inter-pod terms on the resident engine (kb_spec_fed_ok): one selection run whose own commits leave its
// affinity inputs alone (or the cap-1 closed form, traj_key64), on the split engine with resident sweepers (which fold
// the terms into the static cache with the spec's prepared min / max: fed_sweeper), one GPU. Its table commits are the
// placer's (fed_engine_kernel, before the job's publish).
static bool fed_aff_ok(const kb_ctx* c, int spec, bool need_mm) {
  if (!c->use_fed_aff || !c->use_fed_split || !fed_split_ok(c->N.n, c->sharded)) return false;
  // node-sharded: the peer engine (replicated tables: every rank commits every placement's increments); a spec with
  // histograms needs the whole-cluster min / max, reduced through the host all-gather (kb_fed_ipa_prepare)
  if (c->sharded && (!c->peer || (c->spec_hist[spec] && !c->ag_fn))) return false;
  if (c->fed_coop || c->fed_xcc < 0 || c->fed_xcc >= 8 || c->fed_kernel_sweeps) return false;  // (fed_sweepers_now)
  if (c->spec_dyn[spec] && !c->cap1(spec)) return false;
  if (c->spec_aff_err[spec] || c->spec_ipa_err[spec]) return false;
  if (need_mm && c->spec_hist[spec] && !((size_t)spec < c->mm_spec_ok.size() && c->mm_spec_ok[spec])) return false;
  return true;
}

static int spec_fed_ok_impl(kb_ctx* c, int spec, bool need_mm) {
  if (!c || spec < 0 || spec >= c->P.m) return 0;
  if ((c->sharded && !c->peer) || c->use_engine || !c->use_sel || !c->spec_traj_ok[spec]) return 0;
  if (c->sharded && !(c->use_fed_split && fed_split_ok(c->N.n, c->sharded))) return 0;  // the sharded engine is the split one
  const int ns = fed_nsel(c->N.n);  // past one workgroup's key plan: range selectors (split engine only)
  if (ns == 0 || (ns > 1 && !c->use_fed_split)) return 0;
  if (ns == 1 && (!c->sel_ok || !c->traj)) return 0;
  if (c->aff_ok && c->spec_needs_aff[spec] && !fed_aff_ok(c, spec, need_mm)) return 0;
  if (c->host_reasons(spec)) return 0;  // its NO_FIT needs a mid-cycle kb_node_reasons (not beside the engine)
  return c->use_fed ? 1 : 0;
}

int kb_spec_fed_ok(kb_ctx* c, int spec) { return spec_fed_ok_impl(c, spec, true); }
int kb_spec_fed_ok_pre(kb_ctx* c, int spec) { return spec_fed_ok_impl(c, spec, false); }

int kb_fed_ipa_prepare(kb_ctx* c, const int32_t* specs, uint32_t n) {
  if (!c) return KB_E_INVALID;
  if (!c->aff_ok || n == 0) return KB_OK;
  if (c->fed || c->fed_paused) return fail(c, KB_E_STATE, "kb_fed_ipa_prepare: the engine is running");
  for (uint32_t i = 0; i < n; ++i)
    if (specs[i] < 0 || specs[i] >= c->P.m) return fail(c, KB_E_INVALID, "kb_fed_ipa_prepare: spec %d", specs[i]);
  if (n > c->mm_ids_cap) return fail(c, KB_E_INVALID, "kb_fed_ipa_prepare: %u specs, %u uploaded", n, c->mm_ids_cap);
  HIP_OK(c, hipMemcpyAsync(c->d_mm_ids, specs, (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, c->stream));
  hipEvent_t ea;
  c->ev_begin(&ea);
  launch_ipa_minmax(c->N, c->P, c->d_mm_ids, 0, (int)n, c->P.A.mm_spec, nullptr, c->stream, 1);
  c->ev_end(ea, KB_KERNEL_IPA_MINMAX, (uint64_t)c->N.n * n);
  HIP_OK(c, hipGetLastError());
  // (the engine's launch queues behind it on `stream`; the copy's host buffer is read before the call returns)
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (c->sharded) {  // each rank's min / max over its own rows, then the min of the minima and the max of the maxima
    if (!c->ag_fn) return fail(c, KB_E_STATE, "kb_fed_ipa_prepare: node-sharded without the host all-gather");
    const int W = c->shard.world;
    const size_t m2 = 2 * (size_t)std::max(c->P.m, 1);
    std::vector<int64_t> all(m2), mine(2 * (size_t)n), got(2 * (size_t)n * W);
    HIP_OK(c, hipMemcpy(all.data(), c->P.A.mm_spec, m2 * sizeof(int64_t), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) {
      mine[2 * i] = all[2 * (size_t)specs[i]];
      mine[2 * i + 1] = all[2 * (size_t)specs[i] + 1];
    }
    if (int rc = c->ag_fn(c->ag_user, mine.data(), got.data(), mine.size() * sizeof(int64_t)))
      return fail(c, KB_E_HIP, "all-gather callback failed (%d)", rc);
    for (uint32_t i = 0; i < n; ++i) {
      int64_t mn = got[2 * i], mx = got[2 * i + 1];
      for (int w = 1; w < W; ++w) {
        mn = std::min(mn, got[2 * ((size_t)w * n + i)]);
        mx = std::max(mx, got[2 * ((size_t)w * n + i) + 1]);
      }
      all[2 * (size_t)specs[i]] = mn;
      all[2 * (size_t)specs[i] + 1] = mx;
    }
    HIP_OK(c, hipMemcpy(c->P.A.mm_spec, all.data(), m2 * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  if (c->mm_spec_ok.size() < (size_t)c->P.m) c->mm_spec_ok.resize(c->P.m, 0);
  for (uint32_t i = 0; i < n; ++i) c->mm_spec_ok[specs[i]] = 1;
  return KB_OK;
}

int kb_fed_units_indep(const kb_ctx* c, int a, int b) {
  if (!c->aff_ok || a < 0 || b < 0) return 1;
  if ((size_t)b >= c->aff_rd.size() || c->aff_rd[b].empty()) return 1;  // b's sweep reads no table
  if ((size_t)a >= c->aff_wr.size() || c->aff_wr[a].empty()) return 1;  // a's commits write none
  return aff_sweep_indep(c, a, b) ? 1 : 0;
}

uint32_t kb_fed_unit_cap(kb_ctx* c) {
  return c && c->use_fed_split && fed_split_ok(c->N.n, c->sharded) ? (uint32_t)kFedSplitMaxTasks : 0u;
}

int kb_fed_cycle_ok(kb_ctx* c, uint32_t max_job_tasks) {
  if (!c) return 0;
  if (c->sharded && !(c->peer && c->use_fed_split && fed_split_ok(c->N.n, c->sharded) &&
                      max_job_tasks <= (uint32_t)kFedSplitMaxTasks))
    return 0;
  const int ns = fed_nsel(c->N.n);
  return ns == 1 || (ns > 1 && c->use_fed_split && fed_split_ok(c->N.n, c->sharded) && max_job_tasks <= (uint32_t)kFedSplitMaxTasks);
}

int kb_fed_begin(kb_ctx* c, uint32_t max_job_tasks) {
  if (!c) return KB_E_INVALID;
  if (c->fed) return fail(c, KB_E_STATE, "fed engine already running");
  if (!kb_fed_cycle_ok(c, max_job_tasks))
    return fail(c, KB_E_UNSUPPORTED, "fed engine: %d nodes need the split engine with one-segment jobs", c->N.n);
  if (c->any_busy()) return fail(c, KB_E_STATE, "a pipelined job is still in flight");
  if (!c->slot[kJobSlots - 1].h || !c->stream_b) return fail(c, KB_E_STATE, "kb_job_reserve first");
  if (!c->fed_ring) {
    HIP_OK(c, hipMalloc(&c->fed_ring, fed_ring_bytes()));
    HIP_OK(c, memset_sync(c->fed_ring, 0, fed_ring_bytes()));  // (recycled memory: no earlier context's commands)
    HIP_OK(c, hipMalloc((void**)&c->fed_ctr, kJobSlots * sizeof(uint32_t)));
    HIP_OK(c, hipMalloc((void**)&c->fed_exit, sizeof(int32_t)));
    HIP_OK(c, memset_sync(c->fed_ctr, 0, kJobSlots * sizeof(uint32_t)));
    for (int s = 0; s < kJobSlots; ++s) c->fed_count[s] = 0;
  }
  HIP_OK(c, hipMemsetAsync(c->fed_exit, 0, sizeof(int32_t), c->stream));
  c->fed_split_now = false;
  FedSlotPtrs sp;
  for (int s = 0; s < kJobSlots; ++s) {
    sp.keys[s] = c->sel_keys[s];
    sp.stat[s] = c->sel_stat[s];
    sp.commits[s] = c->commits[s];
    sp.js[s] = (JobState*)c->slot[s].d;
    sp.hjs[s] = (JobState*)c->slot[s].hdev;
    sp.hout[s] = (int32_t*)(c->slot[s].hdev + sizeof(JobState));
  }
  c->fed_r = 0;
  c->fed_tasks = 0;
  c->fed_fresh = false;
  if (c->fed_diag) {
    c->dg_iss0.clear();
    c->dg_iss1.clear();
    c->dg_fin0.clear();
    c->dg_fin1.clear();
    c->dg_t0 = std::chrono::steady_clock::now();
  }
  c->fed_ev = nullptr;
  if (c->timing) {  // the engine is one launch per cycle: always timed
    const bool tn = c->timing_now;
    c->timing_now = true;
    c->ev_begin(&c->fed_ev);
    c->timing_now = tn;
  }
  void* xchg = nullptr;
  if (c->use_fed_split && fed_split_ok(c->N.n, c->sharded) && max_job_tasks <= (uint32_t)kFedSplitMaxTasks) {
    if (!c->fed_xchg) HIP_OK(c, hipMalloc(&c->fed_xchg, fed_xchg_bytes()));
    if (!c->h_fed_ctrs) HIP_OK(c, hipHostMalloc((void**)&c->h_fed_ctrs, 24 * sizeof(uint64_t), hipHostMallocDefault));
    HIP_OK(c, hipMemsetAsync(c->fed_xchg, 0, fed_xchg_bytes(), c->stream));  // job numbers restart per cycle
    xchg = c->fed_xchg;
    c->stats.fed_split++;
    c->fed_split_now = true;
  }
  c->stats.fed_cycles++;
  ShardPeers SP{};
  if (c->sharded) {  // (kb_fed_cycle_ok: peer exchange, split engine)
    if (!xchg) return fail(c, KB_E_STATE, "node-sharded fed engine without the split engine");
    for (int w = 0; w < c->shard.world; ++w) SP.inbox[w] = (uint64_t*)c->peer_inbox[w];
    SP.rank = c->shard.rank;
    SP.world = c->shard.world;
    if (((c->shard_epoch + 1) & ((1u << kShardEpochBits) - 1)) == 0)
      if (int rc = shard_inbox_rezero(c)) return rc;
    SP.epoch = ++c->shard_epoch;
    note_peer_epoch(c->shard_epoch + 1);
    SP.self_inbox = c->shard_self_inbox ? 1 : 0;
    c->stats.fed_sharded++;
  }
  // node-sharded: 30 s (every rank's engine waits for the slowest rank's host at each exchange; eight ranks sharing
  // one GPU in the tests once left a rank's engine without progress for over 10 s)
  const uint64_t idle = c->sharded ? 30 * c->fed_idle : c->fed_idle;
  // resident sweepers: the census grid's spare workgroups (split engine, placed on an XCC, plain launch)
  c->fed_sweepers_now = xchg && !c->fed_coop && c->fed_xcc >= 0 && c->fed_xcc < 8 && !c->fed_kernel_sweeps;
  if (c->fed_sweepers_now && !c->fed_hring) {
    HIP_OK(c, hipHostMalloc(&c->fed_hring, kJobSlots * sizeof(FedHostCmd), hipHostMallocMapped | hipHostMallocCoherent));
    memset(c->fed_hring, 0, kJobSlots * sizeof(FedHostCmd));
    HIP_OK(c, hipHostGetDevicePointer(&c->fed_hring_dev, c->fed_hring, 0));
  }
  // the sweepers' level records (the selector forwards them with its candidates; sweep kernels write none)
  const bool lvl_on = c->fed_sweepers_now && !c->no_lvl;
  for (int s = 0; s < kJobSlots; ++s) {
    if (lvl_on && !c->sel_lvl[s]) HIP_OK(c, hipMalloc((void**)&c->sel_lvl[s], (size_t)std::max(c->N.n, 1) * kLvlW * 4));
    sp.lvl[s] = lvl_on ? c->sel_lvl[s] : nullptr;
  }
  c->fed_epoch++;
  c->fed_m = 0;
  c->fed_cmd_m = c->fed_fresh_m = 0;
  HIP_OK(c, (hipError_t)launch_fed_engine(c->N, c->P, c->cfg, c->idx_bits, sp, c->fed_ring, c->fed_ctr,
                                          c->fed_count, idle, c->fed_exit, xchg, c->stream, c->fed_coop, SP,
                                          c->fed_coop || c->fed_xcc < 0 ? -1 : c->fed_xcc | (c->test_one_xcc ? 0x100 : 0),
                                          c->fed_sweepers_now ? c->fed_hring_dev : nullptr, c->fed_epoch));
  HIP_OK(c, hipGetLastError());
  c->fed = true;
  c->prev_listed = false;
  return KB_OK;
}

// Post a command to the engine (sweep: the job's level-0 keys into its slot buffers first).
static int fed_post(kb_ctx* c, const FedCmdArgs& a0, int si, bool sweep) {
  const int r = c->fed_r;
  // the launch's most recent fresh command (the parity selectors: every command before it is final)
  FedCmdArgs a = a0;
  if (a.fresh) c->fed_fresh_m = c->fed_cmd_m;
  a.fresh_m = (int32_t)c->fed_fresh_m;
  c->fed_cmd_m++;
  void* entry = (char*)c->fed_ring + r * (fed_ring_bytes() / kJobSlots);
  if (c->fed_sweepers_now) {  // the resident sweepers take it from the pinned ring: no launch
    fed_host_post(c->fed_hring, r, a, ((uint64_t)c->fed_epoch << 32) | (uint64_t)(c->fed_m + 1));
    c->fed_m++;
  } else if (sweep) {  // the job's level-0 sweep (the launch path's own sweep kernel) carries the command
    hipEvent_t ea;
    c->ev_begin(&ea, c->stream_b);
    launch_sel_sweep(c->N, c->P, c->cfg, a.spec, c->idx_bits, c->sel_keys[si], c->sel_stat[si], nullptr, false,
                     c->stream_b, SpecGuard{nullptr, 0, 0, 0}, c->fed_ctr + r, &a, entry);
    c->ev_end(ea, KB_KERNEL_SEL_SWEEP, (uint64_t)c->N.n, c->stream_b);
  } else {
    launch_fed_cmd(c->N, c->P, c->cfg, c->idx_bits, c->sel_keys[si], c->sel_stat[si], a, entry, c->fed_ctr + r,
                   false, c->stream_b);
  }
  HIP_OK(c, hipGetLastError());
  c->fed_count[r] += (uint32_t)((c->N.n + 63) / 64);
  c->fed_r = r + 1 == kJobSlots ? 0 : r + 1;
  return KB_OK;
}

// Pause the resident engine between two of its commands (nothing in flight): the context's launch paths run on
// stream_alt (a hardware queue of its own: the engine's launch keeps `stream`) while the engine idles, and
// kb_fed_resume hands it the next command flagged fresh.
int kb_fed_pause(kb_ctx* c) {
  if (!c || !c->fed || c->fed_paused) return fail(c, KB_E_STATE, "fed engine not running");
  if (c->any_busy()) return fail(c, KB_E_STATE, "fed engine: a job is still in flight");
  if (!c->stream_alt) {
    hipDeviceProp_t prop;
    HIP_OK(c, hipGetDeviceProperties(&prop, c->device));
    const int cus = std::max(prop.multiProcessorCount, 1);
    std::vector<uint32_t> mask((cus + 31) / 32, 0xffffffffu);
    if (cus % 32) mask.back() = (1u << (cus % 32)) - 1;
    HIP_OK(c, hipExtStreamCreateWithCUMask(&c->stream_alt, (uint32_t)mask.size(), mask.data()));
  }
  std::swap(c->stream, c->stream_alt);
  c->fed = false;
  c->fed_paused = true;
  c->prev_listed = false;
  c->stats.fed_pauses++;
  return KB_OK;
}

int kb_fed_resume(kb_ctx* c) {
  if (!c || !c->fed_paused) return fail(c, KB_E_STATE, "fed engine not paused");
  if (c->any_busy()) return fail(c, KB_E_STATE, "a launch-path job is still in flight");
  HIP_OK(c, hipStreamSynchronize(c->stream));  // the pause's last kernels (a table commit behind a publish)
  std::swap(c->stream, c->stream_alt);
  c->fed = true;
  c->fed_paused = false;
  c->fed_fresh = true;
  c->prev_listed = false;
  return KB_OK;
}

int kb_fed_end(kb_ctx* c) {
  if (c && c->fed_paused) {  // (a pause ends with the engine: the next command is its EXIT)
    HIP_OK(c, hipStreamSynchronize(c->stream));
    std::swap(c->stream, c->stream_alt);
    c->fed = true;
    c->fed_paused = false;
  }
  if (!c || !c->fed) return KB_OK;
  c->fed = false;
  FedCmdArgs a{KB_ENG_EXIT, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  int rc = fed_post(c, a, 0, false);
  if (c->fed_ev) {  // queued behind the engine on the place stream
    c->ev_end(c->fed_ev, KB_KERNEL_FED_ENGINE, c->fed_tasks * (uint64_t)c->N.n);
    c->fed_ev = nullptr;
  }
  // the placer's counters (FedXchg::sphase, sdiag): copied behind the engine on its stream into pinned memory, so
  // reading them adds no device round trip to the cycle
  const bool ctrs = c->fed_xchg && c->fed_split_now && c->h_fed_ctrs;
  constexpr size_t kCtrWords = 24;  // sphase[8] + sdiag[16], the end of FedXchg
  if (ctrs)
    (void)hipMemcpyAsync(c->h_fed_ctrs, (char*)c->fed_xchg + fed_xchg_bytes() - kCtrWords * sizeof(uint64_t),
                         kCtrWords * sizeof(uint64_t), hipMemcpyDeviceToHost, c->stream);
  const hipError_t e = hipStreamSynchronize(c->stream);  // bounded: EXIT, or the engine's idle exit
  if (rc == KB_OK && e != hipSuccess) rc = fail(c, KB_E_HIP, "fed engine: %s", hipGetErrorString(e));
  if (c->timing) c->ev_collect(true);
  if (ctrs && e == hipSuccess) {
    const uint64_t* ph = c->h_fed_ctrs;     // sphase
    const uint64_t* d = c->h_fed_ctrs + 8;  // sdiag
    if (c->fed_diag && d[6]) {  // KB_DIAG builds: the placer's fine stamps (FedXchg::wdiag, ahead of census/sphase)
      uint64_t w[8] = {};
      const size_t off = fed_xchg_bytes() - kCtrWords * sizeof(uint64_t) - fed_census_bytes() - sizeof(w);
      if (hipMemcpy(w, (char*)c->fed_xchg + off, sizeof(w), hipMemcpyDeviceToHost) == hipSuccess && d[6])
        fprintf(stderr, "kb_fed_placer_fine cycles/job cand_scan=%.0f range=%.0f thr_search=%.0f takes=%.0f "
                "late_heads/job=%.3f rounds/job=%.2f search_steps/job=%.2f K/job=%.1f\n", (double)w[0] / d[6],
                (double)w[1] / d[6], (double)w[2] / d[6], (double)w[3] / d[6], (double)w[4] / d[6],
                (double)w[5] / d[6], (double)w[6] / d[6], (double)w[7] / d[6]);
    }
    if (c->fed_diag && fed_trace_offset()) {  // KB_DIAG / KB_TIMELINE builds: the engine's per-job timeline
      const int TJ = fed_trace_jobs();
      constexpr int TW = 16;  // FedXchg::tl's words per job
      std::vector<uint64_t> tl((size_t)TJ * TW);
      const int jobs = (int)std::min<uint64_t>(d[6] ? d[6] : (uint64_t)c->dg_iss0.size(), (uint64_t)TJ);
      if (hipMemcpy(tl.data(), (char*)c->fed_xchg + fed_trace_offset(), tl.size() * 8, hipMemcpyDeviceToHost) ==
              hipSuccess && jobs > 8) {
        // per job m (relative to the placer's end of job m-1 = when it wants job m's head): the selector's command
        // arrival, patch done, selection done, set seen, head; the placer's start and end of job m
        constexpr int NK = 16;
        const char* names[NK] = {"cmd", "patched", "selected", "set_seen", "head", "loop_top", "cmd_decoded",
                                 "placer_start", "merge_loads", "set_published", "node_setup", "e_seq", "winners",
                                 "pub_start", "released", "placer_end"};
        const int ks[NK] = {0, 1, 2, 3, 4, 11, 10, 5, 12, 6, 13, 14, 15, 8, 9, 7};
        std::vector<double> v[NK], lv[NK];
        for (int m = 4; m < jobs - 1; ++m) {
          const double E = (double)tl[(size_t)(m - 1) * TW + 7];
          const bool late = tl[(size_t)m * TW + 4] > tl[(size_t)(m - 1) * TW + 7];
          for (int k = 0; k < NK; ++k) {
            const double x = ((double)tl[(size_t)m * TW + ks[k]] - E) * 0.01;  // us (100 MHz ticks)
            v[k].push_back(x);
            if (late) lv[k].push_back(x);
          }
        }
        const auto pct = [](std::vector<double> x, double q) {
          if (x.empty()) return 0.0;
          std::sort(x.begin(), x.end());
          return x[std::min(x.size() - 1, (size_t)(q * (double)x.size()))];
        };
        fprintf(stderr, "kb_fed_timeline us after the placer's end of job m-1 (p10/p50/p90; late heads %zu of %zu:"
                " their p50)", lv[0].size(), v[0].size());
        for (int k = 0; k < NK; ++k)
          fprintf(stderr, " %s=%.2f/%.2f/%.2f[%.2f]", names[k], pct(v[k], 0.1), pct(v[k], 0.5), pct(v[k], 0.9),
                  pct(lv[k], 0.5));
        fprintf(stderr, "\n");
        // the late heads by job index mod the slot count and their runs; the host's side of the same jobs: the
        // issue call, the gap from seeing job m-kJobSlots's result to issuing job m, and the result intervals
        int bym[8] = {}, run = 0, maxrun = 0, runs = 0;
        std::vector<char> late_m((size_t)jobs, 0);
        for (int m = 4; m < jobs - 1; ++m) {
          const bool late = tl[(size_t)m * TW + 4] > tl[(size_t)(m - 1) * TW + 7];
          late_m[(size_t)m] = late;
          if (late) {
            bym[m % kJobSlots]++;
            runs += run == 0;
            maxrun = std::max(maxrun, ++run);
          } else {
            run = 0;
          }
        }
        fprintf(stderr, "kb_fed_late by m%%%d:", kJobSlots);
        for (int k = 0; k < kJobSlots; ++k) fprintf(stderr, " %d", bym[k]);
        fprintf(stderr, " runs=%d longest=%d\n", runs, maxrun);
        const size_t nh = std::min({c->dg_iss0.size(), c->dg_iss1.size(), (size_t)jobs});
        if (nh > 8 && c->dg_fin1.size() + kJobSlots >= nh) {
          std::vector<double> iss, gap, fin, lgap, liss;
          for (size_t m = kJobSlots; m < nh; ++m) {
            const double is = (double)(c->dg_iss1[m] - c->dg_iss0[m]) * 1e-3;
            const double gp = (double)(c->dg_iss0[m] - c->dg_fin1[m - kJobSlots]) * 1e-3;
            iss.push_back(is);
            gap.push_back(gp);
            if (m < c->dg_fin1.size()) fin.push_back((double)(c->dg_fin1[m] - c->dg_fin1[m - 1]) * 1e-3);
            if (m < late_m.size() && late_m[m]) {
              lgap.push_back(gp);
              liss.push_back(is);
            }
          }
          fprintf(stderr, "kb_fed_host us (p10/p50/p90/max [late heads' p50]) issue=%.2f/%.2f/%.2f/%.2f[%.2f] "
                  "seen_m-%d_to_issue=%.2f/%.2f/%.2f/%.2f[%.2f] result_interval=%.2f/%.2f/%.2f/%.2f\n",
                  pct(iss, 0.1), pct(iss, 0.5), pct(iss, 0.9), pct(iss, 0.999), pct(liss, 0.5), kJobSlots,
                  pct(gap, 0.1), pct(gap, 0.5), pct(gap, 0.9), pct(gap, 0.999), pct(lgap, 0.5), pct(fin, 0.1),
                  pct(fin, 0.5), pct(fin, 0.9), pct(fin, 0.999));
        }
      }
    }
    if (c->fed_diag && d[6]) {  // KB_DIAG builds: the selector's phases
      fprintf(stderr, "kb_fed_placer_merge cycles/job loads=%.0f b_order=%.0f union_rank=%.0f slots=%.0f\n",
              (double)d[8] / d[6], (double)d[9] / d[6], (double)d[10] / d[6], (double)d[11] / d[6]);
      fprintf(stderr, "kb_fed_selector jobs=%llu cycles/job wait_cmd=%.0f key_load=%.0f wait_set_exclude=%.0f "
              "wait_done_patch=%.0f select=%.0f publish=%.0f cmd_gated/job=%.3f\n", (unsigned long long)d[6],
              (double)d[0] / d[6], (double)d[1] / d[6], (double)d[2] / d[6], (double)d[3] / d[6], (double)d[4] / d[6],
              (double)d[5] / d[6], (double)d[7] / d[6]);
    }
    c->stats.shard_wait_ticks += d[12];
    c->stats.shard_xchg += d[13];
    c->stats.fed_clock_ticks += d[14];
    c->stats.fed_real_ticks += d[15];
    if (c->sharded)
      for (int k = 0; k < 6; ++k) c->stats.shard_phase_ticks[k] += ph[k];
    // (the placer's word carries the resident sweeper count in bits 40..47)
    c->stats.fed_wg_place[0] = ph[6] & ~(0xffull << 40);
    c->stats.fed_wg_place[1] = ph[7];
    c->stats.fed_last_sweepers = (int32_t)((ph[6] >> 40) & 0xffu);
  }
  c->prev_listed = false;  // (the launch path's next sweep must not count on the engine's commit lists)
  // an idle exit after every job was served (a host stall before this call) loses nothing
  int32_t idle = 0;
  if (rc == KB_OK && c->any_busy() &&
      hipMemcpy(&idle, c->fed_exit, sizeof(idle), hipMemcpyDeviceToHost) == hipSuccess && idle)
    rc = fail(c, KB_E_HIP, "fed engine exited idle with a job in flight");
  return rc;
}

// The engine idled out while the host stalled (kFedIdleExit from kb_job_finish): it served every command
// before the one the host waits for and none after. Leave fed mode; the caller re-issues the unserved job on
// the launch path (the speculative one, never run, is dropped) and the cycle goes on there.
int kb_fed_abandon(kb_ctx* c) {
  if (c && c->fed_paused) {
    (void)hipStreamSynchronize(c->stream);
    std::swap(c->stream, c->stream_alt);
    c->fed = true;
    c->fed_paused = false;
  }
  if (!c || !c->fed) return KB_OK;
  c->fed = false;
  if (c->sharded) {  // every rank would have to leave at the same job: fail loudly instead
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->stream_b);
    std::string why;
    for (auto& sl : c->slot) {
      sl.busy = false;
      const JobState* hs = (const JobState*)sl.h;
      if (hs && (hs->t_recv & 1)) {  // the placer's note (shard_place): the word it waited for
        char b[200];
        snprintf(b, sizeof(b), " (rank %d waited for rank %d's word %d: tag %08x there, %08x wanted; %d of the "
                 "record's words current; epoch %u)", c->shard.rank, (int)(hs->t_recv >> 56),
                 (int)((hs->t_recv >> 40) & 0xffff), (unsigned)(hs->t_done >> 32), (unsigned)hs->t_done,
                 (int)((hs->t_recv >> 20) & 0xfffff), c->shard_epoch);
        why = b;
      }
    }
    return fail(c, KB_E_STATE, "node-sharded fed engine left (code %d): a rank's proposal did not arrive (a peer "
                "stalled or left)%s", c->fed_exit_code, why.c_str());
  }
  if (c->fed_ev) {
    c->ev_end(c->fed_ev, KB_KERNEL_FED_ENGINE, c->fed_tasks * (uint64_t)c->N.n);
    c->fed_ev = nullptr;
  }
  HIP_OK(c, hipStreamSynchronize(c->stream));
  HIP_OK(c, hipStreamSynchronize(c->stream_b));  // the unserved jobs' sweeps (they only read rows)
  HIP_OK(c, memset_sync(c->fed_exit, 0, sizeof(int32_t)));
  for (auto& sl : c->slot) sl.busy = false;
  c->prev_listed = false;
  c->n_fed_abandon++;
  c->stats.fed_abandon++;
  return KB_OK;
}

int kb_job_issue(kb_ctx* c, const kb_job_req* job, int slot, const kb_job_pred* pred) {
  if (!c || !job || slot < 0 || slot >= kJobSlots) return KB_E_INVALID;
  if (!c->fed && slot > 1) return fail(c, KB_E_INVALID, "the per-job launch path pipelines two slots");
  if (int rc = validate_job(c, job)) return rc;
  if (job->n_tasks == 0) return fail(c, KB_E_INVALID, "empty job");
  if (c->slot[slot].busy) return fail(c, KB_E_STATE, "job slot %d is busy", slot);
  if (job->n_tasks > slots_cap(c))  // growing would free a slot in flight
    return fail(c, KB_E_STATE, "kb_job_reserve(%u) first", job->n_tasks);
  if (int rc = kb_engine_stop(c)) return rc;
  if (int rc = ensure_slots(c, job->n_tasks, true)) return rc;
  if (c->fed) {  // one selection run: the sweep kernel carries the command to the resident engine
    for (uint32_t i = 1; i < job->n_tasks; ++i)
      if (job->task_specs[i] != job->task_specs[0]) return fail(c, KB_E_INVALID, "fed engine: one run per job");
    if (!kb_spec_fed_ok(c, job->task_specs[0])) return fail(c, KB_E_INVALID, "fed engine: spec not eligible");
    if (c->aff_ok && c->spec_needs_aff[job->task_specs[0]]) c->stats.fed_aff_units++;
    kb_ctx::JobSlot& S = c->slot[slot];
    S.t_issue = std::chrono::steady_clock::now();
    if (c->fed_diag) c->dg_iss0.push_back((S.t_issue - c->dg_t0).count());
    c->timing_now = c->timing && (c->issue_count++ % c->timing_every == 0);  // the job's sweep
    memset(((JobState*)S.h)->diag, 0, sizeof(((JobState*)S.h)->diag));
    ((JobState*)S.h)->t_recv = 0;  // (the sharded placer's timeout note)
    FedCmdArgs a{KB_ENG_RUN, job->task_specs[0], 0, (int32_t)job->n_tasks, job->ready_num, job->min_available,
                 job->gang_ready, slot, pred ? 1 : 0, pred ? pred->stop : 0, pred ? pred->placed : 0,
                 pred ? pred->ready : 0, ++c->seq, c->fed_fresh ? 1 : 0,
                 c->fed_fresh || c->spec_rowcols[job->task_specs[0]] ? 1 : 0};
    c->fed_fresh = false;
    if (c->issue_trace)
      fprintf(stderr, "kb_issue rank=%d seq=%u slot=%d spec=%d tasks=%u guard=%d stop=%d placed=%d ready=%d\n",
              c->sharded ? c->shard.rank : 0, c->seq, slot, job->task_specs[0], job->n_tasks, pred ? 1 : 0,
              pred ? pred->stop : 0, pred ? pred->placed : 0, pred ? pred->ready : 0);
    S.ev_b = c->pending.size();
    if (int rc = fed_post(c, a, slot, true)) return rc;
    S.ev_e = c->pending.size();
    S.seq = c->seq;
    S.busy = true;
    S.issue_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - S.t_issue).count();
    if (c->fed_diag) c->dg_iss1.push_back((std::chrono::steady_clock::now() - c->dg_t0).count());
    return KB_OK;
  }
  SpecGuard g{nullptr, 0, 0, 0};
  if (pred) {
    if (!kb_job_guardable(c, job)) return fail(c, KB_E_INVALID, "job cannot be issued speculatively");
    g = SpecGuard{(const JobState*)c->slot[pred->prev_slot].d, pred->stop, pred->placed, pred->ready};
  }
  return c->sharded ? shard_issue(c, job, slot, g) : place_issue(c, job, slot, g);
}

int kb_job_finish(kb_ctx* c, int slot, int32_t* placed_node, int32_t* placed_kind, kb_job_result* result,
                  int skipped) {
  if (!c || !result || slot < 0 || slot >= kJobSlots) return KB_E_INVALID;
  memset(result, 0, sizeof(*result));
  result->fail_task = -1;
  return place_finish(c, slot, placed_node, placed_kind, result, skipped != 0);
}

extern "C++" {
template <class SCORE>
static int eval_impl(kb_ctx* c, const int32_t* spec_ids, uint32_t t, uint32_t* reasons, SCORE* scores);
}

int kb_eval32(kb_ctx* c, const int32_t* spec_ids, uint32_t t, uint32_t* reasons, int32_t* scores) {
  if (c) c->timing_now = c->timing;
  if (c) c->prev_listed = false;
  if (!c || (!spec_ids && t)) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs first");
  const DevCfg& C = c->cfg;
  for (uint32_t i = 0; i < t; ++i) {
    const int s = spec_ids[i];
    if (s < 0 || s >= c->P.m) return fail(c, KB_E_INVALID, "spec id %d", s);
    if (c->spec_needs_aff[s] && !c->aff_ok)
      return fail(c, KB_E_UNSUPPORTED, "spec %d has pod (anti)affinity: upload the affinity tables first", s);
    const int64_t ov = (size_t)s < c->ov_absmax.size() ? c->ov_absmax[s] : 0;
    const long double bound = 10.0L * std::llabs((long long)C.w_lr) + 10.0L * std::llabs((long long)C.w_bra) +
                              (long double)c->spec_pref_weight[s] * std::llabs((long long)C.w_na) + (long double)ov +
                              10.0L * std::llabs((long long)C.w_pa);
    if (bound >= 2147483647.0L || ((size_t)s < c->spec_ipa_err.size() && c->spec_ipa_err[s]))
      return fail(c, KB_E_UNSUPPORTED, "spec %d: its score does not fit int32 (use kb_eval)", s);
  }
  HIP_OK(c, hipSetDevice(c->device));
  return eval_impl(c, spec_ids, t, reasons, scores);
}

int kb_eval(kb_ctx* c, const int32_t* spec_ids, uint32_t t, uint32_t* reasons, int64_t* scores) {
  if (c) c->timing_now = c->timing;
  if (c) c->prev_listed = false;
  if (!c || (!spec_ids && t)) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs first");
  for (uint32_t i = 0; i < t; ++i) {
    if (spec_ids[i] < 0 || spec_ids[i] >= c->P.m) return fail(c, KB_E_INVALID, "spec id %d", spec_ids[i]);
    if (c->spec_needs_aff[spec_ids[i]] && !c->aff_ok)
      return fail(c, KB_E_UNSUPPORTED, "spec %d has pod (anti)affinity: upload the affinity tables first",
                  spec_ids[i]);
  }
  HIP_OK(c, hipSetDevice(c->device));
  return eval_impl(c, spec_ids, t, reasons, scores);
}

int kb_node_reasons(kb_ctx* c, int spec, uint32_t* reasons) {
  const bool tn = c->timing_now;
  c->timing_now = false;
  const int rc = eval_impl<int64_t>(c, &spec, 1, reasons, nullptr);
  c->timing_now = tn;
  return rc;
}

extern "C++" {
template <class SCORE>
static int eval_impl(kb_ctx* c, const int32_t* spec_ids, uint32_t t, uint32_t* reasons, SCORE* scores) {
  const size_t n = (size_t)c->N.n;
  const uint32_t chunk = 8192;
  int32_t* d_ids;
  uint32_t* d_r;
  SCORE* d_s;
  const uint32_t tc = std::min(t, chunk);
  // the output buffers persist in the context (grown, never shrunk): no allocation per call, and one placement of
  // the pages for the context's life
  const size_t need = std::max<size_t>(tc * n, 1);
  if (c->eval_cap < need || c->eval_ids_cap < std::max<uint32_t>(tc, 1)) {
    (void)hipFree(c->eval_ids);
    (void)hipFree(c->eval_r);
    (void)hipFree(c->eval_s);
    c->eval_ids = nullptr, c->eval_r = nullptr, c->eval_s = nullptr, c->eval_cap = 0, c->eval_ids_cap = 0;
    HIP_OK(c, hipMalloc(&c->eval_ids, std::max<uint32_t>(tc, 1) * 4));
    HIP_OK(c, hipMalloc(&c->eval_r, need * 4));
    HIP_OK(c, hipMalloc(&c->eval_s, need * 8));  // (room for 64-bit scores)
    c->eval_cap = need;
    c->eval_ids_cap = std::max<uint32_t>(tc, 1);
  }
  d_ids = (int32_t*)c->eval_ids;
  d_r = (uint32_t*)c->eval_r;
  d_s = (SCORE*)c->eval_s;
  int rc = KB_OK;
  for (uint32_t b = 0; b < t && rc == KB_OK; b += chunk) {
    const uint32_t cnt = std::min(chunk, t - b);
    if (hipMemcpyAsync(d_ids, spec_ids + b, cnt * 4, hipMemcpyHostToDevice, c->stream) != hipSuccess) rc = KB_E_HIP;
    hipEvent_t ea;
    if (c->aff_ok) {  // per-spec InterPodAffinity min / max first
      if (c->mm_eval_cap < cnt) {
        void* q;
        if (hipMalloc(&q, (size_t)cnt * 2 * sizeof(int64_t)) != hipSuccess) { rc = KB_E_HIP; break; }
        c->aff_mem.push_back(q);
        c->mm_eval = (int64_t*)q;
        c->mm_eval_cap = cnt;
      }
      launch_ipa_minmax(c->N, c->P, d_ids, 0, (int)cnt, c->mm_eval, nullptr, c->stream);
    }
    // a batch of plain specs (no overlay rows): the row-only kernel (KB_NO_EVAL_PLAIN: the general one, tests)
    bool plain = c->use_eval_plain;
    for (uint32_t i = 0; i < cnt && plain; ++i) {
      const int s = spec_ids[b + i];
      plain = c->spec_plain[s] && ((size_t)s >= c->ov_slot.size() || c->ov_slot[s] < 0);
    }
    c->ev_begin(&ea);
    if constexpr (sizeof(SCORE) == 8)
      launch_eval(c->N, c->P, c->cfg, d_ids, (int)cnt, d_r, d_s, c->aff_ok ? c->mm_eval : nullptr, plain,
                  c->cus | c->eval_bpc64 << 16, c->eval_spb, c->stream);
    else
      launch_eval32(c->N, c->P, c->cfg, d_ids, (int)cnt, d_r, d_s, c->aff_ok ? c->mm_eval : nullptr, plain,
                    c->cus | c->eval_bpc32 << 16, c->eval_spb, c->stream);
    c->ev_end(ea, KB_KERNEL_EVAL, (uint64_t)cnt * n);
    if (hipGetLastError() != hipSuccess) rc = KB_E_HIP;
    if (reasons && hipMemcpyAsync(reasons + (size_t)b * n, d_r, cnt * n * 4, hipMemcpyDeviceToHost, c->stream))
      rc = KB_E_HIP;
    if (scores && hipMemcpyAsync(scores + (size_t)b * n, d_s, cnt * n * sizeof(SCORE), hipMemcpyDeviceToHost,
                                 c->stream))
      rc = KB_E_HIP;
    if (hipStreamSynchronize(c->stream) != hipSuccess) rc = KB_E_HIP;
  }
  if (c->timing) c->ev_collect(true);
  if (rc) return fail(c, rc, "kb_eval: HIP failure");
  return KB_OK;
}
}  // extern "C++"

// The keys of kb_sort_nodes / kb_predicate_nodes (PredicateFn without allocate's resource check +
// PrioritizeNodes) into h, sorted descending or in node order.
static int pred_keys(kb_ctx* c, int32_t spec, bool sort, std::vector<uint64_t>& h);

int kb_sort_nodes(kb_ctx* c, int32_t spec, int32_t* order, int64_t* scores, uint32_t* n_out) {
  if (!c || !n_out) return KB_E_INVALID;
  *n_out = 0;
  std::vector<uint64_t> h;
  if (int rc = pred_keys(c, spec, true, h)) return rc;
  if (c->cfg.nodeorder && c->spec_ipa_err[spec]) return KB_OK;  // PrioritizeNodes' batch error: no scores
  uint32_t k = 0;
  for (; k < (uint32_t)h.size() && (h[k] & kFeasible); ++k) {
    if (order) order[k] = (int32_t)(kIdxMask - (uint32_t)(h[k] & kIdxMask));
    if (scores) scores[k] = (int64_t)((h[k] >> 24) & ((1ull << 39) - 1)) - kScoreBias;
  }
  *n_out = k;
  return KB_OK;
}

int kb_predicate_nodes(kb_ctx* c, int32_t spec, int32_t* nodes, uint32_t* n_out, uint32_t* reason_hist) {
  if (!c || !n_out) return KB_E_INVALID;
  *n_out = 0;
  std::vector<uint64_t> h;
  if (int rc = pred_keys(c, spec, false, h)) return rc;
  uint32_t k = 0, hist[KB_NUM_REASONS] = {0};
  for (size_t i = 0; i < h.size(); ++i) {
    if (h[i] & kFeasible) {
      if (nodes) nodes[k] = (int32_t)i;
      ++k;
    } else {
      for (int b = 0; b < KB_NUM_REASONS; ++b) hist[b] += (uint32_t)(h[i] >> b) & 1u;
    }
  }
  *n_out = k;
  if (reason_hist) memcpy(reason_hist, hist, sizeof(hist));
  return KB_OK;
}

static int pred_keys(kb_ctx* c, int32_t spec, bool sort, std::vector<uint64_t>& h) {
  c->prev_listed = false;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs first");
  if (c->fed || c->any_busy()) return fail(c, KB_E_STATE, "a job is in flight");
  if (c->sharded) return fail(c, KB_E_UNSUPPORTED, "kb_sort_nodes does not run node-sharded");
  if (spec < 0 || spec >= c->P.m) return fail(c, KB_E_INVALID, "spec %d out of range", spec);
  if (c->spec_needs_aff[spec] && !c->aff_ok)
    return fail(c, KB_E_UNSUPPORTED, "spec %d has pod (anti)affinity: upload the affinity tables first", spec);
  HIP_OK(c, hipSetDevice(c->device));
  const int n = c->N.n;
  int n_pad = kBitonicMin;
  while (n_pad < n) n_pad <<= 1;
  uint64_t* keys = nullptr;
  HIP_OK(c, hipMalloc(&keys, (size_t)n_pad * 8));
  const int64_t* mm = nullptr;
  if (c->aff_ok && c->spec_needs_aff[spec]) {  // this spec's InterPodAffinity min / max first
    if (c->mm_eval_cap < 1) {
      void* q;
      if (hipMalloc(&q, 2 * sizeof(int64_t)) != hipSuccess) {
        (void)hipFree(keys);
        return fail(c, KB_E_HIP, "hipMalloc");
      }
      c->aff_mem.push_back(q);
      c->mm_eval = (int64_t*)q;
      c->mm_eval_cap = 1;
    }
    launch_ipa_minmax(c->N, c->P, nullptr, spec, 1, c->mm_eval, nullptr, c->stream);
    mm = c->mm_eval;
  }
  launch_sort_nodes(c->N, c->P, c->cfg, spec, mm, keys, n_pad, c->stream, sort);
  h.assign(n, 0);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(h.data(), keys, (size_t)n * 8, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  (void)hipFree(keys);
  if (e != hipSuccess) return fail(c, KB_E_HIP, "PredicateNodes sweep: %s", hipGetErrorString(e));
  return KB_OK;
}

// Device copies of the host overlays (after every change; overlays change rarely, between jobs).
static int overlay_upload(kb_ctx* c) {
  // kernels of earlier jobs may still hold the old arrays
  HIP_OK(c, hipStreamSynchronize(c->stream));
  if (c->stream_b) HIP_OK(c, hipStreamSynchronize(c->stream_b));
  free_all(c->ov_mem);
  c->P.ov_slot = nullptr;
  c->P.ov_fail = nullptr;
  c->P.ov_score = nullptr;
  bool any = false;
  for (int32_t sl : c->ov_slot) any = any || sl >= 0;
  if (!any) return KB_OK;
  const size_t n = (size_t)c->N.n, slots = c->ov_fail.size();
  std::vector<uint8_t> f(slots * n);
  std::vector<int32_t> sc(slots * n);
  for (size_t k = 0; k < slots; ++k) {
    memcpy(f.data() + k * n, c->ov_fail[k].data(), n);
    memcpy(sc.data() + k * n, c->ov_score[k].data(), n * 4);
  }
  int rc;
  if ((rc = upload(c, c->ov_mem, &c->P.ov_slot, c->ov_slot.data(), c->ov_slot.size()))) return rc;
  if ((rc = upload(c, c->ov_mem, &c->P.ov_fail, f.data(), f.size()))) return rc;
  if ((rc = upload(c, c->ov_mem, &c->P.ov_score, sc.data(), sc.size()))) return rc;
  return KB_OK;
}

int kb_set_host_overlay(kb_ctx* c, int32_t spec, const uint8_t* fail_in, const int64_t* score_add) {
  if (c) c->prev_listed = false;
  if (!c) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs first");
  if (c->fed || c->any_busy()) return fail(c, KB_E_STATE, "a job is in flight");
  if (spec < 0 || spec >= c->P.m) return fail(c, KB_E_INVALID, "spec %d out of range", spec);
  // node sharding: the overlay's verdicts, its score bound (key width) and the NO_FIT hook's node masks are
  // rank-local, so ranks could take different paths for one job and break the collective sequence
  if (c->sharded) return fail(c, KB_E_UNSUPPORTED, "host overlay on a node-sharded context");
  HIP_OK(c, hipSetDevice(c->device));
  const size_t n = (size_t)c->N.n, m = (size_t)c->P.m;
  if (c->ov_slot.size() != m) {
    c->ov_slot.assign(m, -1);
    c->ov_any_fail.assign(m, 0);
  }
  if (c->ov_absmax.size() != m) c->ov_absmax.assign(m, 0);
  int32_t sl = c->ov_slot[spec];
  if (!fail_in && !score_add) {  // clear
    c->ov_slot[spec] = -1;
    c->ov_any_fail[spec] = 0;
    c->ov_absmax[spec] = 0;
  } else {
    int64_t mx = 0;
    if (score_add)
      for (size_t i = 0; i < n; ++i) {
        const int64_t v = score_add[i] < 0 ? -score_add[i] : score_add[i];
        if (v >= (1ll << 26)) return fail(c, KB_E_UNSUPPORTED, "overlay score %lld at node %zu exceeds 2^26",
                                          (long long)score_add[i], i);
        mx = std::max(mx, v);
      }
    if (sl < 0) {  // a free row (one no spec points at), else a new one
      std::vector<char> used(c->ov_fail.size(), 0);
      for (int32_t x : c->ov_slot)
        if (x >= 0) used[x] = 1;
      sl = (int32_t)(std::find(used.begin(), used.end(), 0) - used.begin());
      if ((size_t)sl == c->ov_fail.size()) {
        c->ov_fail.emplace_back(n, 0);
        c->ov_score.emplace_back(n, 0);
      }
    }
    auto& f = c->ov_fail[sl];
    auto& sc = c->ov_score[sl];
    f.assign(n, 0);
    sc.assign(n, 0);
    char any = 0;
    for (size_t i = 0; i < n; ++i) {
      if (fail_in && fail_in[i]) f[i] = 1, any = 1;
      if (score_add) sc[i] = (int32_t)score_add[i];
    }
    c->ov_slot[spec] = sl;
    c->ov_any_fail[spec] = any;
    c->ov_absmax[spec] = mx;
  }
  kb_update_traj_ok(c);
  if (int rc = kb_check_score_range(c)) {  // refused: take the overlay back
    c->ov_slot[spec] = -1;
    c->ov_any_fail[spec] = 0;
    c->ov_absmax[spec] = 0;
    kb_update_traj_ok(c);
    (void)overlay_upload(c);
    return rc;
  }
  return overlay_upload(c);
}

int kb_apply(kb_ctx* c, const kb_row_delta* d, uint32_t k, const int64_t* sc, uint32_t n_sc, const kb_port* ports,
             uint32_t n_ports) {
  if (c) c->prev_listed = false;  // rows changed outside any job's commit list
  if (!c || (!d && k)) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (!c->nodes_ok || !c->specs_ok) return fail(c, KB_E_STATE, "upload nodes and specs first");
  if (c->fed || c->any_busy()) return fail(c, KB_E_STATE, "a job is in flight");
  if (k == 0) return KB_OK;
  // every index the kernel follows is checked here
  const uint32_t S = (uint32_t)c->N.S;
  for (uint32_t i = 0; i < k; ++i) {
    const kb_row_delta& e = d[i];
    const int64_t lo = c->N.base, hi = (int64_t)c->N.base + c->N.n;
    const int64_t total = c->sharded ? (int64_t)c->shard.n_total : hi;
    if (e.node < 0 || e.node >= total) return fail(c, KB_E_INVALID, "delta %u: node %d", i, e.node);
    (void)lo;
    if (e.sc_off != 0xffffffffu && (uint64_t)e.sc_off + 2ull * S > n_sc)
      return fail(c, KB_E_INVALID, "delta %u: scalar deltas out of range", i);
    if ((uint64_t)e.port_off + e.port_cnt > n_ports) return fail(c, KB_E_INVALID, "delta %u: ports", i);
    for (uint32_t j = 0; j < e.port_cnt; ++j) {
      const kb_port& p = ports[e.port_off + j];
      if (p.slot < 0 || p.slot >= c->N.P || p.ip < 0 || p.ip > 63) return fail(c, KB_E_INVALID, "delta %u port", i);
    }
    if (e.spec >= c->P.m || (e.spec >= 0 && c->spec_needs_aff[e.spec] && !c->aff_ok))
      return fail(c, KB_E_INVALID, "delta %u: spec %d", i, e.spec);
  }
  HIP_OK(c, hipSetDevice(c->device));
  std::vector<void*> tmp;
  kb_row_delta* dd;
  int64_t* dsc;
  kb_port* dp;
  int rc;
  if ((rc = upload(c, tmp, &dd, d, k)) || (rc = upload(c, tmp, &dsc, sc, n_sc, false)) ||
      (rc = upload(c, tmp, &dp, ports, n_ports, false))) {
    free_all(tmp);
    return rc;
  }
  launch_apply(c->N, c->P, dd, (int)k, dsc, dp, c->stream);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  free_all(tmp);
  if (e != hipSuccess) return fail(c, KB_E_HIP, "kb_apply: %s", hipGetErrorString(e));
  return KB_OK;
}

int kb_apply_affinity(kb_ctx* c, const kb_aff_delta* d, uint32_t k) {
  if (!c || (!d && k)) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (c->broken) return fail(c, KB_E_HIP, "context unusable: %s", c->err.c_str());
  if (!c->aff_ok) return fail(c, KB_E_STATE, "upload the affinity tables first");
  if (c->fed || c->any_busy()) return fail(c, KB_E_STATE, "a job is in flight");
  if (k == 0) return KB_OK;
  const auto& D = c->aff_slot_D;
  for (uint32_t i = 0; i < k; ++i) {  // every index the kernel follows
    const kb_aff_delta& e = d[i];
    if (e.node < 0 || e.node >= c->P.A.n) return fail(c, KB_E_INVALID, "affinity delta %u: node %d", i, e.node);
    if (e.table >= 0) {
      if ((uint32_t)e.table >= c->aff_n_tables) return fail(c, KB_E_INVALID, "affinity delta %u: table %d", i, e.table);
    } else if (e.table != -1 || e.slot < 0 || (size_t)e.slot >= D.size() ||
               (int64_t)e.h_off + D[e.slot] > (int64_t)c->aff_n_h) {
      return fail(c, KB_E_INVALID, "affinity delta %u: histogram (slot %d, h_off %u)", i, e.slot, e.h_off);
    }
  }
  HIP_OK(c, hipSetDevice(c->device));
  std::vector<void*> tmp;
  kb_aff_delta* dd;
  if (int rc = upload(c, tmp, &dd, d, k)) {
    free_all(tmp);
    return rc;
  }
  launch_apply_aff(c->P.A, dd, (int)k, c->N.base, c->stream);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  free_all(tmp);
  if (e != hipSuccess) return fail(c, KB_E_HIP, "kb_apply_affinity: %s", hipGetErrorString(e));
  return KB_OK;
}

int kb_set_nofit_hook(kb_ctx* c, kb_nofit_fn fn, void* user) {
  if (!c) return KB_E_INVALID;
  c->nofit_fn = fn;
  c->nofit_user = user;
  return KB_OK;
}

int kb_restore_nodes(kb_ctx* c) {
  if (c) c->prev_listed = false;
  if (!c) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (!c->nodes_ok) return fail(c, KB_E_STATE, "no node table");
  for (auto& col : c->pristine)
    if (col.bytes) HIP_OK(c, hipMemcpyAsync(col.dst, col.src, col.bytes, hipMemcpyDeviceToDevice, c->stream));
  for (auto& col : c->aff_pristine)
    if (col.bytes) HIP_OK(c, hipMemcpyAsync(col.dst, col.src, col.bytes, hipMemcpyDeviceToDevice, c->stream));
  return KB_OK;
}

int kb_get_stats(kb_ctx* c, kb_stats* out, int reset) {
  if (!c || !out) return KB_E_INVALID;
  if (c->timing && !c->broken) c->ev_collect(true);
  *out = c->stats;
  if (reset) c->stats = kb_stats{};
  return KB_OK;
}

int kb_read_nodes(kb_ctx* c, int64_t* idle_cpu, int64_t* idle_mem, int64_t* rel_cpu, int64_t* rel_mem,
                  int32_t* pod_count, int64_t* nz_cpu, int64_t* nz_mem) {
  if (!c) return KB_E_INVALID;
  if (int rc_ = kb_engine_stop(c)) return rc_;
  if (!c->nodes_ok) return fail(c, KB_E_STATE, "no node table");
  HIP_OK(c, hipSetDevice(c->device));
  HIP_OK(c, hipStreamSynchronize(c->stream));
  const size_t n = (size_t)c->N.n;
  if (idle_cpu) HIP_OK(c, hipMemcpy(idle_cpu, c->N.idle_cpu, n * 8, hipMemcpyDeviceToHost));
  if (idle_mem) HIP_OK(c, hipMemcpy(idle_mem, c->N.idle_mem, n * 8, hipMemcpyDeviceToHost));
  if (rel_cpu) HIP_OK(c, hipMemcpy(rel_cpu, c->N.rel_cpu, n * 8, hipMemcpyDeviceToHost));
  if (rel_mem) HIP_OK(c, hipMemcpy(rel_mem, c->N.rel_mem, n * 8, hipMemcpyDeviceToHost));
  if (pod_count) HIP_OK(c, hipMemcpy(pod_count, c->N.pod_count, n * 4, hipMemcpyDeviceToHost));
  if (nz_cpu) HIP_OK(c, hipMemcpy(nz_cpu, c->N.nz_cpu, n * 8, hipMemcpyDeviceToHost));
  if (nz_mem) HIP_OK(c, hipMemcpy(nz_mem, c->N.nz_mem, n * 8, hipMemcpyDeviceToHost));
  return KB_OK;
}

}  // extern "C"
