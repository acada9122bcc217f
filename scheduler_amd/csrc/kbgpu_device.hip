// HIP kernels (gfx950) for kube-batch's allocate hot path.
//
// One (task, node) evaluation = the predicate chain of allocate's predicateFn
// (actions/allocate/allocate.go:80-93) + the predicates plugin
// (plugins/predicates/predicates.go:154-299) and the nodeorder score
// (plugins/nodeorder/nodeorder.go:188-246), read from the struct-of-arrays node
// table in HBM. Integer work only: resource fit is exact int64 (all quantities are
// integral float64 in the reference, resource_info.go:75-93); BalancedResource
// keeps its IEEE double division (balanced_resource_allocation.go:41-77), compiled
// with -ffp-contract=off.
//
// Kernels
//   sweep_keys_kernel : one thread per node; writes the packed argmax key of every
//                       node, the max key of every 64-node chunk (one wave) and the
//                       node's static-predicate / NodeAffinity cache for the spec.
//   place_loop_kernel : ONE wave, persistent for a run of same-spec tasks of a job:
//                       argmax over chunk maxima (LDS) -> commit the winner's row
//                       (Session.Allocate/Pipeline -> NodeInfo.AddTask + AddPod) ->
//                       re-key the winner -> re-reduce its chunk. With no pod
//                       (anti)affinity in the spec only the winner's row changes, so
//                       the incremental argmax is exact (SURVEY.md §7 hard parts).
//   eval_kernel       : parity mode, reasons + scores for T specs x N nodes.
#include <hip/hip_runtime.h>

#include "kbgpu_device.h"

namespace kbgpu {

__device__ __forceinline__ uint64_t wave_max_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t x = __shfl_xor(v, o, 64);
    v = x > v ? x : v;
  }
  return v;
}

// ---- wave-wide scans / reductions on DPP (row shifts + row broadcasts: a few cycles per step, where a
// ds_bpermute shuffle butterfly waits on LDS latency six times). Lanes whose DPP source is out of range
// keep `ident`. Every lane of the wave must be active.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint32_t dpp_src(uint32_t ident, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)ident, (int)v, CTRL, ROW_MASK, 0xf, false);
}
// inclusive prefix combine over the 64 lanes
template <class Op>
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x, uint32_t ident, Op op) {
  x = op(x, dpp_src<0x111>(ident, x));        // row_shr:1
  x = op(x, dpp_src<0x112>(ident, x));        // row_shr:2
  x = op(x, dpp_src<0x114>(ident, x));        // row_shr:4
  x = op(x, dpp_src<0x118>(ident, x));        // row_shr:8
  x = op(x, dpp_src<0x142, 0xa>(ident, x));   // row_bcast:15 -> rows 1, 3
  x = op(x, dpp_src<0x143, 0xc>(ident, x));   // row_bcast:31 -> rows 2, 3
  return x;
}
struct OpAdd { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a + b; } };
struct OpMax { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a > b ? a : b; } };
struct OpMin { __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return a < b ? a : b; } };
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_dpp(v, 0u, OpAdd{}), 63);
}

// Resource.LessEqual per dimension for integral values: r < rr || |rr - r| < tol  <=>  r - rr < tol
// (api/resource_info.go:253-276).
__device__ __forceinline__ bool le_tol(int64_t r, int64_t avail, int64_t tol) { return r - avail < tol; }

__device__ __forceinline__ bool scalars_fit(const DevNodes& N, const kb_spec& sp, const int64_t* sc, bool has_map,
                                            const int64_t* node_sc, int n) {
  if (!(sp.flags & KB_SPEC_INIT_HAS_MAP)) return true;  // r.ScalarResources == nil
  if (!has_map) return false;                            // rr.ScalarResources == nil
  uint64_t m = sp.init_sc_mask;
  while (m) {
    const int s = __builtin_ctzll(m);
    m &= m - 1;
    if (!le_tol(sc[s], node_sc[(size_t)s * N.n + n], 10)) return false;
  }
  return true;
}

__device__ __forceinline__ bool fits_idle(const DevNodes& N, const kb_spec& sp, const int64_t* sci, uint32_t f, int n) {
  return le_tol(sp.init_cpu, N.idle_cpu[n], 10) && le_tol(sp.init_mem, N.idle_mem[n], 10ll * 1024 * 1024) &&
         scalars_fit(N, sp, sci, f & KB_NODE_IDLE_HAS_MAP, N.idle_sc, n);
}
__device__ __forceinline__ bool fits_rel(const DevNodes& N, const kb_spec& sp, const int64_t* sci, uint32_t f, int n) {
  return le_tol(sp.init_cpu, N.rel_cpu[n], 10) && le_tol(sp.init_mem, N.rel_mem[n], 10ll * 1024 * 1024) &&
         scalars_fit(N, sp, sci, f & KB_NODE_REL_HAS_MAP, N.rel_sc, n);
}

// labels.Requirement.Matches (vendor/k8s.io/apimachinery/pkg/labels/selector.go:185-236)
__device__ bool req_match(const DevNodes& N, const DevSpecs& P, const kb_req& r, int n) {
  if (r.op == KB_OP_TRUE) return true;
  if (r.op == KB_OP_FALSE) return false;
  const size_t at = (size_t)r.key * N.n + n;
  const int32_t v = N.label_val[at];
  const bool has = v >= 0;
  switch (r.op) {
    case KB_OP_IN:
    case KB_OP_NOTIN: {
      bool in = false;
      if (has)
        for (uint32_t i = 0; i < r.val_cnt; ++i)
          if (P.vals[r.val_off + i] == v) { in = true; break; }
      return r.op == KB_OP_IN ? in : !in;
    }
    case KB_OP_EXISTS: return has;
    case KB_OP_DNE: return !has;
    case KB_OP_GT:
    case KB_OP_LT: {
      if (!has || !N.label_int_ok[at]) return false;
      const int64_t lv = N.label_int[at];
      return r.op == KB_OP_GT ? lv > r.ival : lv < r.ival;
    }
  }
  return false;
}

// A node-selector term: AND of its requirements; an empty term matches nothing.
__device__ bool term_match(const DevNodes& N, const DevSpecs& P, const kb_term& t, int n) {
  if (t.req_cnt == 0) return false;
  for (uint32_t i = 0; i < t.req_cnt; ++i)
    if (!req_match(N, P, P.reqs[t.req_off + i], n)) return false;
  return true;
}

// leastRequestedScore (priorities/least_requested.go:36-53): ((cap - req) * 10) / cap, q in [0, 10].
// The int64 division is replaced by a double estimate corrected with exact int64 products.
__device__ __forceinline__ int64_t lr_score(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  const int64_t num = (cap - req) * 10;
  if (cap > 0 && cap < (1ll << 52) && num >= 0 && num < (1ll << 62)) {
    int64_t q = (int64_t)((double)num / (double)cap);
    q = q < 0 ? 0 : (q > 11 ? 11 : q);
    if (q * cap > num) --q;
    if ((q + 1) * cap <= num) ++q;
    return q;
  }
  return num / cap;
}
// fractionOfCapacity (balanced_resource_allocation.go:72-77)
__device__ __forceinline__ double frac_cap(int64_t req, int64_t cap) {
  return cap == 0 ? 1.0 : (double)req / (double)cap;
}

// The mutable + per-node numeric columns one evaluation reads (one batch of independent loads).
struct Row {
  uint32_t flags;
  int32_t pod_count, max_pods;
  // (the padding word before the int64 columns) the split engine's hand-off: a selector entry's A (allocations
  // before the node's Idle stops fitting the job's spec, allocs_before_full), -1 where the placer computes it; no
  // node column, never stored back
  int32_t aux;
  int64_t idle_cpu, idle_mem, rel_cpu, rel_mem, nz_cpu, nz_mem, alloc_cpu, alloc_mem;
};
static_assert(sizeof(Row) == 80, "Row: aux fills the padding word");

__device__ __forceinline__ Row load_row(const DevNodes& N, int n) {
  Row r;
  r.flags = N.flags[n];
  r.pod_count = N.pod_count[n];
  r.max_pods = N.max_pods[n];
  r.idle_cpu = N.idle_cpu[n];
  r.idle_mem = N.idle_mem[n];
  r.rel_cpu = N.rel_cpu[n];
  r.rel_mem = N.rel_mem[n];
  r.nz_cpu = N.nz_cpu[n];
  r.nz_mem = N.nz_mem[n];
  r.alloc_cpu = N.alloc_cpu[n];
  r.alloc_mem = N.alloc_mem[n];
  return r;
}

// The columns a commit changes, loaded around the vector L1 (sc1: agent-scope relaxed atomic loads). The selection
// path's commits store them sc1 (store_back_row), so the fed selector reads the placer's commits once it has seen
// the placer's tagged p_done word, without an agent-scope acquire per job (MI355X_MICROARCH.md, the hand-off
// table's first row: sc1 stores, vmcnt(0) and one sc1 signal on the writer's side, sc1 loads on the reader's).
template <class T>
__device__ __forceinline__ T ld_sc1(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void st_sc1(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ Row load_row_sc1(const DevNodes& N, int n) {
  Row r;
  r.flags = N.flags[n];  // (flags, max_pods, allocatable: no commit changes them)
  r.pod_count = ld_sc1(&N.pod_count[n]);
  r.max_pods = N.max_pods[n];
  r.idle_cpu = ld_sc1(&N.idle_cpu[n]);
  r.idle_mem = ld_sc1(&N.idle_mem[n]);
  r.rel_cpu = ld_sc1(&N.rel_cpu[n]);
  r.rel_mem = ld_sc1(&N.rel_mem[n]);
  r.nz_cpu = ld_sc1(&N.nz_cpu[n]);
  r.nz_mem = ld_sc1(&N.nz_mem[n]);
  r.alloc_cpu = N.alloc_cpu[n];
  r.alloc_mem = N.alloc_mem[n];
  return r;
}

// The columns a commit changes (idle / releasing cpu+mem, pod count, non-zero requests).
__device__ __forceinline__ void store_row(const DevNodes& N, int n, const Row& r) {
  N.idle_cpu[n] = r.idle_cpu;
  N.idle_mem[n] = r.idle_mem;
  N.rel_cpu[n] = r.rel_cpu;
  N.rel_mem[n] = r.rel_mem;
  N.pod_count[n] = r.pod_count;
  N.nz_cpu[n] = r.nz_cpu;
  N.nz_mem[n] = r.nz_mem;
}

// ---- inter-pod (anti)affinity lookups (kb_affinity; scheduler_amd/affinity.py) ----
constexpr uint32_t kAffExistingAnti = (1u << KB_R_POD_AFFINITY) | (1u << KB_R_EXISTING_ANTI);
constexpr uint32_t kAffAntiRules = (1u << KB_R_POD_AFFINITY) | (1u << KB_R_ANTI_AFFINITY_RULES);
constexpr uint32_t kAffAffinityRules = (1u << KB_R_POD_AFFINITY) | (1u << KB_R_AFFINITY_RULES);
// a plain error from the reference's predicate (FitErrors.SetNodeError with the error's own string, no
// PredicateFailureReason): the caller supplies the string (kb_set_nofit_hook)
constexpr uint32_t kHostError = 1u << KB_R_HOST_ERROR;

// InterPodAffinityMatches (vendor/.../predicates.go:1155-1185) through the count tables, in the
// reference's order: existing pods' anti-affinity (:1293-1333), then the pod's own anti-affinity and
// affinity (satisfiesPodsAffinityAntiAffinity, :1367-1465).
// Mutable table entries: COH = true reads at L2 (the block-wide place loop updates them with atomics,
// which do not refresh this CU's L1).
template <bool COH>
__device__ __forceinline__ int32_t ld_cnt(const int32_t* p) {
  if (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

template <bool COH = false>
__device__ __forceinline__ uint32_t aff_reasons(const DevAff& A, const kb_aff_spec& as, int n) {
  for (uint32_t i = 0; i < as.check_cnt; ++i) {
    const kb_aff_check c = A.checks[as.check_off + i];
    const kb_aff_table t = A.tables[c.table];
    const int32_t d = A.topo_dom[(size_t)t.slot * A.n + n];
    const int32_t cnt = d >= 0 ? ld_cnt<COH>(&A.counters[t.cnt_off + d]) : 0;
    if (c.kind == KB_AFF_EXISTING_ANTI) {
      if (cnt > 0) return kAffExistingAnti;
    } else if (c.kind == KB_AFF_ANTI) {
      if (cnt > 0) return kAffAntiRules;
    } else if (c.kind == KB_AFF_ERROR) {
      if (cnt > 0) return kHostError;
    } else if (cnt == 0 && (ld_cnt<COH>(&A.totals[c.table]) > 0 || !as.self_match)) {
      return kAffAffinityRules;
    }
  }
  return 0;
}

// counts[node] of CalculateInterPodAffinityPriority (interpod_affinity.go:119-219) as the sum of the
// spec's per-key domain histograms.
template <bool COH = false>
__device__ __forceinline__ int64_t ipa_count(const DevAff& A, const kb_aff_spec& as, int n) {
  int64_t c = 0;
  for (uint32_t i = 0; i < as.hist_cnt; ++i) {
    const kb_ipa_hist h = A.hists[as.hist_off + i];
    const int32_t d = A.topo_dom[(size_t)h.slot * A.n + n];
    if (d >= 0) c += ld_cnt<COH>(&A.h[h.h_off + d]);
  }
  return c;
}

// fScore = MaxPriority * ((count - min) / (max - min)), HostPriority.Score = int(fScore) (:221-238);
// min and max start at 0 and run over every node. Counts are integers, exact in float64.
__device__ __forceinline__ int32_t ipa_score(int64_t c, int64_t mn, int64_t mx) {
  if (mx - mn <= 0) return 0;
  const double f = 10.0 * ((double)(c - mn) / (double)(mx - mn));
  return (int32_t)f;
}

// The table updates of commits of `sp` on node w: n_alloc Allocates join the lister tables
// (PodLister.UpdateTask, plugins/util/util.go:108-130), every commit adds the pod to the node for the
// score (nodeorder.go:161-172).
__device__ void apply_commit_tables(const DevAff& A, const kb_spec& sp, int w, int n_alloc, int n_commit) {
  if (!A.enabled || sp.aff_class < 0) return;
  const kb_aff_spec as = A.specs[sp.aff_class];
  if (n_alloc != 0)  // (negative: kb_apply taking a pod back)
    for (uint32_t i = 0; i < as.lister_cnt; ++i) {
      const int32_t t = A.lister[as.lister_off + i];
      const kb_aff_table tb = A.tables[t];
      const int32_t d = A.topo_dom[(size_t)tb.slot * A.n + w];
      if (d >= 0) atomicAdd(&A.counters[tb.cnt_off + d], n_alloc);
      atomicAdd(&A.totals[t], n_alloc);
    }
  if (n_commit != 0)
    for (uint32_t i = 0; i < as.incr_cnt; ++i) {
      const kb_ipa_incr e = A.incr[as.incr_off + i];
      const int32_t d = A.topo_dom[(size_t)e.slot * A.n + w];
      if (d >= 0) atomicAdd(&A.h[e.h_off + d], e.weight * n_commit);
    }
}

// Static part of the predicate chain and score for (spec, node): everything that no commit changes.
//   bits  0..15: first failing static stage BEFORE the host-port check (conditions, node selector)
//   bits 16..32: first failing static stage AFTER it (taints, pressure, inter-pod affinity, then the host
//                overlay of kb_set_host_overlay: a plugin later in tier order)
//   bits 33..59: NodeAffinity priority count x its weight + the overlay's score (node_affinity.go:34-74),
//                signed 27-bit (the host bounds it)
//   bits 60..63: InterPodAffinity priority (0..10); kIpaErrorField: the batch score errors
// `mm` (this spec's InterPodAffinity min / max) non-null: the spec's affinity inputs do not change
// during its run, so the affinity predicate and priority are folded in here too. A spec with inter-pod
// affinity evaluated without them (the block-wide loops) defers the overlay's predicate to aff_key.
// AFF = false compiles the affinity lookups out (specs without inter-pod affinity: fewer live registers).
constexpr uint32_t kIpaErrorField = 15;
constexpr int64_t kIpaErrorScore = -(1ll << 36);  // every feasible node <= -1: SelectBestNode panics

__device__ __forceinline__ int32_t ov_row(const DevSpecs& P, int spec) {
  return P.ov_slot != nullptr ? P.ov_slot[spec] : -1;
}

template <bool AFF>
__device__ uint64_t static_eval(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const kb_spec& sp,
                                int spec, uint32_t f, int n, const int64_t* mm) {
  uint32_t pre = 0, post = 0;
  const bool aff = AFF && mm != nullptr && sp.aff_class >= 0;
  const int32_t ov = ov_row(P, spec);
  if (C.predicates) {
    // CheckNodeConditionPredicate (vendor/.../predicates.go:1568-1596): one reason per bad condition
    pre = f & ((1u << KB_R_NOT_READY) | (1u << KB_R_OUT_OF_DISK) | (1u << KB_R_NETWORK_UNAVAILABLE) |
               (1u << KB_R_UNSCHEDULABLE));
    // PodMatchNodeSelector: nodeSelector AND required node affinity (vendor/.../predicates.go:807-863)
    if (!pre && (sp.flags & KB_SPEC_HAS_SELECTOR) && !term_match(N, P, P.terms[sp.sel_term], n))
      pre = 1u << KB_R_NODE_SELECTOR;
    if (!pre && (sp.flags & KB_SPEC_HAS_REQUIRED)) {
      bool any = false;
      for (uint32_t i = 0; i < sp.req_term_cnt && !any; ++i) any = term_match(N, P, P.terms[sp.req_term_off + i], n);
      if (!any) pre = 1u << KB_R_NODE_SELECTOR;
    }
    // PodToleratesNodeTaints (vendor/.../predicates.go:1489-1518), then the optional pressure predicates
    if (!P.tolerates[(size_t)sp.tol_set * P.n_taint_sets + N.taint_set[n]]) post = 1u << KB_R_TAINTS;
    else if (C.mem_pressure && (sp.flags & KB_SPEC_BEST_EFFORT) && (f & KB_NODE_MEM_PRESSURE))
      post = 1u << KB_R_MEMORY_PRESSURE;
    else if (C.disk_pressure && (f & KB_NODE_DISK_PRESSURE)) post = 1u << KB_R_DISK_PRESSURE;
    else if (C.pid_pressure && (f & KB_NODE_PID_PRESSURE)) post = 1u << KB_R_PID_PRESSURE;
    // InterPodAffinityMatches, the last predicate (plugins/predicates/predicates.go:278-296)
    if (aff && !pre && !post) post = aff_reasons(P.A, P.A.specs[sp.aff_class], n);
  }
  // the host overlay's predicate (deferred behind the live affinity check when that is not folded in)
  if (ov >= 0 && !pre && !post && (aff || sp.aff_class < 0) && P.ov_fail[(size_t)ov * N.n + n]) post = kHostError;
  int32_t na = 0;
  uint32_t ipa = 0;
  if (C.nodeorder) {
    if (!(sp.flags & KB_SPEC_NA_ERROR))
      for (uint32_t i = 0; i < sp.pref_term_cnt; ++i) {
        const kb_term t = P.terms[sp.pref_term_off + i];
        if (t.weight == 0) continue;
        if (term_match(N, P, t, n)) na += t.weight;
      }
    na *= C.w_na;
    if (sp.flags & KB_SPEC_IPA_ERROR) {
      ipa = kIpaErrorField;
    } else if (aff) {
      const kb_aff_spec as = P.A.specs[sp.aff_class];
      if (as.hist_cnt) ipa = (uint32_t)ipa_score(ipa_count(P.A, as, n), mm[0], mm[1]);
    }
  }
  if (ov >= 0) na += P.ov_score[(size_t)ov * N.n + n];
  return (uint64_t)pre | ((uint64_t)post << 16) | ((uint64_t)((uint32_t)na & 0x07ffffffu) << 33) |
         ((uint64_t)ipa << 60);
}

__device__ __forceinline__ uint32_t stat_pre(uint64_t st) { return (uint32_t)(st & 0xffffu); }
__device__ __forceinline__ uint32_t stat_post(uint64_t st) { return (uint32_t)((st >> 16) & 0x1ffffu); }
// weighted NodeAffinity + overlay score
__device__ __forceinline__ int32_t stat_na(uint64_t st) { return (int32_t)((uint32_t)(st >> 33) << 5) >> 5; }
__device__ __forceinline__ int32_t stat_ipa(uint64_t st) { return (int32_t)(st >> 60); }

__device__ __forceinline__ bool sc_fit(const DevNodes& N, const kb_spec& sp, const int64_t* sci, bool has_map,
                                       const int64_t* node_sc, int n) {
  return scalars_fit(N, sp, sci, has_map, node_sc, n);
}

// Reason mask of the full chain from a loaded row + the static cache (0 = fits). RES = false: Session.PredicateFn
// alone, without allocate's resource check (preempt's sweep, preempt.go:189).
template <bool RES = true>
__device__ __forceinline__ uint32_t row_reasons(const DevNodes& N, const DevSpecs& P, const DevCfg& C,
                                                const kb_spec& sp, const int64_t* sci, const Row& r, uint64_t st,
                                                int n) {
  // allocate.go:88: InitResreq <= Idle || InitResreq <= Releasing
  const bool fi = !RES || (le_tol(sp.init_cpu, r.idle_cpu, 10) && le_tol(sp.init_mem, r.idle_mem, 10ll * 1024 * 1024) &&
                           sc_fit(N, sp, sci, r.flags & KB_NODE_IDLE_HAS_MAP, N.idle_sc, n));
  if (!fi) {
    const bool fr = le_tol(sp.init_cpu, r.rel_cpu, 10) && le_tol(sp.init_mem, r.rel_mem, 10ll * 1024 * 1024) &&
                    sc_fit(N, sp, sci, r.flags & KB_NODE_REL_HAS_MAP, N.rel_sc, n);
    if (!fr) return 1u << KB_R_RESOURCE_FIT;
  }
  if (!C.predicates) return stat_post(st);  // the host overlay only
  if (r.max_pods <= r.pod_count) return 1u << KB_R_POD_NUMBER;  // predicates.go:162-166
  const uint32_t pre = stat_pre(st);
  if (pre) return pre;
  // PodFitsHostPorts (vendor/.../predicates.go:1031-1052; cache/host_ports.go:96-125)
  for (uint32_t i = 0; i < sp.port_cnt; ++i) {
    const kb_port p = P.ports[sp.port_off + i];
    const uint64_t used = N.port_used[(size_t)p.slot * N.n + n];
    const uint64_t hit = p.ip == 0 ? used : (used & (1ull | (1ull << p.ip)));
    if (hit) return 1u << KB_R_HOST_PORTS;
  }
  return stat_post(st);
}

// nodeOrderFn (nodeorder.go:188-226) + the InterPodAffinity batch score (:229-246) from the static cache.
// All terms are integers, so the reference's float64 sum equals this int64 sum.
__device__ __forceinline__ int64_t row_score(const DevCfg& C, const kb_spec& sp, const Row& r, uint64_t st) {
  if (!C.nodeorder) return stat_na(st);  // the host overlay's score only
  if (stat_ipa(st) == (int32_t)kIpaErrorField) return kIpaErrorScore;  // batch error: no scores at all
  const int64_t batch = (int64_t)stat_ipa(st) * C.w_pa;
  if (sp.flags & KB_SPEC_NA_ERROR) return batch;  // map fn error: the node keeps only the batch score
  const int64_t rc = sp.nz_cpu + r.nz_cpu, rm = sp.nz_mem + r.nz_mem;
  const int64_t lr = (lr_score(rc, r.alloc_cpu) + lr_score(rm, r.alloc_mem)) / 2;
  const double cf = frac_cap(rc, r.alloc_cpu), mf = frac_cap(rm, r.alloc_mem);
  const int64_t bra = (cf >= 1.0 || mf >= 1.0) ? 0 : (int64_t)((1.0 - fabs(cf - mf)) * 10.0);
  return lr * C.w_lr + bra * C.w_bra + (int64_t)stat_na(st) + batch;
}

// ---- the same scores with the node's reciprocals precomputed (kb_eval: many specs against one node) ----
// leastRequestedScore with the quotient estimated as num * (1 / cap): the estimate is within one of the exact
// quotient (num / cap <= 10, relative error < 2^-51), which the int64 corrections then fix.
__device__ __forceinline__ int64_t lr_score_inv(int64_t req, int64_t cap, double inv) {
  if (cap == 0 || req > cap) return 0;
  const int64_t num = (cap - req) * 10;
  if (cap > 0 && cap < (1ll << 52) && num >= 0 && num < (1ll << 62)) {
    int64_t q = (int64_t)((double)num * inv);
    q = q < 0 ? 0 : (q > 11 ? 11 : q);
    if (q * cap > num) --q;
    if ((q + 1) * cap <= num) ++q;
    return q;
  }
  return num / cap;
}
// BalancedResourceAllocation (balanced_resource_allocation.go:41-77): fractionOfCapacity >= 1 is the integer
// test req >= cap (cap < 2^53); otherwise int((1 - |cf - mf|) * 10) from the reciprocal estimates, which lie
// within 1e-14 of the IEEE quotients -- unless that value is within 1e-9 of an integer, where the IEEE
// divisions decide (the result must be the reference's bit for bit).
__device__ __forceinline__ int64_t bra_score_inv(int64_t rc, int64_t ac, int64_t rm, int64_t am, double ic,
                                                 double im) {
  const bool exactable = ac > 0 && am > 0 && ac < (1ll << 53) && am < (1ll << 53) && rc >= 0 && rm >= 0;
  if (exactable) {
    if (rc >= ac || rm >= am) return 0;
    const double f = (1.0 - fabs((double)rc * ic - (double)rm * im)) * 10.0;
    const double fl = floor(f);
    if (f - fl > 1e-9 && fl + 1.0 - f > 1e-9) return (int64_t)f;
  }
  const double cf = frac_cap(rc, ac), mf = frac_cap(rm, am);
  return (cf >= 1.0 || mf >= 1.0) ? 0 : (int64_t)((1.0 - fabs(cf - mf)) * 10.0);
}
__device__ __forceinline__ int64_t row_score_inv(const DevCfg& C, const kb_spec& sp, const Row& r, uint64_t st,
                                                 double ic, double im) {
  if (!C.nodeorder) return stat_na(st);
  if (stat_ipa(st) == (int32_t)kIpaErrorField) return kIpaErrorScore;
  const int64_t batch = (int64_t)stat_ipa(st) * C.w_pa;
  if (sp.flags & KB_SPEC_NA_ERROR) return batch;
  const int64_t rc = sp.nz_cpu + r.nz_cpu, rm = sp.nz_mem + r.nz_mem;
  const int64_t lr = (lr_score_inv(rc, r.alloc_cpu, ic) + lr_score_inv(rm, r.alloc_mem, im)) / 2;
  const int64_t bra = bra_score_inv(rc, r.alloc_cpu, rm, r.alloc_mem, ic, im);
  return lr * C.w_lr + bra * C.w_bra + (int64_t)stat_na(st) + batch;
}

__device__ __forceinline__ uint64_t make_key(uint32_t reasons, int64_t score, int n) {
  if (reasons) return reasons;
  return kFeasible | ((uint64_t)(score + kScoreBias) << 24) | (uint64_t)(kIdxMask - (uint32_t)n);
}

// ---- wave reductions over 64-bit keys with DPP (identity 0 for max) ----
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
__device__ __forceinline__ uint64_t umax64(uint64_t a, uint64_t b) { return a > b ? a : b; }
// wave-uniform max of v over the 64 lanes (every lane must be active)
__device__ __forceinline__ uint64_t wave_max_dpp(uint64_t v) {
  v = umax64(v, dpp_u64<0xb1>(v));   // quad_perm [1,0,3,2]
  v = umax64(v, dpp_u64<0x4e>(v));   // quad_perm [2,3,0,1]
  v = umax64(v, dpp_u64<0x124>(v));  // row_ror:4
  v = umax64(v, dpp_u64<0x128>(v));  // row_ror:8
  v = umax64(v, dpp_u64<0x142>(v));  // row_bcast:15
  v = umax64(v, dpp_u64<0x143>(v));  // row_bcast:31
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((uint32_t)v, 63);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((uint32_t)(v >> 32), 63);
  return ((uint64_t)hi << 32) | lo;
}

template <bool AFF>
__global__ __launch_bounds__(256) void sweep_keys_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, uint64_t* keys,
                                                         uint64_t* cmax, uint64_t* stat, const JobState* js) {
  if (js != nullptr && js->stopped) return;
  const kb_spec sp = P.specs[spec];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t k = 0;
  if (n < N.n) {
    const Row r = load_row(N, n);
    const uint64_t st = static_eval<AFF>(N, P, C, sp, spec, r.flags, n, P.A.mm);
    stat[n] = st;
    const uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, n);
    k = make_key(rs, rs ? 0 : row_score(C, sp, r, st), n);
    keys[n] = k;
  }
  const uint64_t m = wave_max_u64(k);
  if ((threadIdx.x & 63) == 0 && (n >> 6) < ((N.n + 63) >> 6)) cmax[n >> 6] = m;
}

// L2-coherent load of a key another lane of this wave may have stored earlier in the launch.
__device__ __forceinline__ uint64_t load_key_l2(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void publish_diag(JobState* hjs, const uint64_t* dg, uint64_t rt) {
  for (int k = 0; k < 7; ++k) hjs->diag[k] += dg[k];
  hjs->diag[7] += rt;
}

// Thread 0, after a block barrier that follows every thread's host-buffer writes and system fence.
__device__ __forceinline__ void publish_state(JobState* js, JobState* hjs, int stopped, int stop, int fail_task,
                                              int placed, int ready, int minav, int gang, int panic,
                                              uint32_t seq) {
  js->stopped = stopped;
  js->stop = stop;
  js->fail_task = fail_task;
  js->n_placed = placed;
  js->ready_num = ready;
  js->min_available = minav;
  js->gang_ready = gang;
  js->panic = panic;
  hjs->stopped = stopped;
  hjs->stop = stop;
  hjs->fail_task = fail_task;
  hjs->n_placed = placed;
  hjs->ready_num = ready;
  hjs->min_available = minav;
  hjs->gang_ready = gang;
  hjs->panic = panic;
  // the host spins on seq: a system-scope release orders every earlier write of the workgroup (each wave
  // waited for its stores before the barrier that precedes this call) ahead of it
  __hip_atomic_store(&hjs->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// A launch that finds its batch already stopped still reports completion.
__device__ __forceinline__ bool guard_fails(const SpecGuard& g) {
  if (g.prev == nullptr) return false;
  const JobState* p = g.prev;
  return p->panic != 0 || p->stop != g.stop || p->n_placed != g.placed || p->ready_num != g.ready;
}

__device__ __forceinline__ void signal_skip(JobState* hjs, uint32_t seq) {
  if (threadIdx.x == 0) __hip_atomic_store(&hjs->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#ifdef KB_DIAG
#define KB_STAMP(k)                                   \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    dg[k] += t_ - dg_last;                            \
    dg_last = t_;                                     \
  } while (0)
#else
#define KB_STAMP(k) \
  do {              \
  } while (0)
#endif


// Selection-kernel stamps: KB_DIAG gives its 7 phases; KB_DIAG_SEL splits node selection finer
// (0 key load, 1 reduce, 2 threshold search, 3 scans, 4 compaction, 5 the rest of the segment).
#if defined(KB_DIAG_SEL)
#define KB_SEL_PH(k) KB_STAMP((k) == 0 ? 0 : (k) == 1 ? 4 : (k) == 6 ? 6 : 5)
#define KB_SEL_FINE(k) KB_STAMP(k)
#else
#define KB_SEL_PH(k) KB_STAMP(k)
#define KB_SEL_FINE(k) \
  do {                 \
  } while (0)
#endif
// KB_DIAG builds: fine stamps inside sel_run's e-sequences and winners (dg[8..12]: time, taken from the phase stamp
// that follows) and counts (dg[13] e-sequence rounds, dg[14] winners threshold-search steps, dg[15] candidates K)
#ifdef KB_DIAG
#define KB_SEL_W(k) KB_STAMP(k)
#define KB_SEL_COUNT(k, v) (dg[k] += (uint64_t)(v))
#else
#define KB_SEL_W(k) \
  do {              \
  } while (0)
#define KB_SEL_COUNT(k, v) \
  do {                     \
  } while (0)
#endif

// Copy the buffered placements to the caller's pinned host buffer (coalesced, once per run / buffer).
__device__ __forceinline__ void flush_placements(const uint64_t* pb, int cnt, int base, int32_t* hout, int lane) {
  __syncthreads();
  for (int i = lane; i < cnt; i += 64) {
    const uint64_t v = pb[i];
    hout[2 * (base + i)] = (int32_t)(uint32_t)v;
    hout[2 * (base + i) + 1] = (int32_t)(uint32_t)(v >> 32);
  }
}

// Loop-exit state of wave 0, handed to the whole block through LDS.
struct alignas(16) LoopOut {  // 48 B: keeps the dynamic LDS base 16-B aligned (guide §6 Guideline 17)
  int32_t stop, fail_task, placed, ready, minav, gang, panic, stopped, pb_n, pb_base, pad0, pad1;
};
static_assert(sizeof(LoopOut) % 16 == 0, "static LDS must stay a multiple of 16 B");
constexpr int kLdsLimit = 160 * 1024 - 256;  // dynamic LDS budget next to the small static block

// ONE wave. Runs a job's same-spec tasks: argmax -> commit (Session.Allocate / Pipeline applied to the
// winner's row: NodeInfo.AddTask, api/node_info.go:165-193, + schedulercache AddPod,
// cache/node_info.go:498-520) -> re-key the winner from registers -> re-reduce its chunk.
// The winner's row is read from HBM once per task; the new key needs no reload.
template <bool KEYS_IN_LDS>
__global__ __launch_bounds__(512) void place_loop_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, int t_begin,
                                                        int t_count, uint64_t* keys, const uint64_t* cmax_g,
                                                        const uint64_t* stat, JobState* js, int first, int ready0,
                                                        int minav0, int gang0, int32_t* hout, JobState* hjs,
                                                        int pb_cap, uint32_t seq) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  __shared__ LoopOut lo;
  if (!first && js->stopped) {
    signal_skip(hjs, seq);
    return;
  }
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int n = N.n;
  const int M = (n + 63) >> 6;
  const int Mp = (M + 1) & ~1;
  uint64_t* cm = lds;                // [Mp] chunk maxima
  uint64_t* pb = lds + Mp;           // [pb_cap] buffered placements (node | kind << 32)
  uint64_t* lk = lds + Mp + pb_cap;  // [n] keys (KEYS_IN_LDS)
  int pb_n = 0, pb_base = t_begin;   // placements buffered since the last flush
  for (int c = tid; c < M; c += 512) cm[c] = cmax_g[c];
  if (KEYS_IN_LDS) {
#pragma unroll 4
    for (int i = tid; i < n; i += 512) lk[i] = keys[i];
  }
  __syncthreads();
  if (tid < 64) {  // only wave 0 runs the sequential loop
  uint64_t lmax = 0;  // max over the chunks this lane owns (c = lane + 64 j)
  for (int c = lane; c < M; c += 64) lmax = umax64(lmax, cm[c]);

  const kb_spec sp = P.specs[spec];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  int ready, minav, gang, placed;
  if (first) {
    ready = ready0;
    minav = minav0;
    gang = gang0;
    placed = 0;
  } else {
    ready = js->ready_num;
    minav = js->min_available;
    gang = js->gang_ready;
    placed = js->n_placed;
  }

  int pw = -1;  // previous winner whose row stores are still pending (lane 0)
  Row pr{};
  uint64_t pst = 0;
#ifdef KB_DIAG
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  for (int t = 0; t < t_count; ++t) {
    KB_STAMP(5);
    const uint64_t best = wave_max_dpp(lmax);
    KB_STAMP(0);
    if (!(best & kFeasible)) {
      // PredicateNodes found nothing (allocate.go:150-153): FitErrors histogram over all nodes.
      uint32_t cnt[KB_NUM_REASONS];
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) cnt[b] = 0;
      for (int i = lane; i < n; i += 64) {
        const uint64_t k = KEYS_IN_LDS ? lk[i] : load_key_l2(&keys[i]);
#pragma unroll
        for (int b = 0; b < KB_NUM_REASONS; ++b) cnt[b] += (uint32_t)(k >> b) & 1u;
      }
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) {
        const uint32_t s = wave_sum_u32(cnt[b]);
        if (lane == 0) {
          js->hist[b] = s;
          hjs->hist[b] = s;
        }
      }
      if (lane == 0 && pw >= 0) store_row(N, pw, pr);
#ifdef KB_DIAG
      if (lane == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
      if (lane == 0) lo = LoopOut{KB_STOP_NO_FIT, t_begin + t, placed, ready, minav, gang, 0, 1, pb_n, pb_base, 0, 0};
      goto done;
    }
    const int64_t score = (int64_t)((best >> 24) & ((1ull << 39) - 1)) - kScoreBias;
    if (score <= -1) {  // SelectBestNode: no bucket with score > -1 -> the reference panics
      if (lane == 0 && pw >= 0) store_row(N, pw, pr);
      if (lane == 0) lo = LoopOut{KB_STOP_DONE, t_begin + t, placed, ready, minav, gang, 1, 1, pb_n, pb_base, 0, 0};
      goto done;
    }
    const int w = (int)(kIdxMask - (uint32_t)(best & kIdxMask));

    uint64_t nk = 0;
    int kind = 0;
    if (lane == 0) {
      // The winner's row: from registers when it won the previous task too, else one batch of loads.
      Row r;
      uint64_t st;
      if (w == pw) {
        r = pr;
        st = pst;
      } else {
        r = load_row(N, w);
        st = stat[w];
        // The previous winner's stores are issued only now, after these loads, so waiting on the
        // loads does not also wait for their acknowledgement (stores and loads share vmcnt).
        if (pw >= 0) store_row(N, pw, pr);
      }
#ifdef KB_DIAG
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      KB_STAMP(1);
      // allocate.go:159: Allocate when InitResreq fits Idle, else Pipeline onto Releasing (:172)
      const bool to_idle = le_tol(sp.init_cpu, r.idle_cpu, 10) &&
                           le_tol(sp.init_mem, r.idle_mem, 10ll * 1024 * 1024) &&
                           scalars_fit(N, sp, sci, r.flags & KB_NODE_IDLE_HAS_MAP, N.idle_sc, w);
      if (to_idle) {
        r.idle_cpu -= sp.req_cpu;
        r.idle_mem -= sp.req_mem;
        if (r.flags & KB_NODE_IDLE_HAS_MAP) {  // Sub leaves a nil map alone (resource_info.go:152-157)
          uint64_t m = sp.req_sc_mask;
          while (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            N.idle_sc[(size_t)q * n + w] -= scr[q];
          }
        }
        kind = KB_PLACE_ALLOCATE;
      } else {
        r.rel_cpu -= sp.req_cpu;
        r.rel_mem -= sp.req_mem;
        if (r.flags & KB_NODE_REL_HAS_MAP) {
          uint64_t m = sp.req_sc_mask;
          while (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            N.rel_sc[(size_t)q * n + w] -= scr[q];
          }
        }
        kind = KB_PLACE_PIPELINE;
      }
      r.pod_count += 1;
      r.nz_cpu += sp.nz_cpu;
      r.nz_mem += sp.nz_mem;
      for (uint32_t i = 0; i < sp.port_cnt; ++i) {  // UpdateUsedPorts (cache/node_info.go:593-606)
        const kb_port p = P.ports[sp.port_off + i];
        N.port_used[(size_t)p.slot * n + w] |= 1ull << p.ip;
      }
      const uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, w);
      nk = make_key(rs, rs ? 0 : row_score(C, sp, r, st), w);
      if (KEYS_IN_LDS) lk[w] = nk;
      else keys[w] = nk;
      pw = w;
      pr = r;
      pst = st;
      pb[pb_n] = (uint32_t)w | ((uint64_t)(uint32_t)kind << 32);
      KB_STAMP(2);
    }
    nk = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)(nk >> 32), 0) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readlane((uint32_t)nk, 0);
    kind = __builtin_amdgcn_readlane(kind, 0);
    if (!KEYS_IN_LDS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");

    // Re-reduce the winner's chunk; its owner lane refreshes its running max.
    const int c = w >> 6;
    const int i = (c << 6) + lane;
    uint64_t v = 0;
    if (i < n) v = (i == w) ? nk : (KEYS_IN_LDS ? lk[i] : load_key_l2(&keys[i]));
    v = wave_max_dpp(v);
    KB_STAMP(3);
    if (lane == (c & 63)) {
      cm[c] = v;
      uint64_t mx = 0;
      for (int cc = lane; cc < M; cc += 64) mx = umax64(mx, cm[cc]);
      lmax = mx;
    }
    KB_STAMP(4);

    ++placed;
    ++pb_n;
    if (kind == KB_PLACE_ALLOCATE) ++ready;
    if (!gang || ready >= minav) {  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
      if (lane == 0 && pw >= 0) store_row(N, pw, pr);
#ifdef KB_DIAG
      if (lane == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
      if (lane == 0) lo = LoopOut{KB_STOP_READY, -1, placed, ready, minav, gang, 0, 1, pb_n, pb_base, 0, 0};
      goto done;
    }
    if (pb_n == pb_cap) {
      for (int k = lane; k < pb_n; k += 64) {
        const uint64_t e = pb[k];
        hout[2 * (pb_base + k)] = (int32_t)(uint32_t)e;
        hout[2 * (pb_base + k) + 1] = (int32_t)(uint32_t)(e >> 32);
      }
      pb_base += pb_n;
      pb_n = 0;
    }
  }
  if (lane == 0 && pw >= 0) store_row(N, pw, pr);
#ifdef KB_DIAG
  if (lane == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
  if (lane == 0) lo = LoopOut{KB_STOP_DONE, -1, placed, ready, minav, gang, 0, 0, pb_n, pb_base, 0, 0};
  }
done:
  __syncthreads();
  for (int k = tid; k < lo.pb_n; k += 512) {
    const uint64_t v = pb[k];
    hout[2 * (lo.pb_base + k)] = (int32_t)(uint32_t)v;
    hout[2 * (lo.pb_base + k) + 1] = (int32_t)(uint32_t)(v >> 32);
  }
  __threadfence_system();
  __syncthreads();
  if (tid == 0)
    publish_state(js, hjs, lo.stopped, lo.stop, lo.fail_task, lo.placed, lo.ready, lo.minav, lo.gang, lo.panic,
                  seq);
}

// Parity / snapshot sweep (kb_eval): reasons + scores for T specs x N nodes. Node-stationary: a thread
// loads its node's row once and evaluates kEvalSpecs specs against it (the spec fields are wave-uniform:
// scalar loads), writing one coalesced 4 B + 8 B pair per spec. HBM traffic is the 12 B/pair of output; the
// 76 B row is read once per kEvalSpecs specs.
constexpr int kEvalSpecs = 16;
template <bool AFF, class SCORE>
__global__ __launch_bounds__(256) void eval_kernel(DevNodes N, DevSpecs P, DevCfg C, const int32_t* spec_ids, int t,
                                                   uint32_t* reasons, SCORE* scores, const int64_t* mm) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N.n) return;
  const int j0 = blockIdx.y * kEvalSpecs;
  const int j1 = j0 + kEvalSpecs < t ? j0 + kEvalSpecs : t;
  const Row r = load_row(N, n);
  const double ic = 1.0 / (double)r.alloc_cpu, im = 1.0 / (double)r.alloc_mem;  // once per node
  for (int j = j0; j < j1; ++j) {
    const int s = spec_ids[j];
    const kb_spec sp = P.specs[s];
    const uint64_t st = static_eval<AFF>(N, P, C, sp, s, r.flags, n, AFF ? mm + 2 * j : nullptr);
    reasons[(size_t)j * N.n + n] = row_reasons(N, P, C, sp, P.sc_init + (size_t)s * N.S, r, st, n);
    scores[(size_t)j * N.n + n] = (SCORE)row_score_inv(C, sp, r, st, ic, im);
  }
}

// kb_eval over a batch of plain specs (the host checks, kb_ctx::spec_plain: no nodeSelector, node affinity, host
// ports, scalar requests, inter-pod terms or overlay, requests below 2^49, and one taint set that every spec
// tolerates). The chain then reads only the row: resource fit, pod count, the node's conditions and pressure,
// LeastRequested + Balanced. The node-only parts are computed once per node; the specs' requests are staged in LDS
// once per block, so the per-spec loop has no dependent scalar loads and no spec-dependent branches. Rows whose
// values lie below 2^49 (all real ones) take the loop in f64, which is exact there: every sum, difference and
// tenfold product of such integers is an integer below 2^53, the LeastRequested quotient is floored from a
// reciprocal estimate and corrected by one exact fma remainder, and Balanced keeps bra_score_inv's estimate with
// its IEEE-division fallback near integers. Other rows take the int64 forms. Same values as eval_kernel on such
// specs (tests/test_gpu_parity.py::test_eval_plain_equals_general, test_eval_plain_matches_oracle).
#ifdef KB_EVAL_TEMPORAL
constexpr int kEvalAux = 0;  // (A/B builds: ordinary stores)
#else
constexpr int kEvalAux = 2;  // buffer stores' cache policy: nt (the output is streamed once, never read back here)
#endif
constexpr int kEvalPlainSpecs = 64;  // (one resident round at 50k nodes needs 43: eval_plain_spb)
constexpr double kPlainMax = 562949953421312.0;  // 2^49
// leastRequestedScore (least_requested.go:36-53) on integers below 2^49 held in doubles. num = (cap - req) * 10
// arrives as the node's (cap - nz_node) * 10 minus the spec's nz * 10 (exact), so req > cap is num < 0. The
// quotient is truncated from a reciprocal estimate (the floor, or one off when num / cap lies within 2^-48 of an
// integer) and corrected by the exact remainder (fma: num - q * cap is an integer below 2^53). cap == 0: the
// caller's node flag.
__device__ __forceinline__ int lr_score_f64(double num, double cap, double inv) {
  const int qe = (int)(num * inv);
  const double rem = fma(-(double)qe, cap, num);
  const int q = qe + (rem >= cap ? 1 : 0) - (rem < 0.0 ? 1 : 0);
  return num < 0.0 ? 0 : q;
}
// The same quotient from a reciprocal biased up by 2^-50 (inv_up = RN(RN(1/cap) * (1 + 2^-50))): num * inv_up then
// exceeds num / cap for num > 0 (the three roundings lose less than 3 * 2^-53 relative) by less than 10 * 2^-49
// (num / cap <= 10), so its truncation is the floor or one above it, and the one exact remainder test corrects it
// (num < 0, req > cap: score 0, as in lr_score_f64; the quotient there may saturate the conversion, hence the
// unsigned step). Two VALU instructions fewer per call than lr_score_f64 (eval_plain_kernel's loop).
__device__ __forceinline__ int lr_score_up(double num, double cap, double inv_up) {
  const int qe = (int)(num * inv_up);
  const double rem = fma(-(double)qe, cap, num);
  const int q = (int)((uint32_t)qe - (rem < 0.0 ? 1u : 0u));
  return num < 0.0 ? 0 : q;
}
constexpr double kInvUp = 1.0 + 0x1p-50;
// BalancedResourceAllocation (balanced_resource_allocation.go:41-77) as bra_score_inv, on such doubles: with
// positive capacities (pos) f = 10 - |rc * 10/ac - rm * 10/am| estimates (1 - |cf - mf|) * 10 within 1e-14, which
// decides the truncation unless f lies within 1e-9 of an integer; then (and for other capacities) the IEEE
// divisions of the reference
__device__ __forceinline__ int bra_score_f64(double rc, double ac, double rm, double am, double ic10, double im10,
                                             bool pos) {
  if (pos) {
    if (rc >= ac || rm >= am) return 0;
    const double f = 10.0 - fabs(fma(rc, ic10, -(rm * im10)));
    const double fr = f - floor(f);
    if (fr > 1e-9 && fr < 1.0 - 1e-9) return (int)f;  // f in [0, 10]: truncation is the floor
  }
  const double cf = ac == 0.0 ? 1.0 : rc / ac, mf = am == 0.0 ? 1.0 : rm / am;
  return (cf >= 1.0 || mf >= 1.0) ? 0 : (int)((1.0 - fabs(cf - mf)) * 10.0);
}
// BUF: the output arrays take under 4 GiB (launch_eval_t): the loop's stores are buffer stores with the row's
// offset in a scalar register (soffset) and the lane's node offset fixed in a VGPR -- no per-store 64-bit address
// arithmetic on the VALU, which this kernel is bound by beside the stores.
template <class SCORE, bool BUF = false>
__global__ __launch_bounds__(256) void eval_plain_kernel(DevNodes N, DevSpecs P, DevCfg C, const int32_t* spec_ids,
                                                         int t, int spb, uint32_t* reasons, SCORE* scores) {
  __shared__ int64_t s_req[4][kEvalPlainSpecs];  // init cpu, init mem, non-zero cpu, non-zero mem
  __shared__ double s_dreq[4][kEvalPlainSpecs];  // init cpu, init mem as doubles; non-zero cpu, mem x 10 (exact)
  __shared__ double s_dnz[2][kEvalPlainSpecs];   // non-zero cpu, mem as doubles
  __shared__ uint32_t s_bem[kEvalPlainSpecs];    // BestEffort: all ones
  __shared__ SCORE s_tab[11 * 11];  // lr * w_lr + bra * w_bra for lr, bra in 0..10 (all 0 without nodeorder)
  const int j0 = blockIdx.y * spb;
  const int nj = t - j0 < spb ? t - j0 : spb;
#ifdef KB_EVAL_NPT2
  const int n = (blockIdx.x * blockDim.x + threadIdx.x) * 2;  // (A/B store probe: two nodes per lane)
#elif defined(KB_EVAL_RUN4)
  const int n = blockIdx.x * blockDim.x * 4 + threadIdx.x;  // (A/B store probe: 4 nodes per lane, 256 apart)
#else
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
#endif
  // the node's row first: its loads overlap the specs' staging (two dependent loads) below
  Row r;
  if (n < N.n) r = load_row(N, n);
  if ((int)threadIdx.x < nj) {
    const kb_spec sp = P.specs[spec_ids[j0 + threadIdx.x]];
    s_req[0][threadIdx.x] = sp.init_cpu;
    s_req[1][threadIdx.x] = sp.init_mem;
    s_req[2][threadIdx.x] = sp.nz_cpu;
    s_req[3][threadIdx.x] = sp.nz_mem;
    s_dreq[0][threadIdx.x] = (double)sp.init_cpu;
    s_dreq[1][threadIdx.x] = (double)sp.init_mem;
    s_dreq[2][threadIdx.x] = (double)sp.nz_cpu * 10.0;
    s_dreq[3][threadIdx.x] = (double)sp.nz_mem * 10.0;
    s_dnz[0][threadIdx.x] = (double)sp.nz_cpu;
    s_dnz[1][threadIdx.x] = (double)sp.nz_mem;
    s_bem[threadIdx.x] = (sp.flags & KB_SPEC_BEST_EFFORT) ? ~0u : 0u;
  }
  if (threadIdx.x >= 128 && threadIdx.x < 128 + 121) {
    const int q = (int)threadIdx.x - 128;
    s_tab[q] = C.nodeorder ? (SCORE)(q / 11) * (SCORE)C.w_lr + (SCORE)(q % 11) * (SCORE)C.w_bra : (SCORE)0;
  }
  __syncthreads();
  if (n >= N.n) return;
  // row_reasons after the resource check, per node: pod count, conditions (static_eval's pre), then the post
  // reasons (no taints: the one taint set is tolerated) -- memory pressure for BestEffort specs only
  uint32_t after = 0, post_be = 0;
  if (C.predicates) {
    const uint32_t f = r.flags;
    const uint32_t pre = f & ((1u << KB_R_NOT_READY) | (1u << KB_R_OUT_OF_DISK) | (1u << KB_R_NETWORK_UNAVAILABLE) |
                              (1u << KB_R_UNSCHEDULABLE));
    uint32_t post = 0;
    if (C.disk_pressure && (f & KB_NODE_DISK_PRESSURE)) post = 1u << KB_R_DISK_PRESSURE;
    else if (C.pid_pressure && (f & KB_NODE_PID_PRESSURE)) post = 1u << KB_R_PID_PRESSURE;
    post_be = (C.mem_pressure && (f & KB_NODE_MEM_PRESSURE)) ? 1u << KB_R_MEMORY_PRESSURE : post;
    after = r.max_pods <= r.pod_count ? 1u << KB_R_POD_NUMBER : (pre ? pre : post);
    if (r.max_pods <= r.pod_count || pre) post_be = after;
  }
  const size_t stride = (size_t)N.n;
  const double d_ic = (double)r.idle_cpu, d_im = (double)r.idle_mem, d_rc = (double)r.rel_cpu,
               d_rm = (double)r.rel_mem, d_nc = (double)r.nz_cpu, d_nm = (double)r.nz_mem,
               d_ac = (double)r.alloc_cpu, d_am = (double)r.alloc_mem;
  const double inv_c = 1.0 / d_ac, inv_m = 1.0 / d_am;
  const bool fast = fabs(d_ic) < kPlainMax && fabs(d_im) < kPlainMax && fabs(d_rc) < kPlainMax &&
                    fabs(d_rm) < kPlainMax && fabs(d_nc) < kPlainMax && fabs(d_nm) < kPlainMax &&
                    fabs(d_ac) < kPlainMax && fabs(d_am) < kPlainMax;
  if (fast) {
    // LessEqual's tolerance folded into the node's side once: r - avail < tol <=> r < avail + tol (exact here)
    const double t_ic = d_ic + 10.0, t_im = d_im + 10485760.0, t_rc = d_rc + 10.0, t_rm = d_rm + 10485760.0;
    const bool pos = d_ac > 0.0 && d_am > 0.0;
    // LeastRequested's operands with the zero-capacity case folded in: numerator -1 (minus the spec's nz * 10, so
    // always negative: score 0), capacity and reciprocal 1
    const bool zc = d_ac == 0.0, zm = d_am == 0.0;
    const double num_c = zc ? -1.0 : (d_ac - d_nc) * 10.0, num_m = zm ? -1.0 : (d_am - d_nm) * 10.0;
    const double cap_c = zc ? 1.0 : d_ac, cap_m = zm ? 1.0 : d_am;
    const double lc_inv = zc ? 1.0 : inv_c, lm_inv = zm ? 1.0 : inv_m;
    const double lc_up = lc_inv * kInvUp, lm_up = lm_inv * kInvUp;  // (lr_score_up)
    // Balanced's estimate on positive capacities only (elsewhere every spec takes the fallback)
    const double ic10 = pos ? 10.0 / d_ac : 0.0, im10 = pos ? 10.0 / d_am : 0.0;
    // The unrolled iterations' LDS reads and f64 chains interleave; Balanced's IEEE-division fallback (f within 1e-9
    // of an integer, or a capacity <= 0) is a branch the wave skips unless one of its lanes needs it
    // (BUF) the output arrays as buffer resources: raw, whole-array record counts (< 4 GiB: launch_eval_t)
    const uint32_t out_pairs = (uint32_t)t * (uint32_t)stride;
    const __amdgpu_buffer_rsrc_t rbuf = __builtin_amdgcn_make_buffer_rsrc(reasons, (short)0, (int)(out_pairs * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t sbuf =
        __builtin_amdgcn_make_buffer_rsrc(scores, (short)0, (int)(out_pairs * (uint32_t)sizeof(SCORE)), 0x00020000);
#pragma unroll 4
    for (int j = 0; j < nj; ++j) {
      const double icpu = s_dreq[0][j], imem = s_dreq[1][j], nzc10 = s_dreq[2][j], nzm10 = s_dreq[3][j];
      const double nzc = s_dnz[0][j], nzm = s_dnz[1][j];
      const uint32_t bem = s_bem[j];
      const bool fit = ((icpu < t_ic) & (imem < t_im)) | ((icpu < t_rc) & (imem < t_rm));
      const uint32_t fm = 0u - (uint32_t)fit;
      const uint32_t rs = (((post_be & bem) | (after & ~bem)) & fm) | ((1u << KB_R_RESOURCE_FIT) & ~fm);
      // row_score_inv with no NodeAffinity, overlay or InterPodAffinity term (the table is 0 without nodeorder)
      const int lc = lr_score_up(num_c - nzc10, cap_c, lc_up);
      const int lm = lr_score_up(num_m - nzm10, cap_m, lm_up);
      const double rc = nzc + d_nc, rm = nzm + d_nm;
      const bool over = (rc >= d_ac) | (rm >= d_am);
      const double f = 10.0 - fabs(fma(rc, ic10, -(rm * im10)));  // in [0, 10]
      const double fr = f - floor(f);
      const bool po = pos & over;
      const bool est = pos & !over & (fr > 1e-9) & (fr < 1.0 - 1e-9);
      const bool fbit = !est & !po;
      // (kb_eval32's host check bounds the int32 sum; kb_eval sums in int64)
      SCORE score = s_tab[((lc + lm) >> 1) * 11 + (po ? 0 : (int)f)];
      // Balanced's IEEE-division fallback (f within 1e-9 of an integer, or a capacity <= 0): rare, in place -- a
      // branch the wave skips when no lane takes it (a deferred bit per spec cost more VALU per pair than it saved)
      if (fbit && C.nodeorder) [[unlikely]]
        score = s_tab[((lc + lm) >> 1) * 11 + bra_score_f64(rc, d_ac, rm, d_am, 0.0, 0.0, false)];
      // uniform row bases: the stores take a scalar base and the lane's offset; non-temporal (the output is
      // streamed once, never read back by this kernel: no point keeping it in the caches)
      if constexpr (BUF) {
        const uint32_t orow = (uint32_t)(j0 + j) * (uint32_t)stride;  // (uniform: scalar)
#if defined(KB_EVAL_STOREONLY) && defined(KB_EVAL_NPT2)
        {
          typedef unsigned int v2u __attribute__((ext_vector_type(2)));
          const v2u rv = {(unsigned)(n ^ j), (unsigned)((n + 1) ^ j)};
          const v2u sv = {(unsigned)(n + j), (unsigned)(n + 1 + j)};
          __builtin_amdgcn_raw_buffer_store_b64(rv, rbuf, n * 4, (int)(orow * 4u), kEvalAux);
          __builtin_amdgcn_raw_buffer_store_b64(sv, sbuf, n * 4, (int)(orow * 4u), kEvalAux);
          (void)rs;
          (void)score;
          continue;
        }
#endif
#if defined(KB_EVAL_STOREONLY) && defined(KB_EVAL_RUN4)
        // (one 4 KB run per spec row per workgroup instead of 1 KB)
        for (int k = 0; k < 4; ++k) {
          const int nk = n + k * 256;
          if (nk < N.n) {
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(nk ^ j), rbuf, nk * 4, (int)(orow * 4u), kEvalAux);
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)(nk + j), sbuf, nk * 4, (int)(orow * 4u), kEvalAux);
          }
        }
        (void)rs;
        (void)score;
        continue;
#endif
#if defined(KB_EVAL_STOREONLY)
        const uint32_t rs_v = (uint32_t)(n ^ j);
        const SCORE sc_v = (SCORE)(n + j);
#else
        const uint32_t rs_v = rs;
        const SCORE sc_v = score;
#endif
        __builtin_amdgcn_raw_buffer_store_b32(rs_v, rbuf, n * 4, (int)(orow * 4u), kEvalAux);
        if constexpr (sizeof(SCORE) == 4) {
          __builtin_amdgcn_raw_buffer_store_b32((uint32_t)sc_v, sbuf, n * 4, (int)(orow * 4u), kEvalAux);
        } else {
          typedef unsigned int v2u __attribute__((ext_vector_type(2)));
          const v2u sv = {(unsigned)(uint64_t)sc_v, (unsigned)((uint64_t)sc_v >> 32)};
          __builtin_amdgcn_raw_buffer_store_b64(sv, sbuf, n * 8, (int)(orow * 8u), kEvalAux);
        }
        continue;
      }
      uint32_t* rrow = reasons + (size_t)(j0 + j) * stride;
      SCORE* srow = scores + (size_t)(j0 + j) * stride;
#if defined(KB_EVAL_STOREONLY)  // (A/B builds: the stores alone, no compute -- the kernel's store bound)
      __builtin_nontemporal_store((uint32_t)(n ^ j), rrow + n);
      __builtin_nontemporal_store((SCORE)(n + j), srow + n);
      (void)rs;
      (void)score;
#elif !defined(KB_EVAL_TEMPORAL)
      __builtin_nontemporal_store(rs, rrow + n);
      __builtin_nontemporal_store(score, srow + n);
#else  // (A/B builds: the plain stores)
      rrow[n] = rs;
      srow[n] = score;
#endif
    }
    return;
  }
  for (int j = 0; j < nj; ++j) {
    const int64_t icpu = s_req[0][j], imem = s_req[1][j];
    const bool fit = (le_tol(icpu, r.idle_cpu, 10) && le_tol(imem, r.idle_mem, 10ll * 1024 * 1024)) ||
                     (le_tol(icpu, r.rel_cpu, 10) && le_tol(imem, r.rel_mem, 10ll * 1024 * 1024));
    const uint32_t rs = !fit ? 1u << KB_R_RESOURCE_FIT : (s_bem[j] ? post_be : after);
    int64_t score = 0;
    if (C.nodeorder) {
      const int64_t rc = s_req[2][j] + r.nz_cpu, rm = s_req[3][j] + r.nz_mem;
      const int64_t lr = (lr_score_inv(rc, r.alloc_cpu, inv_c) + lr_score_inv(rm, r.alloc_mem, inv_m)) / 2;
      score = lr * C.w_lr + bra_score_inv(rc, r.alloc_cpu, rm, r.alloc_mem, inv_c, inv_m) * C.w_bra;
    }
    reasons[(size_t)(j0 + j) * stride + n] = rs;
    scores[(size_t)(j0 + j) * stride + n] = (SCORE)score;
  }
}

// eval_plain_kernel with four consecutive nodes per lane (eval_plain4_kernel): the same per-pair arithmetic, but each
// spec row gets one 16-byte store per lane (reasons; scores: one per 4 B of score) -- a wave writes 1 KB of a row
// per store instruction instead of 256 B, the streaming-store form (MI355X_MICROARCH.md's HBM section), and the four
// nodes' f64 chains are independent work for the same wave. An A/B build (-DKB_EVAL_VEC4, `make evalv4`): taken
// there when N % 4 == 0 (rows start 16-byte aligned and no lane's four nodes straddle two rows) and the output fits
// buffer offsets (launch_eval_t). Measured 36.2 us against 34.2-41.0 us for eval_plain_kernel at 256 x 50k (r06v):
// 214 VGPRs leave two waves per SIMD, and the VALU work per pair is unchanged, so it stays the default's bound.
struct PlainNode {  // a node's side of eval_plain_kernel's fast loop
  uint32_t after, post_be;
  double num_c, num_m, cap_c, cap_m, lc_inv, lm_inv, ic10, im10, t_ic, t_im, t_rc, t_rm, d_nc, d_nm, d_ac, d_am;
  bool pos;
};
// false when some operand leaves the exact-double range (the lane then takes the int64 loop for its four nodes)
__device__ __forceinline__ bool plain_node_init(PlainNode& p, const Row& r, const DevCfg& C) {
  p.after = 0;
  p.post_be = 0;
  if (C.predicates) {
    const uint32_t f = r.flags;
    const uint32_t pre = f & ((1u << KB_R_NOT_READY) | (1u << KB_R_OUT_OF_DISK) | (1u << KB_R_NETWORK_UNAVAILABLE) |
                              (1u << KB_R_UNSCHEDULABLE));
    uint32_t post = 0;
    if (C.disk_pressure && (f & KB_NODE_DISK_PRESSURE)) post = 1u << KB_R_DISK_PRESSURE;
    else if (C.pid_pressure && (f & KB_NODE_PID_PRESSURE)) post = 1u << KB_R_PID_PRESSURE;
    p.post_be = (C.mem_pressure && (f & KB_NODE_MEM_PRESSURE)) ? 1u << KB_R_MEMORY_PRESSURE : post;
    p.after = r.max_pods <= r.pod_count ? 1u << KB_R_POD_NUMBER : (pre ? pre : post);
    if (r.max_pods <= r.pod_count || pre) p.post_be = p.after;
  }
  const double d_ic = (double)r.idle_cpu, d_im = (double)r.idle_mem, d_rc = (double)r.rel_cpu,
               d_rm = (double)r.rel_mem;
  p.d_nc = (double)r.nz_cpu;
  p.d_nm = (double)r.nz_mem;
  p.d_ac = (double)r.alloc_cpu;
  p.d_am = (double)r.alloc_mem;
  const bool fast = fabs(d_ic) < kPlainMax && fabs(d_im) < kPlainMax && fabs(d_rc) < kPlainMax &&
                    fabs(d_rm) < kPlainMax && fabs(p.d_nc) < kPlainMax && fabs(p.d_nm) < kPlainMax &&
                    fabs(p.d_ac) < kPlainMax && fabs(p.d_am) < kPlainMax;
  p.t_ic = d_ic + 10.0;
  p.t_im = d_im + 10485760.0;
  p.t_rc = d_rc + 10.0;
  p.t_rm = d_rm + 10485760.0;
  p.pos = p.d_ac > 0.0 && p.d_am > 0.0;
  const bool zc = p.d_ac == 0.0, zm = p.d_am == 0.0;
  p.num_c = zc ? -1.0 : (p.d_ac - p.d_nc) * 10.0;
  p.num_m = zm ? -1.0 : (p.d_am - p.d_nm) * 10.0;
  p.cap_c = zc ? 1.0 : p.d_ac;
  p.cap_m = zm ? 1.0 : p.d_am;
  p.lc_inv = zc ? 1.0 : 1.0 / p.d_ac;
  p.lm_inv = zm ? 1.0 : 1.0 / p.d_am;
  p.ic10 = p.pos ? 10.0 / p.d_ac : 0.0;
  p.im10 = p.pos ? 10.0 / p.d_am : 0.0;
  return fast;
}
// one (spec, node) pair of the fast loop: eval_plain_kernel's body; fb = Balanced's IEEE fallback is due
template <class SCORE>
__device__ __forceinline__ void plain_pair(const PlainNode& p, double icpu, double imem, double nzc10, double nzm10,
                                           double nzc, double nzm, uint32_t bem, const SCORE* s_tab, uint32_t& rs,
                                           SCORE& score, bool& fb) {
  const bool fit = ((icpu < p.t_ic) & (imem < p.t_im)) | ((icpu < p.t_rc) & (imem < p.t_rm));
  const uint32_t fm = 0u - (uint32_t)fit;
  rs = (((p.post_be & bem) | (p.after & ~bem)) & fm) | ((1u << KB_R_RESOURCE_FIT) & ~fm);
  const int lc = lr_score_f64(p.num_c - nzc10, p.cap_c, p.lc_inv);
  const int lm = lr_score_f64(p.num_m - nzm10, p.cap_m, p.lm_inv);
  const double rc = nzc + p.d_nc, rm = nzm + p.d_nm;
  const bool over = (rc >= p.d_ac) | (rm >= p.d_am);
  const double f = 10.0 - fabs(fma(rc, p.ic10, -(rm * p.im10)));
  const double fr = f - floor(f);
  const bool po = p.pos & over;
  const bool est = p.pos & !over & (fr > 1e-9) & (fr < 1.0 - 1e-9);
  fb = !est & !po;
  score = s_tab[((lc + lm) >> 1) * 11 + (po ? 0 : (int)f)];
}
template <class SCORE>
__global__ __launch_bounds__(256) void eval_plain4_kernel(DevNodes N, DevSpecs P, DevCfg C, const int32_t* spec_ids,
                                                          int t, int spb, uint32_t* reasons, SCORE* scores) {
  __shared__ int64_t s_req[4][kEvalPlainSpecs];
  __shared__ double s_dreq[4][kEvalPlainSpecs];
  __shared__ double s_dnz[2][kEvalPlainSpecs];
  __shared__ uint32_t s_bem[kEvalPlainSpecs];
  __shared__ SCORE s_tab[11 * 11];
  const int j0 = blockIdx.y * spb;
  const int nj = t - j0 < spb ? t - j0 : spb;
  const int n0 = (blockIdx.x * blockDim.x + threadIdx.x) * 4;  // (N % 4 == 0: all four nodes or none)
  Row r[4];
  if (n0 < N.n) {
#pragma unroll
    for (int k = 0; k < 4; ++k) r[k] = load_row(N, n0 + k);
  }
  if ((int)threadIdx.x < nj) {
    const kb_spec sp = P.specs[spec_ids[j0 + threadIdx.x]];
    s_req[0][threadIdx.x] = sp.init_cpu;
    s_req[1][threadIdx.x] = sp.init_mem;
    s_req[2][threadIdx.x] = sp.nz_cpu;
    s_req[3][threadIdx.x] = sp.nz_mem;
    s_dreq[0][threadIdx.x] = (double)sp.init_cpu;
    s_dreq[1][threadIdx.x] = (double)sp.init_mem;
    s_dreq[2][threadIdx.x] = (double)sp.nz_cpu * 10.0;
    s_dreq[3][threadIdx.x] = (double)sp.nz_mem * 10.0;
    s_dnz[0][threadIdx.x] = (double)sp.nz_cpu;
    s_dnz[1][threadIdx.x] = (double)sp.nz_mem;
    s_bem[threadIdx.x] = (sp.flags & KB_SPEC_BEST_EFFORT) ? ~0u : 0u;
  }
  if (threadIdx.x >= 128 && threadIdx.x < 128 + 121) {
    const int q = (int)threadIdx.x - 128;
    s_tab[q] = C.nodeorder ? (SCORE)(q / 11) * (SCORE)C.w_lr + (SCORE)(q % 11) * (SCORE)C.w_bra : (SCORE)0;
  }
  __syncthreads();
  if (n0 >= N.n) return;
  const uint32_t stride = (uint32_t)N.n;
  PlainNode p[4];
  bool fast = true;
#pragma unroll
  for (int k = 0; k < 4; ++k) fast &= plain_node_init(p[k], r[k], C);
  if (fast) {
    const uint32_t out_pairs = (uint32_t)t * stride;
    const __amdgpu_buffer_rsrc_t rbuf = __builtin_amdgcn_make_buffer_rsrc(reasons, (short)0, (int)(out_pairs * 4u), 0x00020000);
    const __amdgpu_buffer_rsrc_t sbuf =
        __builtin_amdgcn_make_buffer_rsrc(scores, (short)0, (int)(out_pairs * (uint32_t)sizeof(SCORE)), 0x00020000);
    uint64_t fb[4] = {0, 0, 0, 0};
    typedef unsigned int v4u __attribute__((ext_vector_type(4)));
#pragma unroll 1
    for (int j = 0; j < nj; ++j) {
      const double icpu = s_dreq[0][j], imem = s_dreq[1][j], nzc10 = s_dreq[2][j], nzm10 = s_dreq[3][j];
      const double nzc = s_dnz[0][j], nzm = s_dnz[1][j];
      const uint32_t bem = s_bem[j];
      uint32_t rs[4];
      SCORE sc[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        bool b;
        plain_pair<SCORE>(p[k], icpu, imem, nzc10, nzm10, nzc, nzm, bem, s_tab, rs[k], sc[k], b);
        fb[k] |= (uint64_t)b << j;
      }
      const uint32_t orow = (uint32_t)(j0 + j) * stride;  // (uniform: scalar)
      const v4u rv = {rs[0], rs[1], rs[2], rs[3]};
      __builtin_amdgcn_raw_buffer_store_b128(rv, rbuf, n0 * 4, (int)(orow * 4u), kEvalAux);
      if constexpr (sizeof(SCORE) == 4) {
        const v4u sv = {(unsigned)sc[0], (unsigned)sc[1], (unsigned)sc[2], (unsigned)sc[3]};
        __builtin_amdgcn_raw_buffer_store_b128(sv, sbuf, n0 * 4, (int)(orow * 4u), kEvalAux);
      } else {
        const v4u s01 = {(unsigned)(uint64_t)sc[0], (unsigned)((uint64_t)sc[0] >> 32), (unsigned)(uint64_t)sc[1],
                         (unsigned)((uint64_t)sc[1] >> 32)};
        const v4u s23 = {(unsigned)(uint64_t)sc[2], (unsigned)((uint64_t)sc[2] >> 32), (unsigned)(uint64_t)sc[3],
                         (unsigned)((uint64_t)sc[3] >> 32)};
        __builtin_amdgcn_raw_buffer_store_b128(s01, sbuf, n0 * 8, (int)(orow * 8u), kEvalAux);
        __builtin_amdgcn_raw_buffer_store_b128(s23, sbuf, n0 * 8 + 16, (int)(orow * 8u), kEvalAux);
      }
    }
    if (!C.nodeorder) return;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint64_t m = fb[k];
      while (m) {  // the deferred Balanced fallbacks (this thread's later store to the same word)
        const int j = __builtin_ctzll(m);
        m &= m - 1;
        const int lc = lr_score_f64(p[k].num_c - s_dreq[2][j], p[k].cap_c, p[k].lc_inv);
        const int lm = lr_score_f64(p[k].num_m - s_dreq[3][j], p[k].cap_m, p[k].lm_inv);
        const double rc = s_dnz[0][j] + p[k].d_nc, rm = s_dnz[1][j] + p[k].d_nm;
        scores[(size_t)(j0 + j) * stride + n0 + k] =
            s_tab[((lc + lm) >> 1) * 11 + bra_score_f64(rc, p[k].d_ac, rm, p[k].d_am, 0.0, 0.0, false)];
      }
    }
    return;
  }
#pragma unroll 1
  for (int k = 0; k < 4; ++k) {  // the int64 forms (eval_plain_kernel's tail loop), node by node
    const int n = n0 + k;
    const Row rk = load_row(N, n);  // (reloaded: no dynamic index into the register arrays)
    PlainNode pk;
    plain_node_init(pk, rk, C);
    const double inv_c = 1.0 / (double)rk.alloc_cpu, inv_m = 1.0 / (double)rk.alloc_mem;
    for (int j = 0; j < nj; ++j) {
      const int64_t icpu = s_req[0][j], imem = s_req[1][j];
      const bool fit = (le_tol(icpu, rk.idle_cpu, 10) && le_tol(imem, rk.idle_mem, 10ll * 1024 * 1024)) ||
                       (le_tol(icpu, rk.rel_cpu, 10) && le_tol(imem, rk.rel_mem, 10ll * 1024 * 1024));
      const uint32_t rs = !fit ? 1u << KB_R_RESOURCE_FIT : (s_bem[j] ? pk.post_be : pk.after);
      int64_t score = 0;
      if (C.nodeorder) {
        const int64_t rc = s_req[2][j] + rk.nz_cpu, rm = s_req[3][j] + rk.nz_mem;
        const int64_t lr = (lr_score_inv(rc, rk.alloc_cpu, inv_c) + lr_score_inv(rm, rk.alloc_mem, inv_m)) / 2;
        score = lr * C.w_lr + bra_score_inv(rc, rk.alloc_cpu, rm, rk.alloc_mem, inv_c, inv_m) * C.w_bra;
      }
      reasons[(size_t)(j0 + j) * stride + n] = rs;
      scores[(size_t)(j0 + j) * stride + n] = (SCORE)score;
    }
  }
}

// ===========================================================================
// Trajectory path (N <= kTrajMaxNodes, scores that fit a 32-bit key).
//
// Within a run of same-spec tasks only the winner's row changes, and a node's state after j commits of
// that spec is closed-form: commits Allocate while InitResreq still fits Idle (monotone in the number of
// allocations A), then Pipeline onto Releasing (allocate.go:159-182; NodeInfo.AddTask, node_info.go:165-193).
// So the key of every node after 0..J commits is computed in parallel up front (traj_sweep_kernel), and
// the sequential loop (traj_place_kernel) is pure LDS work: argmax, swap in the precomputed next key,
// re-reduce one chunk. Rows are written back once per run.
// ===========================================================================
constexpr uint32_t kKey32Feasible = 1u << 31;
constexpr uint32_t kKey32Exhausted = 0x7fffffffu;  // nxt32 sentinel: trajectory ran out, compute on demand

__device__ __forceinline__ uint32_t umax32(uint32_t a, uint32_t b) { return a > b ? a : b; }
__device__ __forceinline__ uint32_t umin32(uint32_t a, uint32_t b) { return a < b ? a : b; }
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ uint32_t wave_max32_dpp(uint32_t v) {
  v = umax32(v, dpp_u32<0xb1>(v));
  v = umax32(v, dpp_u32<0x4e>(v));
  v = umax32(v, dpp_u32<0x124>(v));
  v = umax32(v, dpp_u32<0x128>(v));
  v = umax32(v, dpp_u32<0x142>(v));
  v = umax32(v, dpp_u32<0x143>(v));
  return (uint32_t)__builtin_amdgcn_readlane(v, 63);
}

// Scalars fit after `mul` subtractions of the spec's Resreq scalars.
__device__ __forceinline__ bool scalars_fit_after(const DevNodes& N, const kb_spec& sp, const int64_t* sci,
                                                  const int64_t* scr, bool has_map, const int64_t* node_sc, int n,
                                                  int64_t mul) {
  if (!(sp.flags & KB_SPEC_INIT_HAS_MAP)) return true;
  if (!has_map) return false;
  uint64_t m = sp.init_sc_mask;
  while (m) {
    const int q = __builtin_ctzll(m);
    m &= m - 1;
    const int64_t avail = node_sc[(size_t)q * N.n + n] - mul * scr[q];
    if (!le_tol(sci[q], avail, 10)) return false;
  }
  return true;
}

__device__ __forceinline__ bool idle_fits_after(const DevNodes& N, const kb_spec& sp, const int64_t* sci,
                                                const int64_t* scr, const Row& r, int n, int64_t a) {
  return le_tol(sp.init_cpu, r.idle_cpu - a * sp.req_cpu, 10) &&
         le_tol(sp.init_mem, r.idle_mem - a * sp.req_mem, 10ll * 1024 * 1024) &&
         scalars_fit_after(N, sp, sci, scr, r.flags & KB_NODE_IDLE_HAS_MAP, N.idle_sc, n, a);
}

// A = number of consecutive Allocates before InitResreq stops fitting Idle (capped at 65535).
__device__ __forceinline__ int allocs_before_full_search(const DevNodes& N, const kb_spec& sp, const int64_t* sci,
                                                  const int64_t* scr, const Row& r, int n) {
  if (!idle_fits_after(N, sp, sci, scr, r, n, 0)) return 0;
  int lo = 0, hi = 65535;  // fits(lo) holds; find the largest such lo
  if (idle_fits_after(N, sp, sci, scr, r, n, hi)) return 65535;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (idle_fits_after(N, sp, sci, scr, r, n, mid)) lo = mid;
    else hi = mid;
  }
  return lo + 1;
}

// Allocations of the spec the node's Idle takes before it stops fitting (capped at 65535). Each resource's
// test init - (idle - a * req) < tol (idle_fits_after) is a * req < X with X = tol - init + idle, so for
// req >= 0 the largest fitting a is min over resources of (X - 1) / req: a closed form of the search above
// (which stays as the fallback for negative requests), with one load per scalar instead of one per step.
__device__ __forceinline__ int allocs_before_full(const DevNodes& N, const kb_spec& sp, const int64_t* sci,
                                                  const int64_t* scr, const Row& r, int n) {
  int64_t lo = 65535;
  bool ok = true, neg = false;
  const auto bound = [&](int64_t init, int64_t idle, int64_t req, int64_t tol) {
    const int64_t X = tol - init + idle;
    if (X <= 0) ok = false;
    else if (req > 0) lo = (X - 1) / req < lo ? (X - 1) / req : lo;
    else if (req < 0) neg = true;
  };
  bound(sp.init_cpu, r.idle_cpu, sp.req_cpu, 10);
  bound(sp.init_mem, r.idle_mem, sp.req_mem, 10ll * 1024 * 1024);
  if (sp.flags & KB_SPEC_INIT_HAS_MAP) {
    if (!(r.flags & KB_NODE_IDLE_HAS_MAP)) return 0;  // rr.ScalarResources == nil
    uint64_t m = sp.init_sc_mask;
    while (m) {
      const int q = __builtin_ctzll(m);
      m &= m - 1;
      bound(sci[q], N.idle_sc[(size_t)q * N.n + n], scr[q], 10);
    }
  }
  if (neg) return allocs_before_full_search(N, sp, sci, scr, r, n);
  if (!ok) return 0;
  return lo >= 65535 ? 65535 : (int)lo + 1;
}

// Full 64-bit key of node n after j commits of the spec (A allocations at most, the rest pipelined).
// INV: the score from the node's reciprocal capacities ic / im (row_score_inv: the same value).
template <bool INV = false>
__device__ __forceinline__ uint64_t traj_key64(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const kb_spec& sp,
                               const int64_t* sci, const int64_t* scr, const Row& r0, uint64_t st, int n, int j,
                               int A, double ic = 0.0, double im = 0.0) {
  const int64_t a = j < A ? j : A;
  const int64_t p = j - a;
  Row r = r0;
  r.idle_cpu -= a * sp.req_cpu;
  r.idle_mem -= a * sp.req_mem;
  r.rel_cpu -= p * sp.req_cpu;
  r.rel_mem -= p * sp.req_mem;
  r.pod_count += j;
  r.nz_cpu += (int64_t)j * sp.nz_cpu;
  r.nz_mem += (int64_t)j * sp.nz_mem;
  uint32_t reasons = 0;
  const bool fi = le_tol(sp.init_cpu, r.idle_cpu, 10) && le_tol(sp.init_mem, r.idle_mem, 10ll * 1024 * 1024) &&
                  scalars_fit_after(N, sp, sci, scr, r.flags & KB_NODE_IDLE_HAS_MAP, N.idle_sc, n, a);
  if (!fi) {
    const bool fr = le_tol(sp.init_cpu, r.rel_cpu, 10) && le_tol(sp.init_mem, r.rel_mem, 10ll * 1024 * 1024) &&
                    scalars_fit_after(N, sp, sci, scr, r.flags & KB_NODE_REL_HAS_MAP, N.rel_sc, n, p);
    if (!fr) reasons = 1u << KB_R_RESOURCE_FIT;
  }
  if (!reasons && !C.predicates) reasons = stat_post(st);  // the host overlay only
  if (!reasons && C.predicates) {
    if (r.max_pods <= r.pod_count) {
      reasons = 1u << KB_R_POD_NUMBER;
    } else if (stat_pre(st)) {
      reasons = stat_pre(st);
    } else {
      for (uint32_t i = 0; i < sp.port_cnt && !reasons; ++i) {
        const kb_port q = P.ports[sp.port_off + i];
        uint64_t used = N.port_used[(size_t)q.slot * N.n + n];
        if (j > 0)  // the spec's own ports were taken by its earlier commits here (UpdateUsedPorts)
          for (uint32_t k = 0; k < sp.port_cnt; ++k) {
            const kb_port o = P.ports[sp.port_off + k];
            if (o.slot == q.slot) used |= 1ull << o.ip;
          }
        if (q.ip == 0 ? used : (used & (1ull | (1ull << q.ip)))) reasons = 1u << KB_R_HOST_PORTS;
      }
      if (!reasons) reasons = stat_post(st);
      // a cap-1 spec's own anti-affinity check, after its first Allocate here (InterPodAffinityMatches is
      // the last predicate; a node failing a static one never reaches level 1)
      if (!reasons && j > 0 && A > 0 && (sp.flags & kSpecCap1))
        reasons = (sp.flags & kSpecCapAnti) ? kAffAntiRules : kAffExistingAnti;
    }
  }
  if (reasons) return reasons;
  const int64_t score = INV ? row_score_inv(C, sp, r, st, ic, im) : row_score(C, sp, r, st);
  return kFeasible | ((uint64_t)(score + kScoreBias) << 24);
}

__device__ __forceinline__ uint32_t compress_key(uint64_t k64, int n, int idx_bits) {
  if (!(k64 & kFeasible)) return (uint32_t)k64;
  const int64_t score = (int64_t)((k64 >> 24) & ((1ull << 39) - 1)) - kScoreBias;
  const int64_t bias32 = 1ll << (30 - idx_bits);
  const uint32_t idx_mask = (1u << idx_bits) - 1;
  return kKey32Feasible | ((uint32_t)(score + bias32) << idx_bits) | (idx_mask - (uint32_t)n);
}

// grid (ceil(n/256), J+1): thread (node, j) writes the key after j commits.
template <bool AFF>
__global__ __launch_bounds__(256) void traj_sweep_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, int idx_bits,
                                                         uint32_t* traj, uint32_t* cmax32, uint32_t* amax,
                                                         uint64_t* stat, const JobState* js) {
  if (js != nullptr && js->stopped) return;
  const kb_spec sp = P.specs[spec];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  uint32_t k = 0;
  if (n < N.n) {
    const Row r = load_row(N, n);
    const uint64_t st = static_eval<AFF>(N, P, C, sp, spec, r.flags, n, P.A.mm);
    const int A = allocs_before_full(N, sp, sci, scr, r, n);
    k = compress_key(traj_key64(N, P, C, sp, sci, scr, r, st, n, j, A), n, idx_bits);
    traj[(size_t)j * N.n + n] = k;
    if (j == 0) {
      stat[n] = st;
      amax[n] = (uint32_t)A;
    }
  }
  if (j == 0) {
    const uint32_t m = wave_max32_dpp(k);
    if ((threadIdx.x & 63) == 0 && (n >> 6) < ((N.n + 63) >> 6)) cmax32[n >> 6] = m;
  }
}

// Apply `c` commits (the first min(c, A) Allocate, the rest Pipeline) to node w's row in HBM.
__device__ void write_back_row(const DevNodes& N, const DevSpecs& P, const kb_spec& sp, const int64_t* scr, int w,
                               int c, int A) {
  const int64_t a = c < A ? c : A;
  const int64_t p = c - a;
  const uint32_t f = N.flags[w];
  N.idle_cpu[w] -= a * sp.req_cpu;
  N.idle_mem[w] -= a * sp.req_mem;
  N.rel_cpu[w] -= p * sp.req_cpu;
  N.rel_mem[w] -= p * sp.req_mem;
  N.pod_count[w] += c;
  N.nz_cpu[w] += (int64_t)c * sp.nz_cpu;
  N.nz_mem[w] += (int64_t)c * sp.nz_mem;
  uint64_t m = sp.req_sc_mask;
  while (m) {  // Sub on a nil scalar map is a no-op (resource_info.go:152-157)
    const int q = __builtin_ctzll(m);
    m &= m - 1;
    if (a && (f & KB_NODE_IDLE_HAS_MAP)) N.idle_sc[(size_t)q * N.n + w] -= a * scr[q];
    if (p && (f & KB_NODE_REL_HAS_MAP)) N.rel_sc[(size_t)q * N.n + w] -= p * scr[q];
  }
  if (c > 0)
    for (uint32_t i = 0; i < sp.port_cnt; ++i) {
      const kb_port q = P.ports[sp.port_off + i];
      N.port_used[(size_t)q.slot * N.n + w] |= 1ull << q.ip;
    }
}


constexpr int kPlaceThreads = 512;
static_assert(kTrajDefaultJ <= kTrajMaxJ, "trajectory buffer depth");

// The sequential loop keeps the LDS reads of one task independent of each other (issued together) and
// the chunk maxima in registers (lane l owns chunks l, l+64, l+128, l+192). A node's first commit in the
// run takes its key from nxt[] in LDS; a repeat commit (about 1 in 7 on C2) reads its trajectory level
// from global memory.
__global__ __launch_bounds__(kPlaceThreads) void traj_place_kernel(
    DevNodes N, DevSpecs P, DevCfg C, int spec, int t_begin, int t_count, int J, int idx_bits, const uint32_t* traj,
    const uint32_t* cmax32, const uint32_t* amax, const uint64_t* stat, JobState* js, int first, int ready0,
    int minav0, int gang0, int32_t* hout, JobState* hjs, int pb_cap, uint32_t seq) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  __shared__ LoopOut lo;
  if (!first && js->stopped) {
    signal_skip(hjs, seq);
    return;
  }
#ifdef KB_DIAG
  const uint64_t t_start = __builtin_amdgcn_s_memtime();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int n = N.n;
  const int M = (n + 63) >> 6;            // <= 256 (checked by traj_lds_bytes)
  const int W = (n + 63) >> 6;            // touched-bitmap words
  uint64_t* tb = (uint64_t*)lds32;        // [W] nodes committed to in this run
  uint32_t* cur = lds32 + 2 * W;          // [n] key after the commits so far
  // [n] {key after the node's first commit of the run, commits so far | A << 16}: one 8-B read per task
  uint2* nc = (uint2*)(cur + ((n + 1) & ~1));
  uint32_t* pb = (uint32_t*)(nc + n);     // [pb_cap] placements: node | kind << 30
  // fill LDS with every thread of the block (independent loads in flight)
  for (int i = tid; i < W; i += kPlaceThreads) tb[i] = 0;
  {
    // batches of 8 nodes per thread: all 24 loads are issued before the first LDS store
    constexpr int kB = 8;
    const uint32_t* t1 = J >= 1 ? traj + n : traj;
    for (int base = 0; base < n; base += kB * kPlaceThreads) {
      uint32_t a[kB], b[kB], m[kB];
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const int i = base + u * kPlaceThreads + tid;
        const int ic = i < n ? i : n - 1;  // clamped: unconditional loads keep them all in flight
        a[u] = traj[ic];
        b[u] = t1[ic];
        m[u] = amax[ic];
      }
#pragma unroll
      for (int u = 0; u < kB; ++u) {
        const int i = base + u * kPlaceThreads + tid;
        if (i < n) {
          cur[i] = a[u];
          nc[i] = make_uint2(J >= 1 ? b[u] : kKey32Exhausted, m[u] << 16);
        }
      }
    }
  }
  __syncthreads();

  const kb_spec sp = P.specs[spec];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  if (tid < 64) {  // wave 0 runs the sequential placement loop; LDS ops of one wave retire in order
    uint32_t cm0 = lane < M ? cmax32[lane] : 0u;
    uint32_t cm1 = lane + 64 < M ? cmax32[lane + 64] : 0u;
    uint32_t cm2 = lane + 128 < M ? cmax32[lane + 128] : 0u;
    uint32_t cm3 = lane + 192 < M ? cmax32[lane + 192] : 0u;
    uint32_t lmax = umax32(umax32(cm0, cm1), umax32(cm2, cm3));
    const uint32_t idx_mask = (1u << idx_bits) - 1;
    const int64_t bias32 = 1ll << (30 - idx_bits);
    int ready, minav, gang, placed;
    if (first) {
      ready = ready0;
      minav = minav0;
      gang = gang0;
      placed = 0;
    } else {
      ready = js->ready_num;
      minav = js->min_available;
      gang = js->gang_ready;
      placed = js->n_placed;
    }
    int pb_n = 0, pb_base = t_begin;
    int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
#ifdef KB_DIAG
    // phases: 0 argmax, 1 commit, 2 chunk re-reduce, 3 chunk-max update, 4 unused, 5 loop, 6 fill
    uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
    uint64_t dg_last = __builtin_amdgcn_s_memtime();
    dg[6] = dg_last - t_start;
#endif

    for (int t = 0; t < t_count; ++t) {
      KB_STAMP(5);
      const uint32_t best = wave_max32_dpp(lmax);
      KB_STAMP(0);
      if (!(best & kKey32Feasible)) {
        // PredicateNodes found nothing (allocate.go:150-153): FitErrors histogram over all nodes.
        uint32_t h[KB_NUM_REASONS];
#pragma unroll
        for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] = 0;
        for (int i = lane; i < n; i += 64) {
          const uint32_t k = cur[i];
#pragma unroll
          for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] += (k >> b) & 1u;
        }
#pragma unroll
        for (int b = 0; b < KB_NUM_REASONS; ++b) {
          const uint32_t s = wave_sum_u32(h[b]);
          if (lane == 0) {
            js->hist[b] = s;
            hjs->hist[b] = s;
          }
        }
        stop = KB_STOP_NO_FIT;
        fail_task = t_begin + t;
        stopped = 1;
        break;
      }
      const int64_t score = (int64_t)((best >> idx_bits) & ((1u << (31 - idx_bits)) - 1)) - bias32;
      if (score <= -1) {  // SelectBestNode: no bucket with score > -1 -> the reference panics
        fail_task = t_begin + t;
        panic = 1;
        stopped = 1;
        break;
      }
      const int w = (int)(idx_mask - (best & idx_mask));
      const int ch = w >> 6;
      const int i = (ch << 6) + lane;
      // the three LDS reads of this task, issued together (uniform addresses broadcast)
      const uint32_t cv = i < n ? cur[i] : 0u;
      const uint2 ncw = nc[w];
      const uint32_t s = ncw.y, nx = ncw.x;
      const int c = (int)(s & 0xffff), A = (int)(s >> 16);
      const int kind = c < A ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE;  // commit c+1 Allocates iff c+1 <= A

      // key after c+1 commits: level 1 is in LDS, deeper levels in the trajectory buffer
      uint32_t nk = nx;
      if (c >= 1) nk = c + 1 <= J ? traj[(size_t)(c + 1) * n + w] : kKey32Exhausted;
      if (nk == kKey32Exhausted) {  // beyond the precomputed trajectory: compute in place (rare)
        uint32_t k = 0;
        if (lane == 0) {
          const Row r0 = load_row(N, w);
          k = compress_key(traj_key64(N, P, C, sp, sci, scr, r0, stat[w], w, c + 1, A), w, idx_bits);
        }
        nk = (uint32_t)__builtin_amdgcn_readlane((int)k, 0);
      }
      KB_STAMP(1);
      if (lane == 0) {  // fire-and-forget LDS updates
        cur[w] = nk;
        nc[w].y = (uint32_t)(c + 1) | ((uint32_t)A << 16);
        if (c == 0) atomicOr((unsigned long long*)&tb[w >> 6], 1ull << (w & 63));
        pb[pb_n] = (uint32_t)w | ((uint32_t)kind << 30);
      }

      // Re-reduce the winner's chunk; its owner lane refreshes its running max (registers only).
      const uint32_t v = wave_max32_dpp(i == w ? nk : cv);
      KB_STAMP(2);
      const bool own = lane == (ch & 63);
      const int jj = ch >> 6;
      cm0 = (own && jj == 0) ? v : cm0;
      cm1 = (own && jj == 1) ? v : cm1;
      cm2 = (own && jj == 2) ? v : cm2;
      cm3 = (own && jj == 3) ? v : cm3;
      lmax = umax32(umax32(cm0, cm1), umax32(cm2, cm3));
      KB_STAMP(3);

      ++placed;
      ++pb_n;
      if (kind == KB_PLACE_ALLOCATE) ++ready;
      if (!gang || ready >= minav) {  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
        stop = KB_STOP_READY;
        stopped = 1;
        break;
      }
      if (pb_n == pb_cap) {  // buffer full: hand the placements to the host and keep going
        for (int k = lane; k < pb_n; k += 64) {
          const uint32_t e = pb[k];
          hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
          hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
        }
        pb_base += pb_n;
        pb_n = 0;
      }
    }
#ifdef KB_DIAG
    if (lane == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
    if (lane == 0) lo = LoopOut{stop, fail_task, placed, ready, minav, gang, panic, stopped, pb_n, pb_base, 0, 0};
  }
  __syncthreads();
  // write the run's commits back to the node table: one node per thread (touched nodes cluster at low
  // indices, so a per-bitmap-word walk would serialise their load->store chains on a few threads)
  for (int w = tid; w < n; w += kPlaceThreads) {
    if (!((tb[w >> 6] >> (w & 63)) & 1)) continue;
    const uint32_t s = nc[w].y;
    write_back_row(N, P, sp, scr, w, (int)(s & 0xffff), (int)(s >> 16));
  }
  for (int k = tid; k < lo.pb_n; k += kPlaceThreads) {
    const uint32_t e = pb[k];
    hout[2 * (lo.pb_base + k)] = (int32_t)(e & 0x3fffffffu);
    hout[2 * (lo.pb_base + k) + 1] = (int32_t)(e >> 30);
  }
  __threadfence_system();
  __syncthreads();
  if (tid == 0)
    publish_state(js, hjs, lo.stopped, lo.stop, lo.fail_task, lo.placed, lo.ready, lo.minav, lo.gang, lo.panic,
                  seq);
}

// ===========================================================================
// Selection path (32-bit keys, sel_lds_bytes(n) >= 0): a run of same-spec tasks as a parallel top-T
// selection instead of T dependent argmax steps.
//
// Within the run node x's key after j commits of the spec is k_x(j) (closed form, traj_key64), and the
// reference's loop (SelectBestNode + commit, repeated: scheduler_helper.go:147-158, allocate.go:135-188)
// is a greedy merge: take the largest current key, advance that node. Let e_x(j) = min_{i<=j} k_x(i).
// The e-values of the successive picks never increase (DESIGN.md §3 has the argument), so the picks are
// exactly the elements (x, j) in descending (e, then node ascending, then j ascending) order — node
// indices are part of the key, so e-values of different nodes never tie. Per segment of T <= kSegMax
// tasks the kernel therefore
//   1. takes S = the T nodes with the largest current key (binary search on the score field, lowest
//      index first on the threshold score): an element (x, j) ranks at least j + rank_S(x), so no node
//      outside S and no level j >= T - rank_S(x) can be among the first T picks;
//   2. generates every S node's e-sequence over those levels, in parallel rounds;
//   3. finds the T-th largest element (binary search again), orders the T winners, and applies the
//      stop rules in that order: panic (score <= -1), gang ready (allocate.go:184-187), no fit;
//   4. writes the placements and the touched rows back and re-keys the touched nodes for the next
//      segment.
// ===========================================================================
constexpr int kSelThreads = 512;   // 8 waves: up to 256 VGPRs per lane, no spills
constexpr int kSelWaves = kSelThreads / 64;
#ifndef KB_SEL_DENSE_MAX
#define KB_SEL_DENSE_MAX 32  // winners: rank all candidates pairwise up to this many, else threshold + takes
#endif
constexpr int kSegMax = 100;                           // tasks per segment (slot and level fit 7-bit fields)
static_assert(kSegMax == kFedSplitMaxTasks, "the split fed engine's job bound is one segment");
constexpr int kCandMax = kSegMax * (kSegMax + 1) / 2;  // sum over S of (T - rank): levels that can rank < T
constexpr int kCandCap = 5120;                         // candidate composites: 10 per thread, five uint4 reads
constexpr int kCandV = kCandCap / 2 / kSelThreads;     // uint4 (two composites) groups per thread
constexpr int kSelQ4 = 12;                             // uint4 key groups per thread: n <= 512 * 48
static_assert(kCandMax <= kCandCap && kCandCap == 2 * kCandV * kSelThreads, "candidate layout");

struct SelShared {
  Row row[128];            // segment-start rows of the selected nodes
  uint64_t stat[128];
  uint64_t comp[128];      // composites (e << 14 | (127 - slot) << 7 | (127 - level)) of the taken elements
  uint64_t ord[128];       // the same, in pick order
  union {
    uint64_t dense[kSelThreads];  // winners: the candidates, compacted (when there are at most one per thread)
    double recip[2][128];         // e-sequences: 1 / allocatable cpu, memory of the selected nodes
  };
  int32_t node[128];
  uint32_t key0[128];      // current key of the selected node
  int32_t A[128];          // Allocates before InitResreq stops fitting Idle
  int32_t lmax[128];       // levels that can rank below T: T - rank
  int32_t off[128];        // into the candidate array
  int32_t cnt[128];        // e-values kept (all feasible, and >= the cut-off when S fills the segment)
  int32_t gen[128];        // levels examined
  uint32_t emin[128];      // running prefix minimum
  int32_t done[128];
  int32_t fin[128];        // commits of this node in the segment
  int32_t n_commit;        // rows listed in commit_out so far
  int32_t act[128];        // active slots of a generation round
  uint32_t red[2][4][kSelWaves];  // reduction scratch, alternating halves: one barrier per reduction
  uint32_t hist[KB_NUM_REASONS];
  uint32_t theta0;
  int32_t n_act, s_count, cut, stop_kind, n_alloc;
  int32_t n_sel;      // CAND runs: the selected set published to the fed selector
  int32_t need_hist;  // CAND runs: a no-fit whose histogram the caller computes
  LoopOut lo;
  EngineCmd cmd;  // placement engine: the command being served and its current run
  EngineRun run;
  uint64_t t_recv;
};
constexpr int kSelDynLimit = 160 * 1024 - (int)sizeof(SelShared) - 64;
static_assert(4 * (4 * kSelThreads * kSelQ4) + 8 * kCandCap <= kSelDynLimit,
              "the selection plan's largest node count (512 x 48 keys) must fit LDS");
constexpr int kFedDynLimit = kSelDynLimit - 2048;  // the fed engine's own static LDS beside SelShared

__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t v, int lane) {
  (void)lane;
  return wave_incl_scan_dpp(v, 0u, OpAdd{}) - v;
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_dpp(v, 0u, OpMax{}), 63);
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan_dpp(v, 0xffffffffu, OpMin{}), 63);
}

// Block-wide reductions with one barrier each: the scratch half alternates between calls, and the
// barrier of call k+1 separates call k's reads from call k+2's writes. `rp` is block-uniform.
__device__ __forceinline__ void sel_reduce3(SelShared& sh, int& rp, uint32_t& s, uint32_t& mx, uint32_t& mn) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  s = wave_sum_u32(s);
  mx = wave_max_u32(mx);
  mn = wave_min_u32(mn);
  uint32_t(*r)[kSelWaves] = sh.red[rp];
  rp ^= 1;
  if (lane == 0) {
    r[0][wv] = s;
    r[1][wv] = mx;
    r[2][wv] = mn;
  }
  __syncthreads();
  s = 0, mx = 0, mn = 0xffffffffu;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) {
    s += r[0][w];
    mx = umax32(mx, r[1][w]);
    mn = r[2][w] < mn ? r[2][w] : mn;
  }
}
// Node selection's first reduction: feasible count F, max / min score field MX / MN, and the keys at MX: E in
// total and *pre = those of the threads before this one (thread order = node order). lc: the thread's keys at
// its own maximum mx (its count at MX when mx == MX). One barrier.
__device__ __forceinline__ void sel_reduce_top(SelShared& sh, int& rp, uint32_t& F, uint32_t& MX, uint32_t& MN,
                                               uint32_t& E, uint32_t& pre, uint32_t& e, uint32_t lc) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t mx = MX;
  const uint32_t fw = wave_sum_u32(F), mxw = wave_max_u32(mx), mnw = wave_min_u32(MN);
  const uint32_t ew = mx == mxw ? lc : 0u;
  const uint32_t xw = wave_excl_scan_u32(ew, lane), sw = wave_sum_u32(ew);
  uint32_t(*r)[kSelWaves] = sh.red[rp];
  rp ^= 1;
  if (lane == 0) {
    r[0][wv] = fw;
    r[1][wv] = mxw;
    r[2][wv] = mnw;
    r[3][wv] = sw;
  }
  __syncthreads();
  F = 0, MX = 0, MN = 0xffffffffu;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) {
    F += r[0][w];
    MX = umax32(MX, r[1][w]);
    MN = r[2][w] < MN ? r[2][w] : MN;
  }
  E = 0, pre = 0;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) {
    const uint32_t c = r[1][w] == MX ? r[3][w] : 0u;
    E += c;
    pre += w < wv ? c : 0u;
  }
  const bool top = mxw == MX;
  pre += top ? xw : 0u;
  e = top ? ew : 0u;
}
__device__ __forceinline__ uint32_t sel_sum(SelShared& sh, int& rp, uint32_t v) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  v = wave_sum_u32(v);
  uint32_t* r = sh.red[rp][0];
  rp ^= 1;
  if (lane == 0) r[wv] = v;
  __syncthreads();
  uint32_t s = 0;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) s += r[w];
  return s;
}
// Two block-wide exclusive prefix sums in thread order at once; totals in *ta / *tb.
__device__ __forceinline__ void sel_excl_scan2(SelShared& sh, int& rp, uint32_t& a, uint32_t& b, uint32_t* ta,
                                               uint32_t* tb) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t xa = wave_excl_scan_u32(a, lane), xb = wave_excl_scan_u32(b, lane);
  uint32_t(*r)[kSelWaves] = sh.red[rp];
  rp ^= 1;
  if (lane == 63) {
    r[0][wv] = xa + a;
    r[1][wv] = xb + b;
  }
  __syncthreads();
  uint32_t ba = 0, bb = 0, sa = 0, sb = 0;
#pragma unroll
  for (int w = 0; w < kSelWaves; ++w) {
    const uint32_t ra = r[0][w], rb = r[1][w];
    ba += w < wv ? ra : 0;
    bb += w < wv ? rb : 0;
    sa += ra;
    sb += rb;
  }
  a = ba + xa;
  b = bb + xb;
  *ta = sa;
  *tb = sb;
}

// Elements of slot s's candidate list whose score field is >= v (the list is non-increasing).
__device__ __forceinline__ uint32_t sel_cnt_ge(const SelShared& sh, const uint64_t* cand, int s, int S, uint32_t v,
                                               int idx_bits) {
  if (s >= S) return 0;
  uint32_t lo = 0, hi = (uint32_t)sh.cnt[s];
  const uint64_t* c = cand + sh.off[s];
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if ((uint32_t)(c[mid] >> (14 + idx_bits)) >= v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int sel_slot(uint64_t o) { return 127 - (int)((o >> 7) & 127); }
__device__ __forceinline__ int sel_level(uint64_t o) { return 127 - (int)(o & 127); }

// The row after c commits of the spec from its segment-start state r0 (min(c, A) Allocates, the rest
// Pipelines): stores only, no read-modify-write of the main columns (scalars and ports as
// write_back_row does them).
__device__ void store_back_row(const DevNodes& N, const DevSpecs& P, const kb_spec& sp, const int64_t* scr, int w,
                               int c, int A, const Row& r0) {
#ifdef KB_WA_NO_ROWS  // (write-accounting A/B build only: the committed rows are not written back -- wrong placements)
  return;
#endif
  const int64_t a = c < A ? c : A;
  const int64_t p = c - a;
  // (sc1 stores: the fed selector reads them with load_row_sc1, after the placer's p_done, without an acquire)
  st_sc1(&N.idle_cpu[w], r0.idle_cpu - a * sp.req_cpu);
  st_sc1(&N.idle_mem[w], r0.idle_mem - a * sp.req_mem);
  st_sc1(&N.rel_cpu[w], r0.rel_cpu - p * sp.req_cpu);
  st_sc1(&N.rel_mem[w], r0.rel_mem - p * sp.req_mem);
  st_sc1(&N.pod_count[w], r0.pod_count + c);
  st_sc1(&N.nz_cpu[w], r0.nz_cpu + (int64_t)c * sp.nz_cpu);
  st_sc1(&N.nz_mem[w], r0.nz_mem + (int64_t)c * sp.nz_mem);
  uint64_t m = sp.req_sc_mask;
  while (m) {  // Sub on a nil scalar map is a no-op (resource_info.go:152-157)
    const int q = __builtin_ctzll(m);
    m &= m - 1;
    if (a && (r0.flags & KB_NODE_IDLE_HAS_MAP)) N.idle_sc[(size_t)q * N.n + w] -= a * scr[q];
    if (p && (r0.flags & KB_NODE_REL_HAS_MAP)) N.rel_sc[(size_t)q * N.n + w] -= p * scr[q];
  }
  if (c > 0)
    for (uint32_t i = 0; i < sp.port_cnt; ++i) {
      const kb_port q = P.ports[sp.port_off + i];
      N.port_used[(size_t)q.slot * N.n + w] |= 1ull << q.ip;
    }
}

#ifdef KB_DIAG
#define SEL_DIAG_PARAMS , uint64_t *dg, uint64_t &dg_last
#define SEL_DIAG_ARGS , dg, dg_last
#else
#define SEL_DIAG_PARAMS
#define SEL_DIAG_ARGS
#endif

// Node selection, phase 1 of sel_run: the T best keys of k32 (LDS, 4 * kSelThreads * Q4 positions, zero padding)
// by score field, ties to the lower position. sh.node / sh.key0 [0, S) get node_of(position) and the key, in
// position order (the position is the node). Returns the feasible count (0: nothing fits, S = 0). No barrier
// after the LDS writes.
// no / ko (cap entries, default sh.node / sh.key0): where the selected nodes and keys go.
template <int QN>
__device__ __forceinline__ uint32_t sel_pick(SelShared& sh, const uint32_t* k32, int n, int idx_bits, uint32_t T,
                                             int& rp, uint32_t& S_out SEL_DIAG_PARAMS, int32_t* no = nullptr,
                                             uint32_t* ko = nullptr, int cap = 128) {
  const int tid = threadIdx.x;
  if (no == nullptr) no = sh.node, ko = sh.key0;
  constexpr int QU = QN > 0 ? QN : kSelQ4;  // unroll bound of the key passes
  const int Q4 = QN > 0 ? QN : (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const uint4* k32v = (const uint4*)k32;
  uint4 kv[QU];
#pragma unroll
  for (int c = 0; c < QU; ++c) kv[c] = (QN > 0 || c < Q4) ? k32v[tid * Q4 + c] : make_uint4(0u, 0u, 0u, 0u);
#define SEL_EACH_KEY(BODY)                                       \
  _Pragma("unroll") for (int c_ = 0; c_ < QU; ++c_) {           \
    const uint32_t ks_[4] = {kv[c_].x, kv[c_].y, kv[c_].z, kv[c_].w}; \
    _Pragma("unroll") for (int q_ = 0; q_ < 4; ++q_) {           \
      const uint32_t k = ks_[q_];                                \
      const int ki = (tid * Q4 + c_) * 4 + q_;                   \
      (void)ki;                                                  \
      BODY                                                       \
    }                                                            \
  }
  // branch-free over the keys (a branch per key costs more than the arithmetic): an infeasible key counts
  // as score field 0 for the maximum (below every feasible field) and as ~0 for the minimum
  uint32_t F = 0, MX = 0, MN = 0xffffffffu, LC = 0;
  SEL_EACH_KEY({
    const bool f = (int32_t)k < 0;
    const uint32_t h = f ? k >> idx_bits : 0u;
    F += f;
    LC = h > MX ? 1u : LC + (h == MX);
    MX = umax32(MX, h);
    MN = umin32(MN, f ? h : 0xffffffffu);
  })
  // with the count at the top score: nothing lies above MX, so when at least T nodes share it this is also
  // the greater / equal count of the compaction
  uint32_t Etop, pre_top, e_top;
  sel_reduce_top(sh, rp, F, MX, MN, Etop, pre_top, e_top, LC);
  KB_SEL_FINE(1);
  S_out = 0;
  if (F == 0) return 0;
  // infeasible keys (and padding) have a score field below every feasible one: never counted below
  uint32_t sstar = MN, R = 0xffffffffu;  // F <= T: every feasible node
  uint32_t g = 0, e = 0, tg = 0, te = 0, G = 0, E = 0;
  bool counted = false;
  if (F > T) {
    if (Etop >= T) {
      sstar = MX;
      counted = true;
      e = e_top;
      E = pre_top;
      te = Etop;
    } else {
      uint32_t lo = MN, hi = MX - 1;  // count(>= MN) = F > T; count(>= MX) < T
      while (lo < hi) {
        const uint32_t mid = lo + (hi - lo + 1) / 2;
        uint32_t c = 0;
        SEL_EACH_KEY({ c += (k >> idx_bits) >= mid; })
        if (sel_sum(sh, rp, c) >= T) lo = mid;
        else hi = mid - 1;
      }
      sstar = lo;
    }
  }
  KB_SEL_FINE(2);
  if (!counted) {
    g = 0, e = 0;
    SEL_EACH_KEY({
      const uint32_t h = k >> idx_bits;
      g += h > sstar;
      e += h == sstar;
    })
    G = g, E = e;
    sel_excl_scan2(sh, rp, G, E, &tg, &te);
  }
  KB_SEL_FINE(3);
  if (F > T) R = T - tg;
  const uint32_t selE = R > E ? (R - E < e ? R - E : e) : 0u;
  // slot of this thread's first selected node: selected nodes before it in position order
  uint32_t slot = G + (R > E ? E : R);
  S_out = tg + (R < te ? R : te);
  if (g + selE) {  // most threads hold no selected node
    uint32_t le = 0;
    SEL_EACH_KEY({
      const uint32_t h = k >> idx_bits;
      bool take = h > sstar;
      if (h == sstar) take = le++ < selE;
      if (take) {
        no[slot] = ki;
        ko[slot] = k;
        ++slot;
      }
    })
  }
  if (tid >= (int)S_out && tid < cap) ko[tid] = 0u;  // the rank loops read all cap entries
#undef SEL_EACH_KEY
  return F;
}

// One run of same-spec tasks inside a 1024-thread workgroup (the selection algorithm above).
// k32 (LDS, n_pad entries, zero past n) holds every node's current key at entry and is kept current;
// cand (LDS, kCandCap) is scratch; stat is the run's static cache. Placements go to hout[2 * task];
// ready / placed advance, and the stop state is set when the run stops the job.
// PROPOSE (node sharding): one segment of t_count <= kSegMax tasks, no commit; the rank's best picks go
// to `rec` instead (launch_shard_propose).
// QN > 0: the node count needs exactly QN key groups per thread (compile-time passes over 4 * QN keys);
// QN = 0: the group count is taken from n at run time (passes unrolled to kSelQ4 with the spare groups 0).
// The reason histogram of the infeasible keys among 4 * kSelThreads * Q4 (padding 0) into sh.hist; ends after a
// barrier.
__device__ void sel_hist(SelShared& sh, const uint4* k32v, int Q4) {
  const int tid = threadIdx.x, lane = tid & 63;
  if (tid < KB_NUM_REASONS) sh.hist[tid] = 0;
  __syncthreads();
  uint32_t h[KB_NUM_REASONS];
#pragma unroll
  for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] = 0;
  for (int c = 0; c < Q4; ++c) {
    const uint4 v = k32v[tid * Q4 + c];
    const uint32_t ks[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (ks[q] >> 31) continue;
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] += (ks[q] >> b) & 1u;
    }
  }
#pragma unroll
  for (int b = 0; b < KB_NUM_REASONS; ++b) {
    const uint32_t v = wave_sum_u32(h[b]);
    if (lane == 0 && v) atomicAdd(&sh.hist[b], v);
  }
  __syncthreads();
}

// The fed placer's publication to the selector (fed_engine_kernel): the nodes a job can commit to.
// Tagged words: (tag << 32 | payload), written and read as write-through agent-scope atomics. A reader
// takes a word once its tag is the one it waits for, so a publication needs no store ordering (no waits on
// the writer's side) and a stale word from an earlier job reads as not there yet.
#ifdef KB_TIMELINE
#define KB_PUB_TL(k)                                                                          \
  do {                                                                                        \
    if (CAND && pub.tl != nullptr && threadIdx.x == 0) pub.tl[k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define KB_PUB_TL(k) \
  do {               \
  } while (0)
#endif
__device__ __forceinline__ void tag_store(uint64_t* w, uint32_t tag, uint32_t v) {
  __hip_atomic_store(w, ((uint64_t)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t x_load64(const uint64_t* w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void x_store64(uint64_t* w, uint64_t v) {
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The fed placer's publication to the selector: the nodes a job can commit to (its selected set, in slot order).
constexpr uint32_t kPubModeSet = 0, kPubModeSkipped = 2;
struct FedPub {
  uint64_t* head = nullptr;  // tag << 32 | mode << 16 | count; nullptr: nothing to publish
  uint64_t* node = nullptr;  // [128] tag << 32 | node
  uint32_t tag = 0;
  uint64_t* tl = nullptr;    // KB_TIMELINE builds: the job's timeline row (FedXchg::tl)
  __device__ void set_node(int i, int w) const { tag_store(&node[i], tag, (uint32_t)w); }
  __device__ void set_head(uint32_t mode, int cnt) const { tag_store(head, tag, (mode << 16) | (uint32_t)cnt); }
};

// CAND (the split fed engine's placer, one segment): the caller has chosen the run's nodes (sh.n_sel of them in
// sh.node / key0 / row / stat, slots in node order, with sh.lmax = T - key rank and sh.theta0); they are
// published to the selector through `pub`, and a no-fit sets sh.need_hist instead of the histogram (the caller
// rebuilds every node's key first).
template <bool PROPOSE = false, int QN = 0, bool CAND = false>
__device__ __forceinline__ void sel_run(SelShared& sh, uint32_t* k32, uint64_t* cand, const DevNodes& N,
                                        const DevSpecs& P, const DevCfg& C, const kb_spec& sp, int spec,
                                        int t_begin, int t_count,
                                        int idx_bits, const uint64_t* stat, int& ready, int minav, int gang,
                                        int& placed, int& stop, int& fail_task, int& panic, int& stopped,
                                        int32_t* hout, JobState* js, JobState* hjs, int& rp,
                                        ShardRec* rec, int32_t* commit_out SEL_DIAG_PARAMS,
                                        FedPub pub = FedPub{}, uint32_t* pl = nullptr, const uint32_t* clv = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = N.n;
  const int Q4 = QN > 0 ? QN : (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const uint4* k32v = (const uint4*)k32;
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  const int64_t bias32 = 1ll << (30 - idx_bits);
  const uint32_t score_mask = (1u << (31 - idx_bits)) - 1;
  const uint64_t lt = (1ull << lane) - 1;
  if (PROPOSE && !CAND && tid == 0) rec->kp = 0;
  int done_tasks = 0;
  while (done_tasks < t_count) {
    const uint32_t T = (uint32_t)(t_count - done_tasks < kSegMax ? t_count - done_tasks : kSegMax);
    // ---- 1. S = the T best nodes by current key (CAND: chosen by the caller, slots in key order with their
    //         rows and static cache) ----
    uint32_t S;
    bool no_fit;
    if constexpr (CAND) {
      S = (uint32_t)sh.n_sel;
      no_fit = S == 0;
      if (pub.head != nullptr) {  // the nodes this job can commit to, for the selector's next job
        if (tid < (int)S) pub.set_node(tid, sh.node[tid]);
        if (tid == 0) pub.set_head(kPubModeSet, (int)S);
      }
    } else {
      no_fit = sel_pick<QN>(sh, k32, n, idx_bits, T, rp, S SEL_DIAG_ARGS) == 0;
    }
    if (!no_fit) {
      // zero the candidate lists (an unused entry reads as 0: never counted)
      {
        uint4* cv = (uint4*)cand;
#pragma unroll
        for (int q = 0; q < kCandV; ++q) cv[kCandV * tid + q] = make_uint4(0u, 0u, 0u, 0u);
      }
      __syncthreads();
      KB_SEL_PH(1);
      // ---- 2. selected nodes: rows, A; rank by key (8 threads per node) ----
      if (tid < (int)S) {
        const int w = sh.node[tid];
        Row r;
        if constexpr (CAND) {
          r = sh.row[tid];
        } else {
          r = load_row(N, w);
          sh.row[tid] = r;
          sh.stat[tid] = stat[w];
        }
        // (CAND: the selector computed A for its entries one job ahead -- off this chain; the previous set's rows
        // come with aux -1)
        sh.A[tid] = CAND && r.aux >= 0 ? r.aux : allocs_before_full(N, sp, sci, scr, r, w);
        sh.recip[0][tid] = 1.0 / (double)r.alloc_cpu;
        sh.recip[1][tid] = 1.0 / (double)r.alloc_mem;
        sh.cnt[tid] = 0;
        sh.gen[tid] = 0;
        sh.emin[tid] = 0xffffffffu;
        sh.fin[tid] = 0;
        sh.done[tid] = 0;
      }
      if constexpr (CAND) {
        // lmax and theta0 set by the caller (it ranked the candidates by key)
      } else {
        constexpr int kPer = 32;  // keys compared per thread: 4 threads per node, 128 nodes
        static_assert(kSelThreads == 4 * 128, "rank layout");
        const int s = tid >> 2, part = tid & 3;
        const uint32_t k = s < (int)S ? sh.key0[s] : 0u;
        uint32_t rk = 0;
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
          const int o = part * kPer + q;
          rk += sh.key0[o] > k;  // entries past S are 0 (sel_pick): no bound test, no branch
        }
        rk += dpp_src<0xb1>(0u, rk);  // quad_perm [1,0,3,2]
        rk += dpp_src<0x4e>(0u, rk);  // quad_perm [2,3,0,1]
        if (part == 0 && s < (int)S) {
          sh.lmax[s] = (int)(T - rk);
          if (rk == S - 1) sh.theta0 = k;
        }
      }
      __syncthreads();
      if (wv == 0) {
        const uint32_t a = lane < (int)S ? (uint32_t)sh.lmax[lane] : 0u;
        const uint32_t b = lane + 64 < (int)S ? (uint32_t)sh.lmax[lane + 64] : 0u;
        const uint32_t ea = wave_excl_scan_u32(a, lane), ta = wave_sum_u32(a);
        const uint32_t eb = wave_excl_scan_u32(b, lane);
        sh.off[lane] = (int32_t)ea;
        sh.off[lane + 64] = (int32_t)(ta + eb);
      }
      // ---- 3. e-sequences: rounds of 8 levels per node (64 once <= 16 remain), one lane per level,
      //         segmented prefix-min across the node's lanes ----
      const bool cut0 = S == T;  // level 0 of S fills the segment: elements below theta0 cannot rank < T
      __syncthreads();
      if constexpr (CAND) {
        // level 0 without a lane: every slot's own key is a candidate (the merge took feasible keys only, and when
        // S == T theta0 is the least of them), so the first round starts at level 1 and covers one level more per
        // node -- fewer jobs need a second round
        if (tid < (int)S) {
          const int lm = sh.lmax[tid];
          uint32_t e = sh.key0[tid];
          cand[sh.off[tid]] = ((uint64_t)e << 14) | ((uint64_t)(127 - tid) << 7) | 127u;
          int c = 1, g = 1, dn = lm <= 1;
          const uint64_t ci = clv != nullptr ? sh.comp[tid] : 0ull;
          if (ci != 0 && !dn) {
            // levels 1.. from the sweep's record (clv, the same closed-form keys the rounds below compute): the
            // prefix minimum while it stays feasible and above the cut-off, as a round would take them
            const uint4* lr = (const uint4*)(clv + (ci - 1) * kLvlW);
            const uint4 a = lr[0], b = lr[1];
            const uint32_t lv[kPreLevels] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z};
            const int jm = lm < kPreLevels + 1 ? lm : kPreLevels + 1;
            const uint32_t th = cut0 ? sh.theta0 : 0u;
            int j = 1;
#pragma unroll
            for (int q = 0; q < kPreLevels; ++q) {
              if (j != q + 1 || j >= jm) continue;  // (stopped)
              const uint32_t ee = lv[q] < e ? lv[q] : e;
              if (!(ee >> 31) || ee < th) continue;
              cand[sh.off[tid] + c] = ((uint64_t)ee << 14) | ((uint64_t)(127 - tid) << 7) | (uint64_t)(127 - j);
              ++c;
              e = ee;
              ++j;
            }
            g = j;
            dn = j < jm || j >= lm;
          }
          sh.cnt[tid] = c;
          sh.emin[tid] = e;
          sh.gen[tid] = g;
          if (dn) sh.done[tid] = 1;
        }
        if (wv == 0 && clv == nullptr) {  // the first round's active list beside it (active: lmax > 1), under the same barrier
          const bool a0 = lane < (int)S && sh.lmax[lane] > 1;
          const bool a1 = lane + 64 < (int)S && sh.lmax[lane + 64] > 1;
          const uint64_t m0 = __ballot(a0), m1 = __ballot(a1);
          const int c0 = __popcll(m0);
          if (a0) sh.act[__popcll(m0 & lt)] = lane;
          if (a1) sh.act[c0 + __popcll(m1 & lt)] = lane + 64;
          if (lane == 0) sh.n_act = c0 + __popcll(m1);
        }
        __syncthreads();
      }
      KB_SEL_PH(2);
      KB_PUB_TL(13);
      // (with level records the first round's active list needs the emission's done flags: built in the loop)
      for (bool first = CAND && clv == nullptr;; first = false) {
        if (!first) {
          if (wv == 0) {
            const bool a0 = lane < (int)S && !sh.done[lane];
            const bool a1 = lane + 64 < (int)S && !sh.done[lane + 64];
            const uint64_t m0 = __ballot(a0), m1 = __ballot(a1);
            const int c0 = __popcll(m0);
            if (a0) sh.act[__popcll(m0 & lt)] = lane;
            if (a1) sh.act[c0 + __popcll(m1 & lt)] = lane + 64;
            if (lane == 0) sh.n_act = c0 + __popcll(m1);
          }
          __syncthreads();
        }
        const int na = sh.n_act;
        if (na == 0) break;
        KB_SEL_COUNT(13, 1);
        // levels per active node this round: the largest power of two with na * L <= threads, at most 64
        int shift = 6;
        while (shift > 2 && (na << shift) > kSelThreads) --shift;
        const int L = 1 << shift;
        const int q = tid >> shift, u = tid & (L - 1);
        // whole lane groups of L share q; groups with q >= na idle (wave-uniform when L = 64)
        const bool live = q < na;
        const int s = live ? sh.act[q] : 0;
        const int j = live ? sh.gen[s] + u : 0;
        const int lm = live ? sh.lmax[s] : 0;
        uint32_t x = 0xffffffffu;
        if (live && j < lm) {
          x = sh.key0[s];
          if (j > 0) {
            const int w = sh.node[s];
            x = compress_key(traj_key64<true>(N, P, C, sp, sci, scr, sh.row[s], sh.stat[s], w, j, sh.A[s],
                                              sh.recip[0][s], sh.recip[1][s]),
                             w + N.base, idx_bits);
          }
        }
        // segmented inclusive prefix minimum over the group's lanes (levels in order)
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          if (o >= L) break;
          const uint32_t y = __shfl_up(x, o, L);
          if (u >= o) x = y < x ? y : x;
        }
        const uint32_t em = live ? sh.emin[s] : 0u;
        const uint32_t ee = x < em ? x : em;
        const bool valid = live && j < lm && (ee >> 31) && (!cut0 || ee >= sh.theta0);
        const uint64_t vm = __ballot(valid);
        const int gbase = lane & ~(L - 1) & 63;
        const uint32_t gm = L == 64 ? (uint32_t)__popcll(vm) : (uint32_t)__popcll((vm >> gbase) & ((1ull << L) - 1));
        // validity is a prefix of the group: e never increases, levels only grow
        const int c0 = live ? sh.cnt[s] : 0;
        if (valid) cand[sh.off[s] + c0 + u] = ((uint64_t)ee << 14) | ((uint64_t)(127 - s) << 7) | (uint64_t)(127 - j);
        const uint32_t elast = __shfl(ee, gbase + (gm ? gm - 1 : 0), 64);
        __syncthreads();  // every lane of the group has read the node's state
        if (live && u == 0) {
          sh.cnt[s] = c0 + (int)gm;
          if (gm) sh.emin[s] = elast;
          sh.gen[s] = sh.gen[s] + L;
          if ((int)gm < L || sh.gen[s] >= lm) sh.done[s] = 1;
        }
        __syncthreads();
      }
      KB_SEL_PH(3);
      KB_PUB_TL(14);
      // ---- 4. the T winners in pick order: rank every candidate when they fit one per thread, else a
      //         threshold on the score field plus per-slot takes, then rank the T taken ones ----
      uint64_t cs[2 * kCandV];
#pragma unroll
      for (int q = 0; q < kCandV; ++q) {
        const uint4 v = ((const uint4*)cand)[kCandV * tid + q];
        cs[2 * q] = (uint64_t)v.x | ((uint64_t)v.y << 32);
        cs[2 * q + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
      }
      uint32_t kc = 0;
#pragma unroll
      for (int q = 0; q < 2 * kCandV; ++q) kc += cs[q] != 0;
      uint32_t K, zero = 0, ztot;
      uint32_t pos = kc;
      sel_excl_scan2(sh, rp, pos, zero, &K, &ztot);
      KB_SEL_W(8);  // candidate loads + count scan
      KB_SEL_COUNT(15, K);
      if (K <= (uint32_t)KB_SEL_DENSE_MAX) {
#pragma unroll
        for (int q = 0; q < 2 * kCandV; ++q)
          if (cs[q]) sh.dense[pos++] = cs[q];
        __syncthreads();
        if (tid < (int)K) {  // composites are distinct: rank = number of larger ones
          const uint64_t v = sh.dense[tid];
          uint32_t r = 0;
#pragma unroll
          for (uint32_t q = 0; q < (uint32_t)KB_SEL_DENSE_MAX; ++q) r += (q < K) & (sh.dense[q] > v);
          if (r < T) sh.ord[r] = v;
        }
        if (tid == 0) sh.s_count = (int)(K < T ? K : T);
      } else {
        const int fs = 14 + idx_bits;  // score field of a composite
        uint32_t HX = 0, HN = 0xffffffffu, kk = kc;
#pragma unroll
        for (int q = 0; q < 2 * kCandV; ++q) {
          const uint32_t h = (uint32_t)(cs[q] >> fs);  // 0 for an unused entry
          HX = umax32(HX, h);
          HN = umin32(HN, cs[q] ? h : 0xffffffffu);
        }
        sel_reduce3(sh, rp, kk, HX, HN);
        KB_SEL_W(9);  // score range
        uint32_t lo = HN, hi = HX;  // K < T ends at lo = HN: every candidate
        while (lo < hi) {
          const uint32_t mid = lo + (hi - lo + 1) / 2;
          uint32_t c = 0;
#pragma unroll
          for (int q = 0; q < 2 * kCandV; ++q) c += cs[q] && (uint32_t)(cs[q] >> fs) >= mid;
          if (sel_sum(sh, rp, c) >= T) lo = mid;
          else hi = mid - 1;
          KB_SEL_COUNT(14, 1);
        }
        const uint32_t thr = lo;
        KB_SEL_W(10);  // threshold search
        if (wv == 0) {
          const int a = lane, b = lane + 64;
          const uint32_t ga = sel_cnt_ge(sh, cand, a, S, thr + 1, idx_bits);
          const uint32_t gb = sel_cnt_ge(sh, cand, b, S, thr + 1, idx_bits);
          const uint32_t qa = sel_cnt_ge(sh, cand, a, S, thr, idx_bits) - ga;
          const uint32_t qb = sel_cnt_ge(sh, cand, b, S, thr, idx_bits) - gb;
          const uint32_t R2 = T - wave_sum_u32(ga + gb);
          // ties on the threshold score: lower slot (= lower node index) first, then lower level
          const uint32_t Ea = wave_excl_scan_u32(qa, lane), Qa = wave_sum_u32(qa);
          const uint32_t Eb = Qa + wave_excl_scan_u32(qb, lane);
          const uint32_t ta = ga + (R2 > Ea ? (R2 - Ea < qa ? R2 - Ea : qa) : 0u);
          const uint32_t tb = gb + (R2 > Eb ? (R2 - Eb < qb ? R2 - Eb : qb) : 0u);
          const uint32_t pa = wave_excl_scan_u32(ta, lane), Ta = wave_sum_u32(ta);
          const uint32_t pb = Ta + wave_excl_scan_u32(tb, lane);
          for (uint32_t j = 0; j < ta; ++j) sh.comp[pa + j] = cand[sh.off[a] + j];
          for (uint32_t j = 0; j < tb; ++j) sh.comp[pb + j] = cand[sh.off[b] + j];
          // fewer candidates than tasks (K < T: the threshold is the lowest score and every candidate is
          // taken) fills only K entries
          const uint32_t Kt = K < T ? K : T;
          for (uint32_t p = Kt + lane; p < 128; p += 64) sh.comp[p] = 0;
          if (lane == 0) sh.s_count = (int)Kt;
        }
        __syncthreads();
        KB_SEL_W(11);  // per-slot takes
        {  // rank of every taken element, 4 threads per element
          const int e2 = tid >> 2, part = tid & 3;
          const uint64_t v = sh.comp[e2];
          uint32_t c = 0;
#pragma unroll
          for (int q2 = 0; q2 < 32; ++q2) c += sh.comp[part * 32 + q2] > v;
          c += dpp_src<0xb1>(0u, c);  // quad_perm [1,0,3,2]
          c += dpp_src<0x4e>(0u, c);  // quad_perm [2,3,0,1]
          if (part == 0 && e2 < sh.s_count) sh.ord[c] = v;
        }
      }
      __syncthreads();
      KB_SEL_PH(4);
      KB_PUB_TL(15);
      if constexpr (PROPOSE && CAND) {
        // the node-sharded fed engine's placer: the proposal stays in sh.ord[0..s_count) for the caller's exchange
        // and merge (shard_place)
        break;
      } else if constexpr (PROPOSE) {
        // the rank's proposal: its best picks in order with their global nodes and commit kinds; when it runs
        // out of feasible picks, the reason histogram of its rows after all of them (the no-fit case)
        const int Kp = sh.s_count;
        if (tid < Kp) {
          const uint64_t o = sh.ord[tid];
          const int s = sel_slot(o), j = sel_level(o);
          rec->comp[tid] = o;
          rec->node_kind[tid] = (sh.node[s] + N.base) | ((j < sh.A[s] ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE) << 30);
          if (Kp < (int)T) atomicAdd(&sh.fin[s], 1);
        }
        if (tid == 0) rec->kp = Kp;
        __syncthreads();
        if (Kp == (int)T) {
          if (tid < KB_NUM_REASONS) rec->hist[tid] = 0;
          break;
        }
        if (tid < (int)S && sh.fin[tid] > 0) {
          const int w = sh.node[tid], c = sh.fin[tid], A = sh.A[tid];
          k32[w] = compress_key(traj_key64(N, P, C, sp, sci, scr, sh.row[tid], sh.stat[tid], w, c, A), w + N.base,
                                idx_bits);
        }
        __syncthreads();
        no_fit = true;
      } else {
      // ---- stop rules in pick order (wave 0) ----
      if (wv == 0) {
        const int Kp = sh.s_count;
        const bool va = lane < Kp, vb = lane + 64 < Kp;
        const uint64_t oa = sh.ord[lane], ob = sh.ord[lane + 64];
        const bool aa = va && sel_level(oa) < sh.A[sel_slot(oa)];
        const bool ab = vb && sel_level(ob) < sh.A[sel_slot(ob)];
        const auto neg = [&](uint64_t o) {
          const uint32_t e32 = (uint32_t)(o >> 14);
          return (int64_t)((e32 >> idx_bits) & score_mask) - bias32 <= -1;
        };
        const uint64_t le_mask = lt | (1ull << lane);
        const uint64_t ma = __ballot(aa), mb = __ballot(ab);
        const int ra = ready + __popcll(ma & le_mask);
        const int rb = ready + __popcll(ma) + __popcll(mb & le_mask);
        const uint64_t sta = __ballot(va && (!gang || ra >= minav));
        const uint64_t stb = __ballot(vb && (!gang || rb >= minav));
        const uint64_t nga = __ballot(va && neg(oa)), ngb = __ballot(vb && neg(ob));
        const int first_stop = sta ? __builtin_ctzll(sta) : (stb ? 64 + __builtin_ctzll(stb) : 128);
        const int first_neg = nga ? __builtin_ctzll(nga) : (ngb ? 64 + __builtin_ctzll(ngb) : 128);
        int cut, kind;
        if (first_neg < Kp && first_neg <= first_stop) {
          cut = first_neg;  // SelectBestNode finds no score > -1 there: the reference panics
          kind = 3;
        } else if (first_stop < Kp) {
          cut = first_stop + 1;
          kind = KB_STOP_READY;
        } else if (Kp < (int)T) {
          cut = Kp;
          kind = KB_STOP_NO_FIT;
        } else {
          cut = (int)T;
          kind = -1;  // segment done, the run goes on
        }
        const int al = __popcll(cut >= 64 ? ma : (ma & ((1ull << cut) - 1))) +
                       (cut > 64 ? __popcll(mb & ((1ull << (cut - 64)) - 1)) : 0);
        if (lane == 0) {
          sh.cut = cut;
          sh.stop_kind = kind;
          sh.n_alloc = al;
        }
      }
      __syncthreads();
      // ---- commit: placements, rows, keys ----
      const int cut = sh.cut;
      const int kind = sh.stop_kind;
      const int base_c = sh.n_commit;  // (read before the barrier below: thread 0 rewrites it after it)
      if (tid < cut) {
        const uint64_t o = sh.ord[tid];
        const int s = sel_slot(o), j = sel_level(o);
        atomicAdd(&sh.fin[s], 1);
        const int at = t_begin + done_tasks + tid;
        hout[2 * at] = sh.node[s] + N.base;
        hout[2 * at + 1] = j < sh.A[s] ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE;
        if (pl != nullptr) pl[at - t_begin] = (uint32_t)sh.node[s] | (j < sh.A[s] ? 1u << 31 : 0u);
      }
      __syncthreads();
      // the touched nodes' keys matter only to a later segment or to the no-fit histogram; commit_out
      // lists the rows for the next job, whose level-0 sweep ran before these stores (kb_job_issue)
      const bool rekey = !CAND && (kind == KB_STOP_NO_FIT || (kind == -1 && done_tasks + cut < t_count));
      // the commit list's positions: slot order, from two ballots (S <= 128 slots: waves 0 and 1) -- an LDS
      // atomic counter serialised ~100 lanes on one word (~1 us per job)
      const bool has = tid < (int)S && sh.fin[tid] > 0;
      const uint64_t b_lo = __ballot(lane < (int)S && sh.fin[lane] > 0);
      const uint64_t b_hi = __ballot(lane + 64 < (int)S && sh.fin[lane + 64] > 0);
      if (has) {
        const int w = sh.node[tid], c = sh.fin[tid], A = sh.A[tid];
        store_back_row(N, P, sp, scr, w, c, A, sh.row[tid]);
        if (rekey)
          k32[w] = compress_key(traj_key64(N, P, C, sp, sci, scr, sh.row[tid], sh.stat[tid], w, c, A), w + N.base,
                                idx_bits);
        if (commit_out != nullptr) {
          const int at_c = base_c + (wv == 0 ? __popcll(b_lo & lt) : __popcll(b_lo) + __popcll(b_hi & lt));
          st_sc1(&commit_out[at_c], (int32_t)w);  // (fed_patch: ld_sc1)
        }
      }
      if (tid == 0) sh.n_commit = base_c + __popcll(b_lo) + __popcll(b_hi);
      __syncthreads();
      KB_SEL_PH(5);
      ready += sh.n_alloc;
      placed += cut;
      done_tasks += cut;
      if (kind == 3) {
        fail_task = t_begin + done_tasks;
        panic = 1;
        stopped = 1;
        break;
      }
      if (kind == KB_STOP_READY) {
        stop = KB_STOP_READY;
        stopped = 1;
        break;
      }
      no_fit = kind == KB_STOP_NO_FIT;
      }
    }
    if (no_fit) {
      if constexpr (CAND) {  // the caller rebuilds every node's key for the histogram (sh.need_hist)
        if (tid == 0) {
          sh.need_hist = 1;
          if (PROPOSE) sh.s_count = 0;  // (sharded placer: an empty proposal)
        }
        stop = KB_STOP_NO_FIT;
        fail_task = t_begin + done_tasks;
        stopped = 1;
        break;
      }
      // PredicateNodes found nothing (allocate.go:150-153): FitErrors histogram over all nodes at their
      // current keys (an infeasible key is its reason mask; padding keys are 0).
      sel_hist(sh, k32v, Q4);
      if (PROPOSE) {
        if (tid < KB_NUM_REASONS) rec->hist[tid] = sh.hist[tid];
        break;
      }
      if (tid < KB_NUM_REASONS) {
        js->hist[tid] = sh.hist[tid];
        hjs->hist[tid] = sh.hist[tid];
      }
      KB_SEL_PH(6);
      stop = KB_STOP_NO_FIT;
      fail_task = t_begin + done_tasks;
      stopped = 1;
      break;
    }
  }
}

// The level-0 keys into LDS (zero padding past n): every load of the thread is issued before the first
// LDS store, so the copy costs one memory latency instead of one per element.
template <int QU = kSelQ4>
__device__ __forceinline__ void load_keys_lds(uint32_t* k32, const uint32_t* keys32, int n, int n_pad) {
  const int tid = threadIdx.x;
  const int nv = n_pad >> 2, full = n >> 2;
  const uint4* src = (const uint4*)keys32;
  uint4* dst = (uint4*)k32;
  uint4 x[QU];
#pragma unroll
  for (int c = 0; c < QU; ++c) {
    const int v = tid + c * kSelThreads;
    x[c] = make_uint4(0u, 0u, 0u, 0u);
    if (v < full) {
      x[c] = src[v];
    } else if (v == full) {  // the vector n falls in
      const int b = 4 * v;
      x[c].x = b < n ? keys32[b] : 0u;
      x[c].y = b + 1 < n ? keys32[b + 1] : 0u;
      x[c].z = b + 2 < n ? keys32[b + 2] : 0u;
    }
  }
#pragma unroll
  for (int c = 0; c < QU; ++c) {
    const int v = tid + c * kSelThreads;
    if (v < nv) dst[v] = x[c];
  }
}

template <int QN>
__global__ __launch_bounds__(kSelThreads) void sel_place_kernel(
    DevNodes N, DevSpecs P, DevCfg C, int spec, int t_begin, int t_count, int idx_bits, const uint32_t* keys32,
    const uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0, int32_t* hout, JobState* hjs,
    uint32_t seq, SpecGuard g, int32_t* commit_out, const int32_t* patch, const JobState* patch_js,
    const uint32_t* wait_ctr, uint32_t wait_target, int pl_off) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  __shared__ SelShared sh;
  if ((!first && js->stopped) || guard_fails(g)) {
    if (threadIdx.x == 0) {
      // a skipped speculative job: later runs skip too, nothing for the next job to patch, and n_placed
      // (stale: an older job's) reads as nothing placed for the affinity table commit queued behind it
      if (first) js->n_placed = -1;
      js->stopped = 1;
      js->n_commit = 0;
    }
    signal_skip(hjs, seq);
    return;
  }
  const int tid = threadIdx.x;
  const int n = N.n;
  // node keys in contiguous groups of 4 per thread (index order decides the lowest-index tie-break);
  // the padding past n holds 0, an infeasible key with no reason bits
  const int Q4 = QN > 0 ? QN : (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const int n_pad = 4 * kSelThreads * Q4;
  uint32_t* k32 = lds32;           // [n_pad] current key of every node
  uint64_t* cand = (uint64_t*)(lds32 + n_pad);  // [kCandCap] candidate composites, a list per selected node
  const kb_spec sp = P.specs[spec];
#ifdef KB_DIAG
  // phases: 0 sweep wait + key load + patch (from kernel entry), 1 node selection, 2 selected-node setup,
  // 3 e-sequences, 4 winners + order, 5 stop rules + commit, 6 no-fit histogram (thread 0 stamps after
  // the block barriers); diag[7]: realtime ticks from entry to the publish
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  // the previous job's committed rows are final when this kernel starts: their loads go out before the
  // wait for this job's sweep (one per thread; lists longer than the block finish in the loop below)
  const int np = patch != nullptr ? patch_js->n_commit : 0;
  const int pw = tid < np ? patch[tid] : -1;
  Row prow;
  if (pw >= 0) prow = load_row(N, pw);
  if (wait_ctr != nullptr) {
    // this job's level-0 sweep runs on the other stream: wait for all its blocks (acquire), bounded so a
    // missing signal ends the kernel instead of hanging it (reported to the host through stall)
    if (tid == 0) {
      uint32_t spins = 0;
      while (__hip_atomic_load(wait_ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - wait_target > 0x7fffffffu) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins == (1u << 26)) {
          hjs->stall = 1;
          break;
        }
      }
    }
    __syncthreads();
  }
  const uint64_t pst = pw >= 0 ? stat[pw] : 0;  // issued with the key loads
  load_keys_lds<(QN > 0 ? QN : kSelQ4)>(k32, keys32, n, n_pad);
  if (tid == 0) sh.n_commit = 0;
  if (patch != nullptr) {
    // the level-0 sweep of this job overlapped the previous job's place kernel: re-key the rows that
    // job committed, from their stored state (the static cache is commit-independent)
    __syncthreads();
    const int64_t* sci = P.sc_init + (size_t)spec * N.S;
    if (pw >= 0) {
      const uint32_t rs = row_reasons(N, P, C, sp, sci, prow, pst, pw);
      k32[pw] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, prow, pst), pw), pw + N.base, idx_bits);
    }
    for (int i = tid + kSelThreads; i < np; i += kSelThreads) {
      const int w = patch[i];
      const Row r = load_row(N, w);
      const uint64_t st = stat[w];
      const uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, w);
      k32[w] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, r, st), w), w + N.base, idx_bits);
    }
  }
  int ready = first ? ready0 : js->ready_num;
  const int minav = first ? minav0 : js->min_available;
  const int gang = first ? gang0 : js->gang_ready;
  int placed = first ? 0 : js->n_placed;
  int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
  int rp = 0;
  __syncthreads();
  KB_SEL_PH(0);

  // pl_off > 0: the run's placements also into LDS (node | allocate << 31), for its affinity table commits below
  uint32_t* pl = pl_off > 0 ? lds32 + pl_off / 4 : nullptr;
  sel_run<false, QN>(sh, k32, cand, N, P, C, sp, spec, t_begin, t_count, idx_bits, stat, ready, minav, gang, placed,
                     stop, fail_task, panic, stopped, hout, js, hjs, rp, nullptr, commit_out SEL_DIAG_ARGS, FedPub{},
                     pl);
#ifdef KB_DIAG
  if (tid == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
  if (tid == 0) sh.lo = LoopOut{stop, fail_task, placed, ready, minav, gang, panic, stopped, 0, 0, 0, 0};
  // an affinity spec's commits into the global tables, after the whole run (a cap-1 run's closed form and its
  // later segments' keys read the tables as of the run's start) and before the publish: once the host has read
  // this job, its tables are final (a later job's sweep may start on the other stream then)
  if (pl != nullptr) {
    __syncthreads();
    for (int k = tid; k < sh.lo.placed - t_begin; k += kSelThreads)
      apply_commit_tables(P.A, sp, (int)(pl[k] & 0x7fffffffu), (int)(pl[k] >> 31), 1);
  }
  // every wave's host-buffer, row and table stores are complete before the barrier; one lane then releases
  // at system scope and publishes (the host spins on the sequence number)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if (commit_out != nullptr) js->n_commit = sh.n_commit;
    publish_state(js, hjs, sh.lo.stopped, sh.lo.stop, sh.lo.fail_task, sh.lo.placed, sh.lo.ready, sh.lo.minav,
                  sh.lo.gang, sh.lo.panic, seq);
  }
}

// ===========================================================================
// Placement engine: the selection path as ONE persistent workgroup serving kb_place_job calls.
// A per-job launch pays a cold instruction cache on whichever CU it lands on (the selection kernel's
// first pass over a phase ran 2.6x slower than a repeat of the same code) plus two launch latencies
// (level-0 sweep, selection). The engine keeps its code and the node table hot on one CU and takes
// each job from a mailbox in pinned host memory: per run it sweeps every node for the run's spec
// (keys straight into LDS), then runs the selection. It exits on an EXIT command, or by itself after
// idle_ticks without a command (recording which command it was waiting for in exit_seq), so a host
// that stops talking to it never leaves a kernel running.
// ===========================================================================
__device__ __forceinline__ uint32_t load_sys_u32(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ __launch_bounds__(kSelThreads) void engine_kernel(DevNodes N, DevSpecs P, DevCfg C, int idx_bits,
                                                             uint64_t* stat, const EngineCmd* cmd, JobState* js,
                                                             JobState* hjs, int32_t* hout, uint32_t seq0,
                                                             uint64_t idle_ticks) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  __shared__ SelShared sh;
  const int tid = threadIdx.x;
  const int n = N.n;
  const int Q4 = (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const int n_pad = 4 * kSelThreads * Q4;
  uint32_t* k32 = lds32;           // [n_pad] keys of the current run's spec
  uint64_t* cand = (uint64_t*)(lds32 + n_pad);  // [kCandCap]
  const EngineRun* runs = (const EngineRun*)(cmd + 1);
  for (int i = n + tid; i < n_pad; i += kSelThreads) k32[i] = 0u;  // padding: infeasible, no reasons
  int rp = 0;
#ifdef KB_DIAG
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
#endif
  for (uint32_t want = seq0;; ++want) {
    if (tid == 0) {  // one lane polls the mailbox
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int op = KB_ENG_EXIT_IDLE;
      for (;;) {
        if (load_sys_u32(&cmd->seq) == want) {
          op = cmd->op;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(1);
      }
      sh.cmd.op = op;
      if (op == KB_ENG_RUN) {
        sh.cmd.n_runs = cmd->n_runs;
        sh.cmd.ready0 = cmd->ready0;
        sh.cmd.minav0 = cmd->minav0;
        sh.cmd.gang0 = cmd->gang0;
      }
      sh.t_recv = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const int op = sh.cmd.op;
    if (op != KB_ENG_RUN) {
      if (tid == 0 && op == KB_ENG_EXIT_IDLE)
        __hip_atomic_store(&hjs->exit_seq, want, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      break;
    }
#ifdef KB_DIAG
    for (int k = 0; k < 7; ++k) dg[k] = 0;
    dg_last = __builtin_amdgcn_s_memtime();
    const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
    int ready = sh.cmd.ready0, placed = 0;
    const int minav = sh.cmd.minav0, gang = sh.cmd.gang0, n_runs = sh.cmd.n_runs;
    int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
    for (int r = 0; r < n_runs && !stopped; ++r) {
      if (tid == 0) sh.run = runs[r];
      __syncthreads();
      const int spec = sh.run.spec;
      {  // level-0 keys of the run's spec (every node) into LDS, its static cache into `stat`
        const kb_spec sp = P.specs[spec];
        const int64_t* sci = P.sc_init + (size_t)spec * N.S;
        for (int i = tid; i < n; i += kSelThreads) {
          const Row row = load_row(N, i);
          const uint64_t st = static_eval<false>(N, P, C, sp, spec, row.flags, i, nullptr);
          stat[i] = st;
          const uint32_t rs = row_reasons(N, P, C, sp, sci, row, st, i);
          k32[i] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, row, st), i), i + N.base, idx_bits);
        }
      }
      __syncthreads();
      KB_SEL_PH(0);
      const kb_spec sp = P.specs[spec];
      sel_run(sh, k32, cand, N, P, C, sp, spec, sh.run.t_begin, sh.run.t_count, idx_bits, stat, ready, minav, gang, placed,
              stop, fail_task, panic, stopped, hout, js, hjs, rp, nullptr, nullptr SEL_DIAG_ARGS);
    }
#ifdef KB_DIAG
    if (tid == 0) {
      for (int k = 0; k < 7; ++k) hjs->diag[k] = dg[k];
      hjs->diag[7] = __builtin_amdgcn_s_memrealtime() - rt0;
    }
#endif
    // every wave's placement and row stores are complete before the barrier; one lane then releases at
    // system scope and publishes the job state (the host spins on the sequence number)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      hjs->t_recv = sh.t_recv;
      hjs->t_done = __builtin_amdgcn_s_memrealtime();
      __threadfence_system();
      publish_state(js, hjs, stopped, stop, fail_task, placed, ready, minav, gang, panic, want);
    }
  }
}

void launch_engine(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, uint64_t* stat,
                   const EngineCmd* cmd, JobState* js, JobState* hjs, int32_t* hout, uint32_t seq0,
                   uint64_t idle_ticks, void* stream) {
  hipLaunchKernelGGL(engine_kernel, dim3(1), dim3(kSelThreads), sel_lds_bytes(N.n), (hipStream_t)stream, N, P, C,
                     idx_bits, stat, cmd, js, hjs, hout, seq0, idle_ticks);
}

// Level-0 keys for the selection path: one node per thread, 64-thread blocks (a 10k-node table is
// ~160 workgroups, spread over the chip), no trajectory levels.
// A fed-engine job command (fed_engine_kernel): written by the job's level-0 sweep into a device ring entry.
struct FedCmd {
  int32_t op;  // KB_ENG_RUN / KB_ENG_EXIT
  int32_t spec, t_begin, t_count, ready0, minav0, gang0, slot;
  int32_t g_valid, g_stop, g_placed, g_ready;  // SpecGuard on the previous job's outcome
  uint32_t seq;
  int32_t fresh;  // the first command after the engine was paused (kb_fed_pause): the job's sweep ran after every
                  // earlier job committed and after the launch-path units of the pause, whose commits the engine's
                  // own bookkeeping (the previous jobs' sets, rows and commit lists) does not know: none is used
  int32_t acq;    // the job reads global columns the selection path stores plain (a spec with scalar or host-port
                  // columns), or follows a pause: the selector and the placer take an agent acquire before it
  int32_t fresh_m;  // the launch's most recent fresh command at or before this one: every earlier command is final
};
static_assert(sizeof(FedCmd) == 64, "the split engine's selector forwards commands as 8 words");

// The level-0 sweep of a selection run: every node's 32-bit key and static cache for `spec`. done_ctr: each block
// adds 1 with an agent-scope release once its keys are written (the overlapped sweep of the launch path; the fed
// engine's ring counter). ring (fed engine): block 0 also writes the job's command there before its release.
template <bool AFF>
__global__ __launch_bounds__(64) void sel_sweep_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, int idx_bits,
                                                      uint32_t* keys32, uint64_t* stat, const JobState* js,
                                                      SpecGuard g, uint32_t* done_ctr, FedCmd cmd, FedCmd* ring) {
  if ((js != nullptr && js->stopped) || guard_fails(g)) return;
  const int n = blockIdx.x * 64 + threadIdx.x;
  if (n < N.n) {
    const kb_spec sp = P.specs[spec];
    const Row r = load_row(N, n);
    const uint64_t st = static_eval<AFF>(N, P, C, sp, spec, r.flags, n, P.A.mm);
    stat[n] = st;
    const uint32_t rs = row_reasons(N, P, C, sp, P.sc_init + (size_t)spec * N.S, r, st, n);
    keys32[n] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, r, st), n), n + N.base, idx_bits);
  }
  // overlapped sweep (stream_b): one release per block (the wave's stores, written back to memory for
  // the place kernel on another XCD), counted by the place kernel of the same job (or the fed engine)
  if (threadIdx.x == 0) {
    if (ring != nullptr && blockIdx.x == 0) *ring = cmd;
    if (done_ctr != nullptr) __hip_atomic_fetch_add(done_ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

void launch_sel_sweep(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int idx_bits, uint32_t* keys32,
                      uint64_t* stat, const JobState* js, bool aff, void* stream, SpecGuard g,
                      uint32_t* done_ctr, const FedCmdArgs* fed, void* ring) {
  const int blocks = (N.n + 63) / 64;
  FedCmd cmd{};
  if (fed)
    cmd = FedCmd{fed->op, fed->spec, fed->t_begin, fed->t_count, fed->ready0, fed->minav0, fed->gang0, fed->slot,
                 fed->g_valid, fed->g_stop, fed->g_placed, fed->g_ready, fed->seq, fed->fresh, fed->acq, 0};
  FedCmd* rg = fed ? (FedCmd*)ring : nullptr;
  if (aff)
    hipLaunchKernelGGL(sel_sweep_kernel<true>, dim3(blocks), dim3(64), 0, (hipStream_t)stream, N, P, C, spec, idx_bits,
                       keys32, stat, js, g, done_ctr, cmd, rg);
  else
    hipLaunchKernelGGL(sel_sweep_kernel<false>, dim3(blocks), dim3(64), 0, (hipStream_t)stream, N, P, C, spec,
                       idx_bits, keys32, stat, js, g, done_ctr, cmd, rg);
}

// ===========================================================================
// Node sharding across GPUs. Every rank holds a contiguous block of the canonical node
// table. Because the picks of a run come out in descending composite order (the selection argument
// above), the global first-T picks are the T largest of the union of every rank's own first-T picks:
// one all-gather of the ranks' proposals per segment replaces a collective per task. Each rank then
// merges the same proposals into the same global order, applies the stop rules, and commits the picks
// that land on its own rows.
// ===========================================================================
static_assert(kShardSegMax == kSegMax, "ShardRec holds one segment");

__global__ __launch_bounds__(kSelThreads) void shard_propose_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec,
                                                                    int t_count, int idx_bits,
                                                                    const uint32_t* keys32, const uint64_t* stat,
                                                                    const JobState* js, int first, ShardRec* rec,
                                                                    SpecGuard g, const int32_t* patch,
                                                                    const JobState* patch_js, const uint32_t* wait_ctr,
                                                                    uint32_t wait_target, JobState* hjs, uint4 tag) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  __shared__ SelShared sh;
  // the segment's commit kernel skips too (every rank sees the same job state: the exchange still runs, and
  // only its tag is read)
  const bool skip = (!first && js->stopped) || guard_fails(g);
  if (threadIdx.x == 0) {
    rec->tag[0] = tag.x;
    rec->tag[1] = tag.y;
    rec->tag[2] = tag.z;
    rec->tag[3] = tag.w | (skip ? 0x80000000u : 0u);
  }
  if (skip) return;
  const int tid = threadIdx.x;
  const int n = N.n;
  const int Q4 = (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const int n_pad = 4 * kSelThreads * Q4;
  uint32_t* k32 = lds32;
  uint64_t* cand = (uint64_t*)(lds32 + n_pad);
  const kb_spec sp = P.specs[spec];
  // overlapped sweep (as sel_place_kernel): the previous job's committed rows of this rank load first, then
  // the wait for this job's sweep on the other stream, then those rows are re-keyed from their stored state
  const int np = patch != nullptr ? patch_js->n_commit : 0;
  const int pw = tid < np ? patch[tid] : -1;
  Row prow;
  if (pw >= 0) prow = load_row(N, pw);
  if (wait_ctr != nullptr) {
    if (tid == 0) {
      uint32_t spins = 0;
      while (__hip_atomic_load(wait_ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - wait_target > 0x7fffffffu) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins == (1u << 26)) {
          hjs->stall = 1;
          break;
        }
      }
    }
    __syncthreads();
  }
  const uint64_t pst = pw >= 0 ? stat[pw] : 0;
  load_keys_lds(k32, keys32, n, n_pad);
  if (patch != nullptr) {
    __syncthreads();
    const int64_t* sci = P.sc_init + (size_t)spec * N.S;
    if (pw >= 0) {
      const uint32_t rs = row_reasons(N, P, C, sp, sci, prow, pst, pw);
      k32[pw] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, prow, pst), pw), pw + N.base, idx_bits);
    }
  }
  int ready = 0, placed = 0, stop = 0, fail_task = -1, panic = 0, stopped = 0, rp = 0;
#ifdef KB_DIAG
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
#endif
  __syncthreads();
  sel_run<true>(sh, k32, cand, N, P, C, sp, spec, 0, t_count, idx_bits, stat, ready, 0, 0, placed, stop, fail_task,
                panic, stopped, nullptr, nullptr, nullptr, rp, rec, nullptr SEL_DIAG_ARGS);
}

// Elements of a proposal list (descending) greater than v.
__device__ __forceinline__ int shard_count_gt(const uint64_t* list, int len, uint64_t v) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (list[mid] > v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}


__global__ __launch_bounds__(kSelThreads) void shard_commit_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec,
                                                                   int t_begin, int t_count, int idx_bits,
                                                                   const ShardRec* recs, int world, JobState* js,
                                                                   int first, int ready0, int minav0, int gang0,
                                                                   int32_t* hout, JobState* hjs, uint32_t seq,
                                                                   SpecGuard g, int32_t* commit_out) {
  __shared__ ShardRec r[kShardMaxWorld];
  __shared__ uint64_t ord[128];
  __shared__ int32_t ordnk[128];
  __shared__ int32_t fin[128], fin_node[128];
  __shared__ int32_t s_cut, s_kind, s_alloc, s_ncommit;
  __shared__ LoopOut lo;
  if (threadIdx.x == 0) {  // every rank exchanged the same segment (a divergence would otherwise hang later)
    bool same = true;
    for (int w = 1; w < world; ++w)
      for (int q = 0; q < 4; ++q) same = same && recs[w].tag[q] == recs[0].tag[q];
    if (!same) hjs->stall = 2;
  }
  if ((!first && js->stopped) || guard_fails(g)) {
    if (threadIdx.x == 0 && first) {  // a skipped speculative job (see sel_place_kernel)
      js->stopped = 1;
      js->n_placed = -1;
      js->n_commit = 0;
    }
    signal_skip(hjs, seq);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t T = (uint32_t)t_count;
  const int64_t bias32 = 1ll << (30 - idx_bits);
  const uint32_t score_mask = (1u << (31 - idx_bits)) - 1;
  const uint64_t lt = (1ull << lane) - 1;
  {  // every rank's proposal into LDS
    const uint4* src = (const uint4*)recs;
    uint4* dst = (uint4*)r;
    const int words = world * (int)(sizeof(ShardRec) / 16);
    for (int i = tid; i < words; i += kSelThreads) dst[i] = src[i];
  }
  if (tid == 0) s_ncommit = 0;
  if (tid < 128) fin[tid] = 0;
  const int ready_in = first ? ready0 : js->ready_num;
  const int minav = first ? minav0 : js->min_available;
  const int gang = first ? gang0 : js->gang_ready;
  const int placed_in = first ? 0 : js->n_placed;
  __syncthreads();
  // global pick order: rank of proposal i of rank g = i + the larger proposals of every other rank
  int K = 0;
  for (int g = 0; g < world; ++g) K += r[g].kp;
  for (int e = tid; e < world * kShardSegMax; e += kSelThreads) {
    const int g = e / kShardSegMax, i = e % kShardSegMax;
    if (i >= r[g].kp) continue;
    const uint64_t v = r[g].comp[i];
    int rank = i;
    for (int h = 0; h < world; ++h)
      if (h != g) rank += shard_count_gt(r[h].comp, r[h].kp, v);
    if (rank < (int)T) {
      ord[rank] = v;
      ordnk[rank] = r[g].node_kind[i];
    }
  }
  __syncthreads();
  const int Kp = K < (int)T ? K : (int)T;
  if (wv == 0) {  // stop rules in pick order (as the one-GPU selection kernel applies them)
    const bool va = lane < Kp, vb = lane + 64 < Kp;
    const uint64_t oa = va ? ord[lane] : 0, ob = vb ? ord[lane + 64] : 0;
    const bool aa = va && ((uint32_t)ordnk[lane] >> 30) == KB_PLACE_ALLOCATE;
    const bool ab = vb && ((uint32_t)ordnk[lane + 64] >> 30) == KB_PLACE_ALLOCATE;
    const auto neg = [&](uint64_t o) {
      const uint32_t e32 = (uint32_t)(o >> 14);
      return (int64_t)((e32 >> idx_bits) & score_mask) - bias32 <= -1;
    };
    const uint64_t le_mask = lt | (1ull << lane);
    const uint64_t ma = __ballot(aa), mb = __ballot(ab);
    const int ra = ready_in + __popcll(ma & le_mask);
    const int rb = ready_in + __popcll(ma) + __popcll(mb & le_mask);
    const uint64_t sta = __ballot(va && (!gang || ra >= minav));
    const uint64_t stb = __ballot(vb && (!gang || rb >= minav));
    const uint64_t nga = __ballot(va && neg(oa)), ngb = __ballot(vb && neg(ob));
    const int first_stop = sta ? __builtin_ctzll(sta) : (stb ? 64 + __builtin_ctzll(stb) : 128);
    const int first_neg = nga ? __builtin_ctzll(nga) : (ngb ? 64 + __builtin_ctzll(ngb) : 128);
    int cut, kind;
    if (first_neg < Kp && first_neg <= first_stop) {
      cut = first_neg;
      kind = 3;
    } else if (first_stop < Kp) {
      cut = first_stop + 1;
      kind = KB_STOP_READY;
    } else if (Kp < (int)T) {
      cut = Kp;
      kind = KB_STOP_NO_FIT;
    } else {
      cut = (int)T;
      kind = -1;
    }
    const int al = __popcll(cut >= 64 ? ma : (ma & ((1ull << cut) - 1))) +
                   (cut > 64 ? __popcll(mb & ((1ull << (cut - 64)) - 1)) : 0);
    if (lane == 0) {
      s_cut = cut;
      s_kind = kind;
      s_alloc = al;
    }
  }
  __syncthreads();
  const int cut = s_cut, kind = s_kind;
  // placements (every rank writes the whole sequence) and this rank's commits, counted per local slot
  if (tid < cut) {
    const int nk = ordnk[tid];
    const int node = nk & 0x3fffffff;
    hout[2 * (t_begin + tid)] = node;
    hout[2 * (t_begin + tid) + 1] = (int32_t)((uint32_t)nk >> 30);
    if (node >= N.base && node < N.base + N.n) {
      const int s = sel_slot(ord[tid]);
      atomicAdd(&fin[s], 1);
      fin_node[s] = node - N.base;
    }
  }
  __syncthreads();
  if (tid < 128 && fin[tid] > 0) {  // NodeInfo.AddTask x c on the rank's own row
    const kb_spec sp = P.specs[spec];
    const int64_t* sci = P.sc_init + (size_t)spec * N.S;
    const int64_t* scr = P.sc_req + (size_t)spec * N.S;
    const int w = fin_node[tid];
    const Row row = load_row(N, w);
    store_back_row(N, P, sp, scr, w, fin[tid], allocs_before_full(N, sp, sci, scr, row, w), row);
    if (commit_out != nullptr) commit_out[atomicAdd(&s_ncommit, 1)] = w;  // for the next job's overlapped sweep
  }
  int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
  if (kind == 3) {
    fail_task = t_begin + cut;
    panic = 1;
    stopped = 1;
  } else if (kind == KB_STOP_READY) {
    stop = KB_STOP_READY;
    stopped = 1;
  } else if (kind == KB_STOP_NO_FIT) {  // FitErrors over all ranks' rows
    if (tid < KB_NUM_REASONS) {
      uint32_t h = 0;
      for (int g = 0; g < world; ++g) h += r[g].hist[tid];
      js->hist[tid] = h;
      hjs->hist[tid] = h;
    }
    stop = KB_STOP_NO_FIT;
    fail_task = t_begin + cut;
    stopped = 1;
  }
  if (tid == 0)
    lo = LoopOut{stop, fail_task, placed_in + cut, ready_in + s_alloc, minav, gang, panic, stopped, 0, 0, 0, 0};
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if (commit_out != nullptr) js->n_commit = s_ncommit;
    __threadfence_system();
    publish_state(js, hjs, lo.stopped, lo.stop, lo.fail_task, lo.placed, lo.ready, lo.minav, lo.gang, lo.panic, seq);
  }
}

void launch_shard_propose(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_count,
                          int idx_bits, const uint32_t* keys32, const uint64_t* stat, const JobState* js, int first,
                          ShardRec* rec, SpecGuard g, const int32_t* patch, const JobState* patch_js,
                          const uint32_t* wait_ctr, uint32_t wait_target, JobState* hjs, void* stream,
                          const uint32_t* tag) {
  hipLaunchKernelGGL(shard_propose_kernel, dim3(1), dim3(kSelThreads), sel_lds_bytes(N.n), (hipStream_t)stream, N, P,
                     C, spec, t_count, idx_bits, keys32, stat, js, first, rec, g, patch, patch_js, wait_ctr,
                     wait_target, hjs, make_uint4(tag[0], tag[1], tag[2], tag[3]));
}

void launch_shard_commit(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                         int idx_bits, const ShardRec* recs, int world, JobState* js, int first, int ready0,
                         int minav0, int gang0, int32_t* hout, JobState* hjs, uint32_t seq, SpecGuard g,
                         int32_t* commit_out, void* stream) {
  hipLaunchKernelGGL(shard_commit_kernel, dim3(1), dim3(kSelThreads), 0, (hipStream_t)stream, N, P, C, spec, t_begin,
                     t_count, idx_bits, recs, world, js, first, ready0, minav0, gang0, hout, hjs, seq, g, commit_out);
}

int sel_lds_bytes(int n) {
  const long q4 = ((long)n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const long bytes = 4l * (4 * kSelThreads * q4) + 8l * kCandCap;
  return q4 <= kSelQ4 && bytes <= kSelDynLimit ? (int)bytes : -1;
}

// The sel_place_kernel instance for n: the smallest instantiated group count >= ceil(n / 2048) whose LDS
// plan fits, else the run-time-count instance (0).
static int sel_qn(int n) {
  const int q4 = (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  for (int qn : {1, 2, 3, 4, 5, 6, 8, 10}) {
    if (qn < q4) continue;
    const long bytes = 4l * (4 * kSelThreads * qn) + 8l * kCandCap;
    return bytes <= kSelDynLimit ? qn : 0;
  }
  return 0;
}

void launch_sel_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                      int idx_bits, const uint32_t* keys32, const uint64_t* stat, JobState* js, int first, int ready0,
                      int minav0, int gang0, int32_t* hout, JobState* hjs, uint32_t seq, void* stream,
                      SpecGuard g, int32_t* commit_out, const int32_t* patch, const JobState* patch_js,
                      const uint32_t* wait_ctr, uint32_t wait_target, int aff_pl) {
  const int qn = sel_qn(N.n);
  const int base = qn > 0 ? 4 * (4 * kSelThreads * qn) + 8 * kCandCap : sel_lds_bytes(N.n);
  const int pl_off = aff_pl && base + 4 * t_count <= kSelDynLimit ? base : 0;  // (caller: sel_aff_pl_fits)
  const int bytes = base + (pl_off ? 4 * t_count : 0);
#define KB_SEL_QN(Q)                                                                                                \
  case Q:                                                                                                          \
    hipLaunchKernelGGL(sel_place_kernel<Q>, dim3(1), dim3(kSelThreads), bytes, (hipStream_t)stream, N, P, C, spec,  \
                       t_begin, t_count, idx_bits, keys32, stat, js, first, ready0, minav0, gang0, hout, hjs, seq, \
                       g, commit_out, patch, patch_js, wait_ctr, wait_target, pl_off);                             \
    break;
  switch (qn) {
    KB_SEL_QN(1)
    KB_SEL_QN(2)
    KB_SEL_QN(3)
    KB_SEL_QN(4)
    KB_SEL_QN(5)
    KB_SEL_QN(6)
    KB_SEL_QN(8)
    KB_SEL_QN(10)
    default:
      hipLaunchKernelGGL(sel_place_kernel<0>, dim3(1), dim3(kSelThreads), bytes, (hipStream_t)stream, N, P, C, spec,
                         t_begin, t_count, idx_bits, keys32, stat, js, first, ready0, minav0, gang0, hout, hjs, seq,
                         g, commit_out, patch, patch_js, wait_ctr, wait_target, pl_off);
  }
#undef KB_SEL_QN
}

bool sel_aff_pl_fits(int n, int t_count) {
  const int qn = sel_qn(n);
  const int base = qn > 0 ? 4 * (4 * kSelThreads * qn) + 8 * kCandCap : sel_lds_bytes(n);
  return base + 4 * t_count <= kSelDynLimit;
}


// ===========================================================================
// Fed engine: the selection place kernel as ONE resident workgroup for a whole allocate cycle, fed through
// device memory. Per job (one selection run) the host launches only the run's level-0 sweep (sel_sweep_kernel,
// the launch path's own) on the sweep stream: it computes the keys and static cache into the job slot's buffers, block 0
// writes the run's command into a kJobSlots-entry ring, and every block adds one to the ring entry's
// counter with an agent-scope release. The engine waits for the counter (acquire), checks the command's
// guard against the previous job's outcome, re-keys the rows the previous two jobs committed (its sweep may
// have overlapped both), runs the selection and publishes to the slot's pinned host buffers exactly as
// sel_place_kernel does. No per-job kernel boundary on the place stream: the launch gap, the end-of-
// kernel release and the next kernel's acquire (5.6 us median between place kernels) go away.
// ===========================================================================

constexpr int kFedGridMax = 256;
// Level records (split engine with resident sweepers): for every feasible node the sweep also computes its keys after
// 1..kPreLevels commits of the job's spec (traj_key64, the e-sequences' levels) and A (allocs_before_full), kLvlW words
// per node; the selector forwards them with its candidates, so the placer's first e-sequence round is a prefix
// minimum over loaded values instead of kPreLevels closed-form keys per slot on its critical chain.
// (kPreLevels, kLvlW: kbgpu_device.h)
// a selector entry's first word: key (bits 0..31), node (32..55: the split engine's tables are below 2^24 nodes,
// kFedMaxSel * kFedSelNodes), the node's rank among the list's first T (56..62)
constexpr uint64_t kEntNodeMask = 0xffffffull;  // the split engine's grid: placer, selectors, resident sweepers (one per CU)

struct FedSlots {
  uint32_t* keys[kJobSlots];
  uint64_t* stat[kJobSlots];
  int32_t* commits[kJobSlots];
  JobState* js[kJobSlots];   // device job state per slot
  JobState* hjs[kJobSlots];  // pinned host job state per slot (device addresses)
  int32_t* hout[kJobSlots];  // pinned host placements per slot (device addresses)
  uint32_t tgt[kJobSlots];   // ring counters' targets at launch
  // the resident sweepers' level records per slot ([n][kLvlW]: the node's keys after 1..kPreLevels commits, then A),
  // nullptr when the sweeps come from sweep kernels (no records)
  uint32_t* lvl[kJobSlots];
};

// A command without a sweep (EXIT): the ring entry and the whole block count at once.
template <bool AFF>
__global__ __launch_bounds__(64) void fed_cmd_sweep_kernel(DevNodes N, DevSpecs P, DevCfg C, int idx_bits,
                                                          uint32_t* keys32, uint64_t* stat, FedCmd cmd, FedCmd* ring,
                                                          uint32_t* ctr, int sweep) {
  const int n = blockIdx.x * 64 + threadIdx.x;
  if (sweep && n < N.n) {
    const kb_spec sp = P.specs[cmd.spec];
    const Row r = load_row(N, n);
    const uint64_t st = static_eval<AFF>(N, P, C, sp, cmd.spec, r.flags, n, P.A.mm);
    stat[n] = st;
    const uint32_t rs = row_reasons(N, P, C, sp, P.sc_init + (size_t)cmd.spec * N.S, r, st, n);
    keys32[n] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, r, st), n), n + N.base, idx_bits);
  }
  if (threadIdx.x == 0) {
    if (blockIdx.x == 0) *ring = cmd;
    // a non-sweeping command (EXIT) adds the whole count at once
    const uint32_t add = sweep ? 1u : (uint32_t)((N.n + 63) / 64);
    __hip_atomic_fetch_add(ctr, add, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// The split engine's resident sweepers (the census grid's workgroups that are neither placer nor selector, off the
// placer's XCC): the job's level-0 sweep without a kernel launch per job. The host writes command m of the launch
// into the pinned ring entry m % kJobSlots (FedHostCmd: the command's eight words, then the tag epoch << 32 | m + 1,
// a release store). Sweeper 0 polls that tag (system-scope loads, its thread 0) and relays the words and the tag to
// device memory (sc1 stores, vmcnt(0), then the tag: MI355X_MICROARCH.md's hand-off table, first row), where the
// other sweepers poll it (sc1 loads) -- one reader on the bus. Each sweeper then takes one agent-scope acquire (the
// rows its loads read were committed by the placer and released at its publish, or by the launch path during a
// pause), sweeps its share of the 64-node blocks into the slot's keys and static cache, releases, and adds its block
// count to the ring counter the selector waits on -- the count the sweep kernel's blocks gave. Sweeper 0 also
// writes the command into the device ring (before its release). EXIT ends the loop after its count; a sweeper
// leaves too when the engine's exit flag is set or no command comes within idle_ticks.
// Groups: the sweepers form kSweepGroups groups that take the commands in turn (command m: group m % G), each sweeping
// the whole table with its own members, so a group has G job times for a sweep -- one sweep's latency chain (the
// relay, the acquire, the row loads, the level records, the release) is longer than one placer job (r06f: with the
// level records one group fell behind the placer, the selector's commands came 6 us later). Each group's first member
// polls the host ring for its commands and relays them; the group that takes EXIT raises sw_exit for the others.
constexpr int kSweepGroups = 2;
__device__ __forceinline__ void fed_sweeper(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, const FedSlots& S,
                            const FedHostCmd* hring, uint32_t epoch, FedCmd* ring, uint32_t* ctr,
                            uint64_t idle_ticks, int32_t* exit_flag, int sw, int nsw, uint64_t* relay_cmd,
                            uint64_t* relay_go, uint32_t* sw_exit) {
  static_assert(kJobSlots % kSweepGroups == 0, "a ring entry belongs to one sweeper group");
  __shared__ FedCmd s_cmd;
  __shared__ int32_t s_go;
  const int tid = threadIdx.x;
  const int G = nsw >= 2 * kSweepGroups ? kSweepGroups : 1;
  const int g = sw % G, sg = sw / G, ng = (nsw - g + G - 1) / G;  // group, index in it, its members
  const uint32_t B = (uint32_t)((N.n + 63) / 64);
  const uint32_t b0 = (uint32_t)((uint64_t)sg * B / (uint32_t)ng), b1 = (uint32_t)((uint64_t)(sg + 1) * B / (uint32_t)ng);
  const int n0 = (int)b0 * 64, n1 = min((int)b1 * 64, N.n);
  const bool lead = sg == 0;
  for (uint32_t m = (uint32_t)g;; m += (uint32_t)G) {
    const int r = (int)(m % (uint32_t)kJobSlots);
    if (tid == 0) {
      const uint64_t want = ((uint64_t)epoch << 32) | (uint64_t)(m + 1);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      int go = 0;
      // the group's first member polls the pinned ring over the bus; the others poll its relay in device memory
      const uint64_t* tagp = lead ? &hring[r].tag : &relay_go[r];
      for (;;) {
        if (__hip_atomic_load(tagp, __ATOMIC_RELAXED, lead ? __HIP_MEMORY_SCOPE_SYSTEM : __HIP_MEMORY_SCOPE_AGENT) ==
            want) {
          go = 1;
          break;
        }
        if (__hip_atomic_load(exit_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
        if (__hip_atomic_load(sw_exit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (go) {  // the words stored before the tag
        uint64_t w[8];
        if (lead) {
#pragma unroll
          for (int q = 0; q < 8; ++q) w[q] = __hip_atomic_load(&hring[r].w[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#pragma unroll
          for (int q = 0; q < 8; ++q) st_sc1(&relay_cmd[r * 8 + q], w[q]);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          st_sc1(&relay_go[r], want);
        } else {
#pragma unroll
          for (int q = 0; q < 8; ++q) w[q] = ld_sc1(&relay_cmd[r * 8 + q]);
        }
        __builtin_memcpy(&s_cmd, w, sizeof(FedCmd));
        if (s_cmd.op == KB_ENG_RUN) {
#ifndef KB_WA_NO_SWACQ  // (write-accounting A/B builds only: scripts/write_account.sh)
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
#endif
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (the barrier below holds the other waves' loads)
        }
      }
      s_go = go;
    }
    __syncthreads();
    if (!s_go) return;
    // (the fields the sweep uses, as scalars: a private copy of the whole command went to scratch, and every
    // sweeper's per-job release then wrote those dirty scratch lines back to memory -- 56 B per lane per job, most of
    // the engine's WRITE_SIZE before round 6's write accounting found it)
    const int op = s_cmd.op, cspec = s_cmd.spec, cslot = s_cmd.slot;
    if (op == KB_ENG_RUN) {
      const kb_spec sp = P.specs[cspec];
      uint32_t* keys32 = S.keys[cslot];
      uint64_t* stat = S.stat[cslot];
      const int64_t* sci = P.sc_init + (size_t)cspec * N.S;
      uint32_t* lvl = S.lvl[cslot];
      const int64_t* scr = P.sc_req + (size_t)cspec * N.S;
      for (int n = n0 + tid; n < n1; n += kSelThreads) {
#ifdef KB_WA_NO_SWROWS  // (write-accounting A/B: the sweep without its row loads -- wrong keys)
        Row rw{};
        rw.alloc_cpu = rw.alloc_mem = rw.idle_cpu = rw.idle_mem = 1ll << 40;
        rw.max_pods = 110;
#else
        const Row rw = load_row(N, n);
#endif
        // an affinity unit (kb_spec_fed_ok: its inputs stay as they are through the run) folds the inter-pod checks
        // and its InterPodAffinity score, normalised by the min / max the host prepared for its spec, into the
        // static cache, as the launch path's selection sweep does
        // (inlined: as a call it put the kernel's by-value arguments in scratch)
        uint64_t st;
        if (sp.aff_class >= 0) {
          [[clang::always_inline]] st = static_eval<true>(N, P, C, sp, cspec, rw.flags, n, P.A.mm_spec + 2 * (size_t)cspec);
        } else {
          [[clang::always_inline]] st = static_eval<false>(N, P, C, sp, cspec, rw.flags, n, nullptr);
        }
        const uint32_t rs = row_reasons(N, P, C, sp, sci, rw, st, n);
#ifndef KB_WA_NO_SWSTORES  // (write-accounting A/B: no key / static-cache stores -- stale keys)
        stat[n] = st;
        keys32[n] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, rw, st), n), n + N.base, idx_bits);
#endif
        if (lvl != nullptr && rs == 0) {  // (an infeasible node is never a candidate: no record)
          // the e-sequence levels exactly as sel_run computes them (same row, static cache, A and reciprocals)
          // (one level at a time, each stored as it comes: the sweeper role must not raise the kernel's register
          // count, which the placer's chain pays for)
          const int A = allocs_before_full(N, sp, sci, scr, rw, n);
          const double ic = 1.0 / (double)rw.alloc_cpu, im = 1.0 / (double)rw.alloc_mem;
          uint32_t* o = lvl + (size_t)n * kLvlW;
#pragma unroll 1
          for (int j = 1; j <= kPreLevels; ++j)
            o[j - 1] = compress_key(traj_key64<true>(N, P, C, sp, sci, scr, rw, st, n, j, A, ic, im), n + N.base,
                                    idx_bits);
          o[kLvlW - 1] = (uint32_t)A;
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      if (lead) ring[r] = s_cmd;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&ctr[r], b1 - b0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (op != KB_ENG_RUN && lead) __hip_atomic_store(sw_exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (op != KB_ENG_RUN) return;
    __syncthreads();  // (s_cmd / s_go are rewritten by the next poll)
  }
}

// Split engine (grid 2): workgroup 0, the placer, runs the jobs; workgroup 1, the selector, runs each job's
// node selection one job ahead. For job m the selector takes the sweep's keys, re-keys the rows job m-2
// committed (final by then) and drops the nodes job m-1 can commit to (its selected set S, published by the
// placer at job m-1's node setup), then publishes the T best of the rest in key order, each with its row and
// static cache, and the job's command. The placer re-keys S of job m-1 from the final rows it kept and merges:
// the T best of the union are the T best overall, since job m-1 touches only S. A no-fit rebuilds every key
// for the histogram. Cycles with a job of more than one segment do not use the split engine.
constexpr int32_t kSelExit = -3;  // selector -> placer: the command was EXIT
// Past one workgroup's key plan (fed_fits), the node table is split into kFedMaxSel ranges at most, one selector
// workgroup each (grid 1 + nsel): each publishes the T best of its range, and the placer merges the lists. Every
// range is a multiple of 4 nodes (16-byte key loads) and holds at most kFedSelNodes keys.
constexpr int kFedMaxSel = 4;
constexpr int kFedParity = 2;  // selector workgroups per node range, taking the jobs in turn (fed_selector)
constexpr int kEntWords = 2 + (int)(sizeof(Row) / 8) + 4;  // a selector entry: key/node, static cache, row, levels
constexpr int kFedSelQ = 10;                          // key groups per thread of a range selector
constexpr int kFedSelNodes = 4 * kSelThreads * kFedSelQ;  // 20480
static_assert((uint64_t)kFedMaxSel * kFedSelNodes <= kEntNodeMask, "selector entries pack the node in 24 bits");
constexpr int kFedTraceJobs = 2048;  // KB_DIAG / KB_TIMELINE: the fed engine's per-job timeline (FedXchg::tl)
#if defined(KB_DIAG) && !defined(KB_TIMELINE)
#define KB_TIMELINE
#endif
#ifdef KB_TIMELINE
#define KB_FED_TL(m, k)                                                      \
  do {                                                                       \
    if (tid == 0) X->tl[(m) & (kFedTraceJobs - 1)][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define KB_FED_TL(m, k) \
  do {                  \
  } while (0)
#endif
__host__ __device__ __forceinline__ int fed_sel_chunk(int n, int nsel) { return ((n + nsel - 1) / nsel + 3) & ~3; }
struct FedXchg {
  uint64_t p_head[kJobSlots];        // placer -> selector (tagged, job number + 1): mode << 16 | count
  uint64_t p_done[kJobSlots];        //   (tagged) the job's commit count, once its rows are written back
  uint64_t p_node[kJobSlots][128];   //   the job's selected set (tagged)
  uint64_t s_head[kJobSlots][kFedMaxSel];  // selector k -> placer: (job number + 1) << 32 | candidates (selector
                                           //   0: kSelExit on EXIT), stored once the entries below are drained
  uint64_t s_cmd[kJobSlots][16];     //   (selector 0) the job's command (FedCmd), one tagged word per field
  // selector k's candidates in key order (descending), word-major so that a wave's stores and loads of one word
  // are contiguous: [0] key | node << 32, [1] static cache, [2..] the row
  // [2 + Row/8 ..] the entry's level record: levels 1..kPreLevels (two per word), the last word's high half 1 when
  // the record is valid (the node's row is the sweep's: not on the commit lists the selector patched)
  uint64_t s_ent[kJobSlots][kFedMaxSel][kEntWords][128];
  // (selector 0) the static cache of job m-1's set S(m-1) in its slot order (the placer's B candidates), from
  // job m's sweep: the placer reads it here, behind the head, instead of from the sweep's buffer -- which would
  // need an agent-scope acquire per job on the placer's CU (~1.7 us, MI355X_MICROARCH.md)
  uint64_t s_bst[kJobSlots][128];
#ifdef KB_TIMELINE
  // KB_DIAG / KB_TIMELINE builds (KB_TIMELINE: the stamps alone, without the phase counters' registers): per job (index & (kFedTraceJobs - 1)) s_memrealtime of [0] the selector's command arrival,
  // [1] its patch done (after job m-2's p_done), [2] its selection done, [3] job m-1's set seen, [4] its head
  // published; the placer's [5] job start (head and command read), [6] its set published, [7] p_done written,
  // [8] its publish started (the drain before the release), [9] the release and host state done
  uint64_t tl[kFedTraceJobs][16];  // ... [10] the placer's command decoded (thread 0), [11] its loop top, [12] its merge's
                                   // entries in LDS, in sel_run [13] node setup, [14] e-sequences, [15] winners done
#endif
  // resident sweepers: sweeper 0 relays each host command (its eight words sc1, then the tag) to the others
  uint64_t sw_cmd[kJobSlots][8];
  uint64_t sw_go[kJobSlots];
  uint32_t sw_exit;  // the sweeper group that took EXIT tells the other groups
  uint32_t sel_exit;  // the parity selector that took EXIT tells the other
  uint64_t wdiag[8];                  // KB_DIAG builds: the placer's fine sel_run stamps (dg[8..15])
  uint32_t census_n;                  // place_xcc: workgroups counted in (agent-scope atomic add)
  uint32_t census_xcc[kFedGridMax];   //   each workgroup's XCC id + 1
  uint64_t sphase[8];  // SHARD: [0..5] the placer's exchange phases (kb_stats.shard_phase_ticks); every split launch:
                       // [6] / [7] the placer's / selector 0's placement (kb_stats.fed_wg_place), ahead of sdiag
  uint64_t sdiag[16];  // KB_DIAG builds: [0..6] the selector's phases, [8..11] the placer's merge; [12..15] the placer's
                       // counters for kb_stats (every build: exchange wait / count, clock / realtime ticks)
};

// Thread 0: spin (sleeping) until *w reaches want, at most idle_ticks of s_memrealtime. ACQ: with an
// agent-scope acquire (plain loads after it see other agents' released stores); otherwise relaxed (the
// exchange's own words are written and read as agent-scope atomics, which bypass the non-coherent caches).
template <bool ACQ = true>
__device__ __forceinline__ bool fed_wait_word(const uint32_t* w, uint32_t want, uint64_t idle_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint32_t v = ACQ ? __hip_atomic_load(w, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                           : __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (v - want <= 0x7fffffffu) return true;
    if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// Re-key the rows on two commit lists (n0 entries of l0, then n1 of l1) for `spec` into k32 (positions node - base;
// nodes outside [base, base + nk) are another selector's). Ends after a barrier.
// pbits (LDS, nk bits, zeroed; nullptr: none): marks every re-keyed node, whose level record is stale.
__device__ __forceinline__ void fed_patch(uint32_t* k32, const DevNodes& N, const DevSpecs& P, const DevCfg& C, const kb_spec& sp,
                          int spec, const uint64_t* stat, int idx_bits, const int32_t* l0, int n0, const int32_t* l1,
                          int n1, int base, int nk, uint32_t* pbits = nullptr) {
  const int np = n0 + n1;
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  for (int i = threadIdx.x; i < np; i += kSelThreads) {
    // (sc1: the placer stores its commit lists sc1, and this selector takes no acquire per job)
    const int w = i < n0 ? ld_sc1(&l0[i]) : ld_sc1(&l1[i - n0]);
    if ((uint32_t)(w - base) >= (uint32_t)nk) continue;
    const Row rr = load_row_sc1(N, w);
    const uint64_t st = stat[w];
    const uint32_t rs = row_reasons(N, P, C, sp, sci, rr, st, w);
    k32[w - base] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, rr, st), w), w + N.base, idx_bits);
    if (pbits != nullptr) atomicOr(&pbits[(w - base) >> 5], 1u << ((w - base) & 31));
  }
  __syncthreads();
}

// Thread 0: wait for ring entry r's command and keys (acquire), bounded by idle_ticks; s_op = its op.
// done (the split engine's parity selectors): a word another selector sets when it took EXIT -- this one's next command
// never comes; it leaves as if EXIT had (s_op KB_ENG_EXIT without a command).
__device__ __forceinline__ void fed_wait_cmd(const uint32_t* ctr, uint32_t tgt, const FedCmd* ring, FedCmd& cm,
                                             int32_t& s_op, uint64_t idle_ticks, int32_t* exit_flag,
                                             const uint32_t* done = nullptr) {
  if (threadIdx.x == 0) {
    int op = KB_ENG_EXIT_IDLE;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      const uint32_t v = __hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      if (v - tgt <= 0x7fffffffu) {
        cm = *ring;
        op = cm.op;
        break;
      }
      if (done != nullptr && __hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) {
        op = -KB_ENG_EXIT;  // (another selector's EXIT)
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
      __builtin_amdgcn_s_sleep(1);
    }
    s_op = op;
    if (op == KB_ENG_EXIT_IDLE) atomicMax(exit_flag, 1);
  }
  __syncthreads();
}

// The split engine's selector `sel` of nsel: a workgroup of the engine's launch after the placer (one dispatch, so
// all are resident together; separate kernels on separate streams are not guaranteed separate hardware queues).
// It serves the nodes [base, base + nk) of the table (all of them when nsel == 1).
template <int QN>
__device__ __forceinline__ void fed_selector(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits,
                                             const FedSlots& S, const FedCmd* ring, const uint32_t* ctr,
                                             uint64_t idle_ticks, int32_t* exit_flag, FedXchg* X, uint32_t* k32,
                                             SelShared& sh, FedCmd& cm, int32_t& s_op, int32_t& s_n1, int sel,
                                             int nsel, uint32_t* scratch, int par) {
  const int tid = threadIdx.x;
  // candidate lists (scratch: 4 x 256 words of the candidate space, unused by a selector): by position, by rank
  int32_t* cnode = (int32_t*)scratch;
  uint32_t* ckey = scratch + 256;
  int32_t* rnode = (int32_t*)scratch + 512;
  uint32_t* rkey = scratch + 768;
  uint32_t* pbits = scratch + 1024;  // the nodes fed_patch re-keyed this job (their level records are stale)
  const int chunk = fed_sel_chunk(N.n, nsel);
  const int base = sel * chunk;
  const int n = N.n - base < chunk ? N.n - base : chunk;  // this selector's nodes
  const int Q4 = QN > 0 ? QN : (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const int n_pad = 4 * kSelThreads * Q4;
  const uint32_t blocks = (uint32_t)((N.n + 63) / 64);  // the sweep's blocks over the whole table
  uint32_t tgt[kJobSlots];
#pragma unroll
  for (int k = 0; k < kJobSlots; ++k) tgt[k] = S.tgt[k];
  __shared__ int32_t s_n3, s_ns2, s_ns3;
  int rp = 0;
#ifdef KB_DIAG
  // [0] wait for the command, [1] key load, [3] wait for job m-2 + patch, [2] wait for job m-1's set +
  // exclusion, [4] selection, [5] publish, [6] jobs
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
#define KB_SSTAMP(k) KB_STAMP(k)
#else
#define KB_SSTAMP(k) \
  do {               \
  } while (0)
#endif
  // Parity selectors: two selector workgroups per node range take the jobs in turn (this one: m = par, par + 2, ...),
  // so each has two placer jobs of time for its own chain (keys, patches, selection, exclusion, publication), and
  // the selection of job m starts as soon as job m-2 is done, not when job m-1's selection is. Jobs they did not
  // select themselves are known through the placer's tagged words (sets, done words): nothing per job is kept here.
  uint32_t m = (uint32_t)par;
  for (int r = par;; r = (r + kFedParity) % kJobSlots, m += kFedParity) {
    tgt[r] += blocks;
    fed_wait_cmd(&ctr[r], tgt[r], &ring[r], cm, s_op, idle_ticks, exit_flag, &X->sel_exit);
    KB_SSTAMP(0);
    if (sel == 0) KB_FED_TL(m, 0);
    if (s_op != KB_ENG_RUN) {
      if (s_op == KB_ENG_EXIT && tid == 0) {
        if (sel == 0)  // the placer takes EXIT from here
          x_store64(&X->s_head[r][0], ((uint64_t)(m + 1) << 32) | (uint32_t)kSelExit);
        __hip_atomic_store(&X->sel_exit, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (the other parity)
      }
      break;
    }
    const int slot = cm.slot, spec = cm.spec;
    // the jobs before the launch's last fresh command (the first after a pause, at or before this one) are final: their
    // commits predate this sweep -- nothing to patch, no set to leave out
    const uint32_t fm = (uint32_t)cm.fresh_m;
    const bool has1 = m >= 1 && m - 1 >= fm, has2 = m >= 2 && m - 2 >= fm, has3 = m >= 3 && m - 3 >= fm;
    load_keys_lds<(QN > 0 ? QN : kSelQ4)>(k32, S.keys[slot] + base, n, n_pad);
    const uint32_t* lvl = S.lvl[slot];
    if (lvl != nullptr)
      for (int i = tid; i < (n + 31) >> 5; i += kSelThreads) pbits[i] = 0u;
    __syncthreads();
    KB_SSTAMP(1);
    const int r1 = r == 0 ? kJobSlots - 1 : r - 1;
    const int r2 = r1 == 0 ? kJobSlots - 1 : r1 - 1;
    const int r3 = r2 == 0 ? kJobSlots - 1 : r2 - 1;
    const kb_spec sp = P.specs[spec];
    const uint64_t* stat = S.stat[slot];
    // The host issues job m once job m - kJobSlots is read, so its sweep may predate the commits of jobs m-3, m-2
    // and m-1: the placer re-keys m-1's set (B), this selector the rows m-3 and m-2 committed. Job m-3's are final
    // long before this selector needs them (patched from its commit list first, off the critical path). Job m-2's
    // commits come from its selected set S(m-2) -- published at its start, and seen here as job m-1's set -- so the
    // set's static caches for this job are loaded before m-2 ends, and after its done word only the rows' loads and
    // the keys remain (every node of the set re-keyed: an unchanged row gives its unchanged key). That chain, from
    // m-2's done word to this selection, was the engine's critical loop (r06g: 5 us of patch after the done word).
    if (tid == 0) {
      int n3 = 0, ns2 = 0, ns3 = 0;
      if (has3) {  // job m-3 done
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          const uint64_t h = x_load64(&X->p_done[r3]);
          if ((uint32_t)(h >> 32) == m - 2) {
            n3 = (int)(uint32_t)h;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
            n3 = -1;
            atomicMax(exit_flag, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (n3 >= 0 && has3) {  // S(m-3): its head (published before its done word)
        const uint64_t h = x_load64(&X->p_head[r3]);
        ns3 = (uint32_t)(h >> 32) == m - 2 && (h >> 16 & 0xffffu) == kPubModeSet ? (int)(h & 0xffffu) : 0;
        if ((uint32_t)(h >> 32) != m - 2) n3 = -1;  // (cannot happen)
      }
      if (n3 >= 0 && has2) {  // S(m-2): its head
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          const uint64_t h = x_load64(&X->p_head[r2]);
          if ((uint32_t)(h >> 32) == m - 1) {
            ns2 = (h >> 16 & 0xffffu) == kPubModeSet ? (int)(h & 0xffffu) : 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
            n3 = -1;
            atomicMax(exit_flag, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      // the rows' main columns and the commit lists come through sc1 loads (load_row_sc1 / ld_sc1 of the placer's sc1
      // stores); a spec with scalar or host-port columns reads those with plain loads, and after a pause the launch
      // path's kernels wrote too: then an agent acquire (~1.7 us; the host's flag, FedCmd::acq) -- here for m-3's
      // rows, and again below for m-2's
      if (cm.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      s_n3 = n3;
      s_ns2 = ns2;
      s_ns3 = ns3;
    }
    __syncthreads();
    if (s_n3 < 0) break;  // the placer stopped answering: leave (the host sees the exit flag)
    // this thread's node of S(m-2) / S(m-3) in this selector's range, and its static cache for this job (the sets'
    // words: tagged, the heads stored after them)
    int w2 = -1, w3 = -1;
    uint64_t st2 = 0, st3 = 0;
    if (tid < s_ns2) {
      const uint64_t e = x_load64(&X->p_node[r2][tid]);
      if ((uint32_t)(e >> 32) != m - 1) atomicMax(exit_flag, 2);  // (cannot happen: the head is stored last)
      else if ((uint32_t)e - (uint32_t)base < (uint32_t)n) w2 = (int)(uint32_t)e;
    }
    if (tid < s_ns3) {
      const uint64_t e = x_load64(&X->p_node[r3][tid]);
      if ((uint32_t)(e >> 32) != m - 2) atomicMax(exit_flag, 2);
      else if ((uint32_t)e - (uint32_t)base < (uint32_t)n) w3 = (int)(uint32_t)e;
    }
    if (w2 >= 0) st2 = stat[w2];
    if (w3 >= 0) {  // S(m-3) re-keyed from its final rows (job m-3 is done)
      st3 = stat[w3];
      const Row rr = load_row_sc1(N, w3);
      const uint32_t rs = row_reasons(N, P, C, sp, P.sc_init + (size_t)spec * N.S, rr, st3, w3);
      k32[w3 - base] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, rr, st3), w3), w3 + N.base, idx_bits);
      if (lvl != nullptr) atomicOr(&pbits[(w3 - base) >> 5], 1u << ((w3 - base) & 31));
    }
    __syncthreads();
    if (tid == 0) {  // job m-2 done: its rows are written back
      int n2 = 0;
      // A guarded command right behind a skipped job is skipped as well (the placer's guard fails once the previous
      // job was skipped: it leaves last_panic set). When job m-1's head already reads skipped -- the rest of a
      // speculative chain after a misprediction -- this job publishes its command and an empty candidate list at
      // once instead of a whole selection the placer would throw away (C3: two or three per NO_FIT the driver did
      // not predict). Its head is loaded beside job m-2's done word: no round trip of its own.
      const bool may_skip = cm.g_valid && has1;
      if (has2) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (int spin = 0;; ++spin) {
          const uint64_t h = x_load64(&X->p_done[r2]);
          const uint64_t h1 = may_skip ? x_load64(&X->p_head[r1]) : 0ull;
          if (may_skip && (uint32_t)(h1 >> 32) == m && (h1 >> 16 & 0xffffu) == kPubModeSkipped) {
            n2 = -2;  // (job m-2 is done too: the placer published m-1 after it)
            break;
          }
          if ((uint32_t)(h >> 32) == m - 1) {
            n2 = (int)(uint32_t)h;
#ifdef KB_DIAG
            dg[7] += spin == 0 ? 1 : 0;  // job m-2 had committed when the command came: the command gated this job
#endif
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
            n2 = -1;
            atomicMax(exit_flag, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      if (cm.acq && n2 >= 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      s_n1 = n2;
    }
    __syncthreads();
    if (s_n1 == -2) {  // skipped behind a skipped job: the command and an empty list
      if (sel == 0 && tid < 16) tag_store(&X->s_cmd[r][tid], m + 1, ((const uint32_t*)&cm)[tid]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) x_store64(&X->s_head[r][sel], ((uint64_t)(m + 1) << 32) | 0u);
      if (sel == 0) KB_FED_TL(m, 4);
      __syncthreads();  // cm reused by the next command
      continue;
    }
    if (s_n1 < 0) break;  // the placer stopped answering: leave (the host sees the exit flag)
    if (w2 >= 0) {  // S(m-2) re-keyed from its final rows (while job m-1 may still be choosing its set)
      const Row rr = load_row_sc1(N, w2);
      const uint32_t rs = row_reasons(N, P, C, sp, P.sc_init + (size_t)spec * N.S, rr, st2, w2);
      k32[w2 - base] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, rr, st2), w2), w2 + N.base, idx_bits);
      if (lvl != nullptr) atomicOr(&pbits[(w2 - base) >> 5], 1u << ((w2 - base) & 31));
    }
    __syncthreads();
    if (sel == 0) KB_FED_TL(m, 1);
    KB_SSTAMP(3);
    // the T best of this range outside job m-1's set are among its T + kSegMax best (the set holds at most kSegMax
    // nodes): chosen, ranked and their rows loaded before the set is known -- only the exclusion waits for it
    const uint32_t T = (uint32_t)cm.t_count;
    uint32_t cnt;
#ifdef KB_DIAG
    uint64_t dgp[7] = {0, 0, 0, 0, 0, 0, 0};  // sel_pick's own fine stamps (KB_DIAG_SEL) kept apart
    sel_pick<QN>(sh, k32, n, idx_bits, T + kSegMax, rp, cnt, dgp, dg_last, cnode, ckey, 2 * 128);
#else
    sel_pick<QN>(sh, k32, n, idx_bits, T + kSegMax, rp, cnt, cnode, ckey, 2 * 128);
#endif
    __syncthreads();
    {  // rank by key (2 threads per candidate; entries past cnt are 0)
      const int e = tid >> 1, part = tid & 1;
      const uint32_t k = e < (int)cnt ? ckey[e] : 0u;
      uint32_t rk = 0;
#pragma unroll 16
      for (int q = 0; q < 128; ++q) rk += ckey[part * 128 + q] > k;
      rk += dpp_src<0xb1>(0u, rk);  // quad_perm [1,0,3,2]: the pair's other half
      if (part == 0 && e < (int)cnt) {
        rnode[rk] = cnode[e];
        rkey[rk] = k;
      }
    }
    __syncthreads();
    KB_SSTAMP(4);
    if (sel == 0) KB_FED_TL(m, 2);
    // thread i: the rank-i candidate's row and static cache (final: job m-1 touches only its set)
    Row rw{};
    uint64_t stw = 0;
    int wp = 0;
    uint32_t wk = 0;
    uint4 lv0 = make_uint4(0u, 0u, 0u, 0u), lv1 = lv0;  // its level record (the sweep's), loaded beside the row
    if (tid < (int)cnt) {
      wp = rnode[tid];
      wk = rkey[tid];
      rw = load_row_sc1(N, wp + base);
      stw = stat[wp + base];
      if (lvl != nullptr) {
        const uint4* lr = (const uint4*)(lvl + (size_t)(wp + base) * kLvlW);
        lv0 = lr[0];
        lv1 = lr[1];
      }
    }
    if (tid == 0) {  // job m-1's set (published at its node setup)
      int n1 = 0;
      if (has1) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          const uint64_t h = x_load64(&X->p_head[r1]);
          if ((uint32_t)(h >> 32) == m) {
            n1 = (h >> 16 & 0xffffu) == kPubModeSet ? (int)(h & 0xffffu) : 0;
            break;
          }
          if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
            n1 = -1;
            atomicMax(exit_flag, 1);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      s_n1 = n1;
    }
    __syncthreads();
    KB_SSTAMP(2);
    if (sel == 0) KB_FED_TL(m, 3);
    if (s_n1 < 0) break;  // the placer stopped answering: leave (the host sees the exit flag)
    if (tid < s_n1) {  // job m-1's set is the placer's to re-key (every entry's tag checked: no store order)
      uint64_t e = x_load64(&X->p_node[r1][tid]);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while ((uint32_t)(e >> 32) != m) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {  // (cannot happen: the head is stored last)
          atomicMax(exit_flag, 2);
          break;
        }
        e = x_load64(&X->p_node[r1][tid]);
      }
      const uint32_t w = (uint32_t)e - (uint32_t)base;
      if ((uint32_t)(e >> 32) == m && w < (uint32_t)n) k32[w] = 0u;
      if (sel == 0 && (uint32_t)(e >> 32) == m) x_store64(&X->s_bst[r][tid], stat[(uint32_t)e]);  // (before the head)
    }
    __syncthreads();
    // candidates outside the set (a zeroed key: inside), in rank order; the first T go out
    uint32_t pos = tid < (int)cnt && k32[wp] != 0u ? 1u : 0u, zero = 0, kept, ztot;
    const bool keep = pos != 0;
    sel_excl_scan2(sh, rp, pos, zero, &kept, &ztot);
    const uint32_t nout = kept < T ? kept : T;
    // each outgoing entry's rank by node among the first nout: the placer's slot order when the T best of the
    // union are exactly these (its merge's fast path: no node ranking there)
    // (one selector only: the placer's fast path takes a single list)
    if (nsel == 1 && keep && pos < T) cnode[pos] = wp + base;
    __syncthreads();
    uint32_t nrank = 0;
    if (nsel == 1 && keep && pos < T) {
      const int me = wp + base;
      for (uint32_t q = 0; q < nout; ++q) nrank += cnode[q] < me ? 1u : 0u;
    }
    if (keep && pos < T) {
      uint64_t(*ent)[128] = X->s_ent[r][sel];
      x_store64(&ent[0][pos], (uint64_t)wk | ((uint64_t)(uint32_t)(wp + base) << 32) | ((uint64_t)nrank << 56));
      x_store64(&ent[1][pos], stw);
      // the entry's A for the placer's node setup (allocs_before_full: off the placer's chain) -- the sweep's, with
      // its levels, unless this job's patch re-keyed the node (its row changed after the sweep read it)
      const bool lv_ok = lvl != nullptr && !((pbits[wp >> 5] >> (wp & 31)) & 1u);
      rw.aux = lv_ok ? (int32_t)lv1.w
                     : allocs_before_full(N, sp, P.sc_init + (size_t)spec * N.S, P.sc_req + (size_t)spec * N.S, rw,
                                          wp + base);
      uint64_t words[sizeof(Row) / 8];
      __builtin_memcpy(words, &rw, sizeof(Row));
#pragma unroll
      for (int q = 0; q < (int)(sizeof(Row) / 8); ++q) x_store64(&ent[2 + q][pos], words[q]);
      constexpr int kL = 2 + (int)(sizeof(Row) / 8);
      x_store64(&ent[kL][pos], (uint64_t)lv0.x | ((uint64_t)lv0.y << 32));
      x_store64(&ent[kL + 1][pos], (uint64_t)lv0.z | ((uint64_t)lv0.w << 32));
      x_store64(&ent[kL + 2][pos], (uint64_t)lv1.x | ((uint64_t)lv1.y << 32));
      x_store64(&ent[kL + 3][pos], (uint64_t)lv1.z | ((uint64_t)(lv_ok ? 1u : 0u) << 32));
    } else if (sel == 0 && tid >= 256 && tid < 256 + 16) {  // the command, for the placer (tagged: prefetched)
      tag_store(&X->s_cmd[r][tid - 256], m + 1, ((const uint32_t*)&cm)[tid - 256]);
    }
    // every wave's entry stores drained before the head (a barrier alone waits for LDS only)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) x_store64(&X->s_head[r][sel], ((uint64_t)(m + 1) << 32) | nout);
    KB_SSTAMP(5);
    if (sel == 0) KB_FED_TL(m, 4);
#ifdef KB_DIAG
    dg[6]++;
#endif
    __syncthreads();  // cm reused by the next command
  }
#ifdef KB_DIAG
  if (tid == 0 && sel == 0 && par == 0)
    for (int k = 0; k < 8; ++k) X->sdiag[k] = dg[k];
#endif
#undef KB_SSTAMP
}

// The row after c commits of the spec from r0 (min(c, A) Allocates, the rest Pipelines): store_back_row's
// columns as a Row.
__device__ __forceinline__ Row row_after(const kb_spec& sp, const Row& r0, int c, int A) {
  const int64_t a = c < A ? c : A;
  const int64_t p = c - a;
  Row r = r0;
  r.idle_cpu -= a * sp.req_cpu;
  r.idle_mem -= a * sp.req_mem;
  r.rel_cpu -= p * sp.req_cpu;
  r.rel_mem -= p * sp.req_mem;
  r.pod_count += c;
  r.nz_cpu += (int64_t)c * sp.nz_cpu;
  r.nz_mem += (int64_t)c * sp.nz_mem;
  return r;
}

// The no-fit FitErrors histogram (allocate.go:150-153, unschedule_info.go:57-79) of a table too large for the
// placer's LDS: every node's key is the sweep's (keys, read from memory) unless its row changed since, on one of
// the four commit lists (the three jobs before and this one); those are re-keyed. bits (LDS, n bits) marks them, so a node listed twice counts once
// and the streamed pass skips it. Ends after a barrier with the histogram in sh.hist.
__device__ void fed_hist_stream(SelShared& sh, uint32_t* bits, const DevNodes& N, const DevSpecs& P, const DevCfg& C,
                                const kb_spec& sp, int spec, const uint64_t* stat, const uint32_t* keys,
                                const int32_t* l0, int n0, const int32_t* l1, int n1, const int32_t* l2, int n2,
                                const int32_t* l3, int n3) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int n = N.n, nw = (n + 31) >> 5;
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  for (int i = tid; i < nw; i += kSelThreads) bits[i] = 0u;
  if (tid < KB_NUM_REASONS) sh.hist[tid] = 0;
  __syncthreads();
  for (int i = tid; i < n0 + n1 + n2 + n3; i += kSelThreads) {
    const int w = i < n0 ? l0[i]
                         : (i < n0 + n1 ? l1[i - n0] : (i < n0 + n1 + n2 ? l2[i - n0 - n1] : l3[i - n0 - n1 - n2]));
    const uint32_t b = 1u << (w & 31);
    if (atomicOr(&bits[w >> 5], b) & b) continue;  // listed twice: its row is the same final row
    const uint32_t rs = row_reasons(N, P, C, sp, sci, load_row(N, w), stat[w], w);
    for (uint32_t m = rs; m; m &= m - 1) atomicAdd(&sh.hist[__builtin_ctz(m)], 1u);
  }
  __syncthreads();
  uint32_t h[KB_NUM_REASONS];
#pragma unroll
  for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] = 0;
  for (int i0 = 0; i0 < n; i0 += 4 * kSelThreads) {
    uint32_t k[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // the loads first: one memory latency per four keys
      const int i = i0 + q * kSelThreads + tid;
      k[q] = i < n ? keys[i] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int i = i0 + q * kSelThreads + tid;
      if (i >= n || (k[q] >> 31) || ((bits[i >> 5] >> (i & 31)) & 1u)) continue;
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] += (k[q] >> b) & 1u;
    }
  }
#pragma unroll
  for (int b = 0; b < KB_NUM_REASONS; ++b) {
    const uint32_t v = wave_sum_u32(h[b]);
    if (lane == 0 && v) atomicAdd(&sh.hist[b], v);
  }
  __syncthreads();
}

// ---- node-sharded fed engine: the placer's exchange and global merge ----
// Per job every rank's placer proposes its first T picks (the selection of its own rows), writes the proposal into
// every rank's inbox (stores over xGMI into the peers' HBM) and reads all W proposals from its own inbox. Every
// word carries its tag (epoch << 20 | job + 1), so a reader takes a word once its tag matches: no store order, no
// fence, and a stale word (an earlier job or cycle) reads as not there yet. Record i of rank w (L = 3T + 4 + R
// words): 3 per pick (composite high / low, global node | kind << 30), then kp, three header words (the job's
// spec, tasks and gang inputs: every rank must have issued the same job) and the no-fit histogram. Records are
// numbered by exchange (xn: the cycle's jobs that ran, not skipped speculative ones, which exchange nothing), in
// kJobSlots slots: a rank writes exchange xn + 1 only after every rank wrote exchange xn, so no rank is ever more
// than one exchange ahead of another's reads.
__device__ __forceinline__ uint64_t* shard_word(uint64_t* inbox, uint32_t epoch, int r, int w, int i) {
  return inbox + ((((size_t)(epoch & 1u) * kJobSlots + r) * kShardMaxWorld + w) * kShardRecW + i);
}
// SP.inbox[w] by selects: a dynamic index into the by-value kernel argument would copy it to scratch
__device__ __forceinline__ uint64_t* shard_inbox(const ShardPeers& SP, int w) {
  uint64_t* p = SP.inbox[0];
#pragma unroll
  for (int k = 1; k < kShardMaxWorld; ++k) p = w == k ? SP.inbox[k] : p;
  return p;
}
__device__ __forceinline__ uint32_t shard_tag(uint32_t epoch, uint32_t m) {
  static_assert(kShardEpochBits == 12, "tag layout: 12 epoch bits, 20 exchange bits");
  return ((epoch & 0xfffu) << 20) | ((m + 1) & 0xfffffu);
}
// entries of rank h's proposal list (descending, high / low words in LDS) above v
__device__ __forceinline__ int shard_gt(const uint32_t* ghi, const uint32_t* glo, int len, uint64_t v) {
  int lo = 0, hi = len;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((((uint64_t)ghi[mid] << 32) | glo[mid]) > v) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}
constexpr int kShardNoFitR = KB_NUM_REASONS;
constexpr int kShardHistOff = 3 * kShardSegMax + 4;  // the no-fit round's words in a record
static_assert(kShardHistOff + kShardNoFitR <= kShardRecW, "inbox record layout");
// gathered proposals in the placer's candidate space (free between sel_run and the next job's B rows)
struct ShardGather {
  uint32_t hi[kShardMaxWorld][128], lo[kShardMaxWorld][128];
  int32_t nk[kShardMaxWorld][128];
  int32_t kp[kShardMaxWorld];
  uint32_t hdr[kShardMaxWorld][3];
  uint32_t hist[kShardMaxWorld][kShardNoFitR];
  int32_t fail, diverged, cut, kind, n_alloc;
};
static_assert(sizeof(ShardGather) <= 8 * kCandCap, "the gathered proposals fit the candidate space");

// After sel_run<PROPOSE, QN, CAND> (sh.ord[0..s_count): this rank's proposal): the local no-fit histogram when the
// rank ran out of picks, the exchange, the global first-T picks, the stop rules, and the commits on this rank's
// rows. Returns 0, 1 (a peer's proposal did not arrive within idle_ticks) or 2 (the ranks issued different jobs).
// (inlined: as a call it made the engine pass its by-value kernel arguments through scratch)
__device__ __forceinline__ int shard_place(SelShared& sh, uint32_t* k32, uint64_t* cand, const ShardPeers& SP,
                                          uint32_t xn, const DevNodes& N, const DevSpecs& P, const DevCfg& C,
                                          const kb_spec& sp, int spec, const uint64_t* stat, const uint32_t* keys,
                                          const int32_t* l0, int n0, const int32_t* l1, int n1, const int32_t* l2,
                                          int n2, int t_begin,
                                          int t_count, int ready0, int minav, int gang, int idx_bits, int32_t* hout,
                                          JobState* js, JobState* hjs, int32_t* commit_out, uint64_t idle_ticks,
                                          int& stop, int& fail_task, int& placed, int& ready, int& panic, int& stopped,
                                          uint64_t* ph) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int T = t_count, W = SP.world;
  __syncthreads();  // sel_run's no-fit exit writes sh.s_count = 0 from one thread with no barrier after it
  const int kp = sh.s_count;
  stop = KB_STOP_DONE;  // (sel_run's local no-fit outcome is not the job's)
  fail_task = -1;
  panic = 0;
  stopped = 0;
  ShardGather& G = *(ShardGather*)cand;
  if (tid == 0) {
    G.fail = 0;
    G.diverged = 0;
  }
  const uint32_t tag = shard_tag(SP.epoch, xn);
  const int r = (int)(xn % (uint32_t)kJobSlots);
  const uint64_t th = (uint64_t)tag << 32;
  const uint32_t hdr0 = (uint32_t)spec, hdr1 = (uint32_t)T;
  const uint32_t hdr2 = (uint32_t)ready0 * 65599u + (uint32_t)minav * 31u + (uint32_t)gang;
  const int L = 3 * T + 4;  // (a global no-fit's histograms follow in a second round at kShardHistOff)
  // record word i of this rank, and where a record word goes in the gathered arrays
  const auto word = [&](int i) -> uint32_t {
    if (i < 3 * T) {
      const int e = i / 3, q = i - 3 * e;
      if (e >= kp) return 0u;
      const uint64_t o = sh.ord[e];
      if (q == 0) return (uint32_t)(o >> 32);
      if (q == 1) return (uint32_t)o;
      const int s = sel_slot(o), j = sel_level(o);
      return (uint32_t)(sh.node[s] + N.base) | ((uint32_t)(j < sh.A[s] ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE) << 30);
    }
    if (i == 3 * T) return (uint32_t)kp;
    return i == 3 * T + 1 ? hdr0 : (i == 3 * T + 2 ? hdr1 : hdr2);
  };
  const auto gput = [&](int w, int i, uint32_t v) {
    if (i < 3 * T) {
      const int e = i / 3, q = i - 3 * e;
      if (q == 0) G.hi[w][e] = v;
      else if (q == 1) G.lo[w][e] = v;
      else G.nk[w][e] = (int32_t)v;
    } else if (i == 3 * T) {
      G.kp[w] = (int32_t)v;
    } else {
      G.hdr[w][i - 3 * T - 1] = v;
    }
  };
  // ---- write: this rank's record into every other rank's inbox (its own goes straight to LDS) ----
  // ph (thread 0's s_memrealtime phase sums, kb_stats.shard_phase_ticks): [1] write, [2] wait, [3] merge + stop
  // rules, [4] commit, [5] no-fit round
  const uint64_t t_write0 = __builtin_amdgcn_s_memrealtime();
  for (int idx = tid; idx < W * L; idx += kSelThreads) {
    const int w = idx / L, i = idx - w * L;
    const uint32_t v = word(i);
    if (w == SP.rank && !SP.self_inbox) gput(w, i, v);
    else
      __hip_atomic_store(shard_word(shard_inbox(SP, w), SP.epoch, r, SP.rank, i), th | v, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // ---- read: every other rank's record from this rank's inbox ----
  const uint64_t t_read0 = __builtin_amdgcn_s_memrealtime();
  ph[1] += t_read0 - t_write0;
  {
    const uint64_t t0 = t_read0;
    bool late = false;
    uint64_t* own = shard_inbox(SP, SP.rank);
    for (int idx = tid; idx < W * L && !late; idx += kSelThreads) {
      const int w = idx / L, i = idx - w * L;
      if (w == SP.rank && !SP.self_inbox) continue;
      const uint64_t* p = shard_word(own, SP.epoch, r, w, i);
      uint64_t x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      while ((uint32_t)(x >> 32) != tag) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
          late = true;
          // for the host's error text: the word waited for, the tag found there, and how many of rank w's words
          // carry this job's tag
          int have = 0;
          for (int k = 0; k < L; ++k)
            have += (uint32_t)(__hip_atomic_load(shard_word(own, SP.epoch, r, w, k), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_SYSTEM) >> 32) == tag;
          hjs->t_recv = ((uint64_t)w << 56) | ((uint64_t)i << 40) | ((uint64_t)(uint32_t)have << 20) | 1ull;
          hjs->t_done = ((uint64_t)(uint32_t)(x >> 32) << 32) | tag;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (late) break;
      gput(w, i, (uint32_t)x);
    }
    if (late) G.fail = 1;  // (benign race: every writer stores 1)
  }
  __syncthreads();
  const uint64_t t_merge0 = __builtin_amdgcn_s_memrealtime();
  ph[2] += t_merge0 - t_read0;  // (thread 0's count is the one reported)
  if (G.fail) return 1;
  if (tid < W && (G.hdr[tid][0] != hdr0 || G.hdr[tid][1] != hdr1 || G.hdr[tid][2] != hdr2 || G.kp[tid] > T))
    G.diverged = 1;
  __syncthreads();
  if (G.diverged) return 2;
  // ---- the global pick order: proposal i of rank w ranks i + the larger proposals of every other rank ----
  int K = 0;
  for (int w = 0; w < W; ++w) K += G.kp[w];
  int32_t* ordnk = sh.act;
  for (int e = tid; e < W * T; e += kSelThreads) {
    const int w = e / T, i = e - w * T;
    if (i >= G.kp[w]) continue;
    const uint64_t v = ((uint64_t)G.hi[w][i] << 32) | G.lo[w][i];
    int rank = i;
    for (int h = 0; h < W; ++h)
      if (h != w) rank += shard_gt(G.hi[h], G.lo[h], G.kp[h], v);
    if (rank < T) {
      sh.ord[rank] = v;
      ordnk[rank] = G.nk[w][i];
    }
  }
  if (tid < sh.n_sel) sh.fin[tid] = 0;
  __syncthreads();
  const int Kp = K < T ? K : T;
  if (wv == 0) {  // stop rules in pick order (as sel_run applies them on one GPU)
    const int64_t bias32 = 1ll << (30 - idx_bits);
    const uint32_t score_mask = (1u << (31 - idx_bits)) - 1;
    const uint64_t lt = (1ull << lane) - 1;
    const bool va = lane < Kp, vb = lane + 64 < Kp;
    const uint64_t oa = va ? sh.ord[lane] : 0, ob = vb ? sh.ord[lane + 64] : 0;
    const bool aa = va && ((uint32_t)ordnk[lane] >> 30) == KB_PLACE_ALLOCATE;
    const bool ab = vb && ((uint32_t)ordnk[lane + 64] >> 30) == KB_PLACE_ALLOCATE;
    const auto neg = [&](uint64_t o) {
      const uint32_t e32 = (uint32_t)(o >> 14);
      return (int64_t)((e32 >> idx_bits) & score_mask) - bias32 <= -1;
    };
    const uint64_t le_mask = lt | (1ull << lane);
    const uint64_t ma = __ballot(aa), mb = __ballot(ab);
    const int ra = ready0 + __popcll(ma & le_mask);
    const int rb = ready0 + __popcll(ma) + __popcll(mb & le_mask);
    const uint64_t sta = __ballot(va && (!gang || ra >= minav));
    const uint64_t stb = __ballot(vb && (!gang || rb >= minav));
    const uint64_t nga = __ballot(va && neg(oa)), ngb = __ballot(vb && neg(ob));
    const int first_stop = sta ? __builtin_ctzll(sta) : (stb ? 64 + __builtin_ctzll(stb) : 128);
    const int first_neg = nga ? __builtin_ctzll(nga) : (ngb ? 64 + __builtin_ctzll(ngb) : 128);
    int cut, kind;
    if (first_neg < Kp && first_neg <= first_stop) {
      cut = first_neg;
      kind = 3;
    } else if (first_stop < Kp) {
      cut = first_stop + 1;
      kind = KB_STOP_READY;
    } else if (Kp < T) {
      cut = Kp;
      kind = KB_STOP_NO_FIT;
    } else {
      cut = T;
      kind = -1;
    }
    const int al = __popcll(cut >= 64 ? ma : (ma & ((1ull << cut) - 1))) +
                   (cut > 64 ? __popcll(mb & ((1ull << (cut - 64)) - 1)) : 0);
    if (lane == 0) {
      G.cut = cut;
      G.kind = kind;
      G.n_alloc = al;
    }
  }
  __syncthreads();
  const uint64_t t_commit0 = __builtin_amdgcn_s_memrealtime();
  ph[3] += t_commit0 - t_merge0;
  const int cut = G.cut, kind = G.kind;
  // placements (every rank writes the whole sequence) and the picks on this rank's rows, per local slot
  if (tid < cut) {
    const int nk = ordnk[tid];
    const int node = nk & 0x3fffffff;
    hout[2 * (t_begin + tid)] = node;
    hout[2 * (t_begin + tid) + 1] = (int32_t)((uint32_t)nk >> 30);
    if (node >= N.base && node < N.base + N.n) atomicAdd(&sh.fin[sel_slot(sh.ord[tid])], 1);
  }
  const int base_c = sh.n_commit;  // (read before the barrier: thread 0 rewrites it after)
  __syncthreads();
  {  // the commit list in slot order from two ballots (an LDS atomic counter serialises the lanes on one word)
    const int ns = sh.n_sel;
    const uint64_t lt_ = (1ull << lane) - 1;
    const uint64_t b_lo = __ballot(lane < ns && sh.fin[lane] > 0);
    const uint64_t b_hi = __ballot(lane + 64 < ns && sh.fin[lane + 64] > 0);
    if (tid < ns && sh.fin[tid] > 0) {  // NodeInfo.AddTask x fin on this rank's row
      const int w = sh.node[tid];
      store_back_row(N, P, sp, P.sc_req + (size_t)spec * N.S, w, sh.fin[tid], sh.A[tid], sh.row[tid]);
      const int at_c = base_c + (wv == 0 ? __popcll(b_lo & lt_) : __popcll(b_lo) + __popcll(b_hi & lt_));
      st_sc1(&commit_out[at_c], (int32_t)w);  // (fed_patch reads it ld_sc1)
    }
    if (tid == 0) sh.n_commit = base_c + __popcll(b_lo) + __popcll(b_hi);
  }
  // an affinity unit's table commits, on every rank for every placement (the count tables and histograms are
  // replicated: topo_dom covers the whole cluster from this rank's first row), before the job's publish
  if (sp.aff_class >= 0 && tid < cut) {
    const int nk = ordnk[tid];
    [[clang::always_inline]] apply_commit_tables(P.A, sp, (nk & 0x3fffffff) - N.base,
                                                 ((uint32_t)nk >> 30) == KB_PLACE_ALLOCATE ? 1 : 0, 1);
  }
  placed = cut;
  ready = ready0 + G.n_alloc;
  const uint64_t t_hist0 = __builtin_amdgcn_s_memrealtime();
  ph[4] += t_hist0 - t_commit0;
  if (kind == 3) {
    fail_task = t_begin + cut;
    panic = 1;
    stopped = 1;
  } else if (kind == KB_STOP_READY) {
    stop = KB_STOP_READY;
    stopped = 1;
  } else if (kind == KB_STOP_NO_FIT) {
    // FitErrors over every rank's rows (allocate.go:150-153): each rank's histogram of its rows with the job's
    // commits applied (as the one-GPU engine computes it: the sweep's keys, the rows the last three jobs and this one
    // wrote back re-keyed), then a second round of the exchange (17 tagged words per rank) and the sum
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this job's row stores and the sweep's keys: fresh loads
    __syncthreads();
    fed_hist_stream(sh, k32, N, P, C, sp, spec, stat, keys, l0, n0, l1, n1, l2, n2, commit_out, sh.n_commit);
    if (tid < W * kShardNoFitR) {
      const int w = tid / kShardNoFitR, b = tid - w * kShardNoFitR;
      if (w == SP.rank && !SP.self_inbox) {
        G.hist[w][b] = sh.hist[b];
      } else {
        __hip_atomic_store(shard_word(shard_inbox(SP, w), SP.epoch, r, SP.rank, kShardHistOff + b), th | sh.hist[b],
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    if (tid < W * kShardNoFitR) {
      const int w = tid / kShardNoFitR, b = tid - w * kShardNoFitR;
      if (w != SP.rank || SP.self_inbox) {
        const uint64_t* p = shard_word(shard_inbox(SP, SP.rank), SP.epoch, r, w, kShardHistOff + b);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint64_t x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        while ((uint32_t)(x >> 32) != tag) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
            G.fail = 1;
            hjs->t_recv = ((uint64_t)w << 56) | ((uint64_t)(kShardHistOff + b) << 40) | 1ull;
            hjs->t_done = ((uint64_t)(uint32_t)(x >> 32) << 32) | tag;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          x = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        G.hist[w][b] = (uint32_t)x;
      }
    }
    __syncthreads();
    if (G.fail) return 1;
    if (tid < KB_NUM_REASONS) {
      uint32_t h = 0;
      for (int w = 0; w < W; ++w) h += G.hist[w][tid];
      js->hist[tid] = h;
      hjs->hist[tid] = h;
    }
    stop = KB_STOP_NO_FIT;
    fail_task = t_begin + cut;
    stopped = 1;
    ph[5] += __builtin_amdgcn_s_memrealtime() - t_hist0;
  }
  if (tid == 0) sh.need_hist = 0;
  __syncthreads();
  return 0;
}

// SPLIT: grid 1 + nsel, workgroup 0 the placer and 1.. the selectors (fed_selector) of nsel node ranges; every
// job of the cycle one segment (the host checks). Otherwise one workgroup with every node's key in LDS.
// SHARD (split only): the node-sharded engine -- the placer proposes, exchanges and merges (shard_place).
// MSEL: the most selector workgroups the instance serves (1, or kFedMaxSel range selectors past one workgroup's key
// plan): a one-selector instance carries no range merge code and no per-range registers.
template <int QN, bool SPLIT, bool SHARD = false, int MSEL = 1>
__global__ __launch_bounds__(kSelThreads) void fed_engine_kernel(DevNodes N, DevSpecs P, DevCfg C, int idx_bits,
                                                                 FedSlots S, const FedCmd* ring,
                                                                 const uint32_t* ctr, uint64_t idle_ticks,
                                                                 int32_t* exit_flag, FedXchg* X, int nsel_arg,
                                                                 ShardPeers SP, int place_xcc,
                                                                 const FedHostCmd* hring, uint32_t epoch) {
  static_assert(!SHARD || SPLIT, "the node-sharded engine is the split engine");
  static_assert(MSEL == 1 || (SPLIT && MSEL <= kFedMaxSel), "range selectors belong to the split engine");
  const int nsel = MSEL == 1 ? 1 : nsel_arg;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds32[];
  __shared__ SelShared sh;
  __shared__ FedCmd cm;
  __shared__ int32_t s_op, s_cand;
  __shared__ int32_t bprev[128];  // split: the previous job's selected set, slot order
  __shared__ uint32_t bkey[128];  //   its keys for this job
  __shared__ int32_t s_feas;
  __shared__ uint32_t s_bmax;  // split: the largest B key of the job (the merge's fast path)
  __shared__ int32_t s_na[MSEL];  // split: the selectors' candidate counts for this job
  __shared__ int32_t s_pre_na;    // one selector: the next job's candidate count when its head was already there
  const int tid = threadIdx.x;
  const int n = N.n;
  const int Q4 = QN > 0 ? QN : (n + 4 * kSelThreads - 1) / (4 * kSelThreads);
  const int n_pad = 4 * kSelThreads * Q4;
  uint32_t* k32 = lds32;
  uint64_t* cand = (uint64_t*)(lds32 + n_pad);
  if constexpr (SPLIT) {
    // role: 0 the placer, k >= 1 selector k - 1. place_xcc >= 0: a census of the grid's XCC ids (every workgroup is
    // resident: launch_fed_engine's check) picks the workgroups on XCC place_xcc first, the others in block order
    // after them; every workgroup computes the same assignment and the unpicked ones exit. A census that does not
    // complete within idle_ticks leaves every workgroup out (the host sees the idle exit: launch path).
    __shared__ int32_t s_role, s_nsw, s_all;
    __shared__ uint8_t s_cx[kFedGridMax];  // (XCC id + 1; bit 7: role taken -- the static LDS budget is tight)
    uint32_t xcc, hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t G = gridDim.x;
    // (bit 8 of place_xcc, tests only: every workgroup's census entry reads as the placer's XCC -- a one-XCC layout)
    const bool one_xcc = place_xcc >= 0 && (place_xcc & 0x100) != 0;
    const int pxc = place_xcc >= 0 ? (place_xcc & 0xff) : -1;
    if (tid == 0) {
      int all = 1;
      if (pxc >= 0) {
        __hip_atomic_store(&X->census_xcc[blockIdx.x], (one_xcc ? (uint32_t)pxc : xcc) + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(&X->census_n, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (!(all = __hip_atomic_load(&X->census_n, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= G) &&
               __builtin_amdgcn_s_memrealtime() - t0 <= idle_ticks)
          __builtin_amdgcn_s_sleep(1);
        if (!all) atomicMax(exit_flag, 1);
      }
      s_all = all;
    }
    __syncthreads();
    if (pxc >= 0 && s_all && tid < (int)G)  // every entry in one round trip (agent-scope loads)
      s_cx[tid] = (uint8_t)__hip_atomic_load(&X->census_xcc[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    if (tid == 0) {
      // roles: 0 the placer, 1..kFedParity*nsel the selectors -- the workgroups on XCC place_xcc first, then the others, both in
      // block order; then (resident sweepers) every other workgroup NOT on the placer's XCC, in block order: a
      // sweeper's stores and its per-job release would dirty and write back that XCC's L2 under the placer
      // (measured: C2 19.2 us per job with sweepers there, r05r). The rest exit.
      int role = (int)blockIdx.x, nsw = 0;
      if (pxc >= 0) {
        role = -1;
        if (s_all) {
          int k = 0;
          for (int pass = 0; pass < 2; ++pass)
            for (uint32_t b = 0; b < G && k <= kFedParity * nsel; ++b)
              if (!(s_cx[b] & 0x80u) && ((uint32_t)s_cx[b] == (uint32_t)pxc + 1) == (pass == 0)) {
                if (b == blockIdx.x) role = k;
                s_cx[b] |= 0x80u;  // (taken)
                ++k;
              }
          if (hring != nullptr) {
            for (uint32_t b = 0; b < G; ++b)
              if (!(s_cx[b] & 0x80u) && s_cx[b] != (uint32_t)pxc + 1) {
                if (b == blockIdx.x) role = kFedParity * nsel + 1 + nsw;
                ++nsw;
              }
            // no workgroup off the placer's XCC (a one-XCC device or partition): the sweepers share its XCC rather
            // than leave the host ring undrained (the selector would wait out its idle bound for every command)
            if (nsw == 0)
              for (uint32_t b = 0; b < G; ++b)
                if (!(s_cx[b] & 0x80u)) {
                  if (b == blockIdx.x) role = kFedParity * nsel + 1 + nsw;
                  ++nsw;
                }
            // still none (a grid of placer and selectors only, which launch_fed_engine never sizes): every role leaves
            // with the exit flag set, so the host finishes the cycle on the launch path instead of waiting
            if (nsw == 0) {
              role = -1;
              atomicMax(exit_flag, 1);
            }
          }
        }
      }
      s_role = role;
      s_nsw = nsw;
      // (kb_stats.fed_wg_place; the placer's word also carries the sweeper count, kb_stats.fed_last_sweepers)
      if (role >= 0 && role <= 1) X->sphase[6 + role] = (uint64_t)xcc << 32 | hw | (role == 0 ? (uint64_t)nsw << 40 : 0ull);
    }
    __syncthreads();
    const int role = s_role;
    if (role > kFedParity * nsel) {  // resident sweepers
      fed_sweeper(N, P, C, idx_bits, S, hring, epoch, const_cast<FedCmd*>(ring), const_cast<uint32_t*>(ctr),
                  idle_ticks, exit_flag, role - kFedParity * nsel - 1, s_nsw, &X->sw_cmd[0][0], X->sw_go, &X->sw_exit);
      return;
    }
    if (role < 0) return;
    if (role >= 1) {  // selector (role - 1) % nsel of the node ranges, parity (role - 1) / nsel
      fed_selector<QN>(N, P, C, idx_bits, S, ring, ctr, idle_ticks, exit_flag, X, k32, sh, cm, s_op, s_cand,
                       (role - 1) % nsel, nsel, (uint32_t*)cand, (role - 1) / nsel);
      return;
    }
  }
  // split: the previous job's set's final rows, kept from its commit to this job's merge (the candidate
  // lists' space is free between the two)
  Row* brow = (Row*)cand;
  const uint32_t blocks = (uint32_t)((n + 63) / 64);
  uint32_t tgt[kJobSlots];
#pragma unroll
  for (int k = 0; k < kJobSlots; ++k) tgt[k] = S.tgt[k];
  int last_stop = -1, last_placed = -1, last_ready = -1, last_panic = 1;  // no previous job: guards fail
  // the commit lists of the previous three jobs ([0] the last one): a job's sweep may have run before any of them
  // committed (the host issues a job once the job kJobSlots back is read)
  int prev_slot[3] = {-1, -1, -1}, prev_ncommit[3] = {0, 0, 0};
  int nbprev = 0;
  int rp = 0;
  // split, thread 0: the next job's command words and selector 0's head, then the other selectors' heads, loaded
  // at this job's end
  uint64_t pre[16 + MSEL];
#pragma unroll
  for (int q = 0; q < 16 + MSEL; ++q) pre[q] = 0;
  // one selector: this thread's candidate entry of the next job, loaded at the end of this job when the next head was
  // already there (its latency hides behind the publish), with the count it was loaded for (-1: none)
  constexpr int kEntW = kEntWords - 4;  // (the level words are loaded at the merge, not prefetched: registers)
  uint64_t ent_pf[kEntW];
#pragma unroll
  for (int q = 0; q < kEntW; ++q) ent_pf[q] = 0;
  int ent_pf_na = -1;
  uint64_t bst_pf = 0;  // likewise this thread's B entry's static cache (s_bst, written before the same head)
  // ... and its entry's level words, moved into the LDS records (clv) at the next loop top -- not held in registers
  // through the next job's merge, where the kernel's register budget is spent
  uint64_t lw_pf[4] = {0, 0, 0, 0};
#ifdef KB_DIAG
  uint64_t mg[4] = {0, 0, 0, 0};  // split: the merge's steps (loads, B order, union rank, slots)
  // per job: the KB_SEL_PH phases; [0] also takes the wait for this job's command, [6] the previous job's
  // publish (fence + host writes)
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
  uint64_t t_wait0 = dg_last, pub_prev = 0, rt_wait0 = __builtin_amdgcn_s_memrealtime();
#endif
  uint32_t m = 0;
  uint32_t xn = 0;  // SHARD: exchanges so far (the jobs that ran)
  const uint64_t clk0 = __builtin_amdgcn_s_memtime(), rt0_launch = __builtin_amdgcn_s_memrealtime();
  // SHARD: s_memrealtime ticks per phase of the exchanges (kb_stats.shard_phase_ticks; [2] the wait for every peer's
  // record after writing this rank's, also kb_stats.shard_wait_ticks)
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t t_job0 = 0;
  for (int r = 0;; r = r + 1 == kJobSlots ? 0 : r + 1, ++m) {
    if constexpr (SPLIT) {  // the selector's publication carries the command (and EXIT)
      KB_FED_TL(m, 11);
      if (MSEL == 1 && tid < ent_pf_na) {  // the prefetched entry's level words (they came in during the publish)
        uint4* o = (uint4*)(k32 + 128 + (size_t)tid * kLvlW);  // (clv, below)
        o[0] = make_uint4((uint32_t)lw_pf[0], (uint32_t)(lw_pf[0] >> 32), (uint32_t)lw_pf[1], (uint32_t)(lw_pf[1] >> 32));
        o[1] = make_uint4((uint32_t)lw_pf[2], (uint32_t)(lw_pf[2] >> 32), (uint32_t)lw_pf[3], (uint32_t)(lw_pf[3] >> 32));
      }
      if (tid == 0) {
        int c = -2;
        // the head and command prefetched at the end of the previous job, when they were already there
        bool have = (uint32_t)(pre[16] >> 32) == m + 1;
#pragma unroll
        for (int q = 0; q < 16; ++q) have = have && (uint32_t)(pre[q] >> 32) == m + 1;
        uint64_t h = pre[16];
#ifdef KB_DIAG
        dg[12] += have ? 0 : 1;  // jobs whose head was not there at the previous job's end (kb_fed_placer_fine)
#endif
        // (every load below is consumed inside its own branch -- asm operand uses: the compiler's wait counting
        // merges branches, so a load pending past a merge made the prefetched path wait there too, for every
        // earlier load and store of the wave including the previous job's host release: ~0.9 us per job, r05x)
        if (!have) {
          const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
          for (;;) {
            h = x_load64(&X->s_head[r][0]);
            if ((uint32_t)(h >> 32) == m + 1) break;
            if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) break;
            __builtin_amdgcn_s_sleep(1);
          }
          asm volatile("" ::"v"(h));
        }
        if ((uint32_t)(h >> 32) == m + 1) {
          c = (int32_t)(uint32_t)h;
          s_na[0] = c;
#pragma unroll
          for (int k = 1; k < MSEL; ++k) {  // the other selectors' lists of this job (unrolled: pre in VGPRs)
            if (k >= nsel || c < 0) continue;
            uint64_t hk = pre[16 + k];
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            while ((uint32_t)(hk >> 32) != m + 1) {
              if (__builtin_amdgcn_s_memrealtime() - t0 > idle_ticks) {
                c = -2;
                break;
              }
              __builtin_amdgcn_s_sleep(1);
              hk = x_load64(&X->s_head[r][k]);
              asm volatile("" ::"v"(hk));
            }
            s_na[k] = (int32_t)(uint32_t)hk;
          }
          if (c >= 0) {
            // the selector stored the command's words before its head (vmcnt(0) between): all 16 loads issue at
            // once, and the tags only confirm it (a word-by-word spin made this a chain of 16 L2 round trips
            // whenever the prefetch at the end of the previous job came too early)
            uint32_t fields[16];
            if (have) {
#pragma unroll
              for (int q = 0; q < 16; ++q) fields[q] = (uint32_t)pre[q];
            } else {
              uint64_t wv[16];
#pragma unroll
              for (int q = 0; q < 16; ++q) wv[q] = x_load64(&X->s_cmd[r][q]);
              bool tagged = true;
#pragma unroll
              for (int q = 0; q < 16; ++q) tagged = tagged && (uint32_t)(wv[q] >> 32) == m + 1;
              if (!tagged) {
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
                  while ((uint32_t)(wv[q] >> 32) != m + 1) {  // the tag orders it
                    if (__builtin_amdgcn_s_memrealtime() - t1 > idle_ticks) {  // (cannot happen: the head is last)
                      c = -2;
                      atomicMax(exit_flag, 3);
                      break;
                    }
                    wv[q] = x_load64(&X->s_cmd[r][q]);
                  }
                }
              }
#pragma unroll
              for (int q = 0; q < 16; ++q) {
                asm volatile("" ::"v"(wv[q]));
                fields[q] = (uint32_t)wv[q];
              }
            }
            __builtin_memcpy(&cm, fields, sizeof(FedCmd));
          }
          // The placer's plain loads of global memory: the scalar / host-port columns of a spec that has them (rows
          // its own commits wrote, and after a pause the launch path's), and everything after a pause. Those need
          // an agent-scope acquire on this CU (~1.7 us); a plain spec's job reads nothing but the tagged hand-offs
          // and its own LDS, so it skips it (the B candidates' static cache comes through the selector: s_bst).
          if (c >= 0 && cm.acq) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (the host's flag)
        }
        KB_FED_TL(m, 10);
        if (c == -2) atomicMax(exit_flag, 1);
        s_cand = c;
        s_op = c >= 0 ? KB_ENG_RUN : (c == kSelExit ? KB_ENG_EXIT : KB_ENG_EXIT_IDLE);
      }
      __syncthreads();
    } else {
      tgt[r] += blocks;
      fed_wait_cmd(&ctr[r], tgt[r], &ring[r], cm, s_op, idle_ticks, exit_flag);
    }
    if (s_op != KB_ENG_RUN) break;
    const int slot = cm.slot, spec = cm.spec;
    JobState* js = S.js[slot];
    JobState* hjs = S.hjs[slot];
    if (cm.g_valid && (last_panic || last_stop != cm.g_stop || last_placed != cm.g_placed ||
                       last_ready != cm.g_ready)) {  // mispredicted speculative job: nothing runs
      if (tid == 0) {
        js->stopped = 1;
        js->n_commit = 0;
        __hip_atomic_store(&hjs->seq, cm.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (SPLIT) {
          tag_store(&X->p_head[r], m + 1, kPubModeSkipped << 16);
          tag_store(&X->p_done[r], m + 1, 0u);
        }
      }
      last_panic = 1;
      ent_pf_na = -1;  // (the prefetched entries were this skipped job's)
      prev_slot[2] = prev_slot[1], prev_ncommit[2] = prev_ncommit[1];
      prev_slot[1] = prev_slot[0], prev_ncommit[1] = prev_ncommit[0];
      prev_slot[0] = slot, prev_ncommit[0] = 0;
      nbprev = 0;
      __syncthreads();
      continue;
    }
#ifdef KB_DIAG
    for (int k = 0; k < 7; ++k) dg[k] = 0;
    dg_last = __builtin_amdgcn_s_memtime();
    const uint64_t wait_cycles = dg_last - t_wait0;  // wait for the command (+ guard)
    if constexpr (SPLIT) KB_FED_TL(m, 5);
    dg[5] = pub_prev;
    const uint64_t rt0 = rt_wait0;
#endif
    if constexpr (SHARD) t_job0 = __builtin_amdgcn_s_memrealtime();
    if (cm.fresh) {  // after a pause: the sweep saw every earlier commit, and the launch path's units reused the slots
      prev_slot[0] = prev_slot[1] = prev_slot[2] = -1;
      prev_ncommit[0] = prev_ncommit[1] = prev_ncommit[2] = 0;
      nbprev = 0;
    }
    const kb_spec sp = P.specs[spec];
    const uint64_t* stat = S.stat[slot];
    const int64_t* sci = P.sc_init + (size_t)spec * N.S;
    int ready = cm.ready0, placed = 0;
    const int minav = cm.minav0, gang = cm.gang0;
    int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
    if (tid == 0) {
      sh.n_commit = 0;
      sh.need_hist = 0;
      s_feas = 0;
      s_bmax = 0;
    }
    // split engine with resident sweepers: the selected slots' level records (sh.comp: clv index + 1, 0 none)
    const bool lvl_on = SPLIT && S.lvl[slot] != nullptr;
    const uint32_t* lvl_lds = nullptr;
    if constexpr (SPLIT) {
      // candidates: A, the selector's T best outside the previous job's set (key order, with their static cache
      // and rows); B, that set re-keyed from the final rows kept in brow. Every rank below is a count over at
      // most 128 LDS entries split across 4 threads (unrolled), never a per-thread loop over all of them.
      // lists: the selectors' (k < nsel, s_na[k] entries each, keys descending), then B (nb)
      const int nb = nbprev;
      const uint32_t T = (uint32_t)cm.t_count;  // one segment
#ifdef KB_DIAG
      uint64_t mt = __builtin_amdgcn_s_memtime();
#define KB_MSTAMP(k)                                    \
  do {                                                  \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    mg[k] += t_ - mt;                                   \
    mt = t_;                                            \
  } while (0)
#else
#define KB_MSTAMP(k) \
  do {               \
  } while (0)
#endif
      // the lists' keys (A_k at akey[128 k], descending); one selector: its rows and static caches beside the
      // previous set's rows in the candidate space, else (up to 4 * 128 + 128 rows) in the key space, which a
      // split placer does not otherwise use
      uint32_t* akey = k32;
      Row* crow = MSEL == 1 ? brow + 128 : (Row*)(k32 + MSEL * 128);
      uint64_t* cst = (uint64_t*)(crow + (MSEL == 1 ? 256 : 128 * (MSEL + 1)));
      int32_t* cnd = (int32_t*)(cst + 128 * (MSEL + 1));
      // the A entries' level records (kLvlW words each, by list position), in key space the split placer leaves free
      uint32_t* clv = MSEL == 1 ? k32 + 128 : (uint32_t*)(cnd + 128 * (MSEL + 1));
      lvl_lds = clv;
      uint64_t lw[4] = {0, 0, 0, 0};  // this thread's A entry's level words (its record, valid flag in lw[3] >> 32)
      int na = 0, list = -1, idx = 0;
#pragma unroll
      for (int k = 0; k < MSEL; ++k) {
        const int c = k < nsel ? s_na[k] : 0;
        if (tid >= na && tid < na + c) list = k, idx = tid - na;
        na += c;
      }
      // (prefetched at the previous job's end for this very head: the same count)
      const bool pf = MSEL == 1 && ent_pf_na == na;
      int a_nrank = 0;  // an A entry's rank by node among A's first T (the selector's, entry bits 56..62)
      uint32_t bk_mine = 0;  // a B entry's key (0 elsewhere)
      bool b_feas = false;   // a B entry's key is feasible
      if (list >= 0) {
        const uint64_t(*ent)[128] = X->s_ent[r][list];
        // (the loads of the unprefetched path are consumed inside it: see the command decode above)
        uint64_t ew[kEntW];
        if (pf) {
#pragma unroll
          for (int q = 0; q < kEntW; ++q) ew[q] = ent_pf[q];
        } else {
#pragma unroll
          for (int q = 0; q < kEntW; ++q) ew[q] = x_load64(&ent[q][idx]);
#pragma unroll
          for (int q = 0; q < kEntW; ++q) asm volatile("" ::"v"(ew[q]));
        }
        const uint64_t e0 = ew[0];
        const uint64_t st = ew[1];
        uint64_t words[sizeof(Row) / 8];
#pragma unroll
        for (int q = 0; q < (int)(sizeof(Row) / 8); ++q) words[q] = ew[2 + q];
        __builtin_memcpy(&crow[tid], words, sizeof(Row));
        cst[tid] = st;
        cnd[tid] = (int)((e0 >> 32) & kEntNodeMask);
        if (lvl_on && !pf) {  // its level record (valid flag in the last word): loaded now, stored to LDS after the
                              // merge (prefetched: in LDS already, the loop top)
          constexpr int kL = 2 + (int)(sizeof(Row) / 8);
#pragma unroll
          for (int q = 0; q < 4; ++q) lw[q] = x_load64(&ent[kL + q][idx]);
        }
        a_nrank = (int)(e0 >> 56);
        akey[list * 128 + idx] = (uint32_t)e0;
      } else if (tid >= na && tid - na < nb) {
        const int j = tid - na, w = bprev[j];
        const Row rw = brow[j];
        // (selector 0's, behind its head: no acquire needed)
        uint64_t st = bst_pf;
        if (!pf) {
          st = x_load64(&X->s_bst[r][j]);
          asm volatile("" ::"v"(st));
        }
        const uint32_t rs = row_reasons(N, P, C, sp, sci, rw, st, w);
        // an infeasible key (its reason mask) gets the B index below it, so B's keys are distinct: their ranks
        // are a permutation (still below every feasible key)
        bkey[j] = rs ? (rs << 7) | (uint32_t)j
                     : compress_key(make_key(0, row_score(C, sp, rw, st), w), w + N.base, idx_bits);
        crow[na + j] = rw;
        crow[na + j].aux = -1;  // (A computed at the node setup)
        cst[na + j] = st;
        cnd[na + j] = w;
        b_feas = rs == 0;
        bk_mine = bkey[j];
      }
      {  // the largest B key and B's feasible count: per wave, then one LDS atomic per wave (100 lanes on one word
         // cost ~3k cycles, r05A)
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) bk_mine = umax32(bk_mine, (uint32_t)__shfl_xor((int)bk_mine, o, 64));
        const int nf = __popcll(__ballot(b_feas));
        if ((tid & 63) == 0 && bk_mine) atomicMax(&s_bmax, bk_mine);
        if ((tid & 63) == 0 && nf) atomicAdd(&s_feas, nf);
      }
      if (tid >= nb && tid < 128) bkey[tid] = 0u;  // padding ranks below every key
      __syncthreads();
      KB_MSTAMP(0);
      KB_FED_TL(m, 12);
      // Fast path (one selector list): every B key below A's T-th key -- the previous job's nodes, just loaded,
      // rank below the selector's T best, as they mostly do -- makes the T best of the union A's first T, in A's
      // order: no B order, no union ranks (~1.4 us of barrier-separated LDS ranking, r05z)
      const bool fast_a = MSEL == 1 && na >= (int)T && s_bmax < akey[T - 1];
      int pos = -1;
      uint32_t key = 0;
      if (fast_a) {
        if (tid < na) {
          pos = idx;
          key = akey[idx];
        }
      } else {
      // B's keys in descending order (rank among B: 4 threads per entry; the keys are distinct)
      {
        const int j = tid >> 2, part = tid & 3;
        const uint32_t k = j < nb ? bkey[j] : 0u;
        uint32_t c = 0;
#pragma unroll
        for (int q = 0; q < 32; ++q) c += bkey[part * 32 + q] > k;
        c += dpp_src<0xb1>(0u, c);  // quad_perm [1,0,3,2]
        c += dpp_src<0x4e>(0u, c);  // quad_perm [2,3,0,1]
        if (part == 0 && j < nb) {
          sh.emin[c] = k;  // scratch: B's keys sorted (descending)
          sh.A[j] = (int)c;
        }
      }
      __syncthreads();
      KB_MSTAMP(1);
      // rank in the union (keys carry the node: distinct): the own index plus, in every other list, the entries
      // above the key (binary search)
      const int nc = na + nb;
      if (tid < nc) {
        key = tid < na ? akey[list * 128 + idx] : bkey[tid - na];
        // entries above the key in every list (its own list included: there that is its index), all searches
        // at once: branch-free halving steps over lists of at most 128 (padding past a list's length unread)
        int c[MSEL + 1];
#pragma unroll
        for (int k = 0; k <= MSEL; ++k) c[k] = 0;
        int len[MSEL + 1];
#pragma unroll
        for (int k = 0; k <= MSEL; ++k) len[k] = k < MSEL ? (k < nsel ? s_na[k] : 0) : nb;
#pragma unroll
        for (int step = 64; step >= 1; step >>= 1) {
#pragma unroll
          for (int k = 0; k <= MSEL; ++k) {
            if (k < MSEL && k >= nsel) continue;  // (uniform) lists past the selectors
            const uint32_t* l = k < MSEL ? akey + k * 128 : sh.emin;
            const int p = c[k] + step;
            if (p <= len[k] && l[p - 1] > key) c[k] = p;
          }
        }
        pos = 0;
#pragma unroll
        for (int k = 0; k <= MSEL; ++k) pos += c[k];
      }
      }  // (the general merge)
      // the T best feasible (A is all feasible; infeasible keys rank below every feasible one), slots in node
      // order: the winners' tie rule on equal score fields takes lower slots first, which must be lower nodes
      const int nsel_t = min((int)T, na + s_feas);
      const bool sel = pos >= 0 && pos < nsel_t;
      if (!fast_a) {  // (fast path: the selector's node ranks of its first T entries are the slots)
        __syncthreads();  // the lists read
        if (sel) bprev[pos] = cnd[tid];  // scratch: the selected nodes by rank
        if (tid >= nsel_t && tid < 128) bprev[tid] = 0x7fffffff;  // padding: above every node
        __syncthreads();
        KB_MSTAMP(2);
        {
          const int e = tid >> 2, part = tid & 3;
          const int w = e < nsel_t ? bprev[e] : 0;
          uint32_t c = 0;
#pragma unroll
          for (int q = 0; q < 32; ++q) c += bprev[part * 32 + q] < w;
          c += dpp_src<0xb1>(0u, c);  // quad_perm [1,0,3,2]
          c += dpp_src<0x4e>(0u, c);  // quad_perm [2,3,0,1]
          if (part == 0 && e < nsel_t) sh.gen[e] = (int)c;  // scratch: slot of the rank-e node
        }
        __syncthreads();
      }
      // the selected A entries' level records into LDS (their loads had the merge to arrive; prefetched: there already,
      // the valid flag in the record's last word)
      const bool lv_ok = list >= 0 && (pf ? clv[(size_t)tid * kLvlW + kLvlW - 1] != 0u : (lw[3] >> 32) != 0);
      if (sel && lv_ok && !pf) {
        uint4* o = (uint4*)(clv + (size_t)tid * kLvlW);
        o[0] = make_uint4((uint32_t)lw[0], (uint32_t)(lw[0] >> 32), (uint32_t)lw[1], (uint32_t)(lw[1] >> 32));
        o[1] = make_uint4((uint32_t)lw[2], (uint32_t)(lw[2] >> 32), (uint32_t)lw[3], 1u);
      }
      if (sel) {
        const int slot_s = fast_a ? a_nrank : sh.gen[pos];
        sh.node[slot_s] = cnd[tid];
        sh.key0[slot_s] = key;
        sh.row[slot_s] = crow[tid];
        sh.stat[slot_s] = cst[tid];
        sh.lmax[slot_s] = (int)T - pos;
        sh.comp[slot_s] = lv_ok ? (uint64_t)(tid + 1) : 0ull;  // (sel_run: the slot's level record, clv[comp - 1])
        if (pos == nsel_t - 1) sh.theta0 = key;
      }
      if (tid == 0) sh.n_sel = nsel_t;
      __syncthreads();
      KB_MSTAMP(3);
#undef KB_MSTAMP
    } else {
      // the previous three jobs' commits (final rows) re-keyed for this spec: their loads first
      const int np0 = prev_slot[0] >= 0 ? prev_ncommit[0] : 0;
      const int np01 = np0 + (prev_slot[1] >= 0 ? prev_ncommit[1] : 0);
      const int np = np01 + (prev_slot[2] >= 0 ? prev_ncommit[2] : 0);
      const int32_t* patch0 = prev_slot[0] >= 0 ? S.commits[prev_slot[0]] : nullptr;
      const int32_t* patch1 = prev_slot[1] >= 0 ? S.commits[prev_slot[1]] : nullptr;
      const int32_t* patch2 = prev_slot[2] >= 0 ? S.commits[prev_slot[2]] : nullptr;
      const auto prev_node = [&](int i) {
        return i < np0 ? patch0[i] : (i < np01 ? patch1[i - np0] : patch2[i - np01]);
      };
      const int pw = tid < np ? prev_node(tid) : -1;
      Row prow;
      if (pw >= 0) prow = load_row(N, pw);
      const uint64_t pst = pw >= 0 ? stat[pw] : 0;
      load_keys_lds<(QN > 0 ? QN : kSelQ4)>(k32, S.keys[slot], n, n_pad);
      __syncthreads();
      if (np > 0) {
        if (pw >= 0) {
          const uint32_t rs = row_reasons(N, P, C, sp, sci, prow, pst, pw);
          k32[pw] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, prow, pst), pw), pw + N.base, idx_bits);
        }
        for (int i = tid + kSelThreads; i < np; i += kSelThreads) {
          const int w = prev_node(i);
          const Row rr = load_row(N, w);
          const uint64_t st = stat[w];
          const uint32_t rs = row_reasons(N, P, C, sp, sci, rr, st, w);
          k32[w] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, rr, st), w), w + N.base, idx_bits);
        }
        __syncthreads();
      }
    }
    KB_SEL_PH(0);
    if constexpr (SPLIT) KB_FED_TL(m, 6);  // (sel_run publishes the set first thing)
    FedPub pub;
    if constexpr (SPLIT) {
      pub.head = &X->p_head[r];
      pub.node = X->p_node[r];
      pub.tag = m + 1;
#ifdef KB_TIMELINE
      pub.tl = X->tl[m & (kFedTraceJobs - 1)];
#endif
    }
    if constexpr (SHARD) {
      sel_run<true, QN, true>(sh, k32, cand, N, P, C, sp, spec, cm.t_begin, cm.t_count, idx_bits, stat, ready, minav,
                              gang, placed, stop, fail_task, panic, stopped, S.hout[slot], js, hjs, rp, nullptr,
                              S.commits[slot] SEL_DIAG_ARGS, pub, nullptr, lvl_on ? lvl_lds : nullptr);
      ph[0] += __builtin_amdgcn_s_memrealtime() - t_job0;
      const int rc = shard_place(sh, k32, cand, SP, xn++, N, P, C, sp, spec, stat, S.keys[slot],
                                 prev_slot[0] >= 0 ? S.commits[prev_slot[0]] : nullptr,
                                 prev_slot[0] >= 0 ? prev_ncommit[0] : 0,
                                 prev_slot[1] >= 0 ? S.commits[prev_slot[1]] : nullptr,
                                 prev_slot[1] >= 0 ? prev_ncommit[1] : 0,
                                 prev_slot[2] >= 0 ? S.commits[prev_slot[2]] : nullptr,
                                 prev_slot[2] >= 0 ? prev_ncommit[2] : 0, cm.t_begin, cm.t_count, cm.ready0, minav,
                                 gang, idx_bits, S.hout[slot], js, hjs, S.commits[slot], idle_ticks, stop, fail_task,
                                 placed, ready, panic, stopped, ph);
      t_job0 = __builtin_amdgcn_s_memrealtime();  // (the publish below counts as commit)
      if (rc != 0) {  // a peer never answered (every rank's engine leaves), or the ranks issued different jobs
        if (tid == 0) {
          atomicMax(exit_flag, 1);
          if (rc == 2) {  // the host sees the job finish with the divergence flag (not a silent idle exit)
            hjs->stall = 2;
            js->n_commit = 0;
            publish_state(js, hjs, 1, KB_STOP_DONE, -1, 0, ready, minav, gang, 0, cm.seq);
          }
        }
        break;
      }
    } else {
      sel_run<false, QN, SPLIT>(sh, k32, cand, N, P, C, sp, spec, cm.t_begin, cm.t_count, idx_bits, stat, ready,
                                minav, gang, placed, stop, fail_task, panic, stopped, S.hout[slot], js, hjs, rp,
                                nullptr, S.commits[slot] SEL_DIAG_ARGS, pub, nullptr, lvl_on ? lvl_lds : nullptr);
    }
    if constexpr (SPLIT) {
      __syncthreads();
      // this job's set, with its final rows, is the next job's B
      const int ns = sh.n_sel;
      if (tid < ns) {
        bprev[tid] = sh.node[tid];
        brow[tid] = row_after(sp, sh.row[tid], sh.fin[tid], sh.A[tid]);
      }
      // an affinity unit's commits into the global tables (the first min(fin, A) commits on a node are Allocates,
      // which join the lister tables; every commit adds to the histograms), before the publish below: the host issues
      // a unit whose sweep reads them only after this one is read (the driver's dependency check)
      if constexpr (!SHARD)
        if (sp.aff_class >= 0 && tid < ns && sh.fin[tid] > 0) {
          // (inlined: as a call it put the kernel's by-value arguments in scratch)
          [[clang::always_inline]] apply_commit_tables(P.A, sp, sh.node[tid], min(sh.fin[tid], sh.A[tid]), sh.fin[tid]);
        }
      nbprev = ns;
      if (sh.need_hist && MSEL > 1 && nsel > 1) {  // no fit, the table past one key plan: the histogram streamed (below)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this job's row stores, not stale cached rows
        __syncthreads();
        const int32_t* l0 = prev_slot[0] >= 0 ? S.commits[prev_slot[0]] : nullptr;
        const int32_t* l1 = prev_slot[1] >= 0 ? S.commits[prev_slot[1]] : nullptr;
        const int32_t* l2 = prev_slot[2] >= 0 ? S.commits[prev_slot[2]] : nullptr;
        fed_hist_stream(sh, k32, N, P, C, sp, spec, stat, S.keys[slot], l0, prev_slot[0] >= 0 ? prev_ncommit[0] : 0,
                        l1, prev_slot[1] >= 0 ? prev_ncommit[1] : 0, l2, prev_slot[2] >= 0 ? prev_ncommit[2] : 0,
                        S.commits[slot], sh.n_commit);
        if (tid < KB_NUM_REASONS) {
          js->hist[tid] = sh.hist[tid];
          hjs->hist[tid] = sh.hist[tid];
        }
      } else if (sh.need_hist) {  // no fit: every node's key at this point (the sweep's, then every row changed since)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // this job's row stores, not stale cached rows
        __syncthreads();
        load_keys_lds<(QN > 0 ? QN : kSelQ4)>(k32, S.keys[slot], n, n_pad);
        __syncthreads();
        const int n0 = prev_slot[0] >= 0 ? prev_ncommit[0] : 0, n1 = prev_slot[1] >= 0 ? prev_ncommit[1] : 0;
        const int n2 = prev_slot[2] >= 0 ? prev_ncommit[2] : 0;
        {  // the previous three jobs' commits and this job's own (one loop: two fed_patch calls here trip the
           // ROCm 7.2 inliner)
          const int32_t* l0 = prev_slot[0] >= 0 ? S.commits[prev_slot[0]] : nullptr;
          const int32_t* l1 = prev_slot[1] >= 0 ? S.commits[prev_slot[1]] : nullptr;
          const int32_t* l2 = prev_slot[2] >= 0 ? S.commits[prev_slot[2]] : nullptr;
          const int n3 = sh.n_commit;
          for (int i = tid; i < n0 + n1 + n2 + n3; i += kSelThreads) {
            const int w = i < n0 ? l0[i]
                                 : (i < n0 + n1 ? l1[i - n0]
                                                : (i < n0 + n1 + n2 ? l2[i - n0 - n1] : S.commits[slot][i - n0 - n1 - n2]));
            const Row rr = load_row(N, w);
            const uint64_t st = stat[w];
            const uint32_t rs = row_reasons(N, P, C, sp, sci, rr, st, w);
            k32[w] = compress_key(make_key(rs, rs ? 0 : row_score(C, sp, rr, st), w), w + N.base, idx_bits);
          }
          __syncthreads();
        }
        sel_hist(sh, (const uint4*)k32, Q4);
        if (tid < KB_NUM_REASONS) {
          js->hist[tid] = sh.hist[tid];
          hjs->hist[tid] = sh.hist[tid];
        }
      }
    }
#ifdef KB_DIAG
    // fed engine layout: [0] key load + patch, [1..4] as sel_run, [5] commit + the previous job's publish +
    // the no-fit histogram, [6] waiting for this job's command; [7] realtime ticks including the wait
    dg[5] += dg[6];
    dg[6] = wait_cycles;
    if (tid == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
    // every wave's host-buffer and row stores are complete before the barrier; one lane then releases at
    // system scope and publishes (the host spins on the sequence number)
#ifdef KB_DIAG
    const uint64_t t_pub = __builtin_amdgcn_s_memtime();
#endif
    if constexpr (SPLIT) KB_FED_TL(m, 8);
    if (SPLIT && tid == 0) {  // the next job's head and command: their latency hides in the drain below
      const int rn = r + 1 == kJobSlots ? 0 : r + 1;
#pragma unroll
      for (int q = 0; q < 16; ++q) pre[q] = x_load64(&X->s_cmd[rn][q]);
#pragma unroll
      for (int k = 0; k < MSEL; ++k) pre[16 + k] = k < nsel ? x_load64(&X->s_head[rn][k]) : 0;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (a barrier alone waits for LDS only)
    if constexpr (SPLIT) {
      // the head and command words are in now (the wait above): a use here, on every path (not under tid == 0:
      // the compiler's wait counting merges the lanes' paths), ends its tracking of their loads, so the next job's
      // decode at the loop top waits for nothing -- else it waited there for every later load and store of the
      // wave, the release's host store included (~1 us per job, r05v-w)
#pragma unroll
      for (int q = 0; q < 16 + MSEL; ++q) asm volatile("" ::"v"(pre[q]));
    }
    if (SPLIT && MSEL == 1 && tid == 0) {  // the next job's head already there: its count, for the entry prefetch
      const bool h_ok = (uint32_t)(pre[16] >> 32) == m + 2 && (int32_t)(uint32_t)pre[16] >= 0;
      s_pre_na = h_ok ? (int32_t)(uint32_t)pre[16] : -1;
    }
    __syncthreads();
    if constexpr (SPLIT && MSEL == 1) {
      // every thread's entry of the next job, its head already seen: loads issued before this job's publish, so
      // their latency runs beside the release (which waits for them in thread 0's wave) instead of stalling the
      // next job's start (issued after it, the loop top's wait took ~1 us, r05v)
      ent_pf_na = s_pre_na;
      const int rn = r + 1 == kJobSlots ? 0 : r + 1;
      if (tid < ent_pf_na) {
        const uint64_t(*ent)[128] = X->s_ent[rn][0];
#pragma unroll
        for (int q = 0; q < kEntW; ++q) ent_pf[q] = x_load64(&ent[q][tid]);
#pragma unroll
        for (int q = 0; q < 4; ++q) lw_pf[q] = x_load64(&ent[kEntW + q][tid]);
      } else if (ent_pf_na >= 0 && tid - ent_pf_na < nbprev) {  // (the thread that takes that B entry)
        bst_pf = x_load64(&X->s_bst[rn][tid - ent_pf_na]);
      }
    }
    const int ncommit = sh.n_commit;
    if (tid == 0) {
      js->n_commit = ncommit;
      publish_state(js, hjs, stopped, stop, fail_task, placed, ready, minav, gang, panic, cm.seq);
#ifdef KB_TIMELINE
      if (SPLIT) X->tl[m & (kFedTraceJobs - 1)][9] = __builtin_amdgcn_s_memrealtime();
#endif
      // after that release (the job's rows written back): the selector may re-key them
      if (SPLIT) tag_store(&X->p_done[r], m + 1, (uint32_t)ncommit);
    }
    if constexpr (SPLIT) KB_FED_TL(m, 7);
    if constexpr (SHARD) ph[4] += __builtin_amdgcn_s_memrealtime() - t_job0;
    last_stop = stop, last_placed = placed, last_ready = ready, last_panic = panic;
    prev_slot[2] = prev_slot[1], prev_ncommit[2] = prev_ncommit[1];
    prev_slot[1] = prev_slot[0], prev_ncommit[1] = prev_ncommit[0];
    prev_slot[0] = slot, prev_ncommit[0] = ncommit;
    __syncthreads();  // cm / sh reused by the next command
#ifdef KB_DIAG
    t_wait0 = __builtin_amdgcn_s_memtime();
    rt_wait0 = __builtin_amdgcn_s_memrealtime();
    pub_prev = t_wait0 - t_pub;
#endif
  }
#ifdef KB_DIAG
  if (SPLIT && tid == 0) {
    for (int k = 0; k < 4; ++k) X->sdiag[8 + k] = mg[k];
    for (int k = 0; k < 8; ++k) X->wdiag[k] = dg[8 + k];
  }
#endif
  if (SPLIT && tid == 0) {  // for the host's stats: the exchange's cost (kb_stats.shard_wait_ticks / shard_xchg) and
                           // the shader clock over the launch (fed_clock_ticks / fed_real_ticks)
    X->sdiag[12] = ph[2];
#pragma unroll
    for (int k = 0; k < 6; ++k) X->sphase[k] = ph[k];
    X->sdiag[13] = xn;
    X->sdiag[14] = __builtin_amdgcn_s_memtime() - clk0;
    X->sdiag[15] = __builtin_amdgcn_s_memrealtime() - rt0_launch;
  }
}

int fed_lds_bytes(int n) {
  const int qn = sel_qn(n);
  return qn > 0 ? 4 * (4 * kSelThreads * qn) + 8 * kCandCap : sel_lds_bytes(n);
}

bool fed_fits(int n) {
  const int b = fed_lds_bytes(n);
  return b >= 0 && b <= kFedDynLimit;
}

void launch_fed_cmd(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, uint32_t* keys32,
                    uint64_t* stat, const FedCmdArgs& a, void* ring, uint32_t* ctr, bool sweep, void* stream) {
  FedCmd cmd{a.op, a.spec, a.t_begin, a.t_count, a.ready0, a.minav0, a.gang0, a.slot, a.g_valid, a.g_stop,
             a.g_placed, a.g_ready, a.seq, a.fresh, a.acq, a.fresh_m};
  const int blocks = sweep ? (N.n + 63) / 64 : 1;
  hipLaunchKernelGGL(fed_cmd_sweep_kernel<false>, dim3(blocks), dim3(64), 0, (hipStream_t)stream, N, P, C, idx_bits,
                     keys32, stat, cmd, (FedCmd*)ring, ctr, sweep ? 1 : 0);
}

size_t fed_ring_bytes() { return kJobSlots * sizeof(FedCmd); }
void fed_host_post(void* hring, int r, const FedCmdArgs& a, uint64_t tag) {
  FedCmd cmd{a.op, a.spec, a.t_begin, a.t_count, a.ready0, a.minav0, a.gang0, a.slot, a.g_valid, a.g_stop,
             a.g_placed, a.g_ready, a.seq, a.fresh, a.acq, a.fresh_m};
  FedHostCmd* h = (FedHostCmd*)hring + r;
  uint64_t w[8];
  __builtin_memcpy(w, &cmd, sizeof(cmd));
  for (int q = 0; q < 8; ++q) __atomic_store_n(&h->w[q], w[q], __ATOMIC_RELAXED);
  __atomic_store_n(&h->tag, tag, __ATOMIC_RELEASE);  // (x86: the words are visible first)
}
size_t fed_xchg_bytes() { return sizeof(FedXchg); }
size_t fed_census_bytes() { return offsetof(FedXchg, sphase) - offsetof(FedXchg, census_n); }
#ifdef KB_TIMELINE
size_t fed_trace_offset() { return offsetof(FedXchg, tl); }
#else
size_t fed_trace_offset() { return 0; }
#endif
int fed_trace_jobs() { return kFedTraceJobs; }
// Selector workgroups of the split engine for n nodes: one when every key fits one workgroup's plan, else the
// fewest ranges of at most kFedSelNodes (kFedMaxSel at most); 0: the table is beyond the engine.
int fed_nsel(int n) {
  if (fed_fits(n) && sel_qn(n) > 0) return 1;  // (the run-time group count instance spills when split)
  for (int k = 2; k <= kFedMaxSel; ++k)
    if (fed_sel_chunk(n, k) <= kFedSelNodes) return k;
  return 0;
}
// The placer's candidate keys and nodes (2 x 4 * kSelThreads words) share its key array: n_pad >= 4096.
// Unsharded tables of one key group stay on the one-workgroup engine; a node-sharded rank's block (the sharded engine
// is the split one) may be of any size: its instance then holds two key groups (n_pad = 4096, so the placer's
// candidate keys and nodes still fit its key array).
bool fed_split_ok(int n, bool sharded) { return fed_nsel(n) > 0 && (sharded ? n > 0 : n > 4 * kSelThreads); }

size_t shard_inbox_bytes() { return (size_t)2 * kJobSlots * kShardMaxWorld * kShardRecW * sizeof(uint64_t); }

// kb_set_shard_peer's pre-flight: one tagged word stored into a peer's inbox from this GPU (system scope, as
// shard_place writes its records over xGMI), and this rank's inbox words read back the way the engine polls them.
__global__ void peer_put_kernel(uint64_t* dst, uint64_t v) {
  if (threadIdx.x == 0) __hip_atomic_store(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void peer_get_kernel(const uint64_t* src, int n, uint64_t* out) {
  const int i = threadIdx.x;
  if (i < n) out[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
void launch_peer_put(uint64_t* dst, uint64_t v, void* stream) {
  hipLaunchKernelGGL(peer_put_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, dst, v);
}
void launch_peer_get(const uint64_t* src, int n, uint64_t* out, void* stream) {
  hipLaunchKernelGGL(peer_get_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, src, n, out);
}

int launch_fed_engine(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, const FedSlotPtrs& sp,
                      const void* ring, const uint32_t* ctr, const uint32_t* tgt, uint64_t idle_ticks,
                      int32_t* exit_flag, void* xchg, void* stream, bool coop, const ShardPeers& shard,
                      int place_xcc, const void* hring, uint32_t epoch) {
  FedSlots S;
  for (int s = 0; s < kJobSlots; ++s) {
    S.tgt[s] = tgt[s];
    S.keys[s] = sp.keys[s];
    S.stat[s] = sp.stat[s];
    S.commits[s] = sp.commits[s];
    S.js[s] = sp.js[s];
    S.hjs[s] = sp.hjs[s];
    S.hout[s] = sp.hout[s];
    S.lvl[s] = sp.lvl[s];
  }
  // past one workgroup's key plan: nsel range selectors of kFedSelQ key groups each (split engine only)
  int nsel = xchg ? fed_nsel(N.n) : 1;
  int qn = nsel > 1 ? kFedSelQ : sel_qn(N.n);
  if (xchg && qn == 1) qn = 2;  // a sharded rank's block of one key group: the split instance of two (fed_split_ok)
  const int bytes = qn > 0 ? 4 * (4 * kSelThreads * qn) + 8 * kCandCap : fed_lds_bytes(N.n);
  const FedCmd* ring_c = (const FedCmd*)ring;
  FedXchg* X = (FedXchg*)xchg;
  ShardPeers SP = shard;
  // (bit 8: the tests' one-XCC census, fed_engine_kernel)
  int pxcc = xchg && place_xcc >= 0 && (place_xcc & 0xff) < 8 ? place_xcc : -1;
  const FedHostCmd* hr = (const FedHostCmd*)hring;
  void* args[] = {(void*)&N, (void*)&P, (void*)&C, (void*)&idx_bits, (void*)&S, (void*)&ring_c, (void*)&ctr,
                  (void*)&idle_ticks, (void*)&exit_flag, (void*)&X, (void*)&nsel, (void*)&SP, (void*)&pxcc,
                  (void*)&hr, (void*)&epoch};
  const bool sharded = SP.world > 0;
  if (sharded && !xchg) return (int)hipErrorInvalidValue;  // the node-sharded engine is the split engine
  const void* f = nullptr;
  bool split = false;
#define KB_FED_QN(Q)                                                                                         \
  case Q:                                                                                                   \
    split = xchg && Q != 1;                                                                                 \
    f = split ? (sharded ? (const void*)fed_engine_kernel<Q, Q != 1, Q != 1> : (const void*)fed_engine_kernel<Q, Q != 1>) \
              : (const void*)fed_engine_kernel<Q, false>;                                                  \
    if (Q == kFedSelQ && split && nsel > 1)  /* range selectors: the instance with the lists' merge */       \
      f = sharded ? (const void*)fed_engine_kernel<kFedSelQ, true, true, kFedMaxSel>                          \
                  : (const void*)fed_engine_kernel<kFedSelQ, true, false, kFedMaxSel>;                      \
    break;
  switch (qn) {
    KB_FED_QN(1)
    KB_FED_QN(2)
    KB_FED_QN(3)
    KB_FED_QN(4)
    KB_FED_QN(5)
    KB_FED_QN(6)
    KB_FED_QN(8)
    KB_FED_QN(10)
    default:
      KB_FED_QN(0)
  }
#undef KB_FED_QN
  if (!split) nsel = 1;
  if (sharded && !split) return (int)hipErrorInvalidValue;
  if (!split) pxcc = -1;
  if (pxcc < 0 || coop) hr = nullptr;  // resident sweepers: with the census grid only
  // with sweepers, enough workgroups for about one sweeper thread per node off the placer's XCC (a sweeper's
  // nodes are latency-bound loads and static checks: C3's 20k nodes over 14 sweepers ran 39 us per job, r05q);
  // the dispatcher deals blocks round robin over the 8 XCCs, so ~7/8 of the grid lands off it
  int g = split ? (pxcc >= 0 ? 8 : 1) * (1 + kFedParity * nsel) : 1;
  if (hr != nullptr) {
    const int want_sw = kSweepGroups * ((N.n + kSelThreads - 1) / kSelThreads);  // (fed_sweeper's groups)
    const int g_sw = ((want_sw * 8 + 6) / 7 + 7) / 8 * 8;
    g = g_sw > g ? g_sw : g;
    if (g > kFedGridMax) g = kFedGridMax;
  }
  const dim3 grid(g), block(kSelThreads);
  if (coop) return (int)hipLaunchCooperativeKernel(f, grid, block, args, (unsigned)bytes, (hipStream_t)stream);
  // A plain launch: its workgroups spin on each other, so every one of them must be resident at once. The
  // dispatcher places them as CUs free up (the sweeps they wait for run on another hardware queue and never wait
  // for the engine), so it suffices that the whole grid fits the device at this LDS / register footprint -- the
  // one check a cooperative launch adds (MI355X_MICROARCH.md: same residency for a grid this small).
  int per_cu = 0, cus = 0, dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, f, kSelThreads, (size_t)bytes);
  if (e != hipSuccess) return (int)e;
  if ((long)per_cu * cus < (long)grid.x) return (int)hipErrorCooperativeLaunchTooLarge;
  return (int)hipLaunchKernel(f, grid, block, args, (size_t)bytes, (hipStream_t)stream);
}

// ---------------------------------------------------------------------------
// ===========================================================================
// Inter-pod affinity kernels.
// ===========================================================================
constexpr int kAffThreads = 1024;

__device__ __forceinline__ int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t x = __shfl_xor(v, o, 64);
    v = x < v ? x : v;
  }
  return v;
}
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t x = __shfl_xor(v, o, 64);
    v = x > v ? x : v;
  }
  return v;
}

// Block-wide min / max (starting at 0, as the reference's do) of the InterPodAffinity counts of a spec.
template <bool COH>
__device__ void block_ipa_minmax(const DevAff& A, const kb_aff_spec& as, int n, int64_t* rmin, int64_t* rmax,
                                 int64_t* mn_out, int64_t* mx_out) {
  const int tid = threadIdx.x, nthr = blockDim.x;
  int64_t mn = 0, mx = 0;
  for (int i = tid; i < n; i += nthr) {
    const int64_t c = ipa_count<COH>(A, as, i);
    mn = c < mn ? c : mn;
    mx = c > mx ? c : mx;
  }
  mn = wave_min_i64(mn);
  mx = wave_max_i64(mx);
  if ((tid & 63) == 0) {
    rmin[tid >> 6] = mn;
    rmax[tid >> 6] = mx;
  }
  __syncthreads();
  mn = 0, mx = 0;
  for (int w = 0; w < (nthr + 63) / 64; ++w) {
    mn = rmin[w] < mn ? rmin[w] : mn;
    mx = rmax[w] > mx ? rmax[w] : mx;
  }
  __syncthreads();  // rmin / rmax reusable
  *mn_out = mn;
  *mx_out = mx;
}

// One block per spec: min / max of its InterPodAffinity counts over all nodes into mm[2 * block].
__global__ __launch_bounds__(kAffThreads) void ipa_minmax_kernel(DevNodes N, DevSpecs P, const int32_t* spec_ids,
                                                                 int spec, int64_t* mm, const JobState* js,
                                                                 int by_spec) {
  __shared__ int64_t rmin[16], rmax[16];
  if (js != nullptr && js->stopped) return;
  const int s = spec_ids ? spec_ids[blockIdx.x] : spec;
  const kb_spec sp = P.specs[s];
  int64_t mn = 0, mx = 0;
  if (sp.aff_class >= 0) {
    const kb_aff_spec as = P.A.specs[sp.aff_class];
    if (as.hist_cnt) {
      // batches of 8 nodes per thread, every load of a batch issued before its use
      const int tid = threadIdx.x, n = N.n;
      constexpr int kB = 8;
      for (int i0 = 0; i0 < n; i0 += kB * kAffThreads) {
        int64_t c[kB];
#pragma unroll
        for (int j = 0; j < kB; ++j) c[j] = 0;
        for (uint32_t e = 0; e < as.hist_cnt; ++e) {
          const kb_ipa_hist h = P.A.hists[as.hist_off + e];
          int32_t d[kB];
#pragma unroll
          for (int j = 0; j < kB; ++j) {
            const int i = i0 + j * kAffThreads + tid;
            d[j] = i < n ? P.A.topo_dom[(size_t)h.slot * P.A.n + i] : -1;
          }
#pragma unroll
          for (int j = 0; j < kB; ++j)
            if (d[j] >= 0) c[j] += P.A.h[h.h_off + d[j]];
        }
#pragma unroll
        for (int j = 0; j < kB; ++j)
          if (i0 + j * kAffThreads + tid < n) {
            mn = c[j] < mn ? c[j] : mn;
            mx = c[j] > mx ? c[j] : mx;
          }
      }
      mn = wave_min_i64(mn);
      mx = wave_max_i64(mx);
      if ((tid & 63) == 0) {
        rmin[tid >> 6] = mn;
        rmax[tid >> 6] = mx;
      }
      __syncthreads();
      mn = 0, mx = 0;
      for (int w = 0; w < kAffThreads / 64; ++w) {
        mn = rmin[w] < mn ? rmin[w] : mn;
        mx = rmax[w] > mx ? rmax[w] : mx;
      }
    }
  }
  if (threadIdx.x == 0) {  // (by_spec: into the spec's own pair, mm_spec)
    const size_t o = by_spec ? (size_t)s : (size_t)blockIdx.x;
    mm[2 * o] = mn;
    mm[2 * o + 1] = mx;
  }
}

// The table increments of a run placed by the trajectory / re-key loops (whose spec's own affinity
// inputs do not move): one thread per placement of the run, read back from the placement buffer.
__global__ __launch_bounds__(256) void aff_commit_kernel(DevSpecs P, int spec, int t_begin, int run,
                                                         const JobState* js, const int32_t* hout, int base) {
  const int placed = js->n_placed - t_begin;  // placements of this run (tasks t_begin .. t_begin + run)
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= run || k >= placed) return;
  const int w = hout[2 * (t_begin + k)] - base;  // (node-sharded: possibly another rank's row; A.topo_dom is global)
  const int kind = hout[2 * (t_begin + k) + 1];
  apply_commit_tables(P.A, P.specs[spec], w, kind == KB_PLACE_ALLOCATE, 1);
}

// Key of node i for a spec whose affinity inputs move with its own commits: the cached base key (row
// + static predicates + LR/BRA/NodeAffinity), then the inter-pod affinity predicate (the last one) and
// the InterPodAffinity batch score from the live tables.
// ovf: the spec's host-overlay predicate row (kb_set_host_overlay), checked after the affinity predicate.
__device__ __forceinline__ uint64_t aff_key(const DevAff& A, const kb_aff_spec& as, const DevCfg& C, uint64_t b,
                                            int i, int64_t mn, int64_t mx, const uint8_t* ovf) {
  if (!(b & kFeasible)) return b;
  if (C.predicates) {
    const uint32_t ar = aff_reasons<true>(A, as, i);
    if (ar) return ar;
  }
  if (ovf != nullptr && ovf[i]) return kHostError;
  if (!C.nodeorder || !as.hist_cnt) return b;
  const int64_t score = (int64_t)((b >> 24) & ((1ull << 39) - 1)) - kScoreBias +
                        (int64_t)ipa_score(ipa_count<true>(A, as, i), mn, mx) * C.w_pa;
  return make_key(0, score, i);
}

// Block-wide place loop for a run of a spec whose own commits change its affinity inputs (e.g.
// anti-affinity to its own job on hostname, or preferred affinity to its own job): per task every node
// is re-keyed from the live tables (the reference's full PredicateNodes + PrioritizeNodes sweep,
// scheduler_helper.go:34-129), the block reduces the argmax, thread 0 commits the row, and the block
// applies the commit's table increments before the next task.
__global__ __launch_bounds__(kAffThreads) void aff_place_kernel(
    DevNodes N, DevSpecs P, DevCfg C, int spec, int t_begin, int t_count, uint64_t* base, uint64_t* stat,
    JobState* js, int first, int ready0, int minav0, int gang0, int32_t* hout, JobState* hjs, int pb_cap,
    uint32_t seq) {
  extern __shared__ __attribute__((aligned(16))) uint32_t pbs[];  // [pb_cap] placements: node | kind << 30
  __shared__ uint64_t red[16];
  __shared__ int64_t rmin[16], rmax[16];
  __shared__ uint32_t hist_s[KB_NUM_REASONS];
  __shared__ int32_t sh_kind;
  __shared__ LoopOut lo;
  if (!first && js->stopped) {
    signal_skip(hjs, seq);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = N.n;
  const kb_spec sp = P.specs[spec];
  const kb_aff_spec as = P.A.specs[sp.aff_class];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  const int32_t ov = ov_row(P, spec);
  const uint8_t* ovf = ov >= 0 ? P.ov_fail + (size_t)ov * n : nullptr;
  for (int i = tid; i < n; i += kAffThreads) {  // base keys (no inter-pod affinity)
    const Row r = load_row(N, i);
    const uint64_t st = static_eval<false>(N, P, C, sp, spec, r.flags, i, nullptr);
    stat[i] = st;
    const uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, i);
    base[i] = make_key(rs, rs ? 0 : row_score(C, sp, r, st), i);
  }
  int ready = first ? ready0 : js->ready_num;
  int minav = first ? minav0 : js->min_available;
  int gang = first ? gang0 : js->gang_ready;
  int placed = first ? 0 : js->n_placed;
  int pb_n = 0, pb_base = t_begin;
  int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
  const bool ipa = C.nodeorder && as.hist_cnt;
  __syncthreads();
  for (int t = 0; t < t_count; ++t) {
    int64_t mn = 0, mx = 0;
    if (ipa) block_ipa_minmax<true>(P.A, as, n, rmin, rmax, &mn, &mx);
    uint64_t best = 0;
    for (int i = tid; i < n; i += kAffThreads) best = umax64(best, aff_key(P.A, as, C, base[i], i, mn, mx, ovf));
    best = wave_max_u64(best);
    if (lane == 0) red[wv] = best;
    __syncthreads();
    best = 0;
    for (int k = 0; k < kAffThreads / 64; ++k) best = umax64(best, red[k]);
    if (!(best & kFeasible)) {
      // PredicateNodes found nothing (allocate.go:150-153): FitErrors histogram over all nodes.
      if (tid < KB_NUM_REASONS) hist_s[tid] = 0;
      __syncthreads();
      uint32_t h[KB_NUM_REASONS];
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] = 0;
      for (int i = tid; i < n; i += kAffThreads) {
        const uint64_t k = aff_key(P.A, as, C, base[i], i, mn, mx, ovf);
#pragma unroll
        for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] += (uint32_t)(k >> b) & 1u;
      }
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) {
        const uint32_t v = wave_sum_u32(h[b]);
        if (lane == 0 && v) atomicAdd(&hist_s[b], v);
      }
      __syncthreads();
      if (tid < KB_NUM_REASONS) {
        js->hist[tid] = hist_s[tid];
        hjs->hist[tid] = hist_s[tid];
      }
      stop = KB_STOP_NO_FIT;
      fail_task = t_begin + t;
      stopped = 1;
      break;
    }
    const int64_t score = (int64_t)((best >> 24) & ((1ull << 39) - 1)) - kScoreBias;
    if (score <= -1) {  // SelectBestNode: no bucket with score > -1 -> the reference panics
      fail_task = t_begin + t;
      panic = 1;
      stopped = 1;
      break;
    }
    const int w = (int)(kIdxMask - (uint32_t)(best & kIdxMask));
    if (tid == 0) {  // commit: Session.Allocate / Pipeline on the winner's row (allocate.go:159-182)
      Row r = load_row(N, w);
      const uint64_t st = stat[w];
      const bool to_idle = le_tol(sp.init_cpu, r.idle_cpu, 10) && le_tol(sp.init_mem, r.idle_mem, 10ll * 1024 * 1024) &&
                           scalars_fit(N, sp, sci, r.flags & KB_NODE_IDLE_HAS_MAP, N.idle_sc, w);
      int kind;
      if (to_idle) {
        r.idle_cpu -= sp.req_cpu;
        r.idle_mem -= sp.req_mem;
        if (r.flags & KB_NODE_IDLE_HAS_MAP) {
          uint64_t m = sp.req_sc_mask;
          while (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            N.idle_sc[(size_t)q * n + w] -= scr[q];
          }
        }
        kind = KB_PLACE_ALLOCATE;
      } else {
        r.rel_cpu -= sp.req_cpu;
        r.rel_mem -= sp.req_mem;
        if (r.flags & KB_NODE_REL_HAS_MAP) {
          uint64_t m = sp.req_sc_mask;
          while (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            N.rel_sc[(size_t)q * n + w] -= scr[q];
          }
        }
        kind = KB_PLACE_PIPELINE;
      }
      r.pod_count += 1;
      r.nz_cpu += sp.nz_cpu;
      r.nz_mem += sp.nz_mem;
      for (uint32_t i = 0; i < sp.port_cnt; ++i) {
        const kb_port p = P.ports[sp.port_off + i];
        N.port_used[(size_t)p.slot * n + w] |= 1ull << p.ip;
      }
      store_row(N, w, r);
      const uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, w);
      base[w] = make_key(rs, rs ? 0 : row_score(C, sp, r, st), w);
      pbs[pb_n] = (uint32_t)w | ((uint32_t)kind << 30);
      sh_kind = kind;
    }
    __syncthreads();
    const int kind = sh_kind;
    // this commit's table increments, in parallel (distinct counters per entry)
    const int nl = kind == KB_PLACE_ALLOCATE ? (int)as.lister_cnt : 0;
    for (int i = tid; i < nl + (int)as.incr_cnt; i += kAffThreads) {
      if (i < nl) {
        const int32_t tb = P.A.lister[as.lister_off + i];
        const kb_aff_table ta = P.A.tables[tb];
        const int32_t d = P.A.topo_dom[(size_t)ta.slot * n + w];
        if (d >= 0) atomicAdd(&P.A.counters[ta.cnt_off + d], 1);
        atomicAdd(&P.A.totals[tb], 1);
      } else {
        const kb_ipa_incr e = P.A.incr[as.incr_off + (i - nl)];
        const int32_t d = P.A.topo_dom[(size_t)e.slot * n + w];
        if (d >= 0) atomicAdd(&P.A.h[e.h_off + d], e.weight);
      }
    }
    __threadfence();
    __syncthreads();
    ++placed;
    ++pb_n;
    if (kind == KB_PLACE_ALLOCATE) ++ready;
    if (!gang || ready >= minav) {  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
      stop = KB_STOP_READY;
      stopped = 1;
      break;
    }
    if (pb_n == pb_cap) {
      for (int k = tid; k < pb_n; k += kAffThreads) {
        const uint32_t e = pbs[k];
        hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
        hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
      }
      __syncthreads();
      pb_base += pb_n;
      pb_n = 0;
    }
  }
  for (int k = tid; k < pb_n; k += kAffThreads) {
    const uint32_t e = pbs[k];
    hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
    hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
  }
  if (tid == 0) lo = LoopOut{stop, fail_task, placed, ready, minav, gang, panic, stopped, pb_n, pb_base, 0, 0};
  __threadfence_system();
  __syncthreads();
  if (tid == 0)
    publish_state(js, hjs, lo.stopped, lo.stop, lo.fail_task, lo.placed, lo.ready, lo.minav, lo.gang, lo.panic,
                  seq);
}

int aff_pb_cap(int t_count) { return t_count < 8192 ? (t_count < 1 ? 1 : t_count) : 8192; }

// ---------------------------------------------------------------------------
// Register-resident variant of aff_place_kernel (same semantics, same outputs). Every thread owns the
// nodes i = k * kAffThreads + tid (k < NPT) for the whole run and keeps, in registers, their base keys and
// the live value of every affinity entry of the spec (checks: the count-table entry of the node's domain;
// histograms: the InterPodAffinity histogram entry). Within the run only this kernel's own commits change
// those tables, and a commit changes a handful of (table, domain) entries, all known: thread 0 broadcasts
// them and every thread patches the nodes of those domains (domain ids in LDS). A task therefore reads no
// global memory for its re-sweep: counts, reasons, min / max and keys come from registers. The global
// tables are still updated (atomics) for the kernels that follow. Specs with more than kAffRegE entries,
// more than kAffRegU table updates per commit, or more than NPT * kAffThreads nodes take aff_place_kernel.
// ---------------------------------------------------------------------------
#ifdef KB_DIAG_AFF  // phase stamps of this kernel only (Makefile target diagaff)
#define AFF_STAMP(k)                                  \
  do {                                                \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    dg[k] += t_ - dg_last;                            \
    dg_last = t_;                                     \
  } while (0)
#else
#define AFF_STAMP(k) \
  do {               \
  } while (0)
#endif
constexpr int kAffRegE = 4;  // entries (checks + histograms) per spec, at most
constexpr int kAffRegU = 8;
constexpr int kAffRegMaxNpt = 10;  // n <= 10240 (domain ids < n fit 16 bits)

struct AffUpd {
  int32_t kind;   // 0: count table (lister join), 1: histogram (commit increment)
  int32_t key;    // table id / histogram h_off
  int32_t dom;    // the committed node's domain (-1: none, nothing changes)
  int32_t delta;
};

template <int NPT, int NE>
__global__ __launch_bounds__(kAffThreads) void aff_reg_kernel(
    DevNodes N, DevSpecs P, DevCfg C, int spec, int t_begin, int t_count, uint64_t* stat, JobState* js, int first,
    int ready0, int minav0, int gang0, int32_t* hout, JobState* hjs, int pb_cap, uint32_t seq) {
  // dynamic LDS: [NPT * kAffThreads] u64 base keys, [NE][NPT * kAffThreads] u16 domain ids (0xffff: no
  // domain), then [pb_cap] placements
  extern __shared__ __attribute__((aligned(16))) uint32_t lds_ar[];
  constexpr int kStride = NPT * kAffThreads;
  uint64_t* bkl = (uint64_t*)lds_ar;
  uint16_t* dm16 = (uint16_t*)(bkl + kStride);
  uint32_t* pbs = (uint32_t*)(dm16 + NE * kStride);
  __shared__ uint64_t red[16];
  __shared__ int64_t rmin[16], rmax[16];
  __shared__ uint32_t hist_s[KB_NUM_REASONS];
  __shared__ int32_t sh_kind, sh_w;
  __shared__ uint64_t sh_base;
  __shared__ AffUpd sh_upd[kAffRegU];
  __shared__ int64_t sh_bp[10];
  __shared__ LoopOut lo;
  if (!first && js->stopped) {
    signal_skip(hjs, seq);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = N.n;
  const DevAff& A = P.A;
  const kb_spec sp = P.specs[spec];
  const kb_aff_spec as = A.specs[sp.aff_class];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  const int nc = (int)as.check_cnt, ne = (int)(as.check_cnt + as.hist_cnt);
  // entry e < nc: check (counters[cnt_off + dom] of table e_key); nc <= e < ne: histogram (h[e_key + dom])
  int32_t e_slot[NE], e_off[NE], e_kind[NE], e_key[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    e_slot[e] = 0, e_off[e] = 0, e_kind[e] = 0, e_key[e] = -1;
    if (e < nc) {
      const kb_aff_check c = A.checks[as.check_off + e];
      const kb_aff_table t = A.tables[c.table];
      e_slot[e] = t.slot, e_off[e] = (int32_t)t.cnt_off, e_kind[e] = c.kind, e_key[e] = c.table;
    } else if (e < ne) {
      const kb_ipa_hist h = A.hists[as.hist_off + (e - nc)];
      e_slot[e] = h.slot, e_off[e] = (int32_t)h.h_off, e_key[e] = (int32_t)h.h_off;
    }
  }
#ifdef KB_DIAG_AFF
  // phases: 0 prologue, 1 counts + min/max, 2 keys + argmax, 3 commit (thread 0), 4 table updates,
  // 5 stop rules / flush, 6 no-fit histogram
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  int32_t v[NPT][NE];
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int i = k * kAffThreads + tid;
    bkl[i] = 0;  // padding: infeasible with no reason bits (never wins, adds nothing to the histogram)
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      dm16[e * kStride + i] = 0xffffu;
      v[k][e] = 0;
    }
    if (i < n) {
      const Row r = load_row(N, i);
      const uint64_t st = static_eval<false>(N, P, C, sp, spec, r.flags, i, nullptr);
      stat[i] = st;
      const uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, i);
      bkl[i] = make_key(rs, rs ? 0 : row_score(C, sp, r, st), i);
#pragma unroll
      for (int e = 0; e < NE; ++e)
        if (e < ne) {
          const int32_t d = A.topo_dom[(size_t)e_slot[e] * A.n + i];
          if (d >= 0) {
            dm16[e * kStride + i] = (uint16_t)d;
            v[k][e] = ld_cnt<true>((e < nc ? A.counters : A.h) + e_off[e] + d);
          }
        }
    }
  }
  int32_t tot[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) tot[e] = e < nc ? ld_cnt<true>(&A.totals[e_key[e]]) : 0;
  int ready = first ? ready0 : js->ready_num;
  int minav = first ? minav0 : js->min_available;
  int gang = first ? gang0 : js->gang_ready;
  int placed = first ? 0 : js->n_placed;
  int pb_n = 0, pb_base = t_begin;
  int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
  const bool ipa = C.nodeorder && as.hist_cnt;
  __syncthreads();
  AFF_STAMP(0);
  // The task loop reads the launch's uniform structs from LDS copies (thread 0's commit needs the node
  // columns, the spec and the affinity tables; kept in scalar registers across the loop they spilled).
  __shared__ DevNodes LN;
  __shared__ DevSpecs LP;
  __shared__ DevCfg LC;
  __shared__ kb_spec LS;
  __shared__ kb_aff_spec LAS;
  if (tid == 0) {
    LN = N;
    LP = P;
    LC = C;
    LS = sp;
    LAS = as;
  }
  const DevAff& LA = LP.A;
  const int c_pred = C.predicates;
  const int64_t c_wpa = C.w_pa;
  for (int t = 0; t < t_count; ++t) {
    // counts and reasons of every owned node from the registers (aff_reasons / ipa_count); computed again
    // in the key pass rather than held across the min / max reduction (register budget)
    const auto count_of = [&](int k) -> int32_t {
      int32_t c = 0;
#pragma unroll
      for (int e = 0; e < NE; ++e)
        if (e >= nc) c += v[k][e];
      return c;
    };
    const auto reasons_of = [&](int k) -> uint32_t {
      if (!c_pred) return 0u;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        if (e >= nc) break;
        if (e_kind[e] == KB_AFF_EXISTING_ANTI) {
          if (v[k][e] > 0) return kAffExistingAnti;
        } else if (e_kind[e] == KB_AFF_ANTI) {
          if (v[k][e] > 0) return kAffAntiRules;
        } else if (e_kind[e] == KB_AFF_ERROR) {
          if (v[k][e] > 0) return kHostError;
        } else if (v[k][e] == 0 && (tot[e] > 0 || !LAS.self_match)) {
          return kAffAffinityRules;
        }
      }
      return 0u;
    };
    int64_t mn = 0, mx = 0;
    if (ipa) {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int32_t c = count_of(k);
        if (k * kAffThreads + tid < n) {  // min / max over every node, from 0 (interpod_affinity.go:221-238)
          mn = c < mn ? c : mn;
          mx = c > mx ? c : mx;
        }
      }
      mn = wave_min_i64(mn);
      mx = wave_max_i64(mx);
      if (lane == 0) {
        rmin[wv] = mn;
        rmax[wv] = mx;
      }
      __syncthreads();
      mn = 0, mx = 0;
#pragma unroll
      for (int w = 0; w < kAffThreads / 64; ++w) {
        mn = rmin[w] < mn ? rmin[w] : mn;
        mx = rmax[w] > mx ? rmax[w] : mx;
      }
      // ipa_score is monotone in the count: its 10 breakpoints, exactly. a_s = ceil(s * b / 10) is the
      // first offset with 10 a / b >= s; the float64 formula can only fall short of s where 10 a / b == s
      // exactly (elsewhere the gap is >= 1 / b, far above the rounding error), and then a_s + 1 is it.
      if (tid < 10) {
        const int64_t bb = mx - mn;
        int64_t as_ = INT64_MAX;
        if (bb > 0) {
          const int64_t sb = (int64_t)(tid + 1) * bb;
          as_ = (sb + 9) / 10;
          if (sb % 10 == 0 && ipa_score(mn + as_, mn, mx) < tid + 1) ++as_;
        }
        sh_bp[tid] = as_;
      }
      __syncthreads();
    }
    int64_t bp[10];  // uniform: scalar registers
#pragma unroll
    for (int q = 0; q < 10; ++q) {
      const int64_t x = ipa ? sh_bp[q] : INT64_MAX;
      const uint32_t lo32 = __builtin_amdgcn_readfirstlane((uint32_t)x);
      const uint32_t hi32 = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
      bp[q] = (int64_t)(((uint64_t)hi32 << 32) | lo32);
    }
    AFF_STAMP(1);
    // aff_key on the registers
    const auto key_of = [&](int k) -> uint64_t {
      const uint64_t b = bkl[k * kAffThreads + tid];
      if (!(b & kFeasible)) return b;
      const uint32_t ar = reasons_of(k);
      if (ar) return ar;
      if (!ipa) return b;
      const int64_t off = (int64_t)count_of(k) - mn;
      int32_t sc = 0;  // == ipa_score(count, mn, mx)
#pragma unroll
      for (int q = 0; q < 10; ++q) sc += off >= bp[q];
      const int64_t score = (int64_t)((b >> 24) & ((1ull << 39) - 1)) - kScoreBias + (int64_t)sc * c_wpa;
      return make_key(0, score, k * kAffThreads + tid);
    };
    uint64_t best = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) best = umax64(best, key_of(k));
    best = wave_max_u64(best);
    if (lane == 0) red[wv] = best;
    __syncthreads();
    best = 0;
#pragma unroll
    for (int k = 0; k < kAffThreads / 64; ++k) best = umax64(best, red[k]);
    AFF_STAMP(2);
    if (!(best & kFeasible)) {
      // PredicateNodes found nothing (allocate.go:150-153): FitErrors histogram over all nodes.
      if (tid < KB_NUM_REASONS) hist_s[tid] = 0;
      __syncthreads();
      uint32_t h[KB_NUM_REASONS];
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const uint64_t kk = key_of(k);
#pragma unroll
        for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] += (uint32_t)(kk >> b) & 1u;
      }
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) {
        const uint32_t s = wave_sum_u32(h[b]);
        if (lane == 0 && s) atomicAdd(&hist_s[b], s);
      }
      __syncthreads();
      if (tid < KB_NUM_REASONS) {
        js->hist[tid] = hist_s[tid];
        hjs->hist[tid] = hist_s[tid];
      }
      stop = KB_STOP_NO_FIT;
      fail_task = t_begin + t;
      stopped = 1;
      AFF_STAMP(6);
      break;
    }
    const int64_t score = (int64_t)((best >> 24) & ((1ull << 39) - 1)) - kScoreBias;
    if (score <= -1) {  // SelectBestNode: no bucket with score > -1 -> the reference panics
      fail_task = t_begin + t;
      panic = 1;
      stopped = 1;
      break;
    }
    const int w = (int)(kIdxMask - (uint32_t)(best & kIdxMask));
    if (tid == 0) {  // commit: Session.Allocate / Pipeline on the winner's row (allocate.go:159-182)
      const int64_t* lsci = LP.sc_init + (size_t)spec * LN.S;
      const int64_t* lscr = LP.sc_req + (size_t)spec * LN.S;
      Row r = load_row(LN, w);
      const uint64_t st = stat[w];
      const bool to_idle = le_tol(LS.init_cpu, r.idle_cpu, 10) && le_tol(LS.init_mem, r.idle_mem, 10ll * 1024 * 1024) &&
                           scalars_fit(LN, LS, lsci, r.flags & KB_NODE_IDLE_HAS_MAP, LN.idle_sc, w);
      int kind;
      if (to_idle) {
        r.idle_cpu -= LS.req_cpu;
        r.idle_mem -= LS.req_mem;
        if (r.flags & KB_NODE_IDLE_HAS_MAP) {
          uint64_t m = LS.req_sc_mask;
          while (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            LN.idle_sc[(size_t)q * n + w] -= lscr[q];
          }
        }
        kind = KB_PLACE_ALLOCATE;
      } else {
        r.rel_cpu -= LS.req_cpu;
        r.rel_mem -= LS.req_mem;
        if (r.flags & KB_NODE_REL_HAS_MAP) {
          uint64_t m = LS.req_sc_mask;
          while (m) {
            const int q = __builtin_ctzll(m);
            m &= m - 1;
            LN.rel_sc[(size_t)q * n + w] -= lscr[q];
          }
        }
        kind = KB_PLACE_PIPELINE;
      }
      r.pod_count += 1;
      r.nz_cpu += LS.nz_cpu;
      r.nz_mem += LS.nz_mem;
      for (uint32_t i = 0; i < LS.port_cnt; ++i) {
        const kb_port p = LP.ports[LS.port_off + i];
        LN.port_used[(size_t)p.slot * n + w] |= 1ull << p.ip;
      }
      store_row(LN, w, r);
      const uint32_t rs = row_reasons(LN, LP, LC, LS, lsci, r, st, w);
      sh_base = make_key(rs, rs ? 0 : row_score(LC, LS, r, st), w);
      sh_w = w;
      pbs[pb_n] = (uint32_t)w | ((uint32_t)kind << 30);
      sh_kind = kind;
    } else if (tid <= (int)(LAS.lister_cnt + LAS.incr_cnt)) {
      // the table entries this commit changes (apply_commit_tables), loaded beside thread 0's row work:
      // lister joins (applied on an Allocate only), then the histogram increments (every commit)
      const int u = tid - 1;
      if (u < (int)LAS.lister_cnt) {
        const int32_t tb = LA.lister[LAS.lister_off + u];
        sh_upd[u] = AffUpd{0, tb, LA.topo_dom[(size_t)LA.tables[tb].slot * n + w], 1};
      } else {
        const kb_ipa_incr e = LA.incr[LAS.incr_off + (u - (int)LAS.lister_cnt)];
        sh_upd[u] = AffUpd{1, (int32_t)e.h_off, LA.topo_dom[(size_t)e.slot * n + w], e.weight};
      }
    }
    __syncthreads();
    AFF_STAMP(3);
    const int kind = sh_kind;
    if (tid == 0) bkl[sh_w] = sh_base;  // the committed node's new base key (read after the next barrier)
    // the global tables (read by the kernels after this one): atomics, completed before the final publish
    const int nupd = (int)(LAS.lister_cnt + LAS.incr_cnt);
    const bool joins = kind == KB_PLACE_ALLOCATE;  // a Pipelined task does not join the lister tables
    if (tid < nupd && (joins || sh_upd[tid].kind == 1)) {
      const AffUpd up = sh_upd[tid];
      if (up.kind == 0) {
        if (up.dom >= 0) atomicAdd(&LA.counters[LA.tables[up.key].cnt_off + up.dom], up.delta);
        atomicAdd(&LA.totals[up.key], up.delta);
      } else if (up.dom >= 0) {
        atomicAdd(&LA.h[up.key + up.dom], up.delta);
      }
    }
    // ... and the same updates on the registers: the nodes of the committed node's domains
    for (int u = 0; u < nupd; ++u) {
      const AffUpd up = sh_upd[u];
      if (up.kind == 0 && !joins) continue;
#pragma unroll
      for (int e = 0; e < NE; ++e) {
        const bool hit = up.kind == 0 ? e < nc && e_key[e] == up.key : e >= nc && e < ne && e_key[e] == up.key;
        if (!hit) continue;
        if (up.kind == 0) tot[e] += up.delta;
        if (up.dom < 0) continue;
#pragma unroll
        for (int k = 0; k < NPT; ++k)
          if (dm16[e * kStride + k * kAffThreads + tid] == (uint32_t)up.dom) v[k][e] += up.delta;
      }
    }
    AFF_STAMP(4);
    ++placed;
    ++pb_n;
    if (kind == KB_PLACE_ALLOCATE) ++ready;
    if (!gang || ready >= minav) {  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
      stop = KB_STOP_READY;
      stopped = 1;
      break;
    }
    if (pb_n == pb_cap) {
      for (int k = tid; k < pb_n; k += kAffThreads) {
        const uint32_t e = pbs[k];
        hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
        hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
      }
      __syncthreads();
      pb_base += pb_n;
      pb_n = 0;
    }
    AFF_STAMP(5);
  }
  for (int k = tid; k < pb_n; k += kAffThreads) {
    const uint32_t e = pbs[k];
    hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
    hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
  }
#ifdef KB_DIAG_AFF
  if (tid == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
  if (tid == 0) lo = LoopOut{stop, fail_task, placed, ready, minav, gang, panic, stopped, pb_n, pb_base, 0, 0};
  __threadfence_system();
  __syncthreads();
  if (tid == 0)
    publish_state(js, hjs, lo.stopped, lo.stop, lo.fail_task, lo.placed, lo.ready, lo.minav, lo.gang, lo.panic,
                  seq);
}

int aff_reg_npt(int n) {
  int npt = (n + kAffThreads - 1) / kAffThreads;
  npt = npt < 2 ? 2 : (npt + 1) & ~1;  // instantiated for even counts (padding nodes never win)
  return npt <= kAffRegMaxNpt ? npt : -1;
}

// The register-resident loop takes (n, entries) when its LDS plan (base keys + domain ids + a placement
// buffer of at least 256) fits.
bool aff_reg_fits(int n, int ne) {
  const int npt = aff_reg_npt(n);
  if (npt < 0 || ne < 1 || ne > kAffRegE) return false;
  return (size_t)npt * kAffThreads * (8 + 2 * ne) + 4096 + 256 * 4 <= (size_t)kLdsLimit;
}

#define KB_AFF_REG_NE(K, E)                                                                                       \
  case (K) * 8 + (E):                                                                                             \
    hipLaunchKernelGGL((aff_reg_kernel<K, E>), dim3(1), dim3(kAffThreads), bytes, (hipStream_t)stream, N, P, C,   \
                       spec, t_begin, t_count, stat, js, first, ready0, minav0, gang0, hout, hjs, pb_cap, seq);    \
    break;
#define KB_AFF_REG_CASE(K) KB_AFF_REG_NE(K, 1) KB_AFF_REG_NE(K, 2) KB_AFF_REG_NE(K, 3) KB_AFF_REG_NE(K, 4)

void launch_aff_reg(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int ne, int t_begin,
                    int t_count, uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0,
                    int32_t* hout, JobState* hjs, uint32_t seq, void* stream) {
  const int npt = aff_reg_npt(N.n);
  const int E = ne < 1 ? 1 : ne;
  int pb_cap = aff_pb_cap(t_count);
  const size_t fixed = (size_t)npt * kAffThreads * (8 + 2 * E);  // base keys + domain ids
  const size_t cap_max = ((size_t)kLdsLimit - 4096 - fixed) / 4;  // the kernel's static LDS stays below 4 KB
  if ((size_t)pb_cap > cap_max) pb_cap = (int)cap_max;
  const size_t bytes = fixed + (size_t)pb_cap * 4;
  switch (npt * 8 + E) {
    KB_AFF_REG_CASE(2)
    KB_AFF_REG_CASE(4)
    KB_AFF_REG_CASE(6)
    KB_AFF_REG_CASE(8)
    KB_AFF_REG_CASE(10)
    default:
      break;
  }
}

#define KB_AFF_REG_FN(K) (const void*)aff_reg_kernel<K, 1>, (const void*)aff_reg_kernel<K, 2>, \
                         (const void*)aff_reg_kernel<K, 3>, (const void*)aff_reg_kernel<K, 4>
static const void* const kAffRegFns[] = {KB_AFF_REG_FN(2), KB_AFF_REG_FN(4), KB_AFF_REG_FN(6), KB_AFF_REG_FN(8),
                                        KB_AFF_REG_FN(10)};
#undef KB_AFF_REG_FN
#undef KB_AFF_REG_CASE
#undef KB_AFF_REG_NE

void launch_ipa_minmax(const DevNodes& N, const DevSpecs& P, const int32_t* spec_ids, int spec, int count,
                       int64_t* mm, const JobState* js, void* stream, int by_spec) {
  hipLaunchKernelGGL(ipa_minmax_kernel, dim3(count), dim3(kAffThreads), 0, (hipStream_t)stream, N, P, spec_ids, spec,
                     mm, js, by_spec);
}

void launch_aff_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                      uint64_t* base, uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0,
                      int32_t* hout, JobState* hjs, uint32_t seq, void* stream) {
  const int pb_cap = aff_pb_cap(t_count);
  hipLaunchKernelGGL(aff_place_kernel, dim3(1), dim3(kAffThreads), (size_t)pb_cap * 4, (hipStream_t)stream, N, P, C,
                     spec, t_begin, t_count, base, stat, js, first, ready0, minav0, gang0, hout, hjs, pb_cap, seq);
}

// ---------------------------------------------------------------------------
// Class loop: a spec whose own commits move only its InterPodAffinity histograms (preferred affinity to
// its own job's pods, say "the rack of my job"), every check static. classify_self_dynamic (kbgpu_host.cpp)
// found F, the finest moving slot, with every histogram's domain a function of the node's F-domain. A
// class = the nodes of one F-domain (class K-1: the nodes without one). They share every histogram entry
// all run long, hence the count, the InterPodAffinity score (interpod_affinity.go:221-238: min / max over
// all nodes = over the non-empty classes) and the checks. Inside a class the order is that of the base key
// (row + static predicates + LR / BRA / NodeAffinity, scheduler_helper.go:67-129 without the batch score),
// so a task's argmax (scheduler_helper.go:147-158) is the best over classes of (class best + class score).
// A commit changes the winner's row (its base key: a rescan of its class's members) and the counts of the
// classes in the committed node's domains (nodeorder.go:161-172 AddPod). Per task: one wave, a few lane
// ops per class and per member of the winner's class, no block barriers; aff_reg_kernel re-keys every node.
// Prologue on the whole block: base keys, class member lists (CSR) and class state in LDS. The run's
// global table updates come at its end, from the placements.
// ---------------------------------------------------------------------------
// 4 waves: the task loop's wave gets the whole VGPR file of its SIMD (1024 threads cap it at 128 and spill)
constexpr int kClsThreads = 256;
constexpr int kClsPM = 2;  // a class phase's members per lane (classes of at most 128 nodes)
constexpr int kClsStaticLds = 6144;  // the kernel's static LDS (the phase's level queues, 4 KB) and slack
static_assert(kClsMaxK <= 16 * 64 && kClsMaxK % kClsThreads == 0, "classes per lane: at most 16");

// wave-uniform signed max / min on DPP (ordering-preserving bias to unsigned); |v| < 2^62
__device__ __forceinline__ int64_t wave_max_i64_dpp(int64_t v) {
  return (int64_t)(wave_max_dpp((uint64_t)v ^ (1ull << 63)) ^ (1ull << 63));
}
__device__ __forceinline__ int64_t wave_min_i64_dpp(int64_t v) { return -wave_max_i64_dpp(-v); }

// One wave's LDS accesses complete in issue order (the LDS serves a wave's DS instructions in order), so a
// lane's store is seen by every later load of the wave: only the compiler must not move accesses across.
__device__ __forceinline__ void wave_sync_lds() { __builtin_amdgcn_wave_barrier(); }

static size_t cls_lds_bytes(int n, int K, int pb_cap) {
  return (size_t)n * 8 + (size_t)K * 8 + (size_t)K * 8 + (size_t)kClsE * K * 4 + (size_t)(K + 1) * 4 +
         (size_t)K * 4 + (size_t)pb_cap * 4 + (size_t)n * 4 + 16;
}

bool cls_fits(int n, int K) {
  return n > 0 && n < 65536 && K >= 1 && K <= kClsMaxK && cls_lds_bytes(n, K, 256) + kClsStaticLds <= (size_t)kLdsLimit;
}

// Chip-wide prologue of a class-loop run, grid (nodes, 1 + kClsL): level 0 -> the base key (allocate's
// predicate with every static affinity check, then the host overlay, as aff_key orders them; LR / BRA /
// NodeAffinity without the batch score), the static cache and A (Allocates before Idle stops fitting);
// level j >= 1 -> the key after j commits of the spec (traj_key64's closed form: the first A Allocate, the
// rest Pipeline). A node failing a static check at level 0 never commits, so levels >= 1 leave them out.
constexpr int kClsL = kClsLevels;
__global__ __launch_bounds__(256) void cls_sweep_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, int F, int K,
                                                        uint64_t* bk, uint64_t* stat, uint64_t* lvl, int32_t* amax,
                                                        uint64_t* cbest, const JobState* js, SpecGuard g) {
  if ((js != nullptr && js->stopped) || guard_fails(g)) return;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  const bool in = i < N.n;
  if (j != 0 && !in) return;
  const DevAff& A = P.A;
  const kb_spec sp = P.specs[spec];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  if (j == 0) {
    // level 0: the base key, and each class's best base key (class = the node's F-domain, K - 1 without one)
    // as one atomic max per class present in the wave (the place kernel reads cbest and zeroes it again)
    uint64_t key = 0;
    int c = -1;
    if (in) {
      const Row r = load_row(N, i);
      const uint64_t st = static_eval<false>(N, P, C, sp, spec, r.flags, i, nullptr);
      const kb_aff_spec as = A.specs[sp.aff_class];
      const int32_t ov = ov_row(P, spec);
      uint32_t rs = row_reasons(N, P, C, sp, sci, r, st, i);
      if (!rs && C.predicates) rs = aff_reasons<false>(A, as, i);
      if (!rs && ov >= 0 && P.ov_fail[(size_t)ov * N.n + i]) rs = kHostError;
      key = make_key(rs, rs ? 0 : row_score(C, sp, r, st), i);
      bk[i] = key;
      stat[i] = st;
      amax[i] = allocs_before_full(N, sp, sci, scr, r, i);
      const int32_t d = A.topo_dom[(size_t)F * N.n + i];
      c = d >= 0 ? d : K - 1;
    }
    uint64_t todo = __ballot(c >= 0);
    while (todo) {  // wave-uniform: one class per pass (members are contiguous in a class slot's usual layout)
      const int cl = __builtin_amdgcn_readlane(c, __builtin_ctzll(todo));
      const bool mine = c == cl;
      const uint64_t m = wave_max_u64(mine ? key : 0);
      if (mine && (threadIdx.x & 63) == __builtin_ctzll(todo) && m)
        atomicMax((unsigned long long*)&cbest[cl], (unsigned long long)m);
      todo &= ~__ballot(mine);
    }
  } else {
    const Row r = load_row(N, i);
    const uint64_t st = static_eval<false>(N, P, C, sp, spec, r.flags, i, nullptr);
    const uint64_t k = traj_key64(N, P, C, sp, sci, scr, r, st, i, j, allocs_before_full(N, sp, sci, scr, r, i));
    lvl[(size_t)(j - 1) * N.n + i] = (k & kFeasible) ? (k | (uint64_t)(kIdxMask - (uint32_t)i)) : k;
  }
}

// lane j's key of the hot node: the key after j + 1 more commits (wave-uniform index)
__device__ __forceinline__ uint64_t hk_at(uint64_t hk, int j) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)hk, j);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(hk >> 32), j);
  return ((uint64_t)hi << 32) | lo;
}

// A node's row as HBM holds it mid-run (the run's deltas flushed as atomics; the caller fenced after them).
__device__ __forceinline__ Row cls_row_now(const DevNodes& N, int w) {
  Row r;
  r.flags = N.flags[w];
  r.max_pods = N.max_pods[w];
  r.alloc_cpu = N.alloc_cpu[w];
  r.alloc_mem = N.alloc_mem[w];
  r.pod_count = __hip_atomic_load(&N.pod_count[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.idle_cpu = __hip_atomic_load(&N.idle_cpu[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.idle_mem = __hip_atomic_load(&N.idle_mem[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.rel_cpu = __hip_atomic_load(&N.rel_cpu[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.rel_mem = __hip_atomic_load(&N.rel_mem[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.nz_cpu = __hip_atomic_load(&N.nz_cpu[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  r.nz_mem = __hip_atomic_load(&N.nz_mem[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return r;
}

// The class loop's deep-node path (rare: a node past the sweep's levels).
__device__ __forceinline__ int cls_allocs_deep(const DevNodes& N, const kb_spec& sp, const int64_t* sci,
                                            const int64_t* scr, const Row& r, int n) {
  return allocs_before_full(N, sp, sci, scr, r, n);
}
__device__ __forceinline__ uint64_t cls_key_deep(const DevNodes& N, const DevSpecs& P, const DevCfg& C,
                                              const kb_spec& sp, const int64_t* sci, const int64_t* scr,
                                              const Row& r, uint64_t st, int n, int j, int A) {
  return traj_key64(N, P, C, sp, sci, scr, r, st, n, j, A);
}

template <int KQ>
__global__ __launch_bounds__(kClsThreads) void cls_place_kernel(
    DevNodes N, DevSpecs P, DevCfg C, int spec, int F, int K, int t_begin, int t_count, const uint64_t* bkg,
    const uint64_t* stat, const uint64_t* lvl, const int32_t* amax, const uint32_t* coff_g, const uint16_t* mem_g,
    uint64_t* cbest_g, JobState* js, int first,
    int ready0, int minav0,
    int gang0, int32_t* hout, JobState* hjs, int pb_cap, uint32_t seq, SpecGuard g) {
  // dynamic LDS: bk u64[n] base keys | cbest u64[K] class best base key | cnt i64[K] class counts |
  // cdom i32[kClsE][K] each histogram's domain per class | coff u32[K + 1] member offsets | cur u32[K]
  // populations, then scatter cursors | pbs u32[pb_cap] placements | mem u16[n] members by class
  extern __shared__ __attribute__((aligned(16))) uint64_t lds_cl[];
  const int n = N.n;
  uint64_t* bk = lds_cl;
  uint64_t* cbest = bk + n;
  int64_t* cnt = (int64_t*)(cbest + K);
  int32_t* cdom = (int32_t*)(cnt + K);
  uint32_t* coff = (uint32_t*)(cdom + kClsE * K);
  uint32_t* cur = coff + K + 1;
  uint32_t* pbs = cur + K;
  uint16_t* mem = (uint16_t*)(pbs + pb_cap);
  uint16_t* lv16 = mem + n;  // commits of this run per node
  __shared__ uint32_t s_phq[64 * kClsPM * kClsL];  // a class phase: member p's 32-bit keys of its next levels
  if ((!first && js->stopped) || guard_fails(g)) {
    if (threadIdx.x == 0) {
      if (first) js->n_placed = -1;  // a skipped speculative job (see sel_place_kernel)
      js->stopped = 1;
      js->n_commit = 0;
    }
    for (int c = threadIdx.x; c < K; c += kClsThreads) cbest_g[c] = 0;  // (its sweep skipped too: already 0)
    signal_skip(hjs, seq);
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
#ifdef KB_DIAG_AFF
  // phases: 0 prologue, 1 min / max + class keys + argmax, 2 commit (lane 0), 3 class rescan + counts,
  // 5 stop rules / flush, 6 no-fit histogram
  uint64_t dg[16] = {};  // [0..6] phases; [8..15] sel_run's fine stamps (KB_SEL_W)
  uint64_t dg_last = __builtin_amdgcn_s_memtime();
  const uint64_t rt0 = __builtin_amdgcn_s_memrealtime();
#endif
  const DevAff& A = P.A;
  const kb_spec sp = P.specs[spec];
  const kb_aff_spec as = A.specs[sp.aff_class];
  const int64_t* sci = P.sc_init + (size_t)spec * N.S;
  const int ne = (int)as.hist_cnt;  // <= kClsE (host)
  int32_t e_slot[kClsE], e_off[kClsE];
#pragma unroll
  for (int e = 0; e < kClsE; ++e) {
    e_slot[e] = 0, e_off[e] = -1;
    if (e < ne) {
      const kb_ipa_hist h = A.hists[as.hist_off + e];
      e_slot[e] = h.slot, e_off[e] = (int32_t)h.h_off;
    }
  }
  // the class member lists (static per topology slot: built at kb_upload_affinity), the base keys and each
  // class's best (both from the sweep) into LDS; every load of a thread in flight at once, 16 bytes each
  for (int c = tid; c <= K; c += kClsThreads) coff[c] = coff_g[c];
  for (int c = tid; c < K; c += kClsThreads) {
    cbest[c] = cbest_g[c];
    cbest_g[c] = 0;  // for the next run's sweep
  }
  {
    const uint4* mg = (const uint4*)mem_g;
    const uint4* kg = (const uint4*)bkg;
    const int nv = (n + 7) / 8;  // mem_g is padded to 8 entries
    const int nk = n / 2;        // key pairs (an odd n's last key below)
    constexpr int kV = 4;
    for (int v0 = 0; v0 < 4 * nv; v0 += kV * 4 * kClsThreads) {  // (4 nv >= nk)
      uint4 x[kV], y[4 * kV];
#pragma unroll
      for (int q = 0; q < kV; ++q) {
        const int v = v0 / 4 + q * kClsThreads + tid;
        x[q] = v < nv ? mg[v] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4 * kV; ++q) {
        const int v = v0 + q * kClsThreads + tid;
        y[q] = v < nk ? kg[v] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < kV; ++q) {
        const int v = v0 / 4 + q * kClsThreads + tid;
        if (v < nv) {
          const uint32_t w4[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
#pragma unroll
          for (int h = 0; h < 8; ++h)
            if (8 * v + h < n) mem[8 * v + h] = (uint16_t)(w4[h >> 1] >> (16 * (h & 1)));
        }
      }
#pragma unroll
      for (int q = 0; q < 4 * kV; ++q) {
        const int v = v0 + q * kClsThreads + tid;
        if (v < nk) ((uint4*)bk)[v] = y[q];
      }
    }
    if ((n & 1) && tid == 0) bk[n - 1] = bkg[n - 1];
  }
  for (int j = tid; j < n; j += kClsThreads) lv16[j] = 0;
  __syncthreads();
  // per class (kClsCT per thread in flight together, the rest after): each histogram's domain (class-uniform:
  // read at the first member) and the count
  constexpr int kClsCT = 2;
  int32_t cdd[kClsCT][kClsE];
  int64_t cc0[kClsCT];
#pragma unroll
  for (int u = 0; u < kClsCT; ++u) {
    const int c = tid + u * kClsThreads;
    const bool any = c < K && coff[c + 1] > coff[c];
    const int i0 = any ? mem[coff[c]] : 0;
#pragma unroll
    for (int e = 0; e < kClsE; ++e) cdd[u][e] = any && e < ne ? A.topo_dom[(size_t)e_slot[e] * n + i0] : -1;
  }
#pragma unroll
  for (int u = 0; u < kClsCT; ++u) {
    cc0[u] = 0;
#pragma unroll
    for (int e = 0; e < kClsE; ++e)
      if (cdd[u][e] >= 0) cc0[u] += ld_cnt<false>(&A.h[e_off[e] + cdd[u][e]]);
  }
#pragma unroll
  for (int u = 0; u < kClsCT; ++u) {
    const int c = tid + u * kClsThreads;
    if (c < K) {
#pragma unroll
      for (int e = 0; e < kClsE; ++e) cdom[e * K + c] = cdd[u][e];
      cnt[c] = cc0[u];
    }
  }
  // the classes past kClsCT per thread: the same, after
  for (int c = tid + kClsCT * kClsThreads; c < K; c += kClsThreads) {
    int64_t c0 = 0;
    const bool any = coff[c + 1] > coff[c];
    const int i0 = any ? mem[coff[c]] : 0;
    int32_t dd[kClsE];
#pragma unroll
    for (int e = 0; e < kClsE; ++e) dd[e] = any && e < ne ? A.topo_dom[(size_t)e_slot[e] * n + i0] : -1;
#pragma unroll
    for (int e = 0; e < kClsE; ++e) {
      cdom[e * K + c] = dd[e];
      if (dd[e] >= 0) c0 += ld_cnt<false>(&A.h[e_off[e] + dd[e]]);
    }
    cnt[c] = c0;
  }
  __syncthreads();
  if (wv != 0) return;  // the task loop is wave 0's: no block barrier below

  // ---- task loop (wave 0) ----
  // class c = q * 64 + lane: its count in registers
  int64_t cq[KQ];
  bool live[KQ];
#pragma unroll
  for (int q = 0; q < KQ; ++q) {
    const int c = q * 64 + lane;
    live[q] = c < K && coff[c + 1] > coff[c];
    cq[q] = c < K ? cnt[c] : 0;
  }
  // each histogram's domain of the lane's classes, in registers (a commit compares them with the winner's)
  int32_t cd[kClsE][KQ];
#pragma unroll
  for (int e = 0; e < kClsE; ++e)
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int c = q * 64 + lane;
      cd[e][q] = e < ne && c < K ? cdom[e * K + c] : -1;
    }
  // the spec's increments of its own histograms (entry, weight); the others go to the global tables only
  // (register arrays: every index a constant after unrolling, so nothing goes to scratch)
  int32_t u_e[kClsU], u_w[kClsU];
  int nu = 0;
  int wsign = 0;       // 1: every own increment > 0, -1: every one < 0, else 2
  bool only_f = true;  // every own increment is on the class slot itself: a commit updates its class only
#pragma unroll
  for (int v = 0; v < kClsU; ++v) u_e[v] = -1, u_w[v] = 0;
  for (uint32_t i = 0; i < as.incr_cnt && nu < kClsU; ++i) {
    const kb_ipa_incr u = A.incr[as.incr_off + i];
#pragma unroll
    for (int e = 0; e < kClsE; ++e)
      if (e < ne && (int32_t)u.h_off == e_off[e] && nu < kClsU) {
#pragma unroll
        for (int v = 0; v < kClsU; ++v)
          if (v == nu) u_e[v] = e, u_w[v] = u.weight;
        const int sg = u.weight > 0 ? 1 : (u.weight < 0 ? -1 : 2);
        wsign = nu == 0 ? sg : (wsign == sg ? wsign : 2);
        only_f = only_f && e_slot[e] == F;
        ++nu;
      }
  }
  // the spec's own increments summed per histogram (a commit adds them to the classes sharing the winner's
  // domain in that histogram; integer sums, so the order of the increments does not matter)
  int32_t e_w[kClsE];
  bool e_has[kClsE];
#pragma unroll
  for (int e = 0; e < kClsE; ++e) {
    e_w[e] = 0, e_has[e] = false;
#pragma unroll
    for (int v = 0; v < kClsU; ++v)
      if (v < nu && u_e[v] == e) e_w[e] += u_w[v], e_has[e] = true;
  }
  // Incremental min / max (interpod_affinity.go:221-238 over the classes): when every own increment has one
  // sign, a commit moves counts one way only, so the new max (weights > 0; the min stays 0 if it was) or
  // the new min (weights < 0) is the old one against the updated classes alone; otherwise a full pass.
  const int64_t* scr = P.sc_req + (size_t)spec * N.S;
  int ready = first ? ready0 : js->ready_num;
  int minav = first ? minav0 : js->min_available;
  int gang = first ? gang0 : js->gang_ready;
  int placed = first ? 0 : js->n_placed;
  int pb_n = 0, pb_base = t_begin;
  int stop = KB_STOP_DONE, fail_task = -1, panic = 0, stopped = 0;
  const bool ipa = C.nodeorder && ne > 0;
  const int64_t c_wpa = C.w_pa;
  // The hot node: the last winner, with its next keys one per lane (lane j: the key after j + 1 more
  // commits), read from the sweep's level keys (a gather, prefetched for the winner's class's new best right
  // after its rescan), or -- past kClsL levels -- computed from its row at once (traj_key64, 64 levels). Its
  // first hot_A further commits are Allocates. Its row deltas go to HBM as atomics when another node turns
  // hot and at the end (nothing waits for them; rows are read again only on the deep path, after a fence).
  // A winner keeps its score for several pods (LR / BRA move in steps): most commits read a register.
  int hot = -1, hot_c = 0, hot_A = 0, hot_n = 0, hot_lim = 0, p_node = -1, p_A = 0;
  uint64_t hk = 0, pk = 0;
  // c commits of the spec on node v, the first ac of them Allocates, as row deltas (NodeInfo.AddTask); any lane
  const auto flush_node = [&](int v, int c, int64_t ac) {
    const int64_t pc = c - ac;
    // read before the atomics: a load issued after them would wait for them too (in-order vmcnt)
    const uint32_t fl = sp.req_sc_mask ? N.flags[v] : 0u;
    if (ac) {
      atomicAdd((unsigned long long*)&N.idle_cpu[v], (unsigned long long)(-ac * sp.req_cpu));
      atomicAdd((unsigned long long*)&N.idle_mem[v], (unsigned long long)(-ac * sp.req_mem));
    }
    if (pc) {
      atomicAdd((unsigned long long*)&N.rel_cpu[v], (unsigned long long)(-pc * sp.req_cpu));
      atomicAdd((unsigned long long*)&N.rel_mem[v], (unsigned long long)(-pc * sp.req_mem));
    }
    atomicAdd(&N.pod_count[v], c);
    atomicAdd((unsigned long long*)&N.nz_cpu[v], (unsigned long long)((int64_t)c * sp.nz_cpu));
    atomicAdd((unsigned long long*)&N.nz_mem[v], (unsigned long long)((int64_t)c * sp.nz_mem));
    uint64_t m = sp.req_sc_mask;
    while (m) {  // Sub on a nil scalar map is a no-op (resource_info.go:152-157)
      const int q = __builtin_ctzll(m);
      m &= m - 1;
      if (ac && (fl & KB_NODE_IDLE_HAS_MAP))
        atomicAdd((unsigned long long*)&N.idle_sc[(size_t)q * n + v], (unsigned long long)(-ac * scr[q]));
      if (pc && (fl & KB_NODE_REL_HAS_MAP))
        atomicAdd((unsigned long long*)&N.rel_sc[(size_t)q * n + v], (unsigned long long)(-pc * scr[q]));
    }
    for (uint32_t i = 0; i < sp.port_cnt; ++i) {
      const kb_port q = P.ports[sp.port_off + i];
      atomicOr((unsigned long long*)&N.port_used[(size_t)q.slot * n + v], 1ull << q.ip);
    }
  };
  const auto flush_hot = [&]() {  // lane 0: the hot node's commits
    if (hot < 0 || hot_c == 0) return;
    if (lane == 0) {
      flush_node(hot, hot_c, hot_c < hot_A ? hot_c : hot_A);
      lv16[hot] = (uint16_t)(hot_n + hot_c);
    }
  };
  // Class phases (exact batching of the per-task argmax). When a commit can only raise its own class's count
  // (every own increment > 0 and on the class slot, the min at 0, InterPodAffinity weight >= 0), the winner's
  // class R only gains -- its count grows, and its score with it (ipa_score is monotone in the count; the max
  // follows R's count or stays) -- while every other class only loses (its count is fixed, the max can only
  // grow). So from a task whose winner is in R, as long as R's best base key plus R's score at the phase's start
  // beats S, the best other class's key at the start, the argmax is R's best node: the picks are R's members in
  // base-key order (each member's keys after 1..kClsL commits are the sweep's levels), with no landscape and
  // no class rescan per task. The phase ends at the first pick that is not provably R's (then the per-task
  // path decides, exactly), at a member past the sweep's levels, or at a stop rule.
  const bool phase_ok = (!ipa || (wsign == 1 && only_f && c_wpa >= 0)) && KQ <= 4;
  AFF_STAMP(0);
  int64_t mn = 0, mx = 0;
  bool mm_ok = false;  // mn / mx hold the current min / max
  for (int t = 0; t < t_count; ++t) {
    int64_t bp[10];
#pragma unroll
    for (int q = 0; q < 10; ++q) bp[q] = INT64_MAX;
    if (ipa && !mm_ok) {
      mn = 0, mx = 0;
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        if (live[q]) {
          mn = cq[q] < mn ? cq[q] : mn;
          mx = cq[q] > mx ? cq[q] : mx;
        }
      mn = wave_min_i64_dpp(mn);
      mx = wave_max_i64_dpp(mx);
      mm_ok = true;
    }
    if (ipa && KQ > 2) {
      // ipa_score is monotone in the count: its 10 breakpoints, exactly (as in aff_reg_kernel): a_s =
      // ceil(s * b / 10) is the first offset with 10 a / b >= s; the float64 formula falls short of s only
      // where 10 a / b == s exactly, and then a_s + 1 is it. Lane s - 1 computes a_s.
      const int64_t bb = mx - mn;
      int64_t as_ = INT64_MAX;
      if (bb > 0 && lane < 10) {
        const int64_t sb = (int64_t)(lane + 1) * bb;
        as_ = (sb + 9) / 10;
        if (sb % 10 == 0 && ipa_score(mn + as_, mn, mx) < lane + 1) ++as_;
      }
#pragma unroll
      for (int q = 0; q < 10; ++q) {
        const uint32_t lo32 = __builtin_amdgcn_readlane((uint32_t)as_, q);
        const uint32_t hi32 = __builtin_amdgcn_readlane((uint32_t)((uint64_t)as_ >> 32), q);
        bp[q] = (int64_t)(((uint64_t)hi32 << 32) | lo32);
      }
    }
    uint64_t kq[KQ];
    uint64_t best = 0;
#pragma unroll
    for (int q = 0; q < KQ; ++q) {
      const int c = q * 64 + lane;
      uint64_t k = c < K ? cbest[c] : 0;
      if ((k & kFeasible) && ipa) {
        int32_t sc;
        if (KQ > 2) {  // == ipa_score(cq[q], mn, mx) by the breakpoints
          const int64_t off = cq[q] - mn;
          sc = 0;
#pragma unroll
          for (int s = 0; s < 10; ++s) sc += off >= bp[s];
        } else {  // a division per class is cheaper than the breakpoints for a few classes per lane
          sc = ipa_score(cq[q], mn, mx);
        }
        k += (uint64_t)((int64_t)sc * c_wpa) << 24;
      }
      kq[q] = k;
      best = umax64(best, k);
    }
    best = wave_max_dpp(best);
    if (!(best & kFeasible)) {
      // PredicateNodes found nothing (allocate.go:150-153): FitErrors over every node's base reasons
      uint32_t h[KB_NUM_REASONS];
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] = 0;
      for (int i = lane; i < n; i += 64) {
        const uint64_t k = bk[i];
#pragma unroll
        for (int b = 0; b < KB_NUM_REASONS; ++b) h[b] += (uint32_t)(k >> b) & 1u;
      }
#pragma unroll
      for (int b = 0; b < KB_NUM_REASONS; ++b) {
        const uint32_t s = wave_sum_u32(h[b]);
        if (lane == b) {
          js->hist[b] = s;
          hjs->hist[b] = s;
        }
      }
      stop = KB_STOP_NO_FIT;
      fail_task = t_begin + t;
      stopped = 1;
      AFF_STAMP(6);
      break;
    }
    const int64_t score = (int64_t)((best >> 24) & ((1ull << 39) - 1)) - kScoreBias;
    if (score <= -1) {  // SelectBestNode: no bucket with score > -1 -> the reference panics
      fail_task = t_begin + t;
      panic = 1;
      stopped = 1;
      break;
    }
    const int w = (int)(kIdxMask - (uint32_t)(best & kIdxMask));
    int mine = -1;
#pragma unroll
    for (int q = 0; q < KQ; ++q)
      if (kq[q] == best) mine = q * 64 + lane;
    const uint64_t who = __ballot(mine >= 0);
    const int cw = __builtin_amdgcn_readlane(mine, (int)__builtin_ctzll(who));
    AFF_STAMP(1);
    if (phase_ok && (!ipa || mn == 0) && coff[cw + 1] - coff[cw] <= 64u * kClsPM) {
      const uint32_t m0 = coff[cw], m1 = coff[cw + 1];
      uint64_t s2 = 0;  // S: the best other class (keys are distinct: they carry the node)
#pragma unroll
      for (int q = 0; q < KQ; ++q) s2 = kq[q] != best ? umax64(s2, kq[q]) : s2;
      s2 = wave_max_dpp(s2);
      int64_t cR = 0, incR = 0;  // R's count and the spec's increment of it per commit
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        if (q == (cw >> 6)) {
          const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)cq[q], cw & 63);
          const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)cq[q] >> 32), cw & 63);
          cR = (int64_t)(((uint64_t)hi << 32) | lo);
        }
#pragma unroll
      for (int e = 0; e < kClsE; ++e) {
        if (!e_has[e]) continue;
        int32_t d = -1;
#pragma unroll
        for (int q = 0; q < KQ; ++q)
          if (q == (cw >> 6)) d = (int32_t)__builtin_amdgcn_readlane((uint32_t)cd[e][q], cw & 63);
        if (d >= 0) incR += e_w[e];
      }
      const int64_t lift = ipa ? (int64_t)ipa_score(cR, mn, mx) * c_wpa : 0;  // R's score term at the start
      // A member may be picked here when its biased base score is at least thr: its key plus R's score beats S
      // by the score alone (ties with S go to the per-task path), and its score plus R's is not the panic.
      // The phase's keys are 32-bit: (biased score - thr + 1) << 8 | (255 - position in R's node-ordered list),
      // 1 below thr (never picked), 0 infeasible -- exact order among the pickable keys.
      int64_t thr = (int64_t)kScoreBias - lift;
      if (s2 & kFeasible) {
        const int64_t t2 = (int64_t)((s2 >> 24) & ((1ull << 39) - 1)) - lift + 1;
        thr = t2 > thr ? t2 : thr;
      }
      bool enc_bad = false;
      const auto enc = [&](uint64_t k, uint32_t tie) -> uint32_t {
        if (!(k & kFeasible)) return 0u;
        const int64_t d = (int64_t)((k >> 24) & ((1ull << 39) - 1)) - thr + 1;
        if (d <= 0) return 1u;
        if (d >= (1ll << 23)) {
          enc_bad = true;
          return 1u;
        }
        return ((uint32_t)d << 8) | tie;
      };
      flush_hot();
      wave_sync_lds();
      hot = -1, hot_c = 0, p_node = -1;
      // R's members, kClsPM per lane (position p = j * 64 + lane): node, 32-bit key, commits so far in this run,
      // Allocates before full (the sweep's), and the queue of its next keys from the sweep's levels
      int nd[kClsPM], lev[kClsPM], am[kClsPM], cc[kClsPM], qn[kClsPM];
      uint32_t k32[kClsPM];
      uint64_t key0[kClsPM];
#pragma unroll
      for (int j = 0; j < kClsPM; ++j) {
        const uint32_t ix = m0 + (uint32_t)(j * 64 + lane);
        nd[j] = ix < m1 ? (int)mem[ix] : -1;
        cc[j] = 0;
      }
#pragma unroll
      for (int j = 0; j < kClsPM; ++j) {
        key0[j] = nd[j] >= 0 ? bk[nd[j]] : 0;
        lev[j] = nd[j] >= 0 ? (int)lv16[nd[j]] : kClsL;
      }
      uint64_t Lk[kClsPM][kClsL];
#pragma unroll
      for (int j = 0; j < kClsPM; ++j) {
        am[j] = nd[j] >= 0 ? amax[nd[j]] : 0;
#pragma unroll
        for (int i = 0; i < kClsL; ++i)
          Lk[j][i] = nd[j] >= 0 && lev[j] + i < kClsL ? lvl[(size_t)(lev[j] + i) * n + nd[j]] : 0;
      }
#pragma unroll
      for (int j = 0; j < kClsPM; ++j) {
        const int pj = j * 64 + lane;
        const uint32_t tie = 255u - (uint32_t)pj;
        k32[j] = enc(key0[j], tie);
        qn[j] = kClsL - lev[j];  // queue entries: entry i = the key after lev + i + 1 commits
#pragma unroll
        for (int i = 0; i < kClsL; ++i)
          if (i < qn[j]) s_phq[pj * kClsL + i] = enc(Lk[j][i], tie);
      }
      wave_sync_lds();
      // a member past the sweep's levels: its next 64 keys across the lanes (lane l: the key after rel0 + l + 1 of
      // this phase's commits on its row as HBM holds it -- the commits before the phase, flushed at its start), as
      // the per-task path's deep keys
      int dh = -1, dh_rel0 = 0;
      uint32_t dk32 = 0;
      bool fenced = false;
      int took = 0;
      bool done = false;
#ifdef KB_DIAG_AFF
      uint64_t why = 4;  // the phase's end: 1 below the bound, 2 a deep key out of range, 3 a stop / the run's end
      uint64_t n_rounds = 0, n_deep = 0;
#endif
      AFF_STAMP(2);
      // The merge first in bulk: the picks of a greedy merge of the members' key sequences come out in descending
      // order of each entry's prefix minimum along its member's sequence (the effective key; entries of different
      // members never tie: the low byte is the position), one wave maximum per pick over the members' effective
      // heads. It stops before taking a member's last known entry (the key after it would be a deep key) and at
      // the bound, a stop rule or the run's end; the rounds below go on from its state (same greedy order).
      if (!__ballot(enc_bad)) {
        uint32_t ef[kClsPM][kClsL + 1];  // member j's effective keys from its next pick on (0: none / unknown)
        uint32_t info[kClsPM];           // node | next pick an Allocate << 30 | next entry is the last known << 31
        int ptr[kClsPM];
#pragma unroll
        for (int j = 0; j < kClsPM; ++j) {
          const uint32_t tie = 255u - (uint32_t)(j * 64 + lane);
          ef[j][0] = k32[j];
#pragma unroll
          for (int i = 0; i < kClsL; ++i)
            ef[j][i + 1] = i < qn[j] ? umin32(ef[j][i], enc(Lk[j][i], tie)) : 0u;
          ptr[j] = 0;
          info[j] = (uint32_t)(nd[j] & 0x3fffffff) | (lev[j] < am[j] ? 1u << 30 : 0u) | (qn[j] <= 0 ? 1u << 31 : 0u);
        }
        const int t_left = __builtin_amdgcn_readfirstlane(t_count - t);
        for (;;) {
          took = __builtin_amdgcn_readfirstlane(took);
          placed = __builtin_amdgcn_readfirstlane(placed);
          pb_n = __builtin_amdgcn_readfirstlane(pb_n);
          ready = __builtin_amdgcn_readfirstlane(ready);
          uint32_t h = ef[0][0];
#pragma unroll
          for (int j = 1; j < kClsPM; ++j) h = umax32(h, ef[j][0]);
          const uint32_t m = wave_max32_dpp(h);
          if (m < 256u) break;  // (the rounds end the phase there too)
          int jw = kClsPM - 1;
          uint64_t hit = 0;
#pragma unroll
          for (int j = kClsPM - 1; j >= 0; --j) {
            const uint64_t b = __ballot(ef[j][0] == m);
            if (b) jw = j, hit = b;
          }
          const int wl = (int)__builtin_ctzll(hit);
          uint32_t isel = info[0];
#pragma unroll
          for (int j = 1; j < kClsPM; ++j) isel = j == jw ? info[j] : isel;
          const uint32_t wi = (uint32_t)__builtin_amdgcn_readlane((int)isel, wl);
          // its last known entry: the rounds take it (and its deep keys); a full placement buffer: the rounds
          // flush it (no flush code here, so the loop keeps its few scalars in registers)
          if ((wi >> 31) || pb_n == pb_cap) break;
          const int kind = (wi >> 30) & 1u ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE;
          pbs[pb_n] = (wi & 0x3fffffffu) | ((uint32_t)kind << 30);  // (every lane the same word)
          cR += incR;
          mx = cR > mx ? cR : mx;
          ++took;
          ++placed;
          ++pb_n;
          ready += kind == KB_PLACE_ALLOCATE ? 1 : 0;
          // the winner's lane advances: its effective keys shift by one, its pick count and info follow
          const bool me = lane == wl;
#pragma unroll
          for (int j = 0; j < kClsPM; ++j)
            if (j == jw) {
#pragma unroll
              for (int i = 0; i < kClsL; ++i) ef[j][i] = me ? ef[j][i + 1] : ef[j][i];
              ef[j][kClsL] = me ? 0u : ef[j][kClsL];
              ptr[j] += me ? 1 : 0;
              info[j] = (uint32_t)(nd[j] & 0x3fffffff) | (lev[j] + ptr[j] < am[j] ? 1u << 30 : 0u) |
                        (ptr[j] >= qn[j] ? 1u << 31 : 0u);
            }
          const bool rdy = !gang || ready >= minav;  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
          stop = rdy ? KB_STOP_READY : stop;
          stopped = rdy ? 1 : stopped;
          if (rdy || took == t_left) {
            done = true;
            break;
          }
        }
        // the members' state for the rounds: commits in this phase, in this run, and the actual next key
#pragma unroll
        for (int j = 0; j < kClsPM; ++j)
          if (ptr[j] > 0) {
            cc[j] += ptr[j];
            lev[j] += ptr[j];
            k32[j] = s_phq[(j * 64 + lane) * kClsL + ptr[j] - 1];
          }
        if (pb_n == pb_cap) {  // (the rounds write pbs[pb_n] before they test for a full buffer)
          wave_sync_lds();
          for (int k0 = 0; k0 < pb_n; k0 += 64) {
            const int k = k0 + lane;
            if (k < pb_n) {
              const uint32_t e = pbs[k];
              hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
              hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
            }
          }
          wave_sync_lds();
          pb_base += pb_n;
          pb_n = 0;
        }
#ifdef KB_DIAG_AFF
        if (done) why = 3;
#endif
      }
      // Each round: one wave reduction finds the winner and the runner-up; the winner then takes picks as long as
      // its next key stays above the runner-up's (a node keeps its score for several pods: LR / BRA move in steps),
      // each pick scalar work on its queue, read once into a register across the lanes.
      while (!done && !__ballot(enc_bad)) {
        uint32_t m = k32[0];
#pragma unroll
        for (int j = 1; j < kClsPM; ++j) m = k32[j] > m ? k32[j] : m;
        m = wave_max_u32(m);
        if (m < 256u) {  // not provably R's (or infeasible): the per-task path decides
#ifdef KB_DIAG_AFF
          why = 1;
#endif
          break;
        }
        int jw = -1;
        uint64_t hit = 0;
        uint32_t r2 = 0;
#pragma unroll
        for (int j = 0; j < kClsPM; ++j) {
          const uint64_t h = __ballot(k32[j] == m);
          if (jw < 0 && h) jw = j, hit = h;
          r2 = k32[j] != m && k32[j] > r2 ? k32[j] : r2;
        }
        const uint32_t m2 = wave_max_u32(r2);  // the runner-up (keys are distinct)
        const int wl = (int)__builtin_ctzll(hit);
        const int p = jw * 64 + wl;  // the winner's position in R
        int ml = 0, ma = 0, mq = 0, mc = 0, mn_ = 0;
#pragma unroll
        for (int j = 0; j < kClsPM; ++j)
          if (j == jw) ml = lev[j], ma = am[j], mq = qn[j], mc = cc[j], mn_ = nd[j];
        const int lw = __builtin_amdgcn_readlane(ml, wl);   // its commits in this run so far
        const int aw = __builtin_amdgcn_readlane(ma, wl);   // Allocates before Idle stops fitting (run start)
        const int qw = __builtin_amdgcn_readlane(mq, wl);   // its queue entries
        const int cw0 = __builtin_amdgcn_readlane(mc, wl);  // its commits in this phase so far
        const int wn = __builtin_amdgcn_readlane(mn_, wl);
        // lane i: queue entry cw0 + i (the key after cw0 + i + 1 phase commits)
        const uint32_t hq = cw0 + lane < qw && lane < kClsL ? s_phq[p * kClsL + cw0 + lane] : 0u;
        int c = 0;
        uint32_t nk = m;
#ifdef KB_DIAG_AFF
        ++n_rounds;
#endif
        AFF_STAMP(3);
        bool stop_now = false;
        for (;;) {  // the winner's stretch (its deep keys computed between the inner loop's passes)
          bool need_deep = false;
          for (;;) {
            // (wave-uniform loop state, stated as such, and one exit test: the loop branches on scalars)
            c = __builtin_amdgcn_readfirstlane(c);
            took = __builtin_amdgcn_readfirstlane(took);
            placed = __builtin_amdgcn_readfirstlane(placed);
            pb_n = __builtin_amdgcn_readfirstlane(pb_n);
            ready = __builtin_amdgcn_readfirstlane(ready);
            dh = __builtin_amdgcn_readfirstlane(dh);
            dh_rel0 = __builtin_amdgcn_readfirstlane(dh_rel0);
            const int t_left = __builtin_amdgcn_readfirstlane(t_count - t);
            // the pick: Session.Allocate while InitResreq fits Idle, then Pipeline (the run-start A: the closed form)
            const int kind = lw + c < aw ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE;
            pbs[pb_n] = (uint32_t)wn | ((uint32_t)kind << 30);  // (every lane the same word)
            cR += incR;
            mx = cR > mx ? cR : mx;  // (phase_ok: the min stays 0, the max follows R or stays)
            ++c;
            ++took;
            ++placed;
            ++pb_n;
            ready += kind == KB_PLACE_ALLOCATE ? 1 : 0;
            if (pb_n == pb_cap) {
              wave_sync_lds();
              for (int k0 = 0; k0 < pb_n; k0 += 64) {
                const int k = k0 + lane;
                if (k < pb_n) {
                  const uint32_t e = pbs[k];
                  hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
                  hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
                }
              }
              wave_sync_lds();
              pb_base += pb_n;
              pb_n = 0;
            }
            // its next key: after rel phase commits -- queue entry rel - 1 (lane c - 1 of hq), else the deep keys
            const int rel = cw0 + c;
            const int iq = rel - 1, id = rel - 1 - dh_rel0;
            const uint32_t nq = (uint32_t)__builtin_amdgcn_readlane((int)hq, (c - 1) & 63);
            const uint32_t nd = (uint32_t)__builtin_amdgcn_readlane((int)dk32, id & 63);
            const bool inq = iq < qw;
            need_deep = !inq && !(wn == dh && id < 64);
            nk = inq ? nq : nd;
            const bool rdy = !gang || ready >= minav;  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
            stop = rdy ? KB_STOP_READY : stop;
            stopped = rdy ? 1 : stopped;
            stop_now = rdy || took == t_left;
            // it still beats every other member: the next pick is its own
            if (need_deep || stop_now || nk <= m2 || nk < 256u) break;
          }
          AFF_STAMP(4);
          if (!need_deep) break;
          // past the sweep's levels: its next 64 keys from its row (lane l: the key after rel + l phase commits)
          AFF_STAMP(4);
#ifdef KB_DIAG_AFF
          ++n_deep;
#endif
          const int rel = cw0 + c;
          if (!fenced) {  // the row deltas flushed at the phase's start (atomics): visible to the loads below
            __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
            fenced = true;
          }
          // (an opaque copy of the node: its row addresses are formed here, not hoisted into every round's
          // preamble, where the compiler had spilled them)
          int wq = wn;
          asm volatile("" : "+s"(wq));
          const Row r = cls_row_now(N, wq);
          const int dA = cls_allocs_deep(N, sp, sci, scr, r, wq);
          const uint64_t k = cls_key_deep(N, P, C, sp, sci, scr, r, stat[wq], wq, rel + lane, dA);
          dk32 = enc((k & kFeasible) ? (k | (uint64_t)(kIdxMask - (uint32_t)wq)) : k, 255u - (uint32_t)p);
          dh = wn, dh_rel0 = rel - 1;
          AFF_STAMP(5);
          if (__ballot(enc_bad)) {  // (a deep key out of the 32-bit range: the per-task path from here)
#ifdef KB_DIAG_AFF
            why = 2;
#endif
            stop_now = true;
            nk = 1u;
          } else {
            nk = (uint32_t)__builtin_amdgcn_readlane((int)dk32, 0);
          }
          if (!gang || ready >= minav) {  // (the pick's stop rules, as in the inner loop)
            stop = KB_STOP_READY;
            stopped = 1;
            stop_now = true;
          }
          if (t + took == t_count) stop_now = true;
          if (!stop_now && nk > m2 && nk >= 256u) continue;
          break;
        }
        // the winner's state back into its lane's registers
        if (lane == wl) {
#pragma unroll
          for (int j = 0; j < kClsPM; ++j)
            if (j == jw) k32[j] = nk, lev[j] += c, cc[j] += c;
        }
        done = stop_now;
      }
      AFF_STAMP(4);
#ifdef KB_DIAG_AFF
      if (why == 4 && took > 0) why = 3;
#endif
      // the members' commits: row deltas, levels and 64-bit keys back (the sweep's level key, or past its levels
      // the row's, after the deltas), then R's best and count
      bool deep_any = false;
#pragma unroll
      for (int j = 0; j < kClsPM; ++j) {
        if (cc[j] > 0) {
          const int l0 = lev[j] - cc[j];
          const int ac = am[j] > l0 ? (am[j] - l0 < cc[j] ? am[j] - l0 : cc[j]) : 0;
          flush_node(nd[j], cc[j], ac);
          lv16[nd[j]] = (uint16_t)lev[j];
          deep_any = deep_any || lev[j] > kClsL;
        }
      }
      if (__ballot(deep_any)) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");  // the deltas just flushed
      uint64_t nb = 0;
#pragma unroll
      for (int j = 0; j < kClsPM; ++j) {
        uint64_t k = key0[j];
        if (cc[j] > 0) {
          if (lev[j] <= kClsL) {
            k = lvl[(size_t)(lev[j] - 1) * n + nd[j]];
          } else {
            const Row r = cls_row_now(N, nd[j]);
            const uint64_t kk = cls_key_deep(N, P, C, sp, sci, scr, r, stat[nd[j]], nd[j], 0,
                                             cls_allocs_deep(N, sp, sci, scr, r, nd[j]));
            k = (kk & kFeasible) ? (kk | (uint64_t)(kIdxMask - (uint32_t)nd[j])) : kk;
          }
          bk[nd[j]] = k;
        }
        nb = umax64(nb, k);
      }
      nb = wave_max_dpp(nb);
      if (lane == 0) cbest[cw] = nb;
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        if (q == (cw >> 6) && lane == (cw & 63)) cq[q] = cR;
      wave_sync_lds();
      AFF_STAMP(5);
#ifdef KB_DIAG_AFF
      // counts: picks + 1e6 per round (a reduction and its winner's stretch) + 1e12 per deep-key computation
      dg[6] += (uint64_t)took + 1000000ull * n_rounds + 1000000000000ull * n_deep;
#endif
      if (took > 0) {
        if (stopped) break;
        t += took - 1;
        continue;
      }
    }
    // commit: Session.Allocate / Pipeline on the winner's row (allocate.go:159-182). A new hot node (or the
    // hot one past its keys) first.
    if (w != hot || hot_c == hot_lim) {
      const bool same = w == hot;
      // lv16[w] before the flush: the flush writes the old hot node's entry (w's own only when same)
      const int l0 = same ? hot_n + hot_c : (int)lv16[w];
      if (l0 < kClsL) {  // the sweep's level keys (lane j: level l0 + j + 1)
        // the new node's loads go out before the old node's atomics, so waiting for them does not wait
        // for the atomics
        uint64_t nhk;
        int nA;
        if (w == p_node) {
          nhk = pk, nA = p_A;
        } else {
          nhk = l0 + lane < kClsL ? lvl[(size_t)(l0 + lane) * n + w] : 0;
          const int a0 = amax[w];
          nA = a0 > l0 ? a0 - l0 : 0;
        }
        flush_hot();
        wave_sync_lds();
        hot = w, hot_c = 0, hot_n = l0;
        hk = nhk, hot_A = nA;
        hot_lim = kClsL - l0;
      } else {  // deeper than the sweep went: from the row as it stands (this run's deltas applied)
        flush_hot();
        wave_sync_lds();
        hot = w, hot_c = 0, hot_n = l0;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        Row r;
        r.flags = N.flags[w];
        r.max_pods = N.max_pods[w];
        r.alloc_cpu = N.alloc_cpu[w];
        r.alloc_mem = N.alloc_mem[w];
        r.pod_count = __hip_atomic_load(&N.pod_count[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.idle_cpu = __hip_atomic_load(&N.idle_cpu[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.idle_mem = __hip_atomic_load(&N.idle_mem[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.rel_cpu = __hip_atomic_load(&N.rel_cpu[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.rel_mem = __hip_atomic_load(&N.rel_mem[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.nz_cpu = __hip_atomic_load(&N.nz_cpu[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r.nz_mem = __hip_atomic_load(&N.nz_mem[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        hot_A = cls_allocs_deep(N, sp, sci, scr, r, w);
        const uint64_t k = cls_key_deep(N, P, C, sp, sci, scr, r, stat[w], w, lane + 1, hot_A);
        hk = (k & kFeasible) ? (k | (uint64_t)(kIdxMask - (uint32_t)w)) : k;
        hot_lim = 64;
      }
      if (p_node == w) p_node = -1;
    }
    const int kind = hot_c < hot_A ? KB_PLACE_ALLOCATE : KB_PLACE_PIPELINE;
    const uint64_t nk = hk_at(hk, hot_c);
    ++hot_c;
    const int moved = nk != cbest[cw];  // w was its class's best; an unchanged key keeps it there
    if (lane == 0) {
      bk[w] = nk;
      pbs[pb_n] = (uint32_t)w | ((uint32_t)kind << 30);
    }
    wave_sync_lds();
    AFF_STAMP(1);
    if (moved) {  // the winner's key fell: its class's best again
      const uint32_t m0 = coff[cw], m1 = coff[cw + 1];
      uint64_t b = 0;
      for (uint32_t k = m0 + lane; k < m1; k += 64) b = umax64(b, bk[mem[k]]);
      b = wave_max_dpp(b);
      if (lane == 0) cbest[cw] = b;
      const int bn = (int)(kIdxMask - (uint32_t)(b & kIdxMask));
      if ((b & kFeasible) && bn != hot && bn != p_node) {  // prefetch its level keys (not waited for here)
        const int l0 = lv16[bn];
        if (l0 < kClsL) {
          p_node = bn;
          pk = l0 + lane < kClsL ? lvl[(size_t)(l0 + lane) * n + bn] : 0;
          const int a0 = amax[bn];
          p_A = a0 > l0 ? a0 - l0 : 0;
        }
      }
    }
    // the classes in the committed node's domains: this commit's increments of the spec's own histograms
    bool upd[KQ];
#pragma unroll
    for (int q = 0; q < KQ; ++q) upd[q] = false;
#pragma unroll
    for (int e = 0; e < kClsE; ++e) {
      if (!e_has[e]) continue;
      int32_t d = -1;  // the winner's domain: lane cw % 64 of register q = cw / 64
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        if (q == (cw >> 6)) d = (int32_t)__builtin_amdgcn_readlane((uint32_t)cd[e][q], cw & 63);
      if (d < 0) continue;
#pragma unroll
      for (int q = 0; q < KQ; ++q)
        if (cd[e][q] == d) {  // -1 (no class / no domain) never equals d >= 0
          cq[q] += e_w[e];
          upd[q] = true;
        }
    }
    if (ipa) {
      if (wsign == 1 && mn == 0) {  // counts only grew: the min stays 0, the max is the old one or an updated one
        int64_t um = INT64_MIN;
        if (only_f) {
#pragma unroll
          for (int q = 0; q < KQ; ++q)
            if (q == (cw >> 6)) {
              const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)cq[q], cw & 63);
              const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)cq[q] >> 32), cw & 63);
              um = (int64_t)(((uint64_t)hi << 32) | lo);
            }
        } else {
#pragma unroll
          for (int q = 0; q < KQ; ++q)
            if (upd[q]) um = cq[q] > um ? cq[q] : um;
          um = wave_max_i64_dpp(um);
        }
        mx = um > mx ? um : mx;
      } else if (wsign == -1 && mx == 0) {  // counts only fell: the max stays 0
        int64_t um = INT64_MAX;
#pragma unroll
        for (int q = 0; q < KQ; ++q)
          if (upd[q]) um = cq[q] < um ? cq[q] : um;
        um = wave_min_i64_dpp(um);
        mn = um < mn ? um : mn;
      } else {
        mm_ok = false;
      }
    }
    wave_sync_lds();
    AFF_STAMP(1);
    ++placed;
    ++pb_n;
    if (kind == KB_PLACE_ALLOCATE) ++ready;
    if (!gang || ready >= minav) {  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
      stop = KB_STOP_READY;
      stopped = 1;
      break;
    }
    if (pb_n == pb_cap) {
      for (int k = lane; k < pb_n; k += 64) {
        const uint32_t e = pbs[k];
        hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
        hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
      }
      wave_sync_lds();
      pb_base += pb_n;
      pb_n = 0;
    }
    AFF_STAMP(1);
  }
  flush_hot();
  for (int k = lane; k < pb_n; k += 64) {
    const uint32_t e = pbs[k];
    hout[2 * (pb_base + k)] = (int32_t)(e & 0x3fffffffu);
    hout[2 * (pb_base + k) + 1] = (int32_t)(e >> 30);
  }
#ifdef KB_DIAG_AFF
  if (lane == 0) publish_diag(hjs, dg, __builtin_amdgcn_s_memrealtime() - rt0);
#endif
  __threadfence_system();
  __builtin_amdgcn_wave_barrier();
  // the run's commits into the global tables, now that no key of this run reads them: from pbs when the run
  // never wrapped it, else back from the host buffer (the fence above made every lane's stores visible)
  const int run_n = pb_base + pb_n - t_begin;
  if (run_n <= pb_cap)
    for (int k = lane; k < run_n; k += 64) {
      const uint32_t e = pbs[k];
      apply_commit_tables(P.A, sp, (int)(e & 0x3fffffffu), (int)(e >> 30) == KB_PLACE_ALLOCATE ? 1 : 0, 1);
    }
  else
    for (int p = t_begin + lane; p < pb_base + pb_n; p += 64)
      apply_commit_tables(P.A, sp, hout[2 * p], hout[2 * p + 1] == KB_PLACE_ALLOCATE ? 1 : 0, 1);
  if (lane == 0) publish_state(js, hjs, stopped, stop, fail_task, placed, ready, minav, gang, panic, seq);
}

void launch_cls_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int F, int K, int t_begin,
                      int t_count, uint64_t* bk, uint64_t* stat, uint64_t* lvl, int32_t* amax, const uint32_t* coff,
                      const uint16_t* mem, uint64_t* cbest, JobState* js, int first, int ready0, int minav0,
                      int gang0, int32_t* hout, JobState* hjs, uint32_t seq, SpecGuard g, void* stream) {
  hipLaunchKernelGGL(cls_sweep_kernel, dim3((N.n + 255) / 256, 1 + kClsL), dim3(256), 0, (hipStream_t)stream, N, P,
                     C, spec, F, K, bk, stat, lvl, amax, cbest, first ? (const JobState*)nullptr : js, g);
  int pb_cap = aff_pb_cap(t_count);
  const size_t fixed = cls_lds_bytes(N.n, K, 0);
  const size_t cap_max = ((size_t)kLdsLimit - kClsStaticLds - fixed) / 4;
  if ((size_t)pb_cap > cap_max) pb_cap = (int)cap_max;
  const size_t bytes = cls_lds_bytes(N.n, K, pb_cap);
#define KB_CLS_Q(Q)                                                                                              \
  hipLaunchKernelGGL(cls_place_kernel<Q>, dim3(1), dim3(kClsThreads), bytes, (hipStream_t)stream, N, P, C, spec, F, \
                     K, t_begin, t_count, bk, stat, lvl, amax, coff, mem, cbest, js, first, ready0, minav0, gang0, hout, \
                     hjs, pb_cap, seq, g)
  const int q = (K + 63) / 64;
  if (q <= 1) KB_CLS_Q(1);
  else if (q <= 2) KB_CLS_Q(2);
  else if (q <= 4) KB_CLS_Q(4);
  else if (q <= 8) KB_CLS_Q(8);
  else KB_CLS_Q(16);
#undef KB_CLS_Q
}

// LDS plan of one place-loop launch: chunk maxima + placement buffer (+ all keys when they fit).
static void place_loop_lds_plan(int n, int t_count, int* bytes, int* pb_cap, bool* keys_in_lds) {
  const int M = (n + 63) >> 6;
  const int Mp = (M + 1) & ~1;
  const int limit = kLdsLimit / 8;  // in u64 words
  int pb = t_count < 4096 ? t_count : 4096;
  pb = (pb + 1) & ~1;
  if (Mp + pb + n <= limit) {
    *keys_in_lds = true;
    *pb_cap = pb;
    *bytes = (Mp + pb + n) * 8;
    return;
  }
  *keys_in_lds = false;
  if (Mp + pb > limit) pb = (limit - Mp) & ~1;
  *pb_cap = pb;
  *bytes = (Mp + pb) * 8;
}
int place_loop_lds_bytes(int n) {
  int bytes, pb;
  bool in_lds;
  place_loop_lds_plan(n, 1, &bytes, &pb, &in_lds);
  return in_lds ? bytes : -bytes;
}

void launch_sweep_keys(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, uint64_t* keys,
                       uint64_t* cmax, uint64_t* stat, const JobState* js, bool aff, void* stream) {
  const int blocks = (N.n + 255) / 256;
  if (aff)
    hipLaunchKernelGGL(sweep_keys_kernel<true>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, N, P, C, spec, keys,
                       cmax, stat, js);
  else
    hipLaunchKernelGGL(sweep_keys_kernel<false>, dim3(blocks), dim3(256), 0, (hipStream_t)stream, N, P, C, spec, keys,
                       cmax, stat, js);
}

void launch_place_loop(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                       uint64_t* keys, const uint64_t* cmax, const uint64_t* stat, JobState* js, int first,
                       int ready0, int minav0, int gang0, int32_t* hout, JobState* hjs, uint32_t seq,
                       void* stream) {
  int lds, pb_cap;
  bool keys_in_lds;
  place_loop_lds_plan(N.n, t_count, &lds, &pb_cap, &keys_in_lds);
  if (keys_in_lds)
    hipLaunchKernelGGL(place_loop_kernel<true>, dim3(1), dim3(512), lds, (hipStream_t)stream, N, P, C, spec, t_begin,
                       t_count, keys, cmax, stat, js, first, ready0, minav0, gang0, hout, hjs, pb_cap, seq);
  else
    hipLaunchKernelGGL(place_loop_kernel<false>, dim3(1), dim3(512), lds, (hipStream_t)stream, N, P, C, spec,
                       t_begin, t_count, keys, cmax, stat, js, first, ready0, minav0, gang0, hout, hjs, pb_cap, seq);
}

int configure_kernels() {
  // dynamic LDS opt-in for the single-workgroup place kernels; kLdsLimit leaves room for their static block
  const void* fns[] = {(const void*)place_loop_kernel<true>, (const void*)place_loop_kernel<false>,
                       (const void*)traj_place_kernel};
  for (const void* f : fns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsLimit);
    if (e != hipSuccess) return (int)e;
  }
  for (const void* f : kAffRegFns) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsLimit - 4096);
    if (e != hipSuccess) return (int)e;
  }
  {
    for (const void* f : {(const void*)cls_place_kernel<1>, (const void*)cls_place_kernel<2>,
                          (const void*)cls_place_kernel<4>, (const void*)cls_place_kernel<8>,
                          (const void*)cls_place_kernel<16>}) {
      hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kLdsLimit - kClsStaticLds);
      if (e != hipSuccess) return (int)e;
    }
  }
  for (const void* f :
       {(const void*)sel_place_kernel<0>, (const void*)sel_place_kernel<1>, (const void*)sel_place_kernel<2>,
        (const void*)sel_place_kernel<3>, (const void*)sel_place_kernel<4>, (const void*)sel_place_kernel<5>,
        (const void*)sel_place_kernel<6>, (const void*)sel_place_kernel<8>, (const void*)sel_place_kernel<10>,
        (const void*)engine_kernel, (const void*)shard_propose_kernel}) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kSelDynLimit);
    if (e != hipSuccess) return (int)e;
  }
  // the fed engine's static block also holds its command and the split engine's merge lists: a smaller budget
#define KB_FED_F(Q) \
  (const void*)fed_engine_kernel<Q, false>, (const void*)fed_engine_kernel<Q, true>, (const void*)fed_engine_kernel<Q, true, true>
  for (const void* f : {KB_FED_F(0), (const void*)fed_engine_kernel<1, false>, KB_FED_F(2), KB_FED_F(3), KB_FED_F(4), KB_FED_F(5), KB_FED_F(6),
                        KB_FED_F(8), KB_FED_F(10), (const void*)fed_engine_kernel<kFedSelQ, true, false, kFedMaxSel>,
                        (const void*)fed_engine_kernel<kFedSelQ, true, true, kFedMaxSel>}) {
    hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kFedDynLimit);
    if (e != hipSuccess) return (int)e;
  }
#undef KB_FED_F
  return 0;
}

int traj_lds_bytes(int n, int t_count, int* pb_cap) {
  const int M = (n + 63) >> 6;
  if (M > 256) return -1;  // chunk maxima live in 4 registers per lane
  const int W = (n + 63) >> 6;
  const int fixed = 8 * W + 4 * ((n + 1) & ~1) + 8 * n;  // tb | cur | nc
  const int limit = kLdsLimit;
  int pb = t_count;
  if (fixed + 4 * pb > limit) pb = (limit - fixed) / 4;
  if (pb < 64) return -1;
  *pb_cap = pb;
  return fixed + 4 * pb;
}

void launch_traj_sweep(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int J, int idx_bits,
                       uint32_t* traj, uint32_t* cmax32, uint32_t* amax, uint64_t* stat, const JobState* js,
                       bool aff, void* stream) {
  dim3 grid((N.n + 255) / 256, J + 1);
  if (aff)
    hipLaunchKernelGGL(traj_sweep_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec, idx_bits,
                       traj, cmax32, amax, stat, js);
  else
    hipLaunchKernelGGL(traj_sweep_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec, idx_bits,
                       traj, cmax32, amax, stat, js);
}

void launch_aff_commit(const DevSpecs& P, int spec, int t_begin, int run, const JobState* js, const int32_t* hout,
                       int base, void* stream) {
  hipLaunchKernelGGL(aff_commit_kernel, dim3((run + 255) / 256), dim3(256), 0, (hipStream_t)stream, P, spec, t_begin,
                     run, js, hout, base);
}

void launch_traj_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                       int J, int idx_bits, const uint32_t* traj, const uint32_t* cmax32, const uint32_t* amax,
                       const uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0,
                       int32_t* hout, JobState* hjs, uint32_t seq, void* stream) {
  int pb_cap = 0;
  const int lds = traj_lds_bytes(N.n, t_count, &pb_cap);
  hipLaunchKernelGGL(traj_place_kernel, dim3(1), dim3(kPlaceThreads), lds, (hipStream_t)stream, N, P, C, spec,
                     t_begin, t_count,
                     J, idx_bits, traj, cmax32, amax, stat, js, first, ready0, minav0, gang0, hout, hjs, pb_cap, seq);
}

// eval_plain_kernel's resident blocks per CU (its occupancy: the instance's registers decide it), per instance
int eval_plain_blocks_per_cu(bool i32) {
  int nb = 0;
  const hipError_t e = i32 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, eval_plain_kernel<int32_t, true>, 256, 0)
                           : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, eval_plain_kernel<int64_t, true>, 256, 0);
  return e == hipSuccess && nb > 0 ? nb : 2;
}

// eval_plain_kernel's specs per block: the grid sized to one resident round (cus CUs x bpc resident blocks of 4
// waves: the kernel's occupancy), so no SIMD runs a second, partial round and every SIMD holds as many waves as fit
// to hide the f64 chains' latency. spb_opt > 0 overrides (kb_opts.eval_spb: measurement).
static int eval_plain_spb(int n, int t, int cus, int bpc, int spb_opt) {
  int spb;
  if (spb_opt > 0) {
    spb = spb_opt;
  } else {
    const int xblocks = (n + 255) / 256;
    const int yblocks = ((cus > 0 ? cus : 256) * (bpc > 0 ? bpc : 2)) / xblocks;  // blocks in one round, per column
    spb = yblocks > 0 ? (t + yblocks - 1) / yblocks : kEvalPlainSpecs;
    if (spb < 8) spb = 8;
  }
  return spb < 1 ? 1 : (spb > kEvalPlainSpecs ? kEvalPlainSpecs : spb);
}
template <class SCORE>
static void launch_eval_t(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const int32_t* spec_ids, int t,
                          uint32_t* reasons, SCORE* scores, const int64_t* mm, bool plain, int cus, int spb_opt,
                          void* stream) {
  const bool buf = (uint64_t)t * (uint64_t)N.n * sizeof(SCORE) < (1ull << 31);
#if defined(KB_EVAL_VEC4)  // (A/B build: measured slower than one node per lane)
  if (plain && buf && N.n % 4 == 0) {  // four nodes per lane, 16-byte stores (eval_plain4_kernel)
    static int bpc4 = 0;  // (its own occupancy, once per instance)
    if (bpc4 == 0) {
      int nb = 0;
      bpc4 = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, eval_plain4_kernel<SCORE>, 256, 0) == hipSuccess && nb > 0
                 ? nb : 1;
    }
    const int spb = eval_plain_spb((N.n + 3) / 4, t, cus & 0xffff, bpc4, spb_opt);
    dim3 grid((N.n / 4 + 255) / 256, (t + spb - 1) / spb);
    hipLaunchKernelGGL((eval_plain4_kernel<SCORE>), grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec_ids, t,
                       spb, reasons, scores);
    return;
  }
#endif
  if (plain) {
    const int spb = eval_plain_spb(N.n, t, cus & 0xffff, cus >> 16, spb_opt);
#ifdef KB_EVAL_NPT2
    dim3 grid((N.n + 511) / 512, (t + spb - 1) / spb);
#elif defined(KB_EVAL_RUN4)
    dim3 grid((N.n + 1023) / 1024, (t + spb - 1) / spb);
#else
    dim3 grid((N.n + 255) / 256, (t + spb - 1) / spb);
#endif
    // buffer stores when every output offset fits 32 bits (the record count is a 32-bit byte count)
    if ((uint64_t)t * (uint64_t)N.n * sizeof(SCORE) < (1ull << 31))
      hipLaunchKernelGGL((eval_plain_kernel<SCORE, true>), grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec_ids, t,
                         spb, reasons, scores);
    else
      hipLaunchKernelGGL((eval_plain_kernel<SCORE, false>), grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec_ids,
                         t, spb, reasons, scores);
    return;
  }
  dim3 grid((N.n + 255) / 256, (t + kEvalSpecs - 1) / kEvalSpecs);
  if (mm)
    hipLaunchKernelGGL((eval_kernel<true, SCORE>), grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec_ids, t,
                       reasons, scores, mm);
  else
    hipLaunchKernelGGL((eval_kernel<false, SCORE>), grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec_ids, t,
                       reasons, scores, mm);
}
void launch_eval(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const int32_t* spec_ids, int t,
                 uint32_t* reasons, int64_t* scores, const int64_t* mm, bool plain, int cus, int spb, void* stream) {
  launch_eval_t(N, P, C, spec_ids, t, reasons, scores, mm, plain, cus, spb, stream);
}
void launch_eval32(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const int32_t* spec_ids, int t,
                   uint32_t* reasons, int32_t* scores, const int64_t* mm, bool plain, int cus, int spb,
                   void* stream) {
  launch_eval_t(N, P, C, spec_ids, t, reasons, scores, mm, plain, cus, spb, stream);
}

// kb_apply: one thread per row delta of a commit made outside the device -- NodeInfo.AddTask / RemoveTask
// (api/node_info.go:165-221) and the plugins' schedulercache AddPod / RemovePod (cache/node_info.go:498-630,
// host_ports.go), plus the inter-pod affinity table updates of the pod's spec. Sums are atomics (order-free);
// flags: every set in pass 0, every clear in pass 1.
__global__ __launch_bounds__(256) void apply_kernel(DevNodes N, DevSpecs P, const kb_row_delta* d, int k,
                                                    const int64_t* sc, const kb_port* ports, int pass) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  const kb_row_delta e = d[i];
  const int w = e.node - N.base;
  if (pass == 0 && e.spec >= 0) {  // the replicated affinity tables: every rank (A.topo_dom covers every node)
    const int sign = e.pods < 0 ? -1 : 1;
    apply_commit_tables(P.A, P.specs[e.spec], w, e.kind == KB_PLACE_ALLOCATE ? sign : 0, sign);
  }
  if (w < 0 || w >= N.n) return;  // another rank's row
  if (pass == 1) {
    if (e.flags_clear) atomicAnd(&N.flags[w], ~e.flags_clear);
    return;
  }
  using u64 = unsigned long long;
  atomicAdd((u64*)&N.idle_cpu[w], (u64)e.idle_cpu);
  atomicAdd((u64*)&N.idle_mem[w], (u64)e.idle_mem);
  atomicAdd((u64*)&N.rel_cpu[w], (u64)e.rel_cpu);
  atomicAdd((u64*)&N.rel_mem[w], (u64)e.rel_mem);
  atomicAdd((u64*)&N.nz_cpu[w], (u64)e.nz_cpu);
  atomicAdd((u64*)&N.nz_mem[w], (u64)e.nz_mem);
  atomicAdd(&N.pod_count[w], e.pods);
  if (e.flags_set) atomicOr(&N.flags[w], e.flags_set);
  if (e.sc_off != 0xffffffffu)
    for (int q = 0; q < N.S; ++q) {
      atomicAdd((u64*)&N.idle_sc[(size_t)q * N.n + w], (u64)sc[e.sc_off + q]);
      atomicAdd((u64*)&N.rel_sc[(size_t)q * N.n + w], (u64)sc[e.sc_off + N.S + q]);
    }
  for (uint32_t j = 0; j < e.port_cnt; ++j) {
    const kb_port p = ports[e.port_off + j];
    u64* used = (u64*)&N.port_used[(size_t)p.slot * N.n + w];
    if (e.pods >= 0) atomicOr(used, 1ull << p.ip);
    else atomicAnd(used, ~(1ull << p.ip));
  }
}

void launch_apply(const DevNodes& N, const DevSpecs& P, const kb_row_delta* d, int k, const int64_t* sc,
                  const kb_port* ports, void* stream) {
  const int blocks = (k + 255) / 256;
  for (int pass = 0; pass < 2; ++pass)
    hipLaunchKernelGGL(apply_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, N, P, d, k, sc, ports, pass);
}

// kb_apply_affinity: one thread per table / histogram entry of a pod outside the session's pending specs.
__global__ __launch_bounds__(256) void apply_aff_kernel(DevAff A, const kb_aff_delta* d, int k, int base) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k) return;
  const kb_aff_delta e = d[i];
  const int w = e.node - base;  // canonical id -> A.topo_dom's view (offset by the rank's first row when sharded)
  if (e.table >= 0) {
    const kb_aff_table tb = A.tables[e.table];
    const int32_t dom = A.topo_dom[(size_t)tb.slot * A.n + w];
    if (dom >= 0) atomicAdd(&A.counters[tb.cnt_off + dom], e.weight);
    atomicAdd(&A.totals[e.table], e.weight);
  } else {
    const int32_t dom = A.topo_dom[(size_t)e.slot * A.n + w];
    if (dom >= 0) atomicAdd(&A.h[e.h_off + dom], e.weight);
  }
}

void launch_apply_aff(const DevAff& A, const kb_aff_delta* d, int k, int base, void* stream) {
  hipLaunchKernelGGL(apply_aff_kernel, dim3((k + 255) / 256), dim3(256), 0, (hipStream_t)stream, A, d, k, base);
}

// ---- preempt's sweep (actions/preempt/preempt.go:189-195): PredicateNodes with Session.PredicateFn (no
// resource check), PrioritizeNodes, SortNodes (util/scheduler_helper.go:132-144): every feasible node by score,
// descending, lowest index first among equal scores. The 64-bit keys (score << 24 | ~index) sort in exactly
// that order; infeasible keys (reason masks) sink to the end. Bitonic sort over a power-of-two buffer.
template <bool AFF>
__global__ __launch_bounds__(256) void sort_keys_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, const int64_t* mm,
                                                        uint64_t* keys, int n_pad) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= n_pad) return;
  uint64_t k = 0;  // padding: below every key
  if (n < N.n) {
    const kb_spec sp = P.specs[spec];
    const Row r = load_row(N, n);
    const uint64_t st = static_eval<AFF>(N, P, C, sp, spec, r.flags, n, mm);
    const uint32_t rs = row_reasons<false>(N, P, C, sp, P.sc_init + (size_t)spec * N.S, r, st, n);
    k = make_key(rs, rs ? 0 : row_score(C, sp, r, st), n);
  }
  keys[n] = k;
}

// one compare-exchange stage (stride j of merge size k) across the whole buffer; descending overall
__global__ __launch_bounds__(256) void bitonic_global_kernel(uint64_t* a, int j, int k) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int p = i ^ j;
  if (p <= i) return;
  const uint64_t x = a[i], y = a[p];
  const bool desc = (i & k) == 0;
  if (desc ? x < y : x > y) {
    a[i] = y;
    a[p] = x;
  }
}

// every stage of merge size k with stride <= j0 (< 2048) inside one 2048-key tile in LDS
constexpr int kBitonicTile = 2048;
__global__ __launch_bounds__(1024) void bitonic_tile_kernel(uint64_t* a, int j0, int k) {
  __shared__ uint64_t t[kBitonicTile];
  const int base = blockIdx.x * kBitonicTile, tid = threadIdx.x;
  t[tid] = a[base + tid];
  t[tid + 1024] = a[base + tid + 1024];
  __syncthreads();
  for (int j = j0; j > 0; j >>= 1) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int e = tid + h * 1024, p = e ^ j;
      if (p > e) {
        const uint64_t x = t[e], y = t[p];
        const bool desc = ((base + e) & k) == 0;
        if (desc ? x < y : x > y) {
          t[e] = y;
          t[p] = x;
        }
      }
    }
    __syncthreads();
  }
  a[base + tid] = t[tid];
  a[base + tid + 1024] = t[tid + 1024];
}

void launch_sort_nodes(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, const int64_t* mm,
                       uint64_t* keys, int n_pad, void* stream, bool sort) {
  hipStream_t s = (hipStream_t)stream;
  if (mm)
    hipLaunchKernelGGL(sort_keys_kernel<true>, dim3(n_pad / 256), dim3(256), 0, s, N, P, C, spec, mm, keys, n_pad);
  else
    hipLaunchKernelGGL(sort_keys_kernel<false>, dim3(n_pad / 256), dim3(256), 0, s, N, P, C, spec, mm, keys, n_pad);
  for (int k = 2; sort && k <= n_pad; k <<= 1) {
    int j = k >> 1;
    for (; j >= kBitonicTile; j >>= 1)
      hipLaunchKernelGGL(bitonic_global_kernel, dim3(n_pad / 256), dim3(256), 0, s, keys, j, k);
    hipLaunchKernelGGL(bitonic_tile_kernel, dim3(n_pad / kBitonicTile), dim3(1024), 0, s, keys, j, k);
  }
}

}  // namespace kbgpu
