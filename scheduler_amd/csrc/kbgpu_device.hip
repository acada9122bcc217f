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
//                       node and the max key of every 64-node chunk (one wave).
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

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
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

// The predicate chain; returns the reason mask of the first failing stage (0 = fits).
__device__ uint32_t node_reasons(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const kb_spec& sp, int s,
                                 int n) {
  const uint32_t f = N.flags[n];
  const int64_t* sci = P.sc_init + (size_t)s * N.S;
  // allocate.go:88: InitResreq <= Idle || InitResreq <= Releasing
  if (!fits_idle(N, sp, sci, f, n) && !fits_rel(N, sp, sci, f, n)) return 1u << KB_R_RESOURCE_FIT;
  if (!C.predicates) return 0;
  // pod number (predicates.go:162-166)
  if (N.max_pods[n] <= N.pod_count[n]) return 1u << KB_R_POD_NUMBER;
  // CheckNodeConditionPredicate (vendor/.../predicates.go:1568-1596): one reason per bad condition
  const uint32_t cond = f & ((1u << KB_R_NOT_READY) | (1u << KB_R_OUT_OF_DISK) | (1u << KB_R_NETWORK_UNAVAILABLE) |
                             (1u << KB_R_UNSCHEDULABLE));
  if (cond) return cond;
  // PodMatchNodeSelector: nodeSelector AND required node affinity (vendor/.../predicates.go:807-863)
  if ((sp.flags & KB_SPEC_HAS_SELECTOR) && !term_match(N, P, P.terms[sp.sel_term], n))
    return 1u << KB_R_NODE_SELECTOR;
  if (sp.flags & KB_SPEC_HAS_REQUIRED) {
    bool any = false;
    for (uint32_t i = 0; i < sp.req_term_cnt && !any; ++i) any = term_match(N, P, P.terms[sp.req_term_off + i], n);
    if (!any) return 1u << KB_R_NODE_SELECTOR;
  }
  // PodFitsHostPorts (vendor/.../predicates.go:1031-1052; cache/host_ports.go:96-125)
  for (uint32_t i = 0; i < sp.port_cnt; ++i) {
    const kb_port p = P.ports[sp.port_off + i];
    const uint64_t used = N.port_used[(size_t)p.slot * N.n + n];
    const uint64_t hit = p.ip == 0 ? used : (used & (1ull | (1ull << p.ip)));
    if (hit) return 1u << KB_R_HOST_PORTS;
  }
  // PodToleratesNodeTaints (vendor/.../predicates.go:1489-1518)
  if (!P.tolerates[(size_t)sp.tol_set * P.n_taint_sets + N.taint_set[n]]) return 1u << KB_R_TAINTS;
  // optional pressure predicates (predicates.go:233-276)
  if (C.mem_pressure && (sp.flags & KB_SPEC_BEST_EFFORT) && (f & KB_NODE_MEM_PRESSURE))
    return 1u << KB_R_MEMORY_PRESSURE;
  if (C.disk_pressure && (f & KB_NODE_DISK_PRESSURE)) return 1u << KB_R_DISK_PRESSURE;
  if (C.pid_pressure && (f & KB_NODE_PID_PRESSURE)) return 1u << KB_R_PID_PRESSURE;
  return 0;
}

// leastRequestedScore (priorities/least_requested.go:36-53)
__device__ __forceinline__ int64_t lr_score(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return ((cap - req) * 10) / cap;
}
// fractionOfCapacity (balanced_resource_allocation.go:72-77)
__device__ __forceinline__ double frac_cap(int64_t req, int64_t cap) {
  return cap == 0 ? 1.0 : (double)req / (double)cap;
}

// nodeOrderFn (nodeorder.go:188-226) + InterPodAffinity batch score (0 without pod affinity terms).
// All terms are integers, so the reference's float64 sum is this int64 sum exactly.
__device__ int64_t node_score(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const kb_spec& sp, int n) {
  if (!C.nodeorder) return 0;
  if (sp.flags & KB_SPEC_NA_ERROR) return 0;  // map fn error: node keeps only the batch score
  const int64_t rc = sp.nz_cpu + N.nz_cpu[n], rm = sp.nz_mem + N.nz_mem[n];
  const int64_t ac = N.alloc_cpu[n], am = N.alloc_mem[n];
  const int64_t lr = (lr_score(rc, ac) + lr_score(rm, am)) / 2;
  const double cf = frac_cap(rc, ac), mf = frac_cap(rm, am);
  const int64_t bra = (cf >= 1.0 || mf >= 1.0) ? 0 : (int64_t)((1.0 - fabs(cf - mf)) * 10.0);
  int32_t na = 0;  // CalculateNodeAffinityPriorityMap (priorities/node_affinity.go:34-74)
  for (uint32_t i = 0; i < sp.pref_term_cnt; ++i) {
    const kb_term t = P.terms[sp.pref_term_off + i];
    if (t.weight == 0) continue;
    if (term_match(N, P, t, n)) na += t.weight;
  }
  return lr * C.w_lr + bra * C.w_bra + (int64_t)na * C.w_na;
}

__device__ __forceinline__ uint64_t node_key(const DevNodes& N, const DevSpecs& P, const DevCfg& C,
                                             const kb_spec& sp, int s, int n) {
  const uint32_t r = node_reasons(N, P, C, sp, s, n);
  if (r) return r;
  const int64_t score = node_score(N, P, C, sp, n);
  return kFeasible | ((uint64_t)(score + kScoreBias) << 24) | (uint64_t)(kIdxMask - (uint32_t)n);
}

// Session.Allocate / Session.Pipeline applied to the device row (framework/session.go:199-297):
// NodeInfo.AddTask (api/node_info.go:165-193) + schedulercache.NodeInfo.AddPod (cache/node_info.go:498-520).
__device__ int commit_row(const DevNodes& N, const DevSpecs& P, const kb_spec& sp, int s, int w) {
  const uint32_t f = N.flags[w];
  const int64_t* sci = P.sc_init + (size_t)s * N.S;
  const int64_t* scr = P.sc_req + (size_t)s * N.S;
  int kind;
  if (fits_idle(N, sp, sci, f, w)) {  // allocate.go:159 -> Idle.Sub(Resreq)
    N.idle_cpu[w] -= sp.req_cpu;
    N.idle_mem[w] -= sp.req_mem;
    if (f & KB_NODE_IDLE_HAS_MAP) {  // Sub leaves a nil map alone (resource_info.go:152-157)
      uint64_t m = sp.req_sc_mask;
      while (m) {
        const int q = __builtin_ctzll(m);
        m &= m - 1;
        N.idle_sc[(size_t)q * N.n + w] -= scr[q];
      }
    }
    kind = KB_PLACE_ALLOCATE;
  } else {  // allocate.go:172 -> Releasing.Sub(Resreq)
    N.rel_cpu[w] -= sp.req_cpu;
    N.rel_mem[w] -= sp.req_mem;
    if (f & KB_NODE_REL_HAS_MAP) {
      uint64_t m = sp.req_sc_mask;
      while (m) {
        const int q = __builtin_ctzll(m);
        m &= m - 1;
        N.rel_sc[(size_t)q * N.n + w] -= scr[q];
      }
    }
    kind = KB_PLACE_PIPELINE;
  }
  N.pod_count[w] += 1;
  N.nz_cpu[w] += sp.nz_cpu;
  N.nz_mem[w] += sp.nz_mem;
  for (uint32_t i = 0; i < sp.port_cnt; ++i) {  // UpdateUsedPorts (cache/node_info.go:593-606)
    const kb_port p = P.ports[sp.port_off + i];
    N.port_used[(size_t)p.slot * N.n + w] |= 1ull << p.ip;
  }
  return kind;
}

__global__ __launch_bounds__(256) void sweep_keys_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, uint64_t* keys,
                                                         uint64_t* cmax, const JobState* js) {
  if (js != nullptr && js->stopped) return;
  const kb_spec sp = P.specs[spec];
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t k = 0;
  if (n < N.n) {
    k = node_key(N, P, C, sp, spec, n);
    keys[n] = k;
  }
  const uint64_t m = wave_max_u64(k);
  if ((threadIdx.x & 63) == 0 && (n >> 6) < ((N.n + 63) >> 6)) cmax[n >> 6] = m;
}

__global__ void job_init_kernel(JobState* js, int ready_num, int min_available, int gang_ready) {
  const int i = threadIdx.x;
  if (i == 0) {
    js->stopped = 0;
    js->stop = KB_STOP_DONE;
    js->fail_task = -1;
    js->n_placed = 0;
    js->ready_num = ready_num;
    js->min_available = min_available;
    js->gang_ready = gang_ready;
    js->panic = 0;
  }
  if (i < KB_NUM_REASONS) js->hist[i] = 0;
}

// L2-coherent load of a key another lane of this wave may have stored earlier in the launch.
__device__ __forceinline__ uint64_t load_key_l2(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool KEYS_IN_LDS>
__global__ __launch_bounds__(64) void place_loop_kernel(DevNodes N, DevSpecs P, DevCfg C, int spec, int t_begin,
                                                        int t_count, uint64_t* keys, const uint64_t* cmax_g,
                                                        JobState* js, int32_t* out) {
  extern __shared__ __attribute__((aligned(16))) uint64_t lds[];
  if (js->stopped) return;
  const int lane = threadIdx.x;
  const int n = N.n;
  const int M = (n + 63) >> 6;
  const int Mp = (M + 1) & ~1;  // keep the key block 16-B aligned
  uint64_t* cm = lds;
  uint64_t* lk = lds + Mp;
  for (int c = lane; c < M; c += 64) cm[c] = cmax_g[c];
  if (KEYS_IN_LDS)
    for (int i = lane; i < n; i += 64) lk[i] = keys[i];
  __syncthreads();

  const kb_spec sp = P.specs[spec];
  int ready = js->ready_num;
  const int minav = js->min_available;
  const int gang = js->gang_ready;
  int placed = js->n_placed;

  for (int t = 0; t < t_count; ++t) {
    uint64_t best = 0;
    for (int c = lane; c < M; c += 64) {
      const uint64_t v = cm[c];
      best = v > best ? v : best;
    }
    best = wave_max_u64(best);

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
        if (lane == 0) js->hist[b] = s;
      }
      if (lane == 0) {
        js->stop = KB_STOP_NO_FIT;
        js->fail_task = t_begin + t;
        js->n_placed = placed;
        js->ready_num = ready;
        js->stopped = 1;
      }
      return;
    }
    const int64_t score = (int64_t)((best >> 24) & ((1ull << 39) - 1)) - kScoreBias;
    if (score <= -1) {  // SelectBestNode: no bucket with score > -1 -> the reference panics
      if (lane == 0) {
        js->panic = 1;
        js->fail_task = t_begin + t;
        js->n_placed = placed;
        js->stopped = 1;
      }
      return;
    }
    const int w = (int)(kIdxMask - (uint32_t)(best & kIdxMask));

    uint64_t nk = 0;
    int kind = 0;
    if (lane == 0) {
      kind = commit_row(N, P, sp, spec, w);
      nk = node_key(N, P, C, sp, spec, w);
      if (!KEYS_IN_LDS) keys[w] = nk;
      out[2 * (t_begin + t)] = w;
      out[2 * (t_begin + t) + 1] = kind;
    }
    nk = __shfl(nk, 0, 64);
    kind = __shfl(kind, 0, 64);
    if (!KEYS_IN_LDS) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (KEYS_IN_LDS && lane == 0) lk[w] = nk;

    // Re-reduce the winner's chunk.
    const int c = w >> 6;
    const int i = (c << 6) + lane;
    uint64_t v = 0;
    if (i < n) v = (i == w) ? nk : (KEYS_IN_LDS ? lk[i] : load_key_l2(&keys[i]));
    v = wave_max_u64(v);
    if (lane == 0) cm[c] = v;
    __syncthreads();

    ++placed;
    if (kind == KB_PLACE_ALLOCATE) ++ready;
    if (!gang || ready >= minav) {  // ssn.JobReady(job) (allocate.go:184-187; gang.go:122-125)
      if (lane == 0) {
        js->stop = KB_STOP_READY;
        js->n_placed = placed;
        js->ready_num = ready;
        js->stopped = 1;
      }
      return;
    }
  }
  if (lane == 0) {
    js->n_placed = placed;
    js->ready_num = ready;
  }
}

__global__ __launch_bounds__(256) void eval_kernel(DevNodes N, DevSpecs P, DevCfg C, const int32_t* spec_ids,
                                                   uint32_t* reasons, int64_t* scores) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (n >= N.n) return;
  const int s = spec_ids[j];
  const kb_spec sp = P.specs[s];
  reasons[(size_t)j * N.n + n] = node_reasons(N, P, C, sp, s, n);
  scores[(size_t)j * N.n + n] = node_score(N, P, C, sp, n);
}

// ---------------------------------------------------------------------------
int place_loop_lds_bytes(int n) {
  const int M = (n + 63) >> 6;
  const int Mp = (M + 1) & ~1;
  const size_t keys_bytes = (size_t)(Mp + n) * 8;
  return keys_bytes <= 160 * 1024 ? (int)keys_bytes : -(Mp * 8);
}

void launch_sweep_keys(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, uint64_t* keys,
                       uint64_t* cmax, const JobState* js, void* stream) {
  const int blocks = (N.n + 255) / 256;
  hipLaunchKernelGGL(sweep_keys_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, N, P, C, spec, keys, cmax,
                     js);
}

void launch_job_init(JobState* js, int ready_num, int min_available, int gang_ready, void* stream) {
  hipLaunchKernelGGL(job_init_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, js, ready_num, min_available,
                     gang_ready);
}

void launch_place_loop(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                       uint64_t* keys, const uint64_t* cmax, JobState* js, int32_t* out, void* stream) {
  const int lds = place_loop_lds_bytes(N.n);
  if (lds > 0) {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)place_loop_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024);
      attr_set = true;
    }
    hipLaunchKernelGGL(place_loop_kernel<true>, dim3(1), dim3(64), lds, (hipStream_t)stream, N, P, C, spec, t_begin,
                       t_count, keys, cmax, js, out);
  } else {
    static bool attr_set = false;
    if (!attr_set) {
      (void)hipFuncSetAttribute((const void*)place_loop_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024);
      attr_set = true;
    }
    hipLaunchKernelGGL(place_loop_kernel<false>, dim3(1), dim3(64), -lds, (hipStream_t)stream, N, P, C, spec, t_begin,
                       t_count, keys, cmax, js, out);
  }
}

void launch_eval(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const int32_t* spec_ids, int t,
                 uint32_t* reasons, int64_t* scores, void* stream) {
  dim3 grid((N.n + 255) / 256, t);
  hipLaunchKernelGGL(eval_kernel, grid, dim3(256), 0, (hipStream_t)stream, N, P, C, spec_ids, reasons, scores);
}

}  // namespace kbgpu
