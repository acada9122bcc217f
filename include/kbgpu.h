/*
 * kbgpu.h — C ABI of the MI355X-native allocate hot path for kube-batch.
 *
 * Drop-in boundary. The reference's plugin API stays as it
 * is: framework.Action / framework.Plugin (pkg/scheduler/framework/interface.go:20-41),
 * the Session dispatchers (framework/session_plugins.go:25-492) and the helper
 * trio PredicateNodes / PrioritizeNodes / SelectBestNode
 * (pkg/scheduler/util/scheduler_helper.go:34,67,147). A kube-batch build binds
 * this header through cgo and replaces, per pending task, the
 * three helpers plus Session.Allocate/Pipeline's node-row update with one device
 * sweep + argmax + in-place commit.
 *
 * Two layers:
 *   1. device layer  — kb_create / kb_upload_* / kb_place_job / kb_eval:
 *      the snapshot lives on the GPU as a struct-of-arrays node table; the caller
 *      keeps queue/job/task ordering (allocate.go:95-192) and calls kb_place_job
 *      once per job pop.
 *   2. session layer — kb_allocate: the whole allocateAction.Execute
 *      (actions/allocate/allocate.go:42-193) with the ordering plugins
 *      (priority, gang, drf, proportion) restated in C++ on the host, driving
 *      layer 1 per job.
 *
 * Conventions: every function returns KB_OK (0) or a negative KB_E_* code and
 * never throws; kb_last_error() describes the last failure. All pointers passed
 * in are caller-owned and read only during the call (cgo rule: C keeps no Go
 * pointers). Device memory is owned by the context. A context is used by one
 * thread at a time (the action goroutine). Strings never cross the ABI: the
 * caller interns names into the integer ids below. Node index = canonical node
 * order (nodes sorted by name), which is also the SelectBestNode tie-break:
 * among equal best scores the lowest index wins (the reference picks at random,
 * scheduler_helper.go:157).
 */
#ifndef KBGPU_H_
#define KBGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KBGPU_ABI_VERSION 16

/* ---- return codes ---- */
#define KB_OK 0
#define KB_E_INVALID (-1)     /* bad argument / shape mismatch */
#define KB_E_HIP (-2)         /* HIP runtime failure */
#define KB_E_UNSUPPORTED (-3) /* input uses a feature the device path does not express */
#define KB_E_NOMEM (-4)
#define KB_E_PANIC (-5)       /* the reference would panic: SelectBestNode found no score > -1
                                 (scheduler_helper.go:147-158) or util/assert fired */
#define KB_E_STATE (-6)       /* call out of order (e.g. place before upload) */

/* ---- predicate failure reasons: bit i of a reason mask ----
 * strings: api/unschedule_info.go:11-19, vendor/.../algorithm/predicates/error.go:24-84 */
#define KB_R_RESOURCE_FIT 0        /* "node(s) resource fit failed" */
#define KB_R_POD_NUMBER 1          /* "node(s) pod number exceeded" */
#define KB_R_NOT_READY 2           /* "node(s) were not ready" */
#define KB_R_OUT_OF_DISK 3         /* "node(s) were out of disk space" */
#define KB_R_NETWORK_UNAVAILABLE 4 /* "node(s) had unavailable network" */
#define KB_R_UNSCHEDULABLE 5       /* "node(s) were unschedulable" */
#define KB_R_NODE_SELECTOR 6       /* "node(s) didn't match node selector" */
#define KB_R_HOST_PORTS 7          /* "node(s) didn't have free ports for the requested pod ports" */
#define KB_R_TAINTS 8              /* "node(s) had taints that the pod didn't tolerate" */
#define KB_R_MEMORY_PRESSURE 9     /* "node(s) had memory pressure" */
#define KB_R_DISK_PRESSURE 10      /* "node(s) had disk pressure" */
#define KB_R_PID_PRESSURE 11       /* "node(s) had pid pressure" */
#define KB_R_POD_AFFINITY 12       /* "node(s) didn't match pod affinity/anti-affinity" */
#define KB_R_EXISTING_ANTI 13      /* "node(s) didn't satisfy existing pods anti-affinity rules" */
#define KB_R_AFFINITY_RULES 14     /* "node(s) didn't match pod affinity rules" */
#define KB_R_ANTI_AFFINITY_RULES 15/* "node(s) didn't match pod anti-affinity rules" */
#define KB_R_HOST_ERROR 16         /* a host-evaluated stage failed: a kb_set_host_overlay plugin predicate, or a
                                      predicate the reference fails with a plain error string (inter-pod affinity
                                      with an invalid selector or an empty topologyKey: vendor/.../predicates.go:
                                      1293-1333, 1189-1214, 1401-1413). The strings are the caller's: the per-node
                                      reason masks of the failing task come through kb_set_nofit_hook / kb_eval. */
#define KB_NUM_REASONS 17

/* ---- node flags (kb_nodes.flags) ---- */
#define KB_NODE_IDLE_HAS_MAP (1u << 0) /* Idle.ScalarResources != nil (allocatable lists a scalar) */
#define KB_NODE_REL_HAS_MAP (1u << 1)  /* Releasing.ScalarResources != nil */
#define KB_NODE_NOT_READY (1u << 2)    /* condition Ready != True            (predicates.go:1582) */
#define KB_NODE_OUT_OF_DISK (1u << 3)  /* condition OutOfDisk != False       (:1584) */
#define KB_NODE_NET_UNAVAIL (1u << 4)  /* condition NetworkUnavailable != False (:1586) */
#define KB_NODE_UNSCHEDULABLE (1u << 5)/* node.Spec.Unschedulable            (:1590) */
#define KB_NODE_MEM_PRESSURE (1u << 9) /* MemoryPressure == True */
#define KB_NODE_DISK_PRESSURE (1u << 10)
#define KB_NODE_PID_PRESSURE (1u << 11)

/*
 * Node table, struct-of-arrays, n rows in canonical order. Resource quantities
 * are the reference's integral float64 values as int64: cpu and scalars in
 * milli-units, memory in bytes (api/resource_info.go:75-93).
 * Scalar slot s (0 <= s < n_scalar) is a caller-interned scalar resource name;
 * arrays [n_scalar][n] are slot-major.
 */
typedef struct kb_nodes {
  uint32_t n;
  uint32_t n_scalar;   /* S */
  uint32_t n_label;    /* K: label-key slots referenced by any selector / term */
  uint32_t n_port;     /* P: (protocol, hostPort) slots referenced by any task */
  const int64_t* idle_cpu;  /* api.NodeInfo.Idle        (node_info.go:35-40) */
  const int64_t* idle_mem;
  const int64_t* rel_cpu;   /* api.NodeInfo.Releasing */
  const int64_t* rel_mem;
  const int64_t* idle_sc;   /* [S][n] (absent key = 0) */
  const int64_t* rel_sc;    /* [S][n] */
  const int64_t* alloc_cpu; /* schedulercache allocatable (cache/node_info.go:611), LR/BRA */
  const int64_t* alloc_mem;
  const int64_t* nz_cpu;    /* schedulercache nonzeroRequest (cache/node_info.go:498-520) */
  const int64_t* nz_mem;
  const int32_t* pod_count; /* len(nodeInfo.Pods())  (predicates.go:162) */
  const int32_t* max_pods;  /* Allocatable.MaxTaskNum */
  const uint32_t* flags;    /* KB_NODE_* */
  const int32_t* label_val; /* [K][n] interned value id of label key k, -1 when absent */
  const int64_t* label_int; /* [K][n] strconv.ParseInt of the value (for Gt/Lt) */
  const uint8_t* label_int_ok; /* [K][n] 1 when the value parsed */
  const int32_t* taint_set; /* [n] id of the node's NoSchedule/NoExecute taint set (0 = none) */
  const uint64_t* port_used;/* [P][n] bitmask over the slot's interned host IPs (bit 0 = 0.0.0.0) */
} kb_nodes;

/* Label requirement program (labels.Requirement, labels/selector.go:185-236). */
#define KB_OP_IN 0
#define KB_OP_NOTIN 1
#define KB_OP_EXISTS 2
#define KB_OP_DNE 3
#define KB_OP_GT 4
#define KB_OP_LT 5
#define KB_OP_TRUE 6  /* field requirement decided on the host (non-name field key) */
#define KB_OP_FALSE 7 /* invalid requirement: the term cannot match */

typedef struct kb_req {
  int32_t key;      /* label-key slot */
  int32_t op;       /* KB_OP_* */
  uint32_t val_off; /* into kb_specs.vals */
  uint32_t val_cnt;
  int64_t ival;     /* Gt/Lt operand */
} kb_req;

typedef struct kb_term {
  uint32_t req_off; /* into kb_specs.reqs; AND of requirements */
  uint32_t req_cnt; /* 0 => the term matches nothing (helpers.go:308-311, :222-225) */
  int32_t weight;   /* preferred terms only */
  int32_t pad;
} kb_term;

/* spec flags */
#define KB_SPEC_INIT_HAS_MAP (1u << 0)  /* InitResreq.ScalarResources != nil */
#define KB_SPEC_REQ_HAS_MAP (1u << 1)
#define KB_SPEC_BEST_EFFORT (1u << 2)   /* v1qos BestEffort (memory-pressure predicate) */
#define KB_SPEC_HAS_SELECTOR (1u << 3)  /* len(nodeSelector) > 0 and every pair valid */
#define KB_SPEC_HAS_REQUIRED (1u << 4)  /* nodeAffinity.RequiredDuringScheduling != nil */
#define KB_SPEC_NA_ERROR (1u << 5)      /* a preferred term is invalid: map fn errors (node_affinity.go:59-62) */
#define KB_SPEC_POD_AFFINITY (1u << 6)  /* pod (anti)affinity terms: needs the affinity tables */
#define KB_SPEC_IPA_ERROR (1u << 7)     /* CalculateInterPodAffinityPriority errors for this pod (an invalid label
                                           selector among the terms it meets, interpod_affinity.go:86-93): the batch
                                           score fails, PrioritizeNodes returns no scores and SelectBestNode panics
                                           (scheduler_helper.go:101-105,147-158) -> KB_E_PANIC once a node fits */

/*
 * Task spec: everything the device needs about a pending pod. Pods of one
 * job usually share a spec; the caller deduplicates by signature.
 */
typedef struct kb_spec {
  int64_t init_cpu, init_mem; /* InitResreq (pod_info.go:53-63): the predicate request */
  int64_t req_cpu, req_mem;   /* Resreq (pod_info.go:66-73): what commit subtracts */
  int64_t nz_cpu, nz_mem;     /* getNonZeroRequests (resource_allocation.go:94-103) */
  uint64_t init_sc_mask;      /* scalar slots present in InitResreq */
  uint64_t req_sc_mask;       /* scalar slots present in Resreq */
  uint32_t flags;             /* KB_SPEC_* */
  int32_t tol_set;            /* toleration-set id (row of kb_specs.tolerates) */
  uint32_t sc_off;            /* into kb_specs.sc_init / sc_req: n_scalar values */
  uint32_t sel_term;          /* nodeSelector as one term (index into terms) */
  uint32_t req_term_off, req_term_cnt;   /* required node-affinity terms (ORed) */
  uint32_t pref_term_off, pref_term_cnt; /* preferred node-affinity terms */
  uint32_t port_off, port_cnt;           /* wanted host ports, into kb_specs.ports */
  int32_t aff_class;          /* inter-pod affinity class (kb_affinity), -1 none */
  int32_t pad;
} kb_spec;

typedef struct kb_port {
  int32_t slot; /* (protocol, hostPort) slot */
  int32_t ip;   /* interned host IP within the slot, 0 = 0.0.0.0 */
} kb_port;

typedef struct kb_specs {
  uint32_t m;              /* number of specs */
  const kb_spec* specs;
  const int64_t* sc_init;  /* [m][n_scalar] */
  const int64_t* sc_req;   /* [m][n_scalar] */
  uint32_t n_terms;
  const kb_term* terms;
  uint32_t n_reqs;
  const kb_req* reqs;
  uint32_t n_vals;
  const int32_t* vals;     /* interned label-value ids */
  uint32_t n_ports;
  const kb_port* ports;
  uint32_t n_tol_sets, n_taint_sets;
  const uint8_t* tolerates;/* [n_tol_sets][n_taint_sets]: 1 if the tolerations tolerate every
                              NoSchedule/NoExecute taint of the set (predicates.go:1489-1518) */
} kb_specs;

/* Plugin configuration that shapes the predicate chain and the score. */
typedef struct kb_config {
  int32_t predicates_enabled; /* "predicates" in tiers with EnabledPredicate (session_plugins.go:372-389) */
  int32_t nodeorder_enabled;  /* "nodeorder" in tiers with EnabledNodeOrder */
  int32_t mem_pressure, disk_pressure, pid_pressure; /* predicate.*PressureEnable (predicates.go:72-111) */
  int32_t w_lr, w_bra, w_na, w_pa;                    /* nodeorder weights (nodeorder.go:96-140) */
} kb_config;

typedef struct kb_opts {
  int32_t device;        /* HIP device ordinal */
  uint32_t flags;        /* KB_OPT_* */
  uint32_t timing_every; /* KB_OPT_TIMING: time the launches of every Nth kb_place_job call (0 or 1: all) */
  int32_t fed_idle_ms;   /* the fed engine's idle exit (0: 1 s; tests shorten it) */
  int32_t eval_spb;      /* eval_plain_kernel's specs per block (0: sized from the device's CU count) */
  int32_t test_stall_ms; /* tests: with test_stall_job >= 0, a host stall of this long before that job */
  int64_t test_stall_job;/* tests: -1 off */
  uint32_t shard_epoch0; /* tests: the node-sharded engine's first cycle epoch (0; the inbox tags' wrap) */
  int32_t fed_xcc;       /* ABI 15: the split engine's workgroups: 0 = the library's default (XCC 0, resident sweepers);
                            k + 1 = on XCC k (a census at launch, kbgpu_device.hip fed_engine_kernel); -1 = where the
                            dispatcher puts them (no census, so per-job sweep kernels). A zero-initialised kb_opts gets
                            the production path. */
  int32_t fed_depth;     /* ABI 15: the fed engine's units in flight (the running one + speculative ones), 2..4;
                            0 = chosen per cycle by the driver (kbgpu_allocate.cpp) */
} kb_opts;

typedef struct kb_ctx kb_ctx;

/* ---- layer 1: device ---- */
kb_ctx* kb_create(const kb_opts* opts);
void kb_destroy(kb_ctx* ctx);
const char* kb_last_error(const kb_ctx* ctx);
int kb_abi_version(void);

int kb_set_config(kb_ctx* ctx, const kb_config* cfg);
/* Copies the node table to HBM (replaces any previous one). */
int kb_upload_nodes(kb_ctx* ctx, const kb_nodes* nodes);
/* Copies the spec tables to HBM. */
int kb_upload_specs(kb_ctx* ctx, const kb_specs* specs);

/*
 * Inter-pod (anti)affinity as counts per topology domain (scheduler_amd/affinity.py has the derivation).
 * Replaces the lister scans of InterPodAffinityMatches (vendor/.../predicates/predicates.go:1155-1465,
 * called from plugins/predicates/predicates.go:278-296) and the per-node loops of
 * CalculateInterPodAffinityPriority (vendor/.../priorities/interpod_affinity.go:119-241, called from
 * plugins/nodeorder/nodeorder.go:229-246).
 *
 * A topology slot is a tuple of label keys; topo_dom[slot][node] is the node's domain id (-1: a key is
 * missing). A count table holds, per domain of its slot, the lister pods that carry one required
 * anti-affinity term (EXISTING_ANTI) or match all required (anti-)affinity terms of a spec (ANTI /
 * AFFINITY), plus a total. A spec checks its tables in order (existing anti, anti, affinity: the
 * reference's order) and keeps InterPodAffinity histograms H[h_off + domain] per topology key.
 * Commits apply the committed spec's increment lists: lister tables on Allocate only (Pipelined tasks
 * are not listed, plugins/util/util.go:108-130), histogram increments on every commit.
 * Counts are int32.
 */
#define KB_AFF_EXISTING_ANTI 0 /* fail if count > 0: "didn't satisfy existing pods anti-affinity rules" */
#define KB_AFF_ANTI 1          /* fail if count > 0: "didn't match pod anti-affinity rules" */
#define KB_AFF_AFFINITY 2      /* fail if count == 0 and (total > 0 or !self_match): "...affinity rules" */
#define KB_AFF_ERROR 3         /* fail with KB_R_HOST_ERROR if count > 0: the reference returns a plain error (lister
                                  pods carrying an invalid required anti-affinity selector; the pod's own required
                                  affinity with an invalid selector or an empty topologyKey met by a lister pod) */
#define KB_AFF_SELF_DYNAMIC (1u << 0) /* the spec's own commits change its checks or histograms */

typedef struct kb_aff_table {
  int32_t slot;
  uint32_t cnt_off; /* into counters: one entry per domain of the slot */
} kb_aff_table;
typedef struct kb_aff_check {
  int32_t table;
  int32_t kind; /* KB_AFF_* */
} kb_aff_check;
typedef struct kb_ipa_hist {
  int32_t slot;   /* single-key slot */
  uint32_t h_off; /* into h: one entry per domain */
} kb_ipa_hist;
typedef struct kb_ipa_incr {
  int32_t slot;
  uint32_t h_off;
  int32_t weight; /* added at the committed node's domain, per commit */
  int32_t pad;
} kb_ipa_incr;
typedef struct kb_aff_spec {
  uint32_t check_off, check_cnt;   /* into checks */
  uint32_t lister_off, lister_cnt; /* into lister: tables a committed (Allocated) task of this spec joins */
  uint32_t hist_off, hist_cnt;     /* into hists: this spec's InterPodAffinity histograms */
  uint32_t incr_off, incr_cnt;     /* into incr: histogram updates of one commit of this spec */
  int32_t self_match;              /* targetPodMatchesAffinityOfPod(pod, pod) (metadata.go:498-510) */
  uint32_t flags;                  /* KB_AFF_SELF_DYNAMIC */
} kb_aff_spec;

typedef struct kb_affinity {
  uint32_t n_slots;
  const int32_t* topo_dom; /* [n_slots][n] */
  uint32_t n_tables;
  const kb_aff_table* tables;
  const int32_t* totals;   /* [n_tables] */
  uint32_t n_counters;
  const int32_t* counters;
  uint32_t m;              /* must equal kb_specs.m; kb_spec.aff_class indexes specs */
  const kb_aff_spec* specs;
  uint32_t n_checks;
  const kb_aff_check* checks;
  uint32_t n_lister;
  const int32_t* lister;   /* table ids */
  uint32_t n_hists;
  const kb_ipa_hist* hists;
  uint32_t n_h;
  const int32_t* h;
  uint32_t n_incr;
  const kb_ipa_incr* incr;
} kb_affinity;

/* Copies the affinity tables to HBM (after kb_upload_nodes and kb_upload_specs). Specs flagged
 * KB_SPEC_POD_AFFINITY are refused by kb_place_job / kb_eval until this is called. */
int kb_upload_affinity(kb_ctx* ctx, const kb_affinity* aff);

/* placement kinds */
#define KB_PLACE_ALLOCATE 1 /* Session.Allocate (session.go:242) */
#define KB_PLACE_PIPELINE 2 /* Session.Pipeline (session.go:199) */

/* stop reasons of one job batch (allocate.go:135-188) */
#define KB_STOP_DONE 0   /* every task placed */
#define KB_STOP_NO_FIT 1 /* a task fit no node: job leaves the queue (allocate.go:150-153) */
#define KB_STOP_READY 2  /* ssn.JobReady(job) after a placement: job re-queued (allocate.go:184-187) */

typedef struct kb_job_req {
  const int32_t* task_specs; /* spec id of each task, in TaskOrderFn order */
  uint32_t n_tasks;
  int32_t ready_num;     /* job.ReadyTaskNum() before the batch (job_info.go:367-378) */
  int32_t min_available; /* job.MinAvailable */
  int32_t gang_ready;    /* 1: JobReady = ReadyTaskNum >= MinAvailable (gang.go:122-125);
                            0: no JobReady plugin enabled, JobReady is always true */
} kb_job_req;

typedef struct kb_job_result {
  uint32_t n_placed;       /* placements written */
  int32_t stop;            /* KB_STOP_* */
  int32_t fail_task;       /* index of the task that fit nowhere (KB_STOP_NO_FIT) */
  int32_t pad;
  uint32_t reason_hist[KB_NUM_REASONS]; /* FitErrors histogram over all nodes for fail_task */
} kb_job_result;

/*
 * Place one popped job's pending tasks (allocate.go:135-188): for each task in
 * order, predicate + score every node, pick the best (lowest index on ties),
 * commit Allocate (InitResreq fits Idle) or Pipeline (fits Releasing) to the
 * device node table in place, stop on no-fit or when the job becomes ready.
 * placed_node[i] / placed_kind[i] receive the i-th placement (task i).
 */
int kb_place_job(kb_ctx* ctx, const kb_job_req* job, int32_t* placed_node, int32_t* placed_kind,
                 kb_job_result* result);

/*
 * Parity / snapshot mode: evaluate t specs against every node at the current
 * node-table state without committing. reasons[t][n] = reason mask (0 = feasible),
 * scores[t][n] = total node-order score (PrioritizeNodes' merged score,
 * scheduler_helper.go:107-127).
 */
int kb_eval(kb_ctx* ctx, const int32_t* spec_ids, uint32_t t, uint32_t* reasons, int64_t* scores);

/*
 * kb_eval with 32-bit scores: 8 B per (spec, node) pair instead of 12 (the sweep's output is most of its HBM
 * traffic). KB_E_UNSUPPORTED when a spec's score cannot be held in int32: its |score| bound (the weighted
 * LeastRequested / Balanced / NodeAffinity / InterPodAffinity maxima plus the overlay's) reaches 2^31, or its
 * InterPodAffinity batch score errors (kb_eval reports those with a score below every int32).
 */
int kb_eval32(kb_ctx* ctx, const int32_t* spec_ids, uint32_t t, uint32_t* reasons, int32_t* scores);

/*
 * preempt's use of the sweep (actions/preempt/preempt.go:189-195): PredicateNodes with Session.PredicateFn
 * alone (no allocate resource check), PrioritizeNodes, then SortNodes (util/scheduler_helper.go:132-144) for
 * one spec at the current node-table state. order[0..*n_out) = the feasible nodes by score, descending, and
 * the lowest index first among equal scores (the reference appends a score bucket's nodes in goroutine
 * completion order); scores[i] = order[i]'s score (either array may be NULL; capacity n). A batch-score error
 * (KB_SPEC_IPA_ERROR) gives an empty list: PrioritizeNodes returns no scores there. Not node-sharded.
 */
int kb_sort_nodes(kb_ctx* ctx, int32_t spec, int32_t* order, int64_t* scores, uint32_t* n_out);

/*
 * util.PredicateNodes(task, nodes, ssn.PredicateFn) alone (util/scheduler_helper.go:34-64): the nodes passing
 * Session.PredicateFn for one spec at the current state, in canonical order, and the FitErrors histogram of the
 * rest. reclaim walks this set for victims (actions/reclaim/reclaim.go:122-126), preempt sorts it (above).
 * nodes: capacity n (may be NULL); reason_hist: KB_NUM_REASONS counters (may be NULL).
 */
int kb_predicate_nodes(kb_ctx* ctx, int32_t spec, int32_t* nodes, uint32_t* n_out, uint32_t* reason_hist);

/*
 * Restore the node table to its state at the last kb_upload_nodes (device-to-device copy of the
 * mutable columns). A fresh allocate cycle over the same cache snapshot re-opens its session this way
 * without another host upload.
 */
int kb_restore_nodes(kb_ctx* ctx);

/* Kernel timing (HIP events on the context's stream), enabled by KB_OPT_TIMING in kb_opts.flags. */
#define KB_OPT_TIMING (1u << 0)
#define KB_OPT_NO_TRAJECTORY (1u << 1) /* no trajectory loop: the per-commit re-key loop (testing the device paths) */
#define KB_OPT_NO_SELECT (1u << 2)     /* no top-T selection path: the trajectory loop (testing the device paths) */
#define KB_OPT_ENGINE (1u << 3)        /* serve selection-path jobs from the persistent placement engine */
/* Path selection and measurement switches (ABI 13: kb_opts fields, never the environment). The default (0) is the
 * production path; the rest exist so the tests can drive every device path and the profiler can run. */
#define KB_OPT_NO_FED (1u << 4)             /* a place kernel per job instead of the resident fed engine */
#define KB_OPT_NO_FED_SPLIT (1u << 5)       /* the one-workgroup fed engine (no selector workgroups) */
#define KB_OPT_NO_PIPELINE (1u << 6)        /* the serial driver: no speculative job issue */
#define KB_OPT_NO_AFF_REG (1u << 7)         /* self-dependent affinity runs on the global-memory loop */
#define KB_OPT_NO_CAP1 (1u << 8)            /* cap-1 affinity specs on the re-sweep loops */
#define KB_OPT_NO_CLS (1u << 9)             /* class-loop affinity specs on the re-sweep loops */
#define KB_OPT_NO_EVAL_PLAIN (1u << 10)     /* kb_eval's general kernel on plain batches too */
#define KB_OPT_FED_SHARED_QUEUES (1u << 11) /* the sweep stream without its own hardware queue (the hazard test) */
#define KB_OPT_FED_PLAIN_LAUNCH (1u << 12)  /* (ABI 14: the default; kept so old option sets still parse) */
#define KB_OPT_SHARD_SELF_INBOX (1u << 13)  /* a rank's own record through its inbox too (exchange tests) */
#define KB_OPT_FED_DIAG (1u << 14)          /* KB_DIAG builds: print the selector's phase stamps at kb_fed_end */
/* ABI 14: the resident engine is a plain launch after an explicit residency check (every workgroup of its 2-5
 * workgroup grid fits the device at once: hipOccupancyMaxActiveBlocksPerMultiprocessor x CUs); this flag restores
 * round 4's cooperative launch, for A/B measurements only (rocprofv3 7.2 crashes at exit after one). */
#define KB_OPT_FED_COOP_LAUNCH (1u << 15)
/* ABI 14, tests only: this rank's kb_set_shard_peer pre-flight words carry a wrong tag (every rank must fail). */
#define KB_OPT_TEST_PEER_BADTAG (1u << 16)
/* ABI 14: the split engine's per-job sweeps by sweep kernels on the CU-masked stream (round 4's path) instead of
 * its resident sweepers (the spare workgroups of its census grid, fed commands through a pinned ring); A/B only. */
#define KB_OPT_FED_KERNEL_SWEEPS (1u << 17)
/* ABI 15, tests only: the split engine's census reads every workgroup as on the placer's XCC (a one-XCC device or
 * partition), so its resident sweepers share that XCC */
#define KB_OPT_TEST_ONE_XCC (1u << 18)
/* ABI 15: the split engine without the resident sweepers' level records (the placer computes every e-sequence level
 * itself, round 5's path); A/B only */
#define KB_OPT_FED_NO_LEVELS (1u << 19)
/* ABI 16: inter-pod-affinity units stay off the resident engine (round 5's path: they run on the launch path while
 * the engine pauses); A/B only. By default kb_allocate's engine takes the affinity units whose inputs its sweep can
 * fold in: selection runs whose own commits leave their inputs alone, and the cap-1 runs. */
#define KB_OPT_FED_NO_AFF (1u << 20)
#define KB_KERNEL_SWEEP 0
#define KB_KERNEL_PLACE 1
#define KB_KERNEL_EVAL 2
#define KB_KERNEL_TRAJ_SWEEP 3
#define KB_KERNEL_TRAJ_PLACE 4
#define KB_KERNEL_AFF_PLACE 5 /* block-wide re-sweep loop (specs with self-dependent pod affinity) */
#define KB_KERNEL_IPA_MINMAX 6
#define KB_KERNEL_SEL_PLACE 7 /* a run as one parallel top-T selection (32-bit keys) */
#define KB_KERNEL_ENGINE 8    /* persistent placement engine: device time per served job */
#define KB_KERNEL_SEL_SWEEP 9 /* level-0 keys of every node for the selection path */
#define KB_KERNEL_SHARD_PROPOSE 10 /* node sharding: the rank's proposal for a segment */
#define KB_KERNEL_SHARD_EXCHANGE 11 /* node sharding: the all-gather of the proposals (RCCL) */
#define KB_KERNEL_SHARD_COMMIT 12  /* node sharding: global merge, stop rules, own commits */
#define KB_KERNEL_FED_ENGINE 13    /* kb_allocate: resident selection workgroup fed by the sweeps, one launch per cycle */
#define KB_KERNEL_CLS_PLACE 14      /* class loop: specs whose own commits move only their affinity histograms */
#define KB_NUM_KERNELS 15
typedef struct kb_stats {
  uint64_t launches[KB_NUM_KERNELS];
  double kernel_ms[KB_NUM_KERNELS];   /* summed event time per kernel kind */
  uint64_t pairs[KB_NUM_KERNELS];     /* (task, node) evaluations covered by those launches */
  uint64_t job_calls;
  double device_ms;                   /* wall time inside kb_place_job */
  uint64_t diag[8];                   /* diagnostic builds only: place-loop phase cycles, [7] realtime */
  uint64_t fed_abandon;               /* kb_allocate cycles the resident engine idled out of (host stall > its
                                         idle bound): finished on the launch path */
  uint64_t fed_cycles, fed_split;     /* kb_allocate cycles served by the resident engine; of those, by the
                                         split engine (node selection one job ahead on a second workgroup) */
  uint64_t cap1_runs;                 /* runs of self-dependent specs taken as cap-1 selection runs */
  uint64_t cls_runs;                  /* runs taken by the class loop (KB_KERNEL_CLS_PLACE) */
  uint64_t fed_sharded;               /* of the fed cycles, node-sharded ones (kb_set_shard_peer: the device
                                         exchange between the ranks' engines) */
  uint64_t shard_rezero;              /* inbox re-zeroings at the tags' epoch wrap (every 4096 sharded cycles) */
  uint64_t shard_xchg;                /* node-sharded engine: exchanges (jobs that ran) */
  uint64_t shard_wait_ticks;          /* node-sharded engine: s_memrealtime ticks (100 MHz) this rank's placer spent
                                         between writing its record and holding every peer's */
  uint64_t fed_clock_ticks, fed_real_ticks; /* split fed engine: s_memtime (shader clock) and s_memrealtime (100 MHz)
                                         ticks of the placer's launches, so clock MHz = 100 * clock / real */
  /* ABI 14 */
  uint64_t sweep_overlap;             /* per-job launch path: level-0 sweeps that overlapped the previous job */
  uint64_t overlap_refused_tables;    /* ... sweeps kept in order because a job still in flight writes tables
                                         the sweep reads (aff_sweep_indep, or an affinity-table commit queued
                                         after the publish of the job two back) */
  uint64_t shard_phase_ticks[6];      /* node-sharded engine, s_memrealtime ticks summed over the exchanges:
                                         [0] proposal (the rank's merge, e-sequences and winners), [1] writing
                                         the record into every peer's inbox, [2] waiting for every peer's record,
                                         [3] the global merge and stop rules, [4] commit + publish, [5] no-fit
                                         histogram rounds */
  uint64_t peer_checks;               /* kb_set_shard_peer pre-flight words that passed (2 per peer) */
  uint64_t fed_wg_place[2];           /* the last split engine launch: where its placer [0] and selector 0 [1] ran,
                                         XCC id << 32 | HW_ID (CU id bits 11:8, SIMD 5:4, SE 15:13) */
  uint64_t off_engine_units;          /* kb_allocate units the resident engine does not take (inter-pod affinity,
                                         host-evaluated reasons, ...), run on the launch path while the engine of a
                                         cycle that otherwise runs on it is paused (or between two launches) */
  uint64_t fed_pauses;                /* engine pauses for such units (the engine idles; its next command is fresh) */
  /* ABI 15 */
  uint64_t fed_mispredicts;           /* pipelined driver: units whose outcome differed from the prediction their
                                         successor was guarded on (the speculative chain behind them drained) */
  uint64_t fed_skipped;               /* ... speculative units skipped (guard failed) and drained */
  uint64_t fed_units;                 /* units finished by the pipelined driver in its fed (engine) mode */
  uint64_t nofit_predicted;           /* speculative issues behind a unit predicted NO_FIT (its spec, or a smaller one
                                         of its feasibility class, already found no node this cycle) */
  int32_t fed_last_depth;             /* the last engine cycle's units in flight (kb_opts.fed_depth or the driver's
                                         choice) */
  int32_t fed_last_sweepers;          /* the last split engine launch: resident sweeper workgroups (0: sweep
                                         kernels) */
  /* ABI 16 */
  uint64_t fed_aff_units;             /* engine units of specs with inter-pod terms (their table commits in the
                                         placer) */
  uint64_t fed_aff_waits;             /* engine units issued only after the units in flight finished: their sweep
                                         reads affinity tables an earlier unit's commits write */
} kb_stats;
int kb_get_stats(kb_ctx* ctx, kb_stats* out, int reset);

/* Read back the mutable node columns (for tests and for the Go side's NodeInfo replay). */
int kb_read_nodes(kb_ctx* ctx, int64_t* idle_cpu, int64_t* idle_mem, int64_t* rel_cpu, int64_t* rel_mem,
                  int32_t* pod_count, int64_t* nz_cpu, int64_t* nz_mem);

/*
 * ---- per-node Go fallback ----
 * Session.PredicateFn ANDs every enabled plugin's predicate per node and Session.NodeOrderMapFn sums
 * every plugin's node-order score (framework/session_plugins.go:372-389, 443-469). A plugin the device
 * does not express is evaluated by the caller with the existing Go functions, per node, and handed over
 * here for one spec: fail[i] != 0 rejects node i with KB_R_HOST_ERROR, score_add[i] is added to the
 * node's order score. The stage sits after the device's predicate chain (a plugin later in tier order)
 * and its score is dropped with the rest of the order score where nodeorder's map fn errors
 * (scheduler_helper.go:74-78). Scores must be integral (every in-tree node-order fn is) and
 * |NodeAffinity * weight + score_add| < 2^26. Either array may be NULL; both NULL clears the overlay.
 * The overlay stays until replaced: a plugin whose answer depends on this cycle's commits is re-set by
 * the caller between kb_place_job calls (device layer). n = this context's node rows. KB_E_UNSUPPORTED on a
 * node-sharded context (the verdicts and the NO_FIT hook's masks would be rank-local).
 */
int kb_set_host_overlay(kb_ctx* ctx, int32_t spec, const uint8_t* fail, const int64_t* score_add);

/*
 * Rows changed by commits made outside the device (Go-side backfill, preempt/reclaim evictions, a
 * plugin's own bookkeeping): NodeInfo.AddTask / RemoveTask (api/node_info.go:165-221) plus the
 * schedulercache AddPod / RemovePod the plugins' event handlers apply (cache/node_info.go:498-630).
 * Quantities are deltas (Idle -= Resreq is a negative idle delta). sc (n_scalar idle deltas followed by
 * n_scalar releasing deltas per row that uses it) and ports ((slot, ip) pairs the pod takes when
 * pods > 0, frees when pods < 0) are indexed by sc_off / port_off. spec >= 0 also applies that spec's
 * inter-pod affinity table updates (kind KB_PLACE_ALLOCATE joins the lister, as Session.Allocate does;
 * KB_PLACE_PIPELINE counts for the score only; pods < 0 takes them back). Deltas for the same node are
 * summed (order-free) except flags, where every set is applied before every clear. Node indices are
 * canonical; on a node-sharded context rows outside the rank are skipped.
 */
typedef struct kb_row_delta {
  int32_t node;
  int32_t pods;                /* pod_count delta */
  int64_t idle_cpu, idle_mem, rel_cpu, rel_mem;
  int64_t nz_cpu, nz_mem;      /* schedulercache nonzeroRequest delta */
  uint32_t flags_set, flags_clear; /* KB_NODE_* (e.g. KB_NODE_REL_HAS_MAP when Releasing gains a scalar map) */
  int32_t spec;                /* -1: no inter-pod affinity updates */
  int32_t kind;                /* KB_PLACE_* (with spec) */
  uint32_t sc_off;             /* UINT32_MAX: no scalar deltas */
  uint32_t port_off, port_cnt;
  int32_t pad;
} kb_row_delta;
int kb_apply(kb_ctx* ctx, const kb_row_delta* deltas, uint32_t k, const int64_t* sc, uint32_t n_sc,
             const kb_port* ports, uint32_t n_ports);

/*
 * Inter-pod affinity table updates for a pod that is not one of the session's pending specs (kb_row_delta.spec
 * cannot name it): a pod bound or deleted by the Go side (schedulercache AddPod / RemovePod reach the
 * InterPodAffinity priority's NodeInfo pods, cache/node_info.go:498-630), or a session task entering or leaving
 * the predicate lister (PodLister.UpdateTask, plugins/util/util.go:108-130: an eviction makes a Running task
 * Releasing, so it leaves the lister but stays on its node). table >= 0: the count table's counter at the node's
 * domain of the table's slot (none when the node has no domain there) and the table's total, both += weight.
 * table == -1: the InterPodAffinity histogram entry h[h_off + the node's domain of `slot`] += weight.
 * scheduler_amd/affinity.py Tables.pod_deltas derives the entries from the pod's labels and terms; a pod whose
 * terms would need a table or histogram the session's specs do not have is refused there (re-export instead).
 */
typedef struct kb_aff_delta {
  int32_t node;   /* canonical index */
  int32_t table;  /* count table id, or -1: a histogram entry */
  int32_t slot;   /* histogram: its topology slot (single-key) */
  uint32_t h_off; /* histogram: its offset into kb_affinity.h */
  int32_t weight;
  int32_t pad;
} kb_aff_delta;
int kb_apply_affinity(kb_ctx* ctx, const kb_aff_delta* deltas, uint32_t k);

/*
 * Called by kb_allocate when a task of a spec with host-evaluated stages (an overlay, or KB_AFF_ERROR
 * checks) fits no node: node_reasons[i] is node i's reason mask at the failing task's state (what
 * kb_eval returns there), so the caller can replace the KB_R_HOST_ERROR bucket of the job's histogram
 * with its own per-node strings (FitErrors.SetNodeError, api/unschedule_info.go:40-54). n_events = the
 * cycle's placements made before the failure (kb_cycle_result.event_task order).
 */
typedef void (*kb_nofit_fn)(void* user, int32_t job, int32_t task, uint32_t n_events, const uint32_t* node_reasons,
                            uint32_t n);
int kb_set_nofit_hook(kb_ctx* ctx, kb_nofit_fn fn, void* user);

/*
 * ---- node sharding across GPUs ----
 * The canonical node table is split into contiguous blocks, one per rank (one process per GPU). Every
 * rank uploads only its block (kb_upload_nodes with those rows) plus every spec, and every rank runs the
 * same allocate loop. Per run segment (<= 100 tasks of one spec) each rank proposes its own best picks
 * (the selection path), the ranks exchange the proposals with ONE all-gather (1280 B per rank), and every
 * rank merges them into the same global pick order, applies the stop rules and commits the picks that
 * land on its own rows -- the same placements as one GPU holding the whole table. Node indices in
 * placements are global. Only selection-path jobs (32-bit keys, no inter-pod affinity) run sharded;
 * others return KB_E_UNSUPPORTED. Call before kb_upload_nodes.
 */
typedef struct kb_shard {
  uint32_t n_total;    /* nodes in the whole session */
  uint32_t node_begin; /* this rank's first canonical node */
  int32_t rank, world; /* world <= 16 */
} kb_shard;
/* Host-staged exchange: copy `bytes` from send into recv + r * bytes for every rank r (host memory). */
typedef int (*kb_allgather_fn)(void* user, const void* send, void* recv, size_t bytes);
int kb_set_shard(kb_ctx* ctx, const kb_shard* shard, kb_allgather_fn fn, void* user);
/* Device exchange over RCCL (xGMI): rank 0 makes the id, every rank passes the same bytes. */
#define KB_COMM_ID_BYTES 128
int kb_comm_unique_id(uint8_t id[KB_COMM_ID_BYTES]);
int kb_set_shard_rccl(kb_ctx* ctx, const kb_shard* shard, const uint8_t id[KB_COMM_ID_BYTES]);
/* Device exchange between the ranks' resident engines (ABI 12): every rank's inbox lives in its own GPU's memory
 * and is mapped into every other rank's GPU (IPC handles, all-gathered once through fn); per job each rank's
 * engine writes its proposal into every inbox over xGMI and merges all of them from its own, with no host or
 * collective launch on the path. kb_allocate cycles whose jobs are all fed-engine runs (one <= 100-task selection
 * run each, no inter-pod terms) take it; other jobs use fn as kb_set_shard's host-staged exchange, unpipelined.
 * Replaces the per-task argmax all-reduce of SURVEY.md §8 e1 (scheduler_helper.go:147-158 over every rank's
 * nodes); ranks must run the same cycles (a divergence fails with KB_E_STATE). */
int kb_set_shard_peer(kb_ctx* ctx, const kb_shard* shard, kb_allgather_fn fn, void* user);
/* ABI 14: before it returns, kb_set_shard_peer checks the path every cycle will take. For every peer on another GPU,
 * hipDeviceCanAccessPeer (the peer's GPU found by its PCI bus id); then a tagged-word round trip through every opened
 * inbox: each rank stores a word into every peer's inbox from its GPU (system scope, as the engine's records go),
 * the ranks meet in fn, each reads the words in its own inbox and answers every peer with a second word, and the
 * ranks meet again and check the answers. The outcome is all-gathered, so every rank fails alike: KB_E_HIP (no
 * peer access) or KB_E_STATE (a word missing or wrong), naming the rank pair. kb_stats.peer_checks counts the
 * words that passed. */

/* ---- layer 2: session (allocate action + ordering plugins on the host) ---- */

/* plugin bits of a tier entry */
#define KB_PLUGIN_PRIORITY 0
#define KB_PLUGIN_GANG 1
#define KB_PLUGIN_DRF 2
#define KB_PLUGIN_PROPORTION 3
#define KB_PLUGIN_PREDICATES 4
#define KB_PLUGIN_NODEORDER 5
#define KB_PLUGIN_CONFORMANCE 6
#define KB_PLUGIN_OTHER 7

/* enable bits (conf.PluginOption, conf/scheduler_conf.go:37-56) */
#define KB_EN_JOB_ORDER (1u << 0)
#define KB_EN_JOB_READY (1u << 1)
#define KB_EN_JOB_PIPELINED (1u << 2)
#define KB_EN_TASK_ORDER (1u << 3)
#define KB_EN_PREEMPTABLE (1u << 4)
#define KB_EN_RECLAIMABLE (1u << 5)
#define KB_EN_QUEUE_ORDER (1u << 6)
#define KB_EN_PREDICATE (1u << 7)
#define KB_EN_NODE_ORDER (1u << 8)

typedef struct kb_tier_plugin {
  int32_t tier;    /* tier index (order = position in the array) */
  int32_t plugin;  /* KB_PLUGIN_* */
  uint32_t enable; /* KB_EN_* */
  int32_t pad;
} kb_tier_plugin;

/* task status (api/types.go:23-61) */
#define KB_ST_PENDING (1 << 0)
#define KB_ST_ALLOCATED (1 << 1)
#define KB_ST_PIPELINED (1 << 2)
#define KB_ST_BINDING (1 << 3)
#define KB_ST_BOUND (1 << 4)
#define KB_ST_RUNNING (1 << 5)
#define KB_ST_RELEASING (1 << 6)
#define KB_ST_SUCCEEDED (1 << 7)
#define KB_ST_FAILED (1 << 8)
#define KB_ST_UNKNOWN (1 << 9)

/*
 * Resources for drf/proportion accounting use the reference's float64 Resource
 * with presence semantics: R = 2 + n_rscalar columns (cpu, memory, scalars by
 * slot) plus a presence mask (bit 63 = map non-nil, bit s = scalar slot s present).
 */
typedef struct kb_session {
  uint32_t n_rscalar;          /* scalar slots used for accounting (<= 62) */
  /* tasks of session jobs */
  uint32_t n_tasks;
  const int32_t* task_job;
  const int32_t* task_spec;    /* device spec id (pending tasks), -1 otherwise */
  const int32_t* task_status;  /* KB_ST_* */
  const int32_t* task_priority;
  const int64_t* task_ctime;   /* pod creation timestamp */
  const int32_t* task_uid_rank;/* rank of the task UID in byte order */
  const double* task_resreq;   /* [n_tasks][2 + n_rscalar] Resreq */
  const uint64_t* task_resreq_mask;
  /* jobs */
  uint32_t n_jobs;
  const int32_t* job_queue;
  const int32_t* job_priority;
  const int32_t* job_min_available;
  const int64_t* job_ctime;
  const int32_t* job_uid_rank;
  const int32_t* job_pg_pending; /* PodGroup phase Pending: skipped (allocate.go:50-52) */
  /* queues */
  uint32_t n_queues;
  const int32_t* queue_weight;
  const int64_t* queue_ctime;
  const int32_t* queue_uid_rank;
  /* sum of session nodes' Allocatable (drf.go:62-64, proportion.go:60-62) */
  const double* total_alloc;   /* [2 + n_rscalar] */
  uint64_t total_alloc_mask;
  /* tiers */
  uint32_t n_tier_plugins;
  const kb_tier_plugin* tier_plugins;
} kb_session;

typedef struct kb_cycle_result {
  int32_t* task_node;      /* [n_tasks] node index or -1 */
  int32_t* task_status;    /* [n_tasks] final status */
  int32_t* job_fail_task;  /* [n_jobs] task index that fit nowhere, -1 */
  uint32_t* job_reason_hist; /* [n_jobs][KB_NUM_REASONS] */
  int32_t* event_task;     /* [n_tasks] placement order: task index */
  uint32_t n_events;       /* out */
  int32_t pad;
  double elapsed_ms;       /* out: allocate action wall time */
  double device_ms;        /* out: time inside kb_place_job calls */
} kb_cycle_result;

/* allocateAction.Execute (actions/allocate/allocate.go:42-193) over the uploaded node table. */
int kb_allocate(kb_ctx* ctx, const kb_session* ssn, kb_cycle_result* out);

#ifdef __cplusplus
}
#endif
#endif /* KBGPU_H_ */
