// kb_ctx: one device-resident session snapshot.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <string>
#include <vector>

#include "kbgpu_device.h"

struct kb_ctx {
  int device = 0;
  bool broken = false;
  hipStream_t stream = nullptr;
  std::string err;

  kbgpu::DevNodes N{};
  kbgpu::DevSpecs P{};
  kbgpu::DevCfg cfg{};
  bool nodes_ok = false, specs_ok = false;
  int64_t max_pref_weight = 0;

  std::vector<void*> node_mem, spec_mem, work_mem, aff_mem;
  // inter-pod affinity (kb_upload_affinity)
  bool aff_ok = false;
  std::vector<char> spec_needs_aff;  // per spec: KB_SPEC_POD_AFFINITY / aff_class set
  std::vector<char> spec_dyn;   // per spec: KB_AFF_SELF_DYNAMIC -> block-wide re-sweep loop
  std::vector<char> spec_hist;  // per spec: has InterPodAffinity histograms
  std::vector<char> spec_incr;  // per spec: its commits update affinity tables
  std::vector<char> spec_aff_reg;  // per spec: its entry count when the register-resident loop takes it, else 0
  std::vector<char> spec_cap1;     // per spec: kSpecCap1 (a selection run with at most one Allocate per node)
  std::vector<int32_t> spec_cls;   // per spec: the class loop's finest dynamic slot (-1: not eligible)
  std::vector<int64_t> aff_slot_D;  // per topology slot: its domain count
  // per spec: its feasibility class (kb_upload_specs; -1: inter-pod terms, no class) and InitResreq (cpu, mem, then
  // the scalar slots; spec_init_mask the slots present): the driver's NO_FIT prediction (kbgpu_allocate.cpp)
  std::vector<int32_t> spec_fclass;
  std::vector<int32_t> spec_fparent;  // [m][3]: the classes with the selector / required terms / both dropped (-1)
  std::vector<int64_t> spec_init;
  std::vector<uint64_t> spec_init_mask;
  int32_t n_fclass = 0;
  std::vector<char> spec_rowcols;  // per spec: it reads scalar / host-port columns (the fed engine's acquire, FedCmd::acq)
  std::vector<int32_t> spec_aff_class0;  // per spec: aff_class as kb_upload_specs got it (kb_upload_affinity marks
                                         // specs with an empty affinity entry -1: they run as plain specs)
  uint32_t aff_n_tables = 0, aff_n_h = 0;  // kb_apply_affinity's bounds
  uint64_t* cls_lvl = nullptr;  // [kClsLevels][n] class loop scratch: keys after 1..kClsLevels commits
  int32_t* cls_amax = nullptr;  // [n] class loop scratch: Allocates before Idle stops fitting
  uint64_t* cls_cbest = nullptr;  // [kClsMaxK] class loop: each class's best base key (sweep -> place kernel; 0 between)
  // per topology slot that is some spec's class slot: its classes as member lists (offsets [K + 1], node ids
  // by class [n]; device copies in aff_mem), else null
  std::vector<uint32_t*> cls_coff;
  std::vector<uint16_t*> cls_mem;
  bool use_cap1 = true, use_cls = true;  // KB_NO_CAP1 / KB_NO_CLS unset
  bool cap1(int spec) const { return use_cap1 && spec < (int)spec_cap1.size() && spec_cap1[spec]; }
  int cls_slot(int spec) const { return use_cls && spec < (int)spec_cls.size() ? spec_cls[spec] : -1; }
  bool use_aff_reg = true;
  int64_t* mm_eval = nullptr;   // [2 * chunk] per-spec IPA min / max for kb_eval
  uint32_t mm_eval_cap = 0;
  // the fed engine's affinity units (kb_spec_fed_ok): !KB_OPT_FED_NO_AFF; per spec, whether kb_fed_ipa_prepare has
  // filled its InterPodAffinity min / max (DevAff::mm_spec) this cycle (kb_allocate's driver clears and refills them)
  bool use_fed_aff = true;
  std::vector<char> mm_spec_ok;
  int32_t* d_mm_ids = nullptr;  // kb_fed_ipa_prepare's spec list (device)
  uint32_t mm_ids_cap = 0;
  uint64_t* keys = nullptr;  // [n] packed argmax keys of the current spec
  uint64_t* cmax = nullptr;  // [ceil(n/64)] chunk maxima
  uint64_t* stat = nullptr;  // [n] static predicate / NodeAffinity cache of the current spec
  // trajectory path
  uint32_t* traj = nullptr;    // [kTrajMaxJ + 1][n] compressed keys after j commits
  uint32_t* cmax32 = nullptr;  // [ceil(n/64)]
  uint32_t* amax = nullptr;    // [n] allocations before Idle stops fitting
  int idx_bits = 0;
  std::vector<std::vector<uint32_t>> aff_rd, aff_wr;  // per spec: affinity inputs its sweep reads / its commits write
  int prev_run_spec = -1;                              // the listed previous job's spec (aff_sweep_indep)
  std::vector<char> spec_traj_ok;  // per spec: score range fits the 32-bit key
  std::vector<int64_t> spec_pref_weight;
  std::vector<char> spec_ipa_err;   // per spec: KB_SPEC_IPA_ERROR (the batch score errors: 64-bit keys)
  std::vector<char> spec_plain;     // per spec: no selector / node affinity / ports / scalars / inter-pod terms, and
                                    //   one taint set it tolerates (kb_eval's row-only kernel; an overlay excludes it)
  std::vector<char> spec_aff_err;   // per spec: its affinity checks include KB_AFF_ERROR
  // host overlay (kb_set_host_overlay): per spec the slot of its rows (-1 none), per slot the rows
  std::vector<int32_t> ov_slot;
  std::vector<std::vector<uint8_t>> ov_fail;
  std::vector<std::vector<int32_t>> ov_score;
  std::vector<int64_t> ov_absmax;   // per spec: max |score_add| (score-range bound)
  std::vector<char> ov_any_fail;    // per spec: some node is rejected by the overlay
  std::vector<void*> ov_mem;        // device copies (P.ov_slot / ov_fail / ov_score)
  // NO_FIT hook (kb_set_nofit_hook)
  kb_nofit_fn nofit_fn = nullptr;
  void* nofit_user = nullptr;
  bool host_reasons(int spec) const {  // the NO_FIT histogram of this spec has host-evaluated buckets
    return (spec < (int)ov_any_fail.size() && ov_any_fail[spec]) ||
           (spec < (int)spec_aff_err.size() && spec_aff_err[spec]);
  }
  bool use_traj = true, use_sel = true, use_engine = false;
  // persistent placement engine (the selection path as one resident workgroup)
  bool eng_running = false;
  hipStream_t eng_stream = nullptr;
  hipEvent_t eng_dep = nullptr;  // orders the engine after work already queued on `stream`
  char* h_cmd = nullptr;         // pinned mailbox: EngineCmd + EngineRun[cmd_cap]
  char* h_cmd_dev = nullptr;
  uint32_t cmd_cap = 0;
  // node sharding (kb_set_shard / kb_set_shard_rccl)
  bool sharded = false;
  kb_shard shard{};
  kb_allgather_fn ag_fn = nullptr;
  void* ag_user = nullptr;
  void* comm = nullptr;            // ncclComm_t when the exchange is RCCL
  kbgpu::ShardRec* d_rec = nullptr;     // this rank's proposal
  kbgpu::ShardRec* d_rec_all = nullptr; // [world] all proposals
  kbgpu::ShardRec* h_rec = nullptr;     // host staging (host exchange): [1 + world]
  // kb_set_shard_peer: the node-sharded fed engine's inboxes (this rank's allocation, and every rank's as this GPU
  // addresses it: IPC-mapped for the peers), and the cycle counter its tags carry
  bool peer = false;
  void* inbox = nullptr;
  void* peer_inbox[kbgpu::kShardMaxWorld] = {};
  uint32_t shard_epoch = 0;
  uint32_t shard_epoch0 = 0;  // kb_opts.shard_epoch0 (tests)
  bool traj_full = false;  // trajectory buffers (kTrajMaxJ + 1 levels): chunk maxima fit the place loop
  bool sel_ok = false;     // the node count fits the selection kernel's LDS plan (level-0 keys buffer)
  char* d_job = nullptr;     // device JobState (chains the runs of one job)
  uint32_t seq = 0;           // place launches issued (JobState::seq)
  char* h_job = nullptr;     // pinned host JobState + placement pairs (written by the place kernel)
  char* h_job_dev = nullptr; // device address of h_job
  uint32_t job_cap = 0;
  // Job slots of the pipelined driver (kb_allocate): slot 0 = d_job / h_job above, slots 1.. below. The
  // driver issues job k+1 into a free slot, guarded on job k's predicted outcome, before reading job k (the
  // per-job launch path: two slots; the fed engine: kJobSlots, two speculative jobs ahead).
  struct JobSlot {
    char *d = nullptr, *h = nullptr, *hdev = nullptr;
    uint32_t seq = 0;        // sequence number the slot's last launch reports
    size_t ev_b = 0, ev_e = 0;  // its timing events in `pending`
    bool busy = false;
    std::chrono::steady_clock::time_point t_issue;
    double issue_ms = 0;
    // the spec whose affinity-table commit (aff_commit_kernel) the slot's last job queued after its final place
    // kernel, -1 none: that commit may still run after the host has read the job (the place kernel publishes
    // first), so a later sweep that reads those tables must not overlap it (place_issue)
    int aff_tail_spec = -1;
  };
  JobSlot slot[kbgpu::kJobSlots];
  char* d_jobx[kbgpu::kJobSlots] = {};  // slots 1..: device / pinned host job state (+ placements)
  char* h_jobx[kbgpu::kJobSlots] = {};
  uint32_t jobx_cap[kbgpu::kJobSlots] = {};
  bool any_busy() const {
    for (const JobSlot& s : slot)
      if (s.busy) return true;
    return false;
  }
  uint64_t issue_count = 0;
  // Selection runs of the pipelined driver use per-slot level-0 keys / static cache / commit lists, so the
  // level-0 sweep of job i can run on stream_b while job i-1's place kernel runs on `stream`; job i then
  // re-keys the rows job i-1 committed, from that job's commit list. Every job before job i-1 has been
  // read back by the host when job i is issued (two slots), so the sweep needs no stream dependency; the
  // place kernel waits on sweep_ctr[slot] reaching sweep_target[slot] (device counter, no events).
  uint32_t* sel_keys[kbgpu::kJobSlots] = {};
  uint32_t* sel_lvl[kbgpu::kJobSlots] = {};  // the resident sweepers' level records (kb_fed_begin, lazily)
  uint64_t* sel_stat[kbgpu::kJobSlots] = {};
  int32_t* commits[kbgpu::kJobSlots] = {};
  int32_t sel_n = -1;       // node count the per-slot buffers were sized for
  uint32_t commits_cap = 0;
  hipStream_t stream_b = nullptr;
  uint32_t* sweep_ctr = nullptr;  // [2] device counters
  uint32_t sweep_target[2] = {0, 0};
  // fed engine (kb_fed_begin / kb_fed_end): one resident selection workgroup per allocate cycle, fed by the
  // sweep kernels through a kJobSlots-entry device ring; fed_count[r]: blocks counted into fed_ctr[r] so far
  bool fed = false;
  bool use_fed = true;         // !KB_OPT_NO_FED
  bool use_eval_plain = true;  // !KB_OPT_NO_EVAL_PLAIN
  void* fed_ring = nullptr;
  uint32_t* fed_ctr = nullptr;
  int32_t* fed_exit = nullptr;
  void* fed_xchg = nullptr;   // split engine exchange (fed_xchg_bytes)
  uint64_t* h_fed_ctrs = nullptr;  // pinned: the placer's counters at the end of fed_xchg, copied at kb_fed_end
  bool use_fed_split = true;  // !KB_OPT_NO_FED_SPLIT
  bool fed_split_now = false;  // the running fed cycle is on the split engine (its FedXchg counters)
  // kb_fed_pause: the engine idles between two commands while launch-path units run on stream_alt (swapped into
  // `stream` for the pause); the first command after kb_fed_resume is flagged fresh (FedCmd::fresh)
  bool fed_paused = false, fed_fresh = false;
  hipStream_t stream_alt = nullptr;
  // The resident engine waits for sweeps issued on stream_b: they must never queue behind it on one hardware queue.
  // stream_b is a CU-masked stream (a hardware queue of its own, never shared with other streams of the process),
  // and the engine a plain launch whose every workgroup fits the device at once (launch_fed_engine checks the
  // occupancy first). KB_OPT_FED_SHARED_QUEUES (tests): a plain stream_b, the hazard the dedicated queue removes.
  bool fed_dedicated = true;
  bool fed_coop = false;  // KB_OPT_FED_COOP_LAUNCH (A/B only): the default is a plain launch + residency check
  // kb_opts.fed_depth: the engine's units in flight, 2..kJobSlots (0: the driver's per-cycle choice, kbgpu_allocate.cpp)
  int fed_depth = 0;
  // kb_opts.fed_xcc - 1: the split engine's XCC (-1: the dispatcher's placement). Default XCC 0: measured on C2
  // (r05c), the placer and selector on XCC 0-3 run 17.0-17.1 us per job, on XCC 4-7 17.6-18.1 us, and a plain
  // launch lands wherever the dispatcher's round robin stands
  int fed_xcc = 0;
  // the split engine's resident sweepers (launch_fed_engine's hring): commands go to a pinned ring (fed_hring,
  // tags fed_epoch << 32 | fed_m + 1) instead of a sweep kernel per job; KB_OPT_FED_KERNEL_SWEEPS turns them off
  bool fed_kernel_sweeps = false, fed_sweepers_now = false;
  bool test_one_xcc = false;  // KB_OPT_TEST_ONE_XCC
  bool no_lvl = false;        // KB_OPT_FED_NO_LEVELS
  void* fed_hring = nullptr;      // pinned host ring (kJobSlots FedHostCmd)
  void* fed_hring_dev = nullptr;  // its device address
  uint32_t fed_epoch = 0, fed_m = 0;
  uint32_t fed_cmd_m = 0, fed_fresh_m = 0;  // commands posted this launch; the last fresh one's index (FedCmd::fresh_m)
  // tests only (kb_opts.test_stall_job / test_stall_ms): kb_allocate's driver sleeps before
  // finishing job test_stall_job, a host stall longer than the engine's idle bound
  int64_t test_stall_job = -1;
  int test_stall_ms = 1500;
  bool use_pipeline = true;    // !KB_OPT_NO_PIPELINE
  bool shard_self_inbox = false;  // KB_OPT_SHARD_SELF_INBOX
  bool test_peer_badtag = false;  // KB_OPT_TEST_PEER_BADTAG
  bool fed_diag = false;       // KB_OPT_FED_DIAG
  // KB_OPT_FED_DIAG: host stamps per fed command (ns since kb_fed_begin): issue entry / exit, finish entry /
  // result seen (kb_fed_end's kb_fed_host line, beside the engine's per-job timeline)
  std::vector<int64_t> dg_iss0, dg_iss1, dg_fin0, dg_fin1;
  std::chrono::steady_clock::time_point dg_t0;
  bool issue_trace = false;    // KB_HOST_TRACE: every fed job issue on stderr
  uint64_t fed_idle = 100000000ull;  // the engine's idle exit in s_memrealtime ticks (100 MHz): 1 s
  int eval_spb = 0;            // kb_opts.eval_spb (0: from cus)
  int cus = 256;               // compute units of the context's device
  int eval_bpc32 = 2, eval_bpc64 = 2;  // eval_plain_kernel's resident blocks per CU (kb_eval32 / kb_eval instance)
  uint32_t fed_count[kbgpu::kJobSlots] = {};
  int fed_r = 0;
  uint64_t fed_tasks = 0;  // tasks the engine placed or tried this session (timing pairs)
  hipEvent_t fed_ev = nullptr;
  bool prev_listed = false; // the last issued job was one selection run that lists its commits
  int prev_slot = -1;
  uint64_t n_overlap = 0;   // sweeps that ran overlapped
  int32_t fed_exit_code = 0;   // the engine's exit flag when it left early (wait_seq)
  uint64_t n_fed_abandon = 0;  // cycles finished on the launch path after the engine idled out
  char* h_eval = nullptr;
  void *eval_ids = nullptr, *eval_r = nullptr, *eval_s = nullptr;  // kb_eval's device buffers (persistent)
  size_t eval_cap = 0;        // pairs the output buffers hold
  uint32_t eval_ids_cap = 0;

  double device_ms = 0;  // wall time inside kb_place_job

  // pristine copies of the mutable node columns (kb_restore_nodes)
  struct Col { void* dst; void* src; size_t bytes; };
  std::vector<Col> pristine, aff_pristine;

  // kernel timing (KB_OPT_TIMING)
  bool timing = false;
  uint32_t timing_every = 1;  // sample the launches of every Nth kb_place_job call
  bool timing_now = false;
  std::vector<hipEvent_t> ev_pool;
  struct Pending { hipEvent_t a, b; int kind; uint64_t pairs; };
  std::vector<Pending> pending;
  kb_stats stats{};
  hipEvent_t ev_get();
  void ev_begin(hipEvent_t* a, hipStream_t s = nullptr);  // nullptr: `stream`
  void ev_end(hipEvent_t a, int kind, uint64_t pairs, hipStream_t s = nullptr);
  size_t ev_collect(bool all, size_t limit = (size_t)-1);  // returns the event pairs it folded
  size_t pending_job_begin = 0;  // first pending event pair of the current kb_place_job call
};

// internal helpers (defined inside kbgpu_host.cpp's extern "C" block, not part of the ABI)
extern "C" __attribute__((visibility("hidden"))) int kb_check_score_range(kb_ctx* c);
extern "C" __attribute__((visibility("hidden"))) void kb_update_traj_ok(kb_ctx* c);
// stops the placement engine (if running) before other work touches the device state
extern "C" __attribute__((visibility("hidden"))) int kb_engine_stop(kb_ctx* c);
// per-node reason masks of one spec at the current node-table state (kb_eval without scores), for the
// NO_FIT hook of kb_allocate's driver
extern "C" __attribute__((visibility("hidden"))) int kb_node_reasons(kb_ctx* c, int spec, uint32_t* reasons);

// Pipelined placement for kb_allocate's driver (kbgpu_host.cpp). kb_job_pipeline_ok: the context runs
// jobs through the launch paths (not sharded, no engine). kb_job_guardable: every task of the job takes
// the selection path, whose first launches can carry a SpecGuard. kb_job_issue launches the job into
// `slot`; with `pred` set it runs only if the job of slot pred->prev_slot ended with exactly
// (stop, placed, ready). kb_job_reserve sizes both slots beforehand. kb_job_finish waits for the slot and
// reads its result (skipped: the caller knows the guard failed and only drains the slot).
struct kb_job_pred {
  int prev_slot;
  int32_t stop, placed, ready;
};
extern "C" __attribute__((visibility("hidden"))) int kb_job_pipeline_ok(kb_ctx* c);
extern "C" __attribute__((visibility("hidden"))) int kb_job_guardable(kb_ctx* c, const kb_job_req* job);
extern "C" __attribute__((visibility("hidden"))) int kb_job_reserve(kb_ctx* c, uint32_t max_tasks);
// Fed engine for a cycle whose jobs are all one selection run of a spec without inter-pod terms
// (kb_spec_fed_ok): kb_fed_begin after kb_job_reserve, then kb_job_issue / kb_job_finish as usual (each
// issue launches only the job's sweep kernel), kb_fed_end before anything else runs on the context.
extern "C" __attribute__((visibility("hidden"))) int kb_spec_fed_ok(kb_ctx* c, int spec);
// Affinity units on the engine (kb_spec_fed_ok takes specs with inter-pod terms whose sweep folds them in). A spec with
// InterPodAffinity histograms needs its min / max over the nodes as the cycle has them: kb_fed_ipa_prepare computes
// them for `n` specs into DevAff::mm_spec (on `stream`, before kb_fed_begin), and kb_spec_fed_ok refuses such a spec
// until then -- kb_spec_fed_ok_pre answers as if it were prepared (the driver's pending-list pass). The driver keeps
// the min / max exact: it prepares only specs whose histograms no unit of the cycle writes. kb_fed_units_indep: the
// commits of a unit of spec a leave every input of a sweep of spec b alone (b may be in flight behind a).
extern "C" __attribute__((visibility("hidden"))) int kb_spec_fed_ok_pre(kb_ctx* c, int spec);
extern "C" __attribute__((visibility("hidden"))) int kb_fed_ipa_prepare(kb_ctx* c, const int32_t* specs, uint32_t n);
extern "C" __attribute__((visibility("hidden"))) int kb_fed_units_indep(const kb_ctx* c, int a, int b);
// the engine can serve a cycle whose jobs have at most max_job_tasks tasks (past one selector's key plan only the
// split engine, whose jobs are one segment)
extern "C" __attribute__((visibility("hidden"))) int kb_fed_cycle_ok(kb_ctx* c, uint32_t max_job_tasks);
// the most tasks one engine command may carry: kFedSplitMaxTasks when the cycle would take the split engine, else 0
// (no bound: the one-workgroup engine runs any number of segments per command)
extern "C" __attribute__((visibility("hidden"))) uint32_t kb_fed_unit_cap(kb_ctx* c);
// max_job_tasks: the most tasks any job of the cycle can place (the split engine takes one-segment jobs only)
extern "C" __attribute__((visibility("hidden"))) int kb_fed_begin(kb_ctx* c, uint32_t max_job_tasks);
extern "C" __attribute__((visibility("hidden"))) int kb_fed_end(kb_ctx* c);
// Launch-path units between two engine commands without ending the engine (nothing may be in flight either way)
extern "C" __attribute__((visibility("hidden"))) int kb_fed_pause(kb_ctx* c);
extern "C" __attribute__((visibility("hidden"))) int kb_fed_resume(kb_ctx* c);
// kb_job_finish's code when the resident engine idled out before serving the job (see kb_fed_abandon)
constexpr int kFedIdleExit = -100;
extern "C" __attribute__((visibility("hidden"))) int kb_fed_abandon(kb_ctx* c);
extern "C" __attribute__((visibility("hidden"))) int kb_job_issue(kb_ctx* c, const kb_job_req* job, int slot,
                                                                  const kb_job_pred* pred);
extern "C" __attribute__((visibility("hidden"))) int kb_job_finish(kb_ctx* c, int slot, int32_t* placed_node,
                                                                   int32_t* placed_kind, kb_job_result* result,
                                                                   int skipped);
