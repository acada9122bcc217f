// Device-side data layout shared by the HIP kernels and the host library.
#pragma once
#include <stdint.h>

#include "../../include/kbgpu.h"

namespace kbgpu {

// Packed argmax key:
//   feasible:   bit 63 = 1 | (score + kScoreBias) << 24 | (2^24 - 1 - node)
//   infeasible: bit 63 = 0 | reason mask (bits 0..15)
// max(key) = highest score, then lowest node index (the canonical tie-break).
constexpr uint64_t kFeasible = 1ull << 63;
constexpr int64_t kScoreBias = 1ll << 38;
constexpr uint32_t kIdxMask = (1u << 24) - 1;
constexpr uint32_t kMaxNodes = 1u << 24;

// Internal kb_spec.flags bits, set on the device copy by kb_upload_affinity (never part of the ABI).
// kSpecCap1: the spec's only self-dependent affinity input is a required anti-affinity check over
// single-node domains (hostname): after one Allocate of the spec on a node (a Pipelined task does not join
// the lister) the check fails there, and nothing else moves. Its run is a selection run whose levels j >= 1
// fail once A >= 1, with the reason of the first such check (kSpecCapAnti: "didn't match pod anti-affinity
// rules", else "didn't satisfy existing pods anti-affinity rules").
constexpr uint32_t kSpecCap1 = 1u << 30;
constexpr uint32_t kSpecCapAnti = 1u << 29;
// Class loop (cls_place_kernel): at most kClsE histograms per spec, kClsU of its own histogram increments
// per commit, kClsMaxK classes (the F-domains + one class for the nodes without one).
constexpr int kClsE = 4;
constexpr int kClsU = 8;
constexpr int kClsMaxK = 1024;

struct DevNodes {
  int32_t n, S, K, P;
  int32_t base;  // canonical index of row 0 (node sharding across GPUs; 0 on one GPU)
  int32_t pad;
  int64_t *idle_cpu, *idle_mem, *rel_cpu, *rel_mem;
  int64_t *idle_sc, *rel_sc;
  int64_t *alloc_cpu, *alloc_mem;
  int64_t *nz_cpu, *nz_mem;
  int32_t *pod_count, *max_pods;
  uint32_t* flags;
  int32_t* label_val;
  int64_t* label_int;
  uint8_t* label_int_ok;
  int32_t* taint_set;
  uint64_t* port_used;
};

// Inter-pod affinity tables (kb_affinity). enabled == 0: none uploaded (no spec refers to them).
struct DevAff {
  int32_t enabled;
  int32_t n;            // nodes (topo_dom row length)
  int32_t* topo_dom;    // [slots][n]
  kb_aff_table* tables;
  int32_t* totals;      // mutable
  int32_t* counters;    // mutable
  kb_aff_spec* specs;
  kb_aff_check* checks;
  int32_t* lister;
  kb_ipa_hist* hists;
  int32_t* h;           // mutable
  kb_ipa_incr* incr;
  int64_t* mm;          // [2] InterPodAffinity min / max count of the current run's spec
  int64_t* mm_spec;     // [2 x specs] the same per spec, for the fed engine's sweeps (kb_fed_ipa_prepare)
};

struct DevSpecs {
  DevAff A;
  // host overlay (kb_set_host_overlay): ov_slot[spec] = row of ov_fail / ov_score, -1 none (ov_slot null: none)
  int32_t* ov_slot;
  uint8_t* ov_fail;   // [slots][n]
  int32_t* ov_score;  // [slots][n]
  kb_spec* specs;
  int64_t *sc_init, *sc_req;
  kb_term* terms;
  kb_req* reqs;
  int32_t* vals;
  kb_port* ports;
  uint8_t* tolerates;
  int32_t n_taint_sets;
  int32_t m;
};

struct DevCfg {
  int32_t predicates, nodeorder, mem_pressure, disk_pressure, pid_pressure;
  int32_t w_lr, w_bra, w_na, w_pa;
};

// Per-job device state (one per context), read back after every kb_place_job.
struct JobState {
  int32_t stopped;    // 1 once the batch stopped; later kernels of the batch exit at entry
  int32_t stop;       // KB_STOP_*
  int32_t fail_task;
  int32_t n_placed;
  int32_t ready_num;
  int32_t min_available;
  int32_t gang_ready;
  int32_t panic;      // 1: SelectBestNode would panic (best score <= -1)
  uint32_t hist[KB_NUM_REASONS];
  uint64_t diag[8];   // -DKB_DIAG builds: per-phase shader cycles of the place loop, [7] = realtime ticks
  uint64_t t_recv, t_done;  // placement engine: s_memrealtime (100 MHz) at command receipt / completion
  uint32_t exit_seq;  // placement engine: the command it was waiting for when it exited idle (0: none)
  int32_t n_commit;   // selection place kernel: rows in its commit list (device copy only)
  int32_t stall;      // host copy: 1 = the place kernel gave up waiting for its overlapped sweep; 2 = node-sharded
                      //   ranks exchanged different segments (ShardRec::tag)
  uint32_t seq;       // host copy: sequence number of the last finished place launch (written last)
};

// Speculative issue (kb_allocate's driver): a job launched before the previous job's result is known runs
// only if that job ended as predicted; otherwise every kernel of the speculative job is a no-op.
struct SpecGuard {
  const JobState* prev;  // nullptr: no guard
  int32_t stop, placed, ready;
};

// Node sharding (kb_set_shard): one rank's proposal for a run segment, exchanged by an all-gather.
constexpr int kShardSegMax = 100;  // == the selection path's segment length (kSegMax)
struct ShardRec {
  int32_t kp;                      // proposals (feasible picks, best first)
  int32_t pad;
  uint32_t hist[KB_NUM_REASONS];   // reason histogram of this rank's rows after all kp picks (kp < T only)
  int32_t pad1;
  uint64_t comp[kShardSegMax];     // pick-order composites (global node index inside)
  int32_t node_kind[kShardSegMax]; // global node | kind << 30
  // what the rank issued for this segment (launch sequence number, spec, segment start << 16 | tasks, guard
  // prediction hash | skipped << 31): every rank must exchange the same tag, else the ranks diverged
  uint32_t tag[4];
};
static_assert(sizeof(ShardRec) % 16 == 0, "ShardRec is exchanged as raw bytes");

// Placement engine mailbox (pinned host memory, written by the host): one command per kb_place_job.
#define KB_ENG_RUN 1
#define KB_ENG_EXIT 2
#define KB_ENG_EXIT_IDLE 3
struct EngineRun {
  int32_t spec, t_begin, t_count, pad;
};
struct EngineCmd {
  uint32_t seq;  // written last (release): the engine starts on seq == the number it waits for
  int32_t op;    // KB_ENG_RUN / KB_ENG_EXIT
  int32_t n_runs, ready0, minav0, gang0;
  int32_t pad[2];
  // EngineRun runs[n_runs] follow
};

// Launch wrappers (kbgpu_device.hip).
void launch_sweep_keys(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, uint64_t* keys,
                       uint64_t* cmax, uint64_t* stat, const JobState* js, bool aff, void* stream);
void launch_place_loop(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                       uint64_t* keys, const uint64_t* cmax, const uint64_t* stat, JobState* js, int first,
                       int ready0, int minav0, int gang0, int32_t* hout, JobState* hjs, uint32_t seq, void* stream);
// plain: every spec of the batch is plain (kb_ctx::spec_plain): the row-only kernel (eval_plain_kernel)
// cus: the device's compute units | the plain kernel instance's resident blocks per CU << 16 (its grid is one
// resident round); spb > 0 overrides its specs per block (measurement)
int eval_plain_blocks_per_cu(bool i32);
void launch_eval(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const int32_t* spec_ids, int t,
                 uint32_t* reasons, int64_t* scores, const int64_t* mm, bool plain, int cus, int spb, void* stream);
void launch_eval32(const DevNodes& N, const DevSpecs& P, const DevCfg& C, const int32_t* spec_ids, int t,
                   uint32_t* reasons, int32_t* scores, const int64_t* mm, bool plain, int cus, int spb,
                   void* stream);
int place_loop_lds_bytes(int n);
// trajectory path
constexpr int kTrajMaxJ = 64;
constexpr int kTrajDefaultJ = 16;  // trajectory depth per run; deeper commits are computed in place
// Inter-pod affinity (kbgpu_device.hip): min / max InterPodAffinity count over all nodes for each of
// `count` specs (spec_ids, or the single `spec` when spec_ids is null) into mm[2 * i] (by_spec: mm[2 * spec], the
// per-spec array DevAff::mm_spec), and the block-wide re-sweep place loop for specs whose own commits change their
// affinity inputs.
void launch_ipa_minmax(const DevNodes& N, const DevSpecs& P, const int32_t* spec_ids, int spec, int count,
                       int64_t* mm, const JobState* js, void* stream, int by_spec = 0);
void launch_aff_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                      uint64_t* base, uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0,
                      int32_t* hout, JobState* hjs, uint32_t seq, void* stream);
// The same loop with every thread's nodes (base keys, domain ids) held for the whole run; n <= 10240 and at
// most 4 checks + histograms per spec (ne of them), 8 table updates per commit (aff_reg_npt(n) < 0: use
// launch_aff_place).
int aff_reg_npt(int n);
bool aff_reg_fits(int n, int ne);
void launch_aff_reg(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int ne, int t_begin,
                    int t_count, uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0,
                    int32_t* hout, JobState* hjs, uint32_t seq, void* stream);
// The class loop for specs whose own commits move only their histograms (kbgpu_host.cpp
// classify_self_dynamic): F = the finest moving slot, K = its domain count + 1. cls_fits: the LDS plan
// holds n nodes and K classes. The kernel applies the run's global table updates itself.
bool cls_fits(int n, int K);
// Scratch: bk / stat [n], lvl [kClsLevels][n], amax [n] (the chip-wide prologue's base keys, static cache,
// keys after 1..kClsLevels commits, Allocates before Idle stops fitting). coff [K + 1] / mem [n]: slot F's
// classes as member lists (node ids by class, kb_upload_affinity).
constexpr int kClsLevels = 8;
void launch_cls_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int F, int K, int t_begin,
                      int t_count, uint64_t* bk, uint64_t* stat, uint64_t* lvl, int32_t* amax, const uint32_t* coff,
                      const uint16_t* mem, uint64_t* cbest, JobState* js, int first, int ready0, int minav0,
                      int gang0, int32_t* hout, JobState* hjs, uint32_t seq, SpecGuard g, void* stream);

// A fed-engine job command (launch_sel_sweep's `fed` / launch_fed_cmd).
struct FedCmdArgs {
  int32_t op, spec, t_begin, t_count, ready0, minav0, gang0, slot;
  int32_t g_valid, g_stop, g_placed, g_ready;
  uint32_t seq;
  int32_t fresh = 0;  // the first command after a pause (FedCmd::fresh)
  int32_t acq = 0;    // FedCmd::acq
  int32_t fresh_m = 0;  // FedCmd::fresh_m (fed_post fills it in)
};

// Selection path (kbgpu_device.hip): the run's tasks as a parallel top-T selection over the level-0
// keys of launch_sel_sweep. sel_lds_bytes(n) < 0: the node count does not fit its LDS plan.
int sel_lds_bytes(int n);
// A guard (g.prev set) replaces the JobState gate of a job's first run. commit_out: the place kernel lists
// every row it commits (count in js->n_commit); patch / patch_js: the previous job's list, whose rows this
// run re-keys after loading keys32 (its sweep ran concurrently with that job). done_ctr: the sweep's
// blocks each add 1 when their keys are written; wait_ctr / wait_target: the place kernel waits for the
// counter to reach the target first.
// fed / ring (the fed engine): the job's command, written to the ring entry before block 0's release.
void launch_sel_sweep(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int idx_bits, uint32_t* keys32,
                      uint64_t* stat, const JobState* js, bool aff, void* stream,
                      SpecGuard g = SpecGuard{nullptr, 0, 0, 0}, uint32_t* done_ctr = nullptr,
                      const FedCmdArgs* fed = nullptr, void* ring = nullptr);
void launch_sel_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                      int idx_bits, const uint32_t* keys32, const uint64_t* stat, JobState* js, int first, int ready0,
                      int minav0, int gang0, int32_t* hout, JobState* hjs, uint32_t seq, void* stream,
                      SpecGuard g = SpecGuard{nullptr, 0, 0, 0}, int32_t* commit_out = nullptr,
                      const int32_t* patch = nullptr, const JobState* patch_js = nullptr,
                      const uint32_t* wait_ctr = nullptr, uint32_t wait_target = 0, int aff_pl = 0);
// aff_pl: the kernel applies the run's affinity table commits itself (needs sel_aff_pl_fits)
bool sel_aff_pl_fits(int n, int t_count);

// Placement engine (kbgpu_device.hip): the selection path as one persistent workgroup serving the
// commands posted to `cmd` from sequence number seq0 on; exits on KB_ENG_EXIT or after idle_ticks
// (s_memrealtime, 100 MHz) without a command.
void launch_engine(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, uint64_t* stat,
                   const EngineCmd* cmd, JobState* js, JobState* hjs, int32_t* hout, uint32_t seq0,
                   uint64_t idle_ticks, void* stream);

// Fed engine (kbgpu_device.hip): one resident selection workgroup per allocate cycle; each job's sweep
// kernel (launch_fed_cmd, on the sweep stream) also posts the job's command to a kJobSlots-entry device ring and
// counts its blocks in ctr[ring entry]; the engine serves commands in order until an EXIT command (or
// idle_ticks without one: *exit_flag = 1).
// Job slots: the fed engine keeps up to kJobSlots jobs in flight (the running one and three speculative ones:
// a job's sweep may predate the commits of the three before it -- the selector re-keys m-2's and m-3's rows, the
// placer m-1's set); the per-job launch path uses two of them.
constexpr int kJobSlots = 4;  // the fed engine's units in flight: the running one and three speculative ones
struct FedSlotPtrs {
  uint32_t* keys[kJobSlots];
  uint64_t* stat[kJobSlots];
  int32_t* commits[kJobSlots];
  JobState* js[kJobSlots];
  JobState* hjs[kJobSlots];
  int32_t* hout[kJobSlots];
  uint32_t* lvl[kJobSlots];  // the resident sweepers' level records per slot (kLvlW words per node), nullptr: none
};
// the split engine's level records (kbgpu_device.hip fed_sweeper): a node's keys after 1..kPreLevels commits, then A
constexpr int kPreLevels = 7;
constexpr int kLvlW = 8;
size_t fed_ring_bytes();
bool fed_fits(int n);  // the engine's LDS plan fits n nodes
void launch_fed_cmd(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, uint32_t* keys32,
                    uint64_t* stat, const FedCmdArgs& a, void* ring, uint32_t* ctr, bool sweep, void* stream);
// xchg (fed_xchg_bytes(), zeroed): the split engine, a second workgroup choosing each job's candidate nodes
// one job ahead (fed_split_ok(n)); nullptr: one workgroup.
constexpr int kFedSplitMaxTasks = 100;  // one selection segment (kbgpu_device.hip kSegMax)
size_t fed_xchg_bytes();
size_t fed_census_bytes();  // FedXchg's census words, between wdiag and sphase (KB_DIAG's host read)
size_t fed_trace_offset();  // KB_DIAG builds: FedXchg::tl (the per-job timeline), else 0
int fed_trace_jobs();
bool fed_split_ok(int n, bool sharded);
// selector workgroups of the split engine for n nodes (1: one holds every key; up to 4 node ranges past that;
// 0: beyond the engine)
int fed_nsel(int n);
// Node-sharded fed engine (kb_set_shard_peer): per job every rank's placer writes its proposal into every rank's
// inbox (device memory of each GPU, the peers' mapped through IPC handles: stores over xGMI) and merges all of
// them from its own inbox. Inbox: [2 cycle halves][kJobSlots][kShardMaxWorld][kShardRecW] tagged 64-bit words
// (tag = epoch << 20 | job + 1 in the high half, so every word validates itself and needs no store order).
constexpr int kShardMaxWorld = 16;
constexpr int kShardEpochBits = 12;  // of the cycle epoch in an inbox word's tag (the host re-zeroes at the wrap)
constexpr int kShardRecW = 3 * kShardSegMax + 24;  // 3 words per pick + kp + 3 header words + the histogram
static_assert(3 * kShardSegMax + 4 + KB_NUM_REASONS <= kShardRecW, "inbox record layout");
struct ShardPeers {
  uint64_t* inbox[kShardMaxWorld];  // every rank's inbox as this GPU addresses it (its own included)
  int32_t rank, world;              // world 0: not sharded
  uint32_t epoch;                   // this cycle's number (the same on every rank)
  int32_t self_inbox;               // testing (KB_SHARD_SELF_INBOX=1): the rank's own record through its inbox too
};
size_t shard_inbox_bytes();
// kb_set_shard_peer's pre-flight (n <= 64 words read)
void launch_peer_put(uint64_t* dst, uint64_t v, void* stream);
void launch_peer_get(const uint64_t* src, int n, uint64_t* out, void* stream);
// coop: a cooperative launch (every workgroup co-resident, on the device's cooperative queue); returns the
// launch's hipError_t. shard.world > 0: the node-sharded engine (split engine only). place_xcc >= 0 (split engine):
// a grid of 8 x (1 + nsel) workgroups takes a census of their XCC ids and the placer and selectors are the ones on
// XCC place_xcc (others where it has too few), the rest exit at once.
// hring (pinned, kJobSlots FedHostCmd entries; place_xcc >= 0 only): the census grid's other workgroups stay as
// resident sweepers (fed_sweeper) that take command m of this launch from hring[m % kJobSlots] once its tag is
// epoch << 32 | m + 1 (fed_host_post) -- no sweep kernel per job; nullptr: they exit, and every command comes
// through a sweep kernel (fed_post's launch_sel_sweep / launch_fed_cmd).
int launch_fed_engine(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int idx_bits, const FedSlotPtrs& sp,
                      const void* ring, const uint32_t* ctr, const uint32_t* tgt, uint64_t idle_ticks,
                      int32_t* exit_flag, void* xchg, void* stream, bool coop, const ShardPeers& shard,
                      int place_xcc = -1, const void* hring = nullptr, uint32_t epoch = 0);
// A command for the resident sweepers: the eight words, then the tag (release).
struct FedHostCmd {
  uint64_t w[8];
  uint64_t tag;
  uint64_t pad[7];
};
void fed_host_post(void* hring, int r, const FedCmdArgs& a, uint64_t tag);

// Node sharding: per segment, the rank's local proposal (after launch_sel_sweep), then, after the
// all-gather of every rank's ShardRec, the global merge + stop rules + commit of the rank's own rows.
void launch_shard_propose(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_count,
                          int idx_bits, const uint32_t* keys32, const uint64_t* stat, const JobState* js, int first,
                          ShardRec* rec, SpecGuard g, const int32_t* patch, const JobState* patch_js,
                          const uint32_t* wait_ctr, uint32_t wait_target, JobState* hjs, void* stream,
                          const uint32_t* tag);
// commit_out (single-segment jobs): the rank's rows this job committed, for the next job's overlapped sweep
void launch_shard_commit(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                         int idx_bits, const ShardRec* recs, int world, JobState* js, int first, int ready0,
                         int minav0, int gang0, int32_t* hout, JobState* hjs, uint32_t seq, SpecGuard g,
                         int32_t* commit_out, void* stream);

constexpr int kBitonicMin = 2048;  // == the sort's LDS tile
// kb_sort_nodes: the spec's keys (PredicateFn + PrioritizeNodes) sorted descending into keys[0..n_pad), n_pad a
// power of two >= max(n, 2048); mm: the spec's InterPodAffinity min / max (affinity tables) or null.
void launch_sort_nodes(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, const int64_t* mm,
                       uint64_t* keys, int n_pad, void* stream, bool sort = true);
// kb_apply_affinity: table / histogram entries of a pod outside the session's specs (indices checked by the host).
void launch_apply_aff(const DevAff& A, const kb_aff_delta* d, int k, int base, void* stream);
// kb_apply: row deltas of commits made outside the device (one thread per delta, atomics).
void launch_apply(const DevNodes& N, const DevSpecs& P, const kb_row_delta* d, int k, const int64_t* sc,
                  const kb_port* ports, void* stream);

// Opt the place kernels into the dynamic LDS they need; returns 0 or the hipError_t.
int configure_kernels();
int traj_lds_bytes(int n, int t_count, int* pb_cap);
void launch_traj_sweep(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int J, int idx_bits,
                       uint32_t* traj, uint32_t* cmax32, uint32_t* amax, uint64_t* stat, const JobState* js,
                       bool aff, void* stream);
// Table increments of a run placed by the trajectory / re-key loops (affinity specs with increments).
// base: the placements' node ids minus base index this context's rows (node-sharded: global ids, A.topo_dom offset)
void launch_aff_commit(const DevSpecs& P, int spec, int t_begin, int run, const JobState* js, const int32_t* hout,
                       int base, void* stream);
void launch_traj_place(const DevNodes& N, const DevSpecs& P, const DevCfg& C, int spec, int t_begin, int t_count,
                       int J, int idx_bits, const uint32_t* traj, const uint32_t* cmax32, const uint32_t* amax,
                       const uint64_t* stat, JobState* js, int first, int ready0, int minav0, int gang0,
                       int32_t* hout, JobState* hjs, uint32_t seq, void* stream);

}  // namespace kbgpu
