// kb_ctx: one device-resident session snapshot.
#pragma once
#include <hip/hip_runtime.h>

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

  std::vector<void*> node_mem, spec_mem, work_mem;
  uint64_t* keys = nullptr;  // [n] packed argmax keys of the current spec
  uint64_t* cmax = nullptr;  // [ceil(n/64)] chunk maxima
  uint64_t* stat = nullptr;  // [n] static predicate / NodeAffinity cache of the current spec
  char* d_job = nullptr;     // device JobState (chains the runs of one job)
  char* h_job = nullptr;     // pinned host JobState + placement pairs (written by the place kernel)
  char* h_job_dev = nullptr; // device address of h_job
  uint32_t job_cap = 0;
  char* h_eval = nullptr;

  double device_ms = 0;  // wall time inside kb_place_job

  // pristine copies of the mutable node columns (kb_restore_nodes)
  struct Col { void* dst; void* src; size_t bytes; };
  std::vector<Col> pristine;

  // kernel timing (KB_OPT_TIMING)
  bool timing = false;
  std::vector<hipEvent_t> ev_pool;
  struct Pending { hipEvent_t a, b; int kind; uint64_t pairs; };
  std::vector<Pending> pending;
  kb_stats stats{};
  hipEvent_t ev_get();
  void ev_begin(hipEvent_t* a);
  void ev_end(hipEvent_t a, int kind, uint64_t pairs);
  void ev_collect();
};

extern "C" int kb_check_score_range(kb_ctx* c);
