// Session layer: allocateAction.Execute (pkg/scheduler/actions/allocate/allocate.go:42-193)
// with the ordering plugins restated on the host in C++ -- priority (plugins/priority/priority.go),
// gang (plugins/gang/gang.go), drf (plugins/drf/drf.go), proportion (plugins/proportion/proportion.go)
// -- dispatched through the tiers exactly as framework/session_plugins.go does. Every job pop hands
// the job's ordered pending tasks to kb_place_job (device), then replays the placements into the
// host-side job / share state the ordering reads.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "kbgpu_ctx.h"

namespace {

// Host helper threads (four per process): kb_allocate builds the cycle's pending lists on one and walks the last three
// quarters of the tasks for the session-open state on the others while its own thread walks the first quarter
// (independent passes over the session's task arrays, ~0.3 ms in one piece on C2's 100k tasks, before the first job
// can be issued). A
// driver that finds no worker free (another context's cycle in another thread) runs the work itself. A worker spins
// for kSpin after its last job before it sleeps, and join() spins before it waits: a futex wake-up costs as much as
// the work (cycles come every ~16 ms on C2, so a serving loop's workers never sleep).
class HostPool {
 public:
  static constexpr int kWorkers = 4;
  static constexpr auto kSpin = std::chrono::milliseconds(40);
  static HostPool& get() {
    static HostPool h;
    return h;
  }
  // the worker that takes f, or -1 (none free: run it yourself)
  int post(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu_);
    for (int i = 0; i < kWorkers; ++i) {
      Worker& w = w_[i];
      if (w.busy.load(std::memory_order_relaxed)) continue;
      if (!w.th.joinable()) w.th = std::thread([this, i] { loop(i); });
      w.job = std::move(f);
      w.busy.store(true, std::memory_order_relaxed);
      w.has_job.store(true, std::memory_order_release);
      cv_.notify_all();
      return i;
    }
    return -1;
  }
  void join(int i) {
    if (i < 0) return;
    Worker& w = w_[i];
    const auto t0 = std::chrono::steady_clock::now();
    while (w.busy.load(std::memory_order_acquire) && std::chrono::steady_clock::now() - t0 < kSpin) __builtin_ia32_pause();
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return !w.busy.load(std::memory_order_acquire); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
    }
    cv_.notify_all();
    for (Worker& w : w_)
      if (w.th.joinable()) w.th.join();
  }

 private:
  struct Worker {
    std::thread th;
    std::function<void()> job;
    std::atomic<bool> busy{false}, has_job{false};
  };
  void loop(int i) {
    Worker& w = w_[i];
    for (;;) {
      const auto t0 = std::chrono::steady_clock::now();
      while (!w.has_job.load(std::memory_order_acquire) && !stop_.load(std::memory_order_relaxed) &&
             std::chrono::steady_clock::now() - t0 < kSpin)
        __builtin_ia32_pause();
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_.load() || w.job != nullptr; });
        if (stop_.load()) return;
        f = std::move(w.job);
        w.job = nullptr;
        w.has_job.store(false, std::memory_order_relaxed);
      }
      f();
      {
        std::lock_guard<std::mutex> lk(mu_);
        w.busy.store(false, std::memory_order_release);
      }
      done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_;
  Worker w_[kWorkers];
  std::atomic<bool> stop_{false};
};

constexpr double kMinMilliCPU = 10, kMinMemory = 10 * 1024 * 1024, kMinMilliScalar = 10;  // resource_info.go:70-72
constexpr uint64_t kHasMap = 1ull << 63;

// api.Resource with fixed slots: v[0] cpu, v[1] memory, v[2 + s] scalar slot s; presence mask bit s
// (+ bit 63 = ScalarResources map non-nil). Restates api/resource_info.go.
struct Res {
  int S = 0;
  double v[64] = {0};
  uint64_t mask = 0;

  bool has(int s) const { return (mask >> s) & 1; }
  double sc(int s) const { return has(s) ? v[2 + s] : 0.0; }
  void add(const Res& r) { add_raw(r.v, r.mask); }
  void add_raw(const double* p, uint64_t m) {  // Add (:131-143) of a resreq row (cpu, mem, scalars) + its mask
    v[0] += p[0];
    v[1] += p[1];
    add_scalars(p, m);
  }
  void add_scalars(const double* p, uint64_t m) {  // add_raw's scalar part (the caller adds cpu and memory)
    for (int s = 0; s < S; ++s)
      if ((m >> s) & 1) {
        mask |= kHasMap | (1ull << s);
        v[2 + s] += p[2 + s];
      }
  }
  bool less_equal(const Res& rr) const {  // LessEqual (:253-276)
    bool ok = (v[0] < rr.v[0] || std::fabs(rr.v[0] - v[0]) < kMinMilliCPU) &&
              (v[1] < rr.v[1] || std::fabs(rr.v[1] - v[1]) < kMinMemory);
    if (!ok) return false;
    if (!(mask & kHasMap)) return true;
    for (int s = 0; s < S; ++s) {
      if (!has(s)) continue;
      if (!(rr.mask & kHasMap)) return false;
      double q = rr.sc(s);
      if (!(v[2 + s] < q || std::fabs(q - v[2 + s]) < kMinMilliScalar)) return false;
    }
    return true;
  }
  bool sub(const Res& r) {  // Sub (:145-159); false = util/assert panic
    if (!r.less_equal(*this)) return false;
    v[0] -= r.v[0];
    v[1] -= r.v[1];
    if (!(mask & kHasMap)) return true;
    for (int s = 0; s < S; ++s)
      if (r.has(s)) {
        mask |= 1ull << s;
        v[2 + s] -= r.v[2 + s];
      }
    return true;
  }
  bool less(const Res& rr) const {  // Less (:228-251)
    if (!(v[0] < rr.v[0] && v[1] < rr.v[1])) return false;
    if (!(mask & kHasMap)) return (rr.mask & kHasMap) != 0;
    for (int s = 0; s < S; ++s) {
      if (!has(s)) continue;
      if (!(rr.mask & kHasMap)) return false;
      if (v[2 + s] >= rr.sc(s)) return false;
    }
    return true;
  }
  bool is_empty() const {  // IsEmpty (:96-108)
    if (!(v[0] < kMinMilliCPU && v[1] < kMinMemory)) return false;
    for (int s = 0; s < S; ++s)
      if (has(s) && v[2 + s] >= kMinMilliScalar) return false;
    return true;
  }
  Res& multi(double ratio) {  // Multi (:218-225)
    v[0] = v[0] * ratio;
    v[1] = v[1] * ratio;
    for (int s = 0; s < S; ++s)
      if (has(s)) v[2 + s] = v[2 + s] * ratio;
    return *this;
  }
  double get(int col) const { return col < 2 ? v[col] : ((mask & kHasMap) ? sc(col - 2) : 0.0); }
};

Res res_min(const Res& l, const Res& r) {  // helpers.Min (api/helpers/helpers.go:27-45)
  Res o;
  o.S = l.S;
  o.v[0] = std::min(l.v[0], r.v[0]);
  o.v[1] = std::min(l.v[1], r.v[1]);
  if (!(l.mask & kHasMap) || !(r.mask & kHasMap)) return o;
  o.mask = kHasMap;
  for (int s = 0; s < l.S; ++s)
    if (l.has(s)) {
      o.mask |= 1ull << s;
      o.v[2 + s] = std::min(l.v[2 + s], r.sc(s));
    }
  return o;
}

double share(double l, double r) {  // helpers.Share (helpers.go:48-63)
  if (r == 0) return l == 0 ? 0 : 1;
  return l / r;
}

// max over ResourceNames() of share(allocated.Get(rn), total.Get(rn)) (drf.go:161-171, proportion.go:265-277)
double dominant_share(const Res& alloc, const Res& total) {
  double res = 0;
  int cols[66];
  int nc = 0;
  cols[nc++] = 0;
  cols[nc++] = 1;
  if (total.mask & kHasMap)
    for (int s = 0; s < total.S; ++s)
      if (total.has(s)) cols[nc++] = 2 + s;
  for (int i = 0; i < nc; ++i) {
    double x = share(alloc.get(cols[i]), total.get(cols[i]));
    if (x > res) res = x;
  }
  return res;
}

bool allocated_status(int s) {  // api/helpers.go:72-79
  return s == KB_ST_BOUND || s == KB_ST_BINDING || s == KB_ST_RUNNING || s == KB_ST_ALLOCATED;
}

// Go container/heap (src/container/heap/heap.go) -- Push = append + up, Pop = swap + down.
template <class T>
struct GoHeap {
  std::vector<T> items;
  std::function<bool(const T&, const T&)> less;
  void up(int j) {
    for (;;) {
      int i = (j - 1) / 2;
      if (i == j || !less(items[j], items[i])) break;
      std::swap(items[i], items[j]);
      j = i;
    }
  }
  void down(int i, int n) {
    for (;;) {
      int j1 = 2 * i + 1;
      if (j1 >= n || j1 < 0) break;
      int j = j1;
      if (j1 + 1 < n && less(items[j1 + 1], items[j1])) j = j1 + 1;
      if (!less(items[j], items[i])) break;
      std::swap(items[i], items[j]);
      i = j;
    }
  }
  void push(T x) {
    items.push_back(x);
    up((int)items.size() - 1);
  }
  T pop() {
    int n = (int)items.size() - 1;
    std::swap(items[0], items[n]);
    down(0, n);
    T x = items.back();
    items.pop_back();
    return x;
  }
  bool empty() const { return items.empty(); }
};

struct JobS {
  std::vector<int> pending;  // pending tasks in TaskOrderFn order (static during the cycle)
  size_t cursor = 0;
  bool pending_built = false;
  int ready = 0, waiting = 0, valid = 0;
  Res drf_alloc;
  double drf_share = 0;
};

struct QueueS {
  double share = 0;
  Res deserved, allocated, request;
};

struct Driver {
  kb_ctx* ctx;
  const kb_session& s;
  kb_cycle_result* out;
  int S;
  std::vector<JobS> jobs;
  std::vector<QueueS> queues;
  std::vector<int> task_status;
  std::vector<std::vector<int>> job_allocated;  // tasks with status Allocated per job (dispatch set)
  bool has[8] = {false};
  bool task_prio = false;
  Res total;

  Driver(kb_ctx* c, const kb_session& ss, kb_cycle_result* o) : ctx(c), s(ss), out(o), S((int)ss.n_rscalar) {}

  const double* task_req(int t) const { return s.task_resreq + (size_t)t * (2 + S); }
  bool task_res_empty(int t) const {  // Resource.IsEmpty (resource_info.go:96-108) on the raw row
    const double* p = task_req(t);
    const uint64_t m = s.task_resreq_mask[t];
    if (!(p[0] < kMinMilliCPU && p[1] < kMinMemory)) return false;
    for (int k = 0; k < S; ++k)
      if (((m >> k) & 1) && p[2 + k] >= kMinMilliScalar) return false;
    return true;
  }
  Res task_res(int t) const {
    Res r;
    r.S = S;
    const double* p = s.task_resreq + (size_t)t * (2 + S);
    for (int i = 0; i < 2 + S; ++i) r.v[i] = p[i];
    r.mask = s.task_resreq_mask[t];
    return r;
  }
  bool enabled(int plugin, uint32_t bit) const {
    for (uint32_t i = 0; i < s.n_tier_plugins; ++i)
      if (s.tier_plugins[i].plugin == plugin && (s.tier_plugins[i].enable & bit)) return true;
    return false;
  }

  // JobOrderFn (session_plugins.go:281-305)
  bool job_less(int l, int r) const {
    for (uint32_t i = 0; i < s.n_tier_plugins; ++i) {
      const kb_tier_plugin& p = s.tier_plugins[i];
      if (!(p.enable & KB_EN_JOB_ORDER)) continue;
      int j = 0;
      if (p.plugin == KB_PLUGIN_PRIORITY) {  // priority.go:60-78
        int a = s.job_priority[l], b = s.job_priority[r];
        j = a > b ? -1 : (a < b ? 1 : 0);
      } else if (p.plugin == KB_PLUGIN_GANG) {  // gang.go:96-119
        bool lr = jobs[l].ready >= s.job_min_available[l], rr = jobs[r].ready >= s.job_min_available[r];
        j = (lr && rr) ? 0 : lr ? 1 : rr ? -1 : 0;
      } else if (p.plugin == KB_PLUGIN_DRF) {  // drf.go:114-130
        double a = jobs[l].drf_share, b = jobs[r].drf_share;
        j = a == b ? 0 : (a < b ? -1 : 1);
      } else {
        continue;
      }
      if (j != 0) return j < 0;
    }
    if (s.job_ctime[l] == s.job_ctime[r]) return s.job_uid_rank[l] < s.job_uid_rank[r];
    return s.job_ctime[l] < s.job_ctime[r];
  }
  // QueueOrderFn (session_plugins.go:308-333)
  bool queue_less(int l, int r) const {
    for (uint32_t i = 0; i < s.n_tier_plugins; ++i) {
      const kb_tier_plugin& p = s.tier_plugins[i];
      if (!(p.enable & KB_EN_QUEUE_ORDER) || p.plugin != KB_PLUGIN_PROPORTION) continue;
      double a = queues[l].share, b = queues[r].share;  // proportion.go:171-184
      int j = a == b ? 0 : (a < b ? -1 : 1);
      if (j != 0) return j < 0;
    }
    if (s.queue_ctime[l] == s.queue_ctime[r]) return s.queue_uid_rank[l] < s.queue_uid_rank[r];
    return s.queue_ctime[l] < s.queue_ctime[r];
  }
  // TaskOrderFn (session_plugins.go:336-369)
  // Only the priority plugin orders tasks, so the tier walk reduces to one flag (task_prio, set in init).
  bool task_less(int l, int r) const {
    if (task_prio) {
      int a = s.task_priority[l], b = s.task_priority[r];  // priority.go:40-56
      if (a != b) return a > b;
    }
    if (s.task_ctime[l] == s.task_ctime[r]) return s.task_uid_rank[l] < s.task_uid_rank[r];
    return s.task_ctime[l] < s.task_ctime[r];
  }
  bool job_ready(int j) const {  // JobReady (session_plugins.go:202-220) -> gang Ready()
    if (has[KB_PLUGIN_GANG] && enabled(KB_PLUGIN_GANG, KB_EN_JOB_READY)) return jobs[j].ready >= s.job_min_available[j];
    return true;
  }
  bool overused(int q) const {  // Overused (session_plugins.go:185-199) -> proportion.go:221-233
    if (!has[KB_PLUGIN_PROPORTION]) return false;
    return queues[q].deserved.less_equal(queues[q].allocated);
  }

  // init()'s task pass over a range of the tasks (the first part on init()'s thread, the others on helpers): the
  // jobs' counts, the allocated-status tasks (their DRF sums and Allocated lists are then replayed in task order), and
  // the queues' proportion sums of the range (proportion.go:72-81, OnSessionOpen's task walk). Counts and sums stay in
  // registers while the job stays the same, the sums in two accumulators. exact: every cpu / memory request summed is
  // a non-negative integer and none has scalars -- then, with the totals below 2^53, every partial sum is exact and
  // the split sums equal the task-order sums bit for bit; else init() sums every task again in task order. The parts
  // are contiguous and ascending, so replaying their allocated-status lists part by part is task order.
  struct TaskPass {
    uint32_t t0 = 0, t1 = 0;
    std::vector<int32_t> ready, waiting, valid;
    std::vector<int> alloc;
    std::vector<double> q;  // per queue: allocated cpu, memory, request cpu, memory
    bool exact = true;
  };
  static constexpr int kTaskParts = 4;
  TaskPass part[kTaskParts];
  static bool exact_int(double x) { return x >= 0 && x < 9007199254740992.0 && x == (double)(int64_t)x; }
  void task_pass(TaskPass& T, bool prop) {
    T.ready.assign(s.n_jobs, 0);
    T.waiting.assign(s.n_jobs, 0);
    T.valid.assign(s.n_jobs, 0);
    T.alloc.clear();
    T.q.assign(4 * (size_t)s.n_queues, 0.0);
    const uint64_t sc_bits = S >= 64 ? ~0ull : (1ull << S) - 1;  // (add_scalars reads these bits only)
    bool exact = true;
    int cj = -1;
    int32_t r = 0, w = 0, v = 0;
    double a[2][2] = {}, q[2][2] = {};  // [accumulator][cpu, memory]: allocated, request
    const auto flush = [&]() {
      if (cj < 0) return;
      T.ready[cj] += r;
      T.waiting[cj] += w;
      T.valid[cj] += v;
      double* x = T.q.data() + 4 * (size_t)s.job_queue[cj];
      x[0] += a[0][0] + a[1][0];
      x[1] += a[0][1] + a[1][1];
      x[2] += q[0][0] + q[1][0];
      x[3] += q[0][1] + q[1][1];
      r = w = v = 0;
      a[0][0] = a[0][1] = a[1][0] = a[1][1] = q[0][0] = q[0][1] = q[1][0] = q[1][1] = 0;
    };
    for (uint32_t t = T.t0; t < T.t1; ++t) {
      const int j = s.task_job[t], st = s.task_status[t];
      if (j != cj) {
        flush();
        cj = j;
      }
      const bool al = allocated_status(st);
      r += (al || st == KB_ST_SUCCEEDED) ? 1 : 0;
      w += st == KB_ST_PIPELINED ? 1 : 0;
      v += (al || st == KB_ST_SUCCEEDED || st == KB_ST_PIPELINED || st == KB_ST_PENDING) ? 1 : 0;
      if (al) T.alloc.push_back((int)t);
      if (prop && (al || st == KB_ST_PENDING)) {
        const double* p = task_req(t);
        exact = exact && exact_int(p[0]) && exact_int(p[1]) && (s.task_resreq_mask[t] & sc_bits) == 0;
        const int k = t & 1;
        if (al) {
          a[k][0] += p[0];
          a[k][1] += p[1];
        }
        q[k][0] += p[0];
        q[k][1] += p[1];
      }
    }
    flush();
    T.exact = exact;
  }

  int init() {
    const auto i0 = std::chrono::steady_clock::now();
    // the pending lists (run()) on a helper thread, beside this task pass (both only read the session)
    const int w_pend = HostPool::get().post([this] { build_pend(); });
    for (uint32_t i = 0; i < s.n_tier_plugins; ++i) {
      int p = s.tier_plugins[i].plugin;
      if (p >= 0 && p < 8) has[p] = true;
      if (p == KB_PLUGIN_PRIORITY && (s.tier_plugins[i].enable & KB_EN_TASK_ORDER)) task_prio = true;
    }
    const bool prop = has[KB_PLUGIN_PROPORTION];
    // parts 1.. of the task pass on the other helpers (large sessions: the split pays for the thread hand-off; a part
    // no worker takes runs on init()'s thread after part 0)
    const int np = s.n_tasks >= 32768 ? kTaskParts : 1;
    int w_part[kTaskParts] = {-1, -1, -1, -1};
    for (int i = 0; i < np; ++i) {
      part[i].t0 = (uint32_t)((uint64_t)s.n_tasks * i / np);
      part[i].t1 = (uint32_t)((uint64_t)s.n_tasks * (i + 1) / np);
    }
    for (int i = 1; i < np; ++i) {
      TaskPass* T = &part[i];
      w_part[i] = HostPool::get().post([this, prop, T] { task_pass(*T, prop); });
    }
    total.S = S;
    for (int i = 0; i < 2 + S; ++i) total.v[i] = s.total_alloc[i];
    total.mask = s.total_alloc_mask;
    jobs.assign(s.n_jobs, JobS());
    queues.assign(s.n_queues, QueueS());
    job_allocated.assign(s.n_jobs, {});
    task_status.assign(s.task_status, s.task_status + s.n_tasks);
    for (auto& j : jobs) j.drf_alloc.S = S;
    for (auto& q : queues) {
      q.deserved.S = q.allocated.S = q.request.S = S;
    }
    const auto ia = std::chrono::steady_clock::now();
    task_pass(part[0], prop);
    for (int i = 1; i < np; ++i)
      if (w_part[i] < 0) task_pass(part[i], prop);
    const auto ib = std::chrono::steady_clock::now();
    for (int i = 1; i < np; ++i) HostPool::get().join(w_part[i]);
    // the jobs' counts; the allocated-status tasks' DRF sums and Allocated lists in task order
    for (uint32_t j = 0; j < s.n_jobs; ++j) {
      int32_t r = 0, w = 0, v = 0;
      for (int i = 0; i < np; ++i) r += part[i].ready[j], w += part[i].waiting[j], v += part[i].valid[j];
      jobs[j].ready = r;
      jobs[j].waiting = w;
      jobs[j].valid = v;
    }
    for (int i = 0; i < np; ++i)
      for (int t : part[i].alloc) {
        const int j = s.task_job[t];
        if (task_status[t] == KB_ST_ALLOCATED) job_allocated[j].push_back(t);
        jobs[j].drf_alloc.add_raw(task_req(t), s.task_resreq_mask[t]);
      }
    if (prop) {  // the queues' allocated / request sums: the split sums when exact, else in task order
      bool ok = true;
      for (int i = 0; i < np; ++i) ok = ok && part[i].exact;
      std::vector<double> sum(4 * (size_t)s.n_queues);
      for (size_t k = 0; ok && k < sum.size(); ++k) {
        double x = 0;
        for (int i = 0; i < np; ++i) x += part[i].q[k];
        sum[k] = x;
        ok = exact_int(sum[k]);
      }
      if (ok) {
        for (uint32_t q = 0; q < s.n_queues; ++q) {
          queues[q].allocated.v[0] = sum[4 * q];
          queues[q].allocated.v[1] = sum[4 * q + 1];
          queues[q].request.v[0] = sum[4 * q + 2];
          queues[q].request.v[1] = sum[4 * q + 3];
        }
      } else {  // one add per task in task order, cpu and memory in registers while the queue stays the same
        int cq = -1;
        double ac = 0, am = 0, rc = 0, rm = 0;
        const auto qflush = [&]() {
          if (cq < 0) return;
          queues[cq].allocated.v[0] = ac;
          queues[cq].allocated.v[1] = am;
          queues[cq].request.v[0] = rc;
          queues[cq].request.v[1] = rm;
        };
        for (uint32_t t = 0; t < s.n_tasks; ++t) {
          const int st = task_status[t];
          const bool al = allocated_status(st);
          if (!(al || st == KB_ST_PENDING)) continue;
          const int qi = s.job_queue[s.task_job[t]];
          if (qi != cq) {
            qflush();
            cq = qi;
            ac = queues[qi].allocated.v[0];
            am = queues[qi].allocated.v[1];
            rc = queues[qi].request.v[0];
            rm = queues[qi].request.v[1];
          }
          const double* p = task_req(t);
          const uint64_t m = s.task_resreq_mask[t];
          if (al) {
            ac += p[0];
            am += p[1];
            queues[qi].allocated.add_scalars(p, m);
          }
          rc += p[0];
          rm += p[1];
          queues[qi].request.add_scalars(p, m);
        }
        qflush();
      }
    }
    const auto ic = std::chrono::steady_clock::now();
    if (w_pend >= 0) HostPool::get().join(w_pend);
    else build_pend();
    const auto i1 = std::chrono::steady_clock::now();
    for (uint32_t j = 0; j < s.n_jobs; ++j) jobs[j].drf_share = dominant_share(jobs[j].drf_alloc, total);
    const auto i2 = std::chrono::steady_clock::now();
    if (prop) open_proportion();
    if (ctx->issue_trace)
      fprintf(stderr,
              "kb_host_trace init tasks_ms=%.3f drf_ms=%.3f proportion_ms=%.3f parts=%d (setup %.3f first part %.3f "
              "merge %.3f pending-list join %.3f)\n",
              std::chrono::duration<double, std::milli>(i1 - i0).count(),
              std::chrono::duration<double, std::milli>(i2 - i1).count(),
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - i2).count(),
              np, std::chrono::duration<double, std::milli>(ia - i0).count(),
              std::chrono::duration<double, std::milli>(ib - ia).count(),
              std::chrono::duration<double, std::milli>(ic - ib).count(),
              std::chrono::duration<double, std::milli>(i1 - ic).count());
    return KB_OK;
  }

  // proportion.OnSessionOpen (proportion.go:58-169); queues visited in UID order.
  void open_proportion() {
    std::vector<char> in_use(s.n_queues, 0);
    for (uint32_t j = 0; j < s.n_jobs; ++j) in_use[s.job_queue[j]] = 1;
    // (the queues' allocated / request sums come from init()'s task pass)
    std::vector<int> order;
    for (uint32_t q = 0; q < s.n_queues; ++q)
      if (in_use[q]) order.push_back((int)q);
    std::sort(order.begin(), order.end(), [&](int a, int b) { return s.queue_uid_rank[a] < s.queue_uid_rank[b]; });
    Res remaining = total;
    std::vector<char> meet(s.n_queues, 0);
    for (;;) {
      int32_t tw = 0;
      for (int q : order)
        if (!meet[q]) tw += s.queue_weight[q];
      if (tw == 0) break;
      Res inc, dec;
      inc.S = dec.S = S;
      for (int q : order) {
        if (meet[q]) continue;
        QueueS& a = queues[q];
        Res old = a.deserved;
        Res part = remaining;
        a.deserved.add(part.multi((double)s.queue_weight[q] / (double)tw));
        if (a.request.less(a.deserved)) {
          a.deserved = res_min(a.deserved, a.request);
          meet[q] = 1;
        }
        a.share = dominant_share(a.allocated, a.deserved);
        // Resource.Diff (resource_info.go:278-309)
        Res i2, d2;
        i2.S = d2.S = S;
        if (a.deserved.v[0] > old.v[0]) i2.v[0] += a.deserved.v[0] - old.v[0]; else d2.v[0] += old.v[0] - a.deserved.v[0];
        if (a.deserved.v[1] > old.v[1]) i2.v[1] += a.deserved.v[1] - old.v[1]; else d2.v[1] += old.v[1] - a.deserved.v[1];
        if (a.deserved.mask & kHasMap)
          for (int sl = 0; sl < S; ++sl) {
            if (!a.deserved.has(sl)) continue;
            double rq = old.sc(sl);
            if (a.deserved.v[2 + sl] > rq) {
              i2.mask |= kHasMap | (1ull << sl);
              i2.v[2 + sl] += a.deserved.v[2 + sl] - rq;
            } else {
              d2.mask |= kHasMap | (1ull << sl);
              d2.v[2 + sl] += rq - a.deserved.v[2 + sl];
            }
          }
        inc.add(i2);
        dec.add(d2);
      }
      remaining.sub(inc);
      remaining.add(dec);
      if (remaining.is_empty()) break;
    }
  }

  // drf.go:135-144, proportion.go:236-246. The allocated sums take every task in event order, as the
  // handlers do; the shares they feed are read only by the job / queue orders at the next heap push, so
  // share_update() computes them once per job instead of once per event (same value).
  void on_allocate_event(int t) {
    int j = s.task_job[t];
    const double* p = task_req(t);
    const uint64_t m = s.task_resreq_mask[t];
    if (has[KB_PLUGIN_DRF]) jobs[j].drf_alloc.add_raw(p, m);
    if (has[KB_PLUGIN_PROPORTION]) queues[s.job_queue[j]].allocated.add_raw(p, m);
  }
  void share_update(int j) {
    if (has[KB_PLUGIN_DRF]) jobs[j].drf_share = dominant_share(jobs[j].drf_alloc, total);
    if (has[KB_PLUGIN_PROPORTION]) {
      QueueS& q = queues[s.job_queue[j]];
      q.share = dominant_share(q.allocated, q.deserved);
    }
  }

  // ---- the allocate loop (actions/allocate/allocate.go:40-176) ----
  double loop_ms = 0;  // KB_HOST_TRACE: time in the job loop of run()
  // The jobs in UID order and every job's Pending tasks as one CSR array, with the cycle's largest pending list and
  // the pending tasks with requests (pend_all), of which the fed engine takes pend_eng. Reads only the session (the
  // input task statuses: init() copies them beside it) and the context's per-spec eligibility, so it runs on the
  // host helper thread during init()'s task pass.
  std::vector<int> jorder;
  uint32_t max_pending = 1;
  uint64_t pend_all = 0, pend_eng = 0;
  uint32_t jobs_pend = 0, jobs_off = 0;  // jobs with pending tasks, and those whose first one the engine does not take
  void build_pend() {
    jorder.resize(s.n_jobs);
    for (uint32_t j = 0; j < s.n_jobs; ++j) jorder[j] = (int)j;
    std::sort(jorder.begin(), jorder.end(), [&](int a, int b) { return s.job_uid_rank[a] < s.job_uid_rank[b]; });
    pend_all = pend_eng = 0;
    jobs_pend = jobs_off = 0;
    // tasks grouped by job in job order (the exporters' layout): one pass appends each job's pending tasks and closes
    // its CSR range; otherwise (the pass meets a smaller job index) the count pass and the fill pass
    pend_off.assign(s.n_jobs + 1, 0);
    pend.resize(s.n_tasks);
    bool grouped = true;
    {
      uint32_t k = 0;
      int last = -1;
      for (uint32_t t = 0; t < s.n_tasks; ++t) {
        const int j = s.task_job[t];
        if (j != last) {
          if (j < last) {
            grouped = false;
            break;
          }
          for (int jj = last + 1; jj <= j; ++jj) pend_off[jj] = k;
          last = j;
        }
        if (s.task_status[t] == KB_ST_PENDING) {
          pend[k++] = (int)t;
          if (!task_res_empty(t)) {
            ++pend_all;
            pend_eng += spec_fed_ok(s.task_spec[t]) ? 1 : 0;
          }
        }
      }
      if (grouped)
        for (uint32_t jj = (uint32_t)(last + 1); jj <= s.n_jobs; ++jj) pend_off[jj] = k;
    }
    if (!grouped) {
      pend_all = pend_eng = 0;
      pend_off.assign(s.n_jobs + 1, 0);
      for (uint32_t t = 0; t < s.n_tasks; ++t)
        if (s.task_status[t] == KB_ST_PENDING) ++pend_off[s.task_job[t] + 1];
      for (uint32_t j = 0; j < s.n_jobs; ++j) pend_off[j + 1] += pend_off[j];
      std::vector<uint32_t> cur(pend_off.begin(), pend_off.end() - 1);
      for (uint32_t t = 0; t < s.n_tasks; ++t)
        if (s.task_status[t] == KB_ST_PENDING) {
          pend[cur[s.task_job[t]]++] = (int)t;
          if (!task_res_empty(t)) {
            ++pend_all;
            pend_eng += spec_fed_ok(s.task_spec[t]) ? 1 : 0;
          }
        }
    }
    pend.resize(pend_off[s.n_jobs]);
    max_pending = 1;
    for (uint32_t j = 0; j < s.n_jobs; ++j) max_pending = std::max<uint32_t>(max_pending, pend_off[j + 1] - pend_off[j]);
    for (uint32_t j = 0; j < s.n_jobs; ++j)
      if (pend_off[j + 1] > pend_off[j]) {
        ++jobs_pend;
        jobs_off += spec_fed_ok(s.task_spec[pend[pend_off[j]]]) ? 0 : 1;
      }
  }
  GoHeap<int> qheap;
  std::vector<GoHeap<int>> jheaps;
  // each job's Pending tasks in task order, as one CSR array (job j: pend[pend_off[j] .. pend_off[j + 1]))
  std::vector<int> pend;
  std::vector<uint32_t> pend_off;
  struct Span {
    const int* b;
    const int* e;
    const int* begin() const { return b; }
    const int* end() const { return e; }
    size_t size() const { return (size_t)(e - b); }
  };
  Span job_pending(int j) const { return Span{pend.data() + pend_off[j], pend.data() + pend_off[j + 1]}; }
  std::vector<int32_t> specs, pn, pk;
  std::vector<uint32_t> node_reasons;  // NO_FIT hook
  int hook_rc = KB_OK;
  uint32_t n_events = 0;
  bool gang_ready_on = false;

  void build_pending(int j) {  // allocate.go:114-129 (BestEffort tasks skipped)
    JobS& js = jobs[j];
    if (js.pending_built) return;
    js.pending.reserve(job_pending(j).size());
    for (int t : job_pending(j))
      if (!task_res_empty(t)) js.pending.push_back(t);
    std::sort(js.pending.begin(), js.pending.end(), [this](int a, int b) { return task_less(a, b); });
    js.pending_built = true;
  }

  // The loop head: pop queues / jobs until a job with pending tasks comes out (allocate.go:90-112).
  // Queues that are overused or out of jobs are dropped; a job without pending tasks is dropped and its
  // queue pushed back. `jh` maps a queue to the job heap to use (the real ones, or scratch copies).
  template <class JH>
  bool next_job(GoHeap<int>& qh, JH&& jh, int& q, int& j) {
    while (!qh.empty()) {
      q = qh.pop();
      if (overused(q)) continue;
      GoHeap<int>& h = jh(q);
      if (h.empty()) continue;
      j = h.pop();
      build_pending(j);
      if (jobs[j].cursor < jobs[j].pending.size()) return true;
      qh.push(q);
    }
    return false;
  }

  // A unit: what one device call places. On the fed engine, one run of one spec (at most unit_cap tasks: the split
  // engine's segment); on the launch paths, the rest of the job (they chain a job's runs on the device). A job pop
  // is one or more units: a unit that places all its tasks without the job becoming ready is followed, in the same
  // pop, by the job's next unit (allocate.go:135-188 goes on with the next task) with no heap operation between.
  struct Unit {
    int q = -1, j = -1;
    size_t cur = 0;
    uint32_t len = 0;
    bool last = true, fed = false;
    bool operator==(const Unit& o) const {
      return q == o.q && j == o.j && cur == o.cur && len == o.len && fed == o.fed;
    }
  };
  bool fed_allowed = false;  // the cycle may run units on the resident engine
  uint32_t unit_cap = 0;     // kb_fed_unit_cap: 0 = any length
  // per spec: -1 not asked yet, else kb_spec_fed_ok_pre (affinity specs with histograms: as if their min / max were
  // prepared; run() prepares them, or drops the ones whose histograms the cycle's commits write: prepare_fed_aff)
  std::vector<int8_t> spec_fed;
  bool spec_fed_ok(int sp) {
    if (sp < 0) return false;
    if ((size_t)sp >= spec_fed.size()) spec_fed.resize(sp + 1, -1);
    if (spec_fed[sp] < 0) spec_fed[sp] = (int8_t)kb_spec_fed_ok_pre(ctx, sp);
    return spec_fed[sp] != 0;
  }
  // The engine's affinity units with InterPodAffinity histograms: their sweep normalises by the min / max over the
  // nodes (interpod_affinity.go:221-238) as the tables stand when the unit runs. Computed once, before the engine's
  // launch, they stay exact through the cycle when no pending spec's commits write the histograms they read
  // (aff_wr / aff_rd, kb_upload_affinity); the other such specs run on the launch path (its own min / max pass per
  // run). Returns the first error.
  int prepare_fed_aff() {
    ctx->mm_spec_ok.assign(ctx->mm_spec_ok.size(), 0);
    if (!ctx->aff_ok) return KB_OK;
    std::vector<char> seen(ctx->spec_needs_aff.size(), 0);
    std::vector<int> cyc;  // the cycle's distinct pending specs
    for (int t : pend) {
      const int sp = s.task_spec[t];
      if (sp < 0 || (size_t)sp >= seen.size() || seen[sp]) continue;
      seen[sp] = 1;
      cyc.push_back(sp);
    }
    std::vector<uint32_t> w_all;  // every table / histogram the cycle's commits may write
    for (int sp : cyc)
      if ((size_t)sp < ctx->aff_wr.size()) w_all.insert(w_all.end(), ctx->aff_wr[sp].begin(), ctx->aff_wr[sp].end());
    std::sort(w_all.begin(), w_all.end());
    w_all.erase(std::unique(w_all.begin(), w_all.end()), w_all.end());
    std::vector<int32_t> prep;
    for (int sp : cyc) {
      if (!ctx->spec_needs_aff[sp] || !ctx->spec_hist[sp] || !spec_fed_ok(sp)) continue;
      bool clash = false;
      for (uint32_t x : ctx->aff_rd[sp])
        if ((x >> 31) && std::binary_search(w_all.begin(), w_all.end(), x)) clash = true;
      if (clash) spec_fed[sp] = 0;
      else prep.push_back(sp);
    }
    return kb_fed_ipa_prepare(ctx, prep.data(), (uint32_t)prep.size());
  }
  // the unit job j's pending list has at its cursor (j popped from queue q)
  Unit unit_at(int q, int j) {
    const JobS& js = jobs[j];
    Unit u;
    u.q = q, u.j = j, u.cur = js.cursor;
    const size_t n = js.pending.size();
    const int sp0 = s.task_spec[js.pending[u.cur]];
    if (fed_allowed && spec_fed_ok(sp0)) {
      const size_t lim = unit_cap ? std::min(n, u.cur + unit_cap) : n;
      size_t e = u.cur + 1;
      while (e < lim && s.task_spec[js.pending[e]] == sp0) ++e;
      u.len = (uint32_t)(e - u.cur);
      u.fed = true;
    } else {
      u.len = (uint32_t)(n - u.cur);
    }
    u.last = u.cur + u.len == n;
    return u;
  }
  kb_job_req make_req(const Unit& u) {
    const JobS& js = jobs[u.j];
    specs.resize(u.len);
    for (uint32_t i = 0; i < u.len; ++i) specs[i] = s.task_spec[js.pending[u.cur + i]];
    return kb_job_req{specs.data(), u.len, js.ready, s.job_min_available[u.j], gang_ready_on ? 1 : 0};
  }
  int check_specs(int j) const {
    const JobS& js = jobs[j];
    for (size_t i = js.cursor; i < js.pending.size(); ++i)
      if (s.task_spec[js.pending[i]] < 0) return KB_E_INVALID;
    return KB_OK;
  }

  // Session.Allocate / Session.Pipeline for the unit's placements, then the heap pushes of the loop tail. Returns
  // true when the pop goes on with the job's next unit (the unit placed all its tasks, the job is not ready, and
  // it has more pending tasks): no loop tail then.
  bool apply(const Unit& u, const kb_job_result& res) {
    const int q = u.q, j = u.j;
    JobS& js = jobs[j];
    for (uint32_t i = 0; i < res.n_placed; ++i) {
      int t = js.pending[js.cursor + i];
      out->task_node[t] = pn[i];
      out->event_task[n_events++] = t;
      if (pk[i] == KB_PLACE_ALLOCATE) {  // Session.Allocate (session.go:242-297)
        task_status[t] = KB_ST_ALLOCATED;
        js.ready++;
        job_allocated[j].push_back(t);
        on_allocate_event(t);
        if (job_ready(j)) {  // dispatch every Allocated task (session.go:286-294)
          for (int a : job_allocated[j]) task_status[a] = KB_ST_BINDING;
          job_allocated[j].clear();
        }
      } else {  // Session.Pipeline (session.go:199-239)
        task_status[t] = KB_ST_PIPELINED;
        js.waiting++;
        on_allocate_event(t);
      }
    }
    if (res.n_placed) share_update(j);
    js.cursor += res.n_placed;
    if (res.stop == KB_STOP_NO_FIT) {
      const int ft = js.pending[js.cursor];
      out->job_fail_task[j] = ft;
      note_dead(s.task_spec[ft]);
      memcpy(out->job_reason_hist + (size_t)j * KB_NUM_REASONS, res.reason_hist, sizeof(res.reason_hist));
      // host-evaluated stages: the caller turns the KB_R_HOST_ERROR bucket into its per-node strings from
      // the reason masks at this state (nothing has run since the failing task)
      const int sp = s.task_spec[ft];
      if (ctx->nofit_fn && ctx->host_reasons(sp)) {
        node_reasons.resize((size_t)ctx->N.n);
        if (int rc = kb_node_reasons(ctx, sp, node_reasons.data())) hook_rc = rc;
        else ctx->nofit_fn(ctx->nofit_user, j, ft, n_events, node_reasons.data(), (uint32_t)ctx->N.n);
      }
    } else if (res.stop == KB_STOP_READY) {
      jheaps[q].push(j);
    } else if (!u.last && res.n_placed == u.len && js.cursor < js.pending.size()) {
      return true;
    }
    qheap.push(q);
    return false;
  }

  // The place call's outcome when every task it places is Allocated (the stop rules of the place
  // kernels): a gang job stops READY at the task that brings ready to minAvailable, a job without the
  // gang JobReady check after its first task; otherwise every task places and the call ends DONE.
  // A unit whose first task's spec is dead (below) stops NO_FIT before placing anything.
  void predict(const Unit& u, int& stop, int& placed) {
    const int j = u.j;
    const JobS& js = jobs[j];
    const int nt = (int)u.len;
    if (is_dead(s.task_spec[js.pending[u.cur]])) {
      stop = KB_STOP_NO_FIT;
      placed = 0;
      return;
    }
    if (!gang_ready_on) {
      stop = KB_STOP_READY;
      placed = 1;
      return;
    }
    const int need = std::max(1, s.job_min_available[j] - js.ready);
    stop = need <= nt ? KB_STOP_READY : KB_STOP_DONE;
    placed = std::min(need, nt);
  }

  // NO_FIT prediction. A spec that stopped a unit NO_FIT found no node at that state; within the cycle every node's
  // Idle, Releasing, pod count and used host ports only move toward failure (Allocate / Pipeline commits, session.go:
  // 199-297), so it finds none later either, and neither does a spec of its feasibility class (kb_upload_specs: the
  // same PredicateFn inputs apart from InitResreq) whose InitResreq is at least as large in every resource
  // (resource_info.go:253-276). Such units are predicted NO_FIT with no placement, so the speculative chain behind
  // them survives (C3: each NO_FIT job used to drain the chain). A dead spec of a parent class (kb_upload_specs: the
  // same filters without the selector or the required node affinity) kills likewise. Specs with inter-pod terms (required affinity can
  // turn true as pods land) or host-evaluated reasons have no class. dead[c]: the minimal dead specs of class c.
  std::vector<std::vector<int>> dead;
  std::vector<int8_t> spec_dead;  // per spec: 0 unknown, 1 dead
  bool dead_any = false;
  bool dead_eligible(int sp) const {
    return sp >= 0 && (size_t)sp < ctx->spec_fclass.size() && ctx->spec_fclass[sp] >= 0 &&
           !(ctx->aff_ok && ctx->spec_needs_aff[sp]) && !ctx->host_reasons(sp);
  }
  bool init_geq(int a, int b) const {  // InitResreq(a) >= InitResreq(b) in every resource b requests
    const uint64_t ma = ctx->spec_init_mask[a], mb = ctx->spec_init_mask[b];
    if (mb & ~ma) return false;
    const size_t w = 2 + (size_t)ctx->N.S;
    const int64_t* va = ctx->spec_init.data() + (size_t)a * w;
    const int64_t* vb = ctx->spec_init.data() + (size_t)b * w;
    if (va[0] < vb[0] || va[1] < vb[1]) return false;
    for (uint64_t m = mb; m; m &= m - 1)
      if (va[2 + __builtin_ctzll(m)] < vb[2 + __builtin_ctzll(m)]) return false;
    return true;
  }
  void note_dead(int sp) {
    if (!dead_eligible(sp)) return;
    std::vector<int>& d = dead[(size_t)ctx->spec_fclass[sp]];
    for (int x : d)
      if (init_geq(sp, x)) return;  // implied by a smaller dead spec
    d.erase(std::remove_if(d.begin(), d.end(), [&](int x) { return init_geq(x, sp); }), d.end());
    d.push_back(sp);
    spec_dead[(size_t)sp] = 1;
    dead_any = true;
  }
  bool is_dead(int sp) {
    if (!dead_any || !dead_eligible(sp)) return false;
    if (spec_dead[(size_t)sp]) return true;
    // its own class, then the parent classes (kb_upload_specs: fewer node filters, so a superset of its nodes)
    for (int k = -1; k < 3; ++k) {
      const int c = k < 0 ? ctx->spec_fclass[sp] : ctx->spec_fparent[(size_t)sp * 3 + k];
      if (c < 0) continue;
      for (int x : dead[(size_t)c])
        if (init_geq(sp, x)) {
          spec_dead[(size_t)sp] = 1;
          return true;
        }
    }
    return false;
  }

  // Units in flight on the device (pipelined driver), oldest first. Entry i > 0 was issued speculatively, guarded on
  // entry i-1 ending as predicted; `pred` is the entry's own predicted outcome (set by the replay that issued the
  // entry after it).
  struct Flight {
    Unit u;
    int slot;
    kb_job_pred pred;
  };
  std::vector<Flight> fl;

  // Speculation: find the unit the loop runs next IF every unit in flight ends as predicted, and issue it into
  // `free_slot` guarded on the last one's prediction. The predictions are applied to the driver state in order and
  // the loop tail / head (or the job's next unit) replayed on scratch copies of the heaps; then the state is put back.
  // Returns false (nothing issued) when there is no next unit, it cannot be guarded, or it belongs to the other
  // device mode (mode_fed: the resident engine runs the chain; the chain ends where the mode changes).
  GoHeap<int> sq;
  std::vector<std::pair<int, GoHeap<int>>> sjh;
  struct SavedJob {
    int j, ready;
    size_t cursor;
    Res drf;
    double share;
  };
  struct SavedQueue {
    int q;
    Res allocated;
    double share;
  };
  std::vector<SavedJob> saved_jobs;
  std::vector<SavedQueue> saved_queues;
  bool speculate(int free_slot, bool mode_fed) {
    saved_jobs.clear();
    saved_queues.clear();
    sq.items = qheap.items;
    sjh.clear();
    auto jh = [&](int qq) -> GoHeap<int>& {
      for (auto& e : sjh)
        if (e.first == qq) return e.second;
      sjh.emplace_back(qq, jheaps[qq]);
      return sjh.back().second;
    };
    bool ok = true;
    Unit nu;
    for (size_t i = 0; i < fl.size() && ok; ++i) {
      Flight& f = fl[i];
      int stop, placed;
      predict(f.u, stop, placed);
      if (stop == KB_STOP_NO_FIT && i + 1 == fl.size()) ctx->stats.nofit_predicted++;
      JobS& js = jobs[f.u.j];
      bool seen = false;
      for (const auto& e : saved_jobs) seen = seen || e.j == f.u.j;
      if (!seen) saved_jobs.push_back(SavedJob{f.u.j, js.ready, js.cursor, js.drf_alloc, js.drf_share});
      seen = false;
      for (const auto& e : saved_queues) seen = seen || e.q == f.u.q;
      if (!seen) saved_queues.push_back(SavedQueue{f.u.q, queues[f.u.q].allocated, queues[f.u.q].share});
      const int ready0 = js.ready;
      for (int k = 0; k < placed; ++k) on_allocate_event(js.pending[js.cursor + k]);
      js.ready += placed;
      js.cursor += placed;
      share_update(f.u.j);
      f.pred = kb_job_pred{f.slot, stop, placed, ready0 + placed};
      if (stop == KB_STOP_DONE && !f.u.last) {  // the pop goes on with the job's next unit
        nu = unit_at(f.u.q, f.u.j);
      } else {  // the loop tail of the predicted outcome, then the next loop head
        if (stop == KB_STOP_READY) jh(f.u.q).push(f.u.j);
        sq.push(f.u.q);
        int nq, nj;
        ok = next_job(sq, jh, nq, nj) && check_specs(nj) == KB_OK;
        if (ok) nu = unit_at(nq, nj);
      }
      if (ok && i + 1 < fl.size()) ok = nu == fl[i + 1].u;  // issued by the same replay
    }
    ok = ok && nu.fed == mode_fed;
    // an engine unit whose sweep reads affinity tables a unit in flight commits to waits for the chain to drain (it is
    // issued after the last one is read: the placer commits the tables before it publishes)
    if (ok && mode_fed && ctx->aff_ok) {
      const int sb = s.task_spec[jobs[nu.j].pending[nu.cur]];
      for (const Flight& f : fl)
        if (!kb_fed_units_indep(ctx, s.task_spec[jobs[f.u.j].pending[f.u.cur]], sb)) ok = false;
      if (!ok) ctx->stats.fed_aff_waits++;
    }
    if (ok) {
      const kb_job_req req = make_req(nu);
      ok = kb_job_guardable(ctx, &req) != 0;
      if (ok) {
        const kb_job_pred pred = fl.back().pred;
        ok = kb_job_issue(ctx, &req, free_slot, &pred) == KB_OK;
      }
    }
    for (const auto& e : saved_jobs) {
      JobS& js = jobs[e.j];
      js.ready = e.ready;
      js.cursor = e.cursor;
      js.drf_alloc = e.drf;
      js.drf_share = e.share;
    }
    for (const auto& e : saved_queues) {
      queues[e.q].allocated = e.allocated;
      queues[e.q].share = e.share;
    }
    if (ok) fl.push_back(Flight{nu, free_slot, kb_job_pred{}});
    return ok;
  }

  // The unit after u (cont: u's job goes on), or the next loop head's. 1: nu set, 0: the cycle is over, < 0: error.
  int advance(const Unit& u, bool cont, Unit& nu) {
    if (cont) {
      nu = unit_at(u.q, u.j);
      return 1;
    }
    int nq, nj;
    if (!next_job(qheap, [this](int qq) -> GoHeap<int>& { return jheaps[qq]; }, nq, nj)) return 0;
    if (check_specs(nj)) return KB_E_INVALID;
    nu = unit_at(nq, nj);
    return 1;
  }

  // The engine's units in flight (the running one + speculative ones): kb_opts.fed_depth, else kJobSlots.
  int fed_depth() const { return ctx->fed_depth >= 2 ? ctx->fed_depth : kbgpu::kJobSlots; }

  int run() {
    const auto r0 = std::chrono::steady_clock::now();
    qheap.less = [this](const int& a, const int& b) { return queue_less(a, b); };
    sq.less = qheap.less;
    jheaps.assign(s.n_queues, GoHeap<int>());
    dead.assign((size_t)ctx->n_fclass, {});
    spec_dead.assign(ctx->spec_fclass.size(), 0);
    dead_any = false;
    for (auto& h : jheaps) h.less = [this](const int& a, const int& b) { return job_less(a, b); };
    gang_ready_on = has[KB_PLUGIN_GANG] && enabled(KB_PLUGIN_GANG, KB_EN_JOB_READY);
    // (jorder, pend_off / pend, max_pending, pend_all, pend_eng: build_pend, during init)
    for (int j : jorder) {
      if (s.job_pg_pending[j]) continue;                                              // allocate.go:50-52
      if (has[KB_PLUGIN_GANG] && jobs[j].valid < s.job_min_available[j]) continue;  // JobValid, gang.go:48-69
      int q = s.job_queue[j];
      if (q < 0 || (uint32_t)q >= s.n_queues) continue;
      qheap.push(q);
      jheaps[q].push(j);
    }
    const auto rq = std::chrono::steady_clock::now();
    pn.resize(max_pending);
    pk.resize(max_pending);
    // Pipelined: unit k+1 is launched (guarded) before unit k's result is read, so the device runs them back to
    // back while the host does the bookkeeping. Otherwise one kb_place_job per unit.
    const bool pipe = kb_job_pipeline_ok(ctx) && ctx->use_pipeline;
    if (pipe)
      if (int rc = kb_job_reserve(ctx, max_pending)) return rc;
    // The resident fed engine runs every unit whose spec it takes (kb_spec_fed_ok: one selection run, no inter-pod
    // terms); a unit it does not take (inter-pod affinity, host-evaluated reasons, ...) runs on the launch path
    // between two engine launches. node-sharded with the peer exchange: the launch path's units go one at a time
    // through the host-staged exchange.
    unit_cap = kb_fed_unit_cap(ctx);
    const uint32_t max_unit = unit_cap ? std::min(max_pending, unit_cap) : max_pending;
    fed_allowed = pipe && kb_fed_cycle_ok(ctx, max_unit);
    // worth it when most of the cycle's tasks are engine units (the counts come from the pending-list pass, build_pend)
    // and when few jobs leave it: each one the engine does not take pauses it (its chain drains, the launch path
    // runs the job, the chain refills: ~50 us on C4, whose 28 % class-loop jobs made the engine cycle slower than the
    // launch path's, r06r: 49.4 against 47.9 ms)
    if (fed_allowed) fed_allowed = 2 * pend_eng > pend_all && 4 * (uint64_t)jobs_off <= jobs_pend;
    if (fed_allowed)
      if (int rc = prepare_fed_aff()) return rc;
    const bool launch_pipe = pipe && !(ctx->sharded && !ctx->comm);
    const auto r1 = std::chrono::steady_clock::now();
    if (ctx->issue_trace)
      fprintf(stderr, "kb_host_trace pre order_pend_heaps_ms=%.3f reserve_fedok_ms=%.3f\n",
              std::chrono::duration<double, std::milli>(rq - r0).count(),
              std::chrono::duration<double, std::milli>(r1 - rq).count());
    using clk = std::chrono::steady_clock;
    struct FedEnd {  // the engine is stopped on every way out of the loop (paused or not)
      kb_ctx* c;
      bool on = false, paused = false;
      ~FedEnd() {
        if (on) (void)kb_fed_end(c);
      }
    } engine{ctx};
    clk::time_point pause_t0{};
    uint64_t pause_units = 0;  // off-engine units run since the pause began
    // A pause ends the engine instead of resuming it once it has gone on too long (the engine's idle exit is 1 s, 30 s
    // node-sharded). One GPU: 200 ms of wall clock. Node-sharded: every rank must end and relaunch its engine at the
    // same unit (a relaunch bumps the exchange epoch), so the bound is a unit count, which every rank's driver sees
    // alike -- never a rank's own clock.
    constexpr auto kMaxPause = std::chrono::milliseconds(200);
    constexpr uint64_t kMaxPauseUnitsSharded = 64;
    const auto pause_over = [&]() {
      return ctx->sharded ? pause_units >= kMaxPauseUnitsSharded : clk::now() - pause_t0 > kMaxPause;
    };
    double fed_begin_ms = 0;
    Unit u;
    int hv;
    {
      int q, j;
      hv = next_job(qheap, [this](int qq) -> GoHeap<int>& { return jheaps[qq]; }, q, j) ? 1 : 0;
      if (hv && check_specs(j)) return KB_E_INVALID;
      if (hv) u = unit_at(q, j);
    }
    // KB_HOST_TRACE=1: per-unit host timings on stderr at the end of the cycle (speculative issue, wait in
    // finish, bookkeeping after it)
    const bool trace = getenv("KB_HOST_TRACE") != nullptr;
    const int64_t stall_job = ctx->test_stall_job;  // tests (read once at kb_create): a host stall before unit k
    const int stall_ms = ctx->test_stall_ms;
    uint64_t n_iter_all = 0;
    const auto loop0 = std::chrono::steady_clock::now();
    double t_spec = 0, t_fin = 0, t_apply = 0;
    uint64_t n_iter = 0;
    const auto us = [](clk::time_point a, clk::time_point b) {
      return std::chrono::duration<double, std::micro>(b - a).count();
    };
    int n_slots = 2;
    const auto free_slot = [&]() {
      for (int sl = 0; sl < n_slots; ++sl) {
        bool used = false;
        for (const Flight& f : fl) used = used || f.slot == sl;
        if (!used) return sl;
      }
      return -1;
    };
    while (hv > 0) {
      // the unit's device mode: start the engine for a fed unit, stop it for the others (every unit in flight has
      // drained: the speculation never crosses a mode change)
      // (a unit the engine does not take pauses it: the launch paths run beside the idle engine, whose next
      // command comes fresh; a pause longer than kMaxPause ends the engine instead, before its idle exit)
      bool mode = u.fed;
      if (mode && engine.paused) {
        if (int rc = kb_fed_resume(ctx)) return rc;
        engine.paused = false;
      } else if (mode && !engine.on) {
        const auto b0 = clk::now();
        if (int rc = kb_fed_begin(ctx, max_unit)) return rc;
        engine.on = true;
        fed_begin_ms += us(b0, clk::now()) * 1e-3;
      } else if (!mode && engine.on && !engine.paused) {
        if (int rc = kb_fed_pause(ctx)) return rc;
        engine.paused = true;
        pause_t0 = clk::now();
        pause_units = 0;
      } else if (!mode && engine.paused && pause_over()) {
        engine.on = engine.paused = false;
        if (int rc = kb_fed_end(ctx)) return rc;
      }
      if (!mode && engine.paused) ++pause_units;
      if (!mode && !launch_pipe) {  // one kb_place_job per unit
        if (fed_allowed) ctx->stats.off_engine_units++;
        const kb_job_req req = make_req(u);
        kb_job_result res;
        if (int rc = kb_place_job(ctx, &req, pn.data(), pk.data(), &res)) return rc;
        const bool cont = apply(u, res);
        if (hook_rc) return hook_rc;
        Unit nu;
        hv = advance(u, cont, nu);
        if (hv < 0) return hv;
        u = nu;
        continue;
      }
      // pipelined (the fed engine: two units ahead, kJobSlots slots; the launch path: one ahead, two slots)
      n_slots = mode ? fed_depth() : 2;
      if (mode) ctx->stats.fed_last_depth = n_slots;
      fl.clear();
      {
        const kb_job_req req = make_req(u);
        if (int rc = kb_job_issue(ctx, &req, 0, nullptr)) return rc;
        fl.push_back(Flight{u, 0, kb_job_pred{}});
      }
      while (!fl.empty()) {
        const auto c0 = clk::now();
        // (a launch-path chain during a pause stops growing once the pause is over: it drains, and the loop top
        // ends the engine before its idle exit)
        const bool grow = mode || !engine.paused || !pause_over();
        for (; grow;) {  // top up the speculative chain
          const int fs = (int)fl.size() < n_slots ? free_slot() : -1;
          if (fs < 0 || !speculate(fs, mode)) break;
        }
        const auto c1 = clk::now();
        if (stall_job >= 0 && (int64_t)n_iter_all == stall_job)  // KB_TEST_STALL_JOB: a host stall (GC pause, ...)
          std::this_thread::sleep_for(std::chrono::milliseconds(stall_ms));
        ++n_iter_all;
        Flight f0 = fl.front();
        kb_job_result res;
        int rc = kb_job_finish(ctx, f0.slot, pn.data(), pk.data(), &res, 0);
        if (rc == kFedIdleExit) {  // the engine idled out during a host stall: this unit and the rest of the chain
          rc = kb_fed_abandon(ctx);  // run on the launch path (the speculative units never ran)
          engine.on = engine.paused = false;
          mode = false;
          fl.assign(1, f0);
          fl[0].slot = 0;
          n_slots = 2;
          if (rc == KB_OK) {
            const kb_job_req req = make_req(f0.u);
            rc = kb_job_issue(ctx, &req, 0, nullptr);
          }
          if (rc == KB_OK) rc = kb_job_finish(ctx, 0, pn.data(), pk.data(), &res, 0);
        }
        const kb_job_pred& pred = fl.front().pred;
        const bool chained = fl.size() > 1;
        const bool match = chained && rc == KB_OK && res.stop == pred.stop && (int)res.n_placed == pred.placed &&
                           jobs[f0.u.j].ready + (int)std::count(pk.begin(), pk.begin() + res.n_placed,
                                                                (int32_t)KB_PLACE_ALLOCATE) == pred.ready;
        if (mode) ctx->stats.fed_units++;
        if (chained && !match) {  // every later guard fails on the device as well: drain the skipped units
          if (mode) {
            ctx->stats.fed_mispredicts++;
            ctx->stats.fed_skipped += fl.size() - 1;
          }
          for (size_t i = 1; i < fl.size(); ++i) {
            kb_job_result skip;
            int rc2 = kb_job_finish(ctx, fl[i].slot, nullptr, nullptr, &skip, 1);
            if (rc2 == kFedIdleExit) {  // it never ran, nor did the ones after it: nothing to drain
              rc2 = kb_fed_abandon(ctx);
              engine.on = engine.paused = false;
              mode = false;
              n_slots = 2;
              if (rc == KB_OK) rc = rc2;
              break;
            }
            if (rc == KB_OK) rc = rc2;
          }
          fl.resize(1);
        }
        if (rc) return rc;
        const auto c2 = clk::now();
        if (!f0.u.fed && fed_allowed) ctx->stats.off_engine_units++;
        const bool cont = apply(f0.u, res);
        if (hook_rc) return hook_rc;
        Unit nu;
        hv = advance(f0.u, cont, nu);
        if (hv < 0) return hv;
        fl.erase(fl.begin());
        if (!fl.empty()) {
          if (hv == 0 || !(nu == fl[0].u)) {  // cannot happen: the speculation replays the loop
            for (const Flight& f : fl) {
              kb_job_result drain;
              (void)kb_job_finish(ctx, f.slot, nullptr, nullptr, &drain, 1);
            }
            ctx->err = "speculative unit does not match the loop order";
            return KB_E_STATE;
          }
        } else if (hv > 0 && nu.fed == mode && (mode || !engine.paused || !pause_over())) {
          const kb_job_req req = make_req(nu);
          const int fs = free_slot();
          if (int rc3 = kb_job_issue(ctx, &req, fs, nullptr)) return rc3;
          fl.push_back(Flight{nu, fs, kb_job_pred{}});
        }  // else the chain ends: no next unit, or the next one runs in the other mode (u, below)
        if (hv > 0) u = nu;
        if (trace) {
          const auto c3 = clk::now();
          t_spec += us(c0, c1), t_fin += us(c1, c2), t_apply += us(c2, c3);
          ++n_iter;
        }
      }
    }
    loop_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - loop0).count();
    if (trace && n_iter)
      fprintf(stderr, "kb_host_trace jobs=%llu speculate_issue_us=%.2f finish_wait_us=%.2f apply_next_us=%.2f\n",
              (unsigned long long)n_iter, t_spec / n_iter, t_fin / n_iter, t_apply / n_iter);
    out->n_events = n_events;
    const auto r3 = std::chrono::steady_clock::now();
    for (uint32_t t = 0; t < s.n_tasks; ++t) out->task_status[t] = task_status[t];
    if (engine.on) {
      engine.on = engine.paused = false;
      if (int rc = kb_fed_end(ctx)) return rc;
    }
    if (trace)
      fprintf(stderr, "kb_host_trace pre_ms=%.3f fed_begin_ms=%.3f post_ms=%.3f\n", us(r0, r1) * 1e-3,
              fed_begin_ms, us(r3, clk::now()) * 1e-3);
    return KB_OK;
  }
};

}  // namespace

extern "C" int kb_allocate(kb_ctx* ctx, const kb_session* ssn, kb_cycle_result* out) {
  if (!ctx || !ssn || !out) return KB_E_INVALID;
  if (ssn->n_rscalar > 62) {
    ctx->err = "more than 62 accounting scalar slots";
    return KB_E_UNSUPPORTED;
  }
  auto t0 = std::chrono::steady_clock::now();
  double dev0 = ctx->device_ms;
  for (uint32_t t = 0; t < ssn->n_tasks; ++t) out->task_node[t] = -1;
  for (uint32_t j = 0; j < ssn->n_jobs; ++j) out->job_fail_task[j] = -1;
  memset(out->job_reason_hist, 0, sizeof(uint32_t) * KB_NUM_REASONS * ssn->n_jobs);
  Driver d(ctx, *ssn, out);
  const auto ti = std::chrono::steady_clock::now();
  int rc = d.init();
  const auto tr = std::chrono::steady_clock::now();
  if (rc == KB_OK) rc = d.run();
  if (getenv("KB_HOST_TRACE"))
    fprintf(stderr, "kb_host_trace fill_ms=%.3f init_ms=%.3f run_ms=%.3f loop_ms=%.3f\n",
            std::chrono::duration<double, std::milli>(ti - t0).count(),
            std::chrono::duration<double, std::milli>(tr - ti).count(),
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr).count(), d.loop_ms);
  out->elapsed_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  out->device_ms = ctx->device_ms - dev0;
  return rc;
}
