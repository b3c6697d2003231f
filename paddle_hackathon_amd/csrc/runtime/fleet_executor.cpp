// Fleet executor carrier: credit-based dataflow over a task graph (reference
// paddle/fluid/distributed/fleet_executor/: Carrier, Interceptor (Compute / Amplifier / Source /
// Sink), TaskNode with upstream/downstream buffer sizes, the DATA_IS_READY / DATA_IS_USELESS
// message protocol).
//
// Every local task runs its micro-batch steps on its own thread. Step i of task t may start
// once (a) each upstream u has finished step i (DATA_IS_READY) and (b) each downstream d still
// has buffer credit: steps_done[t] - steps_consumed_by[d] < buff_size(t -> d) (DATA_IS_USELESS
// returns the credit when d finishes the step that read it). The step body is a callback into
// the host (Python: run a sub-Program / a stage function, or a send / recv over RCCL for an
// edge to another rank's carrier); this thread blocks in it without holding any carrier lock,
// so communication of one task overlaps computation of the others. An amplifier task runs one
// step every `amplify` upstream steps (gradient-accumulation style).
#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <map>
#include <mutex>
#include <thread>
#include <vector>

#include "runtime.h"

namespace {

struct Edge {
  int to;
  int buff;
};

struct FeTask {
  int id = 0, max_run = 0, amplify = 1;
  std::vector<int> ups;
  std::vector<Edge> downs;
  int64_t done = 0;                  // steps finished
  std::map<int, int64_t> consumed;   // downstream id -> steps of ours it has consumed
};

typedef int (*FeStepFn)(int task, int64_t step, void* ctx);

struct Carrier {
  std::mutex mu;
  std::condition_variable cv;
  std::map<int, FeTask> tasks;
  bool failed = false;
  int status = 0;
  std::vector<std::pair<int, int64_t>> trace;   // (task, step) in completion order

  int64_t ups_needed(const FeTask& t, int64_t step) const {   // upstream steps that must be done first
    return (step + 1) * t.amplify;
  }
  bool ready(const FeTask& t, int64_t step) {
    for (int u : t.ups) {
      auto it = tasks.find(u);
      if (it == tasks.end()) continue;
      if (it->second.done < std::min<int64_t>(ups_needed(t, step), it->second.max_run)) return false;
    }
    for (const Edge& e : t.downs) {
      auto it = t.consumed.find(e.to);
      const int64_t used = it == t.consumed.end() ? 0 : it->second;
      if (t.done - used >= e.buff) return false;   // no credit on this edge
    }
    return true;
  }
};

void run_task(Carrier* c, int id, FeStepFn fn, void* ctx) {
  for (;;) {
    int64_t step;
    {
      std::unique_lock<std::mutex> g(c->mu);
      FeTask& t = c->tasks[id];
      if (t.done >= t.max_run || c->failed) return;
      step = t.done;
      c->cv.wait(g, [&] { return c->failed || c->ready(t, step); });
      if (c->failed) return;
    }
    const int rc = fn(id, step, ctx);   // the step body runs without the carrier lock
    std::lock_guard<std::mutex> g(c->mu);
    FeTask& t = c->tasks[id];
    if (rc != 0) {
      c->failed = true;
      c->status = rc;
      c->cv.notify_all();
      return;
    }
    t.done = step + 1;
    c->trace.emplace_back(id, step);
    // DATA_IS_USELESS: our upstreams regain the credit of the steps this one consumed
    for (int u : t.ups) {
      auto it = c->tasks.find(u);
      if (it != c->tasks.end())
        it->second.consumed[id] = std::min<int64_t>(c->ups_needed(t, step), it->second.max_run);
    }
    c->cv.notify_all();   // DATA_IS_READY to the downstreams
  }
}

}  // namespace

PHA_API void* pha_fe_create() { return new Carrier(); }

PHA_API void pha_fe_destroy(void* h) { delete static_cast<Carrier*>(h); }

PHA_API int pha_fe_add_task(void* h, int id, int max_run, int amplify) {
  auto* c = static_cast<Carrier*>(h);
  if (max_run < 0 || amplify < 1 || c->tasks.count(id)) return -1;
  FeTask& t = c->tasks[id];
  t.id = id;
  t.max_run = max_run;
  t.amplify = amplify;
  return 0;
}

// edge up -> down with `buff` steps of credit; only local tasks are known to the carrier: an
// edge to a remote task is the host's send / recv task pair
PHA_API int pha_fe_add_edge(void* h, int up, int down, int buff) {
  auto* c = static_cast<Carrier*>(h);
  auto iu = c->tasks.find(up), id = c->tasks.find(down);
  if (iu == c->tasks.end() || id == c->tasks.end() || buff < 1) return -1;
  iu->second.downs.push_back({down, buff});
  id->second.ups.push_back(up);
  return 0;
}

// run every task to max_run on its own thread; returns 0 or the first failing step's code
PHA_API int pha_fe_run(void* h, FeStepFn fn, void* ctx) {
  auto* c = static_cast<Carrier*>(h);
  std::vector<std::thread> ths;
  std::vector<int> ids;
  for (auto& kv : c->tasks) ids.push_back(kv.first);
  for (int id : ids) ths.emplace_back(run_task, c, id, fn, ctx);
  for (auto& t : ths) t.join();
  return c->failed ? (c->status ? c->status : -1) : 0;
}

PHA_API int64_t pha_fe_trace_len(void* h) { return (int64_t) static_cast<Carrier*>(h)->trace.size(); }

PHA_API void pha_fe_trace(void* h, int32_t* task, int64_t* step) {
  auto* c = static_cast<Carrier*>(h);
  for (size_t i = 0; i < c->trace.size(); ++i) {
    task[i] = c->trace[i].first;
    step[i] = c->trace[i].second;
  }
}
