// Batch collation: copy N equally-sized samples into one contiguous buffer using a
// persistent thread pool. The destination is usually a pinned (hipHostMalloc'd) tensor so
// the following H2D copy is a single async DMA on a side stream
// (reference behaviour: paddle/fluid/operators/reader/buffered_reader.cc + the Python
// default_collate_fn in python/paddle/fluid/dataloader/collate.py).
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "runtime.h"

namespace pha {
namespace {

class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) workers_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  int size() const { return static_cast<int>(workers_.size()); }

  // Run fn(i) for i in [0, tasks) on the pool plus the calling thread; blocks until done.
  void run(int tasks, const std::function<void(int)>& fn) {
    std::unique_lock<std::mutex> lk(run_mu_);
    uint64_t g;
    {
      std::lock_guard<std::mutex> l(mu_);
      fn_ = &fn;
      next_ = 0;
      tasks_ = tasks;
      pending_ = tasks;
      g = ++gen_;
    }
    cv_.notify_all();
    work(g);
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [this] { return pending_ == 0; });
    fn_ = nullptr;
  }

 private:
  // Claims are made under the lock and tagged with the generation, so a worker that wakes
  // late can never execute a task of a different run.
  void work(uint64_t g) {
    for (;;) {
      int i;
      const std::function<void(int)>* f;
      {
        std::lock_guard<std::mutex> l(mu_);
        if (g != gen_ || next_ >= tasks_) return;
        i = next_++;
        f = fn_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> l(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      uint64_t g;
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        g = seen = gen_;
      }
      work(g);
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int next_ = 0, tasks_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

Pool& pool() {
  static Pool p(std::max(1u, std::min(8u, std::thread::hardware_concurrency())) - 1);
  return p;
}

}  // namespace

void parallel_for(int64_t n, int nthreads, void (*fn)(int64_t, int64_t, void*), void* ctx) {
  if (n <= 0) return;
  int chunks = std::max(1, std::min<int>(nthreads > 0 ? nthreads : pool().size() + 1, (int)n));
  if (chunks == 1) {
    fn(0, n, ctx);
    return;
  }
  int64_t per = (n + chunks - 1) / chunks;
  std::function<void(int)> body = [&](int c) {
    int64_t b = c * per, e = std::min<int64_t>(n, b + per);
    if (b < e) fn(b, e, ctx);
  };
  pool().run(chunks, body);
}

}  // namespace pha

namespace {
struct StackCtx {
  const void* const* srcs;
  char* dst;
  size_t bytes;
};
struct GatherCtx {
  const char* src;
  const int64_t* idx;
  char* dst;
  size_t row_bytes;
};
}  // namespace

// dst[i*bytes : (i+1)*bytes] = srcs[i][0:bytes]. Small batches run inline; large ones fan out.
PHA_API int pha_stack_arrays(const void* const* srcs, int64_t n, size_t bytes, void* dst, int nthreads) {
  if (!srcs || !dst) return -1;
  StackCtx c{srcs, static_cast<char*>(dst), bytes};
  const size_t total = bytes * static_cast<size_t>(n);
  if (total < (1u << 20)) nthreads = 1;  // below 1 MiB threading costs more than it saves
  pha::parallel_for(n, nthreads, [](int64_t b, int64_t e, void* p) {
    auto* c = static_cast<StackCtx*>(p);
    for (int64_t i = b; i < e; ++i) std::memcpy(c->dst + i * c->bytes, c->srcs[i], c->bytes);
  }, &c);
  return 0;
}

// dst[i] = src[idx[i]] for row-major rows of row_bytes (embedding-table / dataset gathers).
PHA_API int pha_gather_rows(const void* src, const int64_t* idx, int64_t n, size_t row_bytes, void* dst,
                            int nthreads) {
  GatherCtx c{static_cast<const char*>(src), idx, static_cast<char*>(dst), row_bytes};
  if (row_bytes * static_cast<size_t>(n) < (1u << 20)) nthreads = 1;
  pha::parallel_for(n, nthreads, [](int64_t b, int64_t e, void* p) {
    auto* c = static_cast<GatherCtx*>(p);
    for (int64_t i = b; i < e; ++i) std::memcpy(c->dst + i * c->row_bytes, c->src + c->idx[i] * c->row_bytes, c->row_bytes);
  }, &c);
  return 0;
}

PHA_API int pha_runtime_version() { return 1; }
