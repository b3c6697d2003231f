// Host event tracer (reference behaviour: paddle/fluid/platform/profiler/host_tracer.cc,
// host_event_recorder.h and chrometracing_logger.cc).
//
// Each thread appends completed ranges to its own buffer (one uncontended mutex per
// thread), so RecordEvent costs ~100 ns when enabled and one relaxed load when disabled.
// Export writes chrome://tracing / Perfetto JSON; the Python profiler merges these host
// ranges with the HIP kernel timeline collected by roctracer (torch.profiler/kineto).
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <mutex>
#include <string>
#include <sys/syscall.h>
#include <unistd.h>
#include <vector>

#include "runtime.h"

namespace {

struct Event {
  std::string name;
  int64_t start_ns, end_ns;
  int32_t type;
};

struct ThreadBuf {
  std::mutex mu;
  std::vector<Event> events;
  std::vector<std::pair<std::string, int64_t>> stack;  // open ranges (name, start)
  std::vector<int32_t> stack_types;
  int64_t tid;
};

std::atomic<int> g_enabled{0};
std::mutex g_mu;
std::vector<std::shared_ptr<ThreadBuf>> g_bufs;

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::system_clock::now().time_since_epoch()).count();
}

ThreadBuf& tbuf() {
  thread_local std::shared_ptr<ThreadBuf> b;
  if (!b) {
    b = std::make_shared<ThreadBuf>();
    b->tid = static_cast<int64_t>(syscall(SYS_gettid));
    std::lock_guard<std::mutex> g(g_mu);
    g_bufs.push_back(b);
  }
  return *b;
}

void json_escape(FILE* f, const std::string& s) {
  for (char c : s) {
    if (c == '"' || c == '\\') {
      fputc('\\', f);
      fputc(c, f);
    } else if (static_cast<unsigned char>(c) < 0x20) {
      fprintf(f, "\\u%04x", c);
    } else {
      fputc(c, f);
    }
  }
}

const char* type_name(int32_t t) {
  switch (t) {
    case 1: return "Operator";
    case 2: return "Dataloader";
    case 3: return "ProfileStep";
    case 4: return "Forward";
    case 5: return "Backward";
    case 6: return "Optimization";
    case 7: return "Communication";
    case 8: return "PythonOp";
    default: return "UserDefined";
  }
}

}  // namespace

PHA_API void pha_tracer_enable(int on) { g_enabled.store(on, std::memory_order_release); }
PHA_API int pha_tracer_enabled() { return g_enabled.load(std::memory_order_relaxed); }
PHA_API int64_t pha_tracer_now_ns() { return now_ns(); }

PHA_API void pha_tracer_push(const char* name, int32_t type) {
  if (!g_enabled.load(std::memory_order_relaxed)) return;
  ThreadBuf& b = tbuf();
  std::lock_guard<std::mutex> g(b.mu);
  b.stack.emplace_back(name, now_ns());
  b.stack_types.push_back(type);
}

PHA_API void pha_tracer_pop() {
  ThreadBuf& b = tbuf();
  std::lock_guard<std::mutex> g(b.mu);
  if (b.stack.empty()) return;
  auto top = std::move(b.stack.back());
  int32_t t = b.stack_types.back();
  b.stack.pop_back();
  b.stack_types.pop_back();
  if (g_enabled.load(std::memory_order_relaxed)) b.events.push_back({std::move(top.first), top.second, now_ns(), t});
}

// Record an already-timed range (e.g. measured in Python or converted from device timestamps).
PHA_API void pha_tracer_record(const char* name, int32_t type, int64_t start_ns, int64_t end_ns) {
  if (!g_enabled.load(std::memory_order_relaxed)) return;
  ThreadBuf& b = tbuf();
  std::lock_guard<std::mutex> g(b.mu);
  b.events.push_back({name, start_ns, end_ns, type});
}

PHA_API int64_t pha_tracer_count() {
  std::lock_guard<std::mutex> g(g_mu);
  int64_t n = 0;
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> l(b->mu);
    n += static_cast<int64_t>(b->events.size());
  }
  return n;
}

PHA_API void pha_tracer_clear() {
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> l(b->mu);
    b->events.clear();
  }
}

// Write {"traceEvents":[...]} ("X" complete events, microsecond timestamps). Returns the
// number of events written or -1 if the file could not be opened.
PHA_API int64_t pha_tracer_export_chrome(const char* path, int64_t pid) {
  FILE* f = fopen(path, "w");
  if (!f) return -1;
  fputs("{\"traceEvents\":[\n", f);
  int64_t n = 0;
  std::lock_guard<std::mutex> g(g_mu);
  for (auto& b : g_bufs) {
    std::lock_guard<std::mutex> l(b->mu);
    for (const Event& e : b->events) {
      fputs(n ? ",\n{\"name\":\"" : "{\"name\":\"", f);
      json_escape(f, e.name);
      fprintf(f, "\",\"cat\":\"%s\",\"ph\":\"X\",\"pid\":%lld,\"tid\":%lld,\"ts\":%.3f,\"dur\":%.3f}", type_name(e.type),
              static_cast<long long>(pid), static_cast<long long>(b->tid), e.start_ns / 1000.0,
              (e.end_ns - e.start_ns) / 1000.0);
      ++n;
    }
  }
  fputs("\n],\"displayTimeUnit\":\"ms\"}\n", f);
  fclose(f);
  return n;
}
