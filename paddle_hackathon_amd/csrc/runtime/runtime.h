// Host-side native runtime for paddle_hackathon_amd (C ABI, loaded with ctypes).
//
//   collate.cpp  - multi-threaded batch stacking / gather into (pinned) staging buffers
//   shm_ring.cpp - shared-memory slot ring used by multi-process DataLoader workers
//   bucket.cpp   - gradient bucket planner for DataParallel / sharding collectives
//   tracer.cpp   - low-overhead host event tracer with chrome-trace export (profiler)
//   arena.cpp    - best-fit, coalescing offset allocator (memory planner / flat buffers)
//   fleet_executor.cpp - credit-based dataflow carrier over a task graph (fleet executor)
#pragma once
#include <cstddef>
#include <cstdint>

#define PHA_API extern "C" __attribute__((visibility("default")))

namespace pha {
// Fixed-size worker pool shared by the collate helpers.
void parallel_for(int64_t n, int nthreads, void (*fn)(int64_t begin, int64_t end, void* ctx), void* ctx);
}  // namespace pha
