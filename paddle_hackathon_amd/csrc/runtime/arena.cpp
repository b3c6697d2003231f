// Best-fit, coalescing offset allocator over one contiguous region, plus an offline
// lifetime-based memory planner (reference behaviour:
// paddle/fluid/memory/allocation/auto_growth_best_fit_allocator.cc and the static-graph
// memory-reuse passes in paddle/fluid/framework/ir/memory_optimize_pass).
//
// The arena only does the bookkeeping: the caller owns the backing buffer (a single large
// torch allocation in HBM3E or pinned host memory) and turns offsets into views. Sizing one
// flat buffer for a whole step avoids allocator fragmentation at 288 GB scale and lets a
// HIP-graph capture see stable addresses.
#include <algorithm>
#include <map>
#include <numeric>
#include <set>
#include <vector>

#include "runtime.h"

namespace {

struct Arena {
  int64_t capacity, align, used = 0, peak = 0;
  std::map<int64_t, int64_t> free_by_off;         // offset -> size
  std::set<std::pair<int64_t, int64_t>> free_set;  // (size, offset)
  std::map<int64_t, int64_t> live;                 // offset -> size

  void add_free(int64_t off, int64_t size) {
    free_by_off[off] = size;
    free_set.insert({size, off});
  }
  void del_free(std::map<int64_t, int64_t>::iterator it) {
    free_set.erase({it->second, it->first});
    free_by_off.erase(it);
  }
};

int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

}  // namespace

PHA_API void* pha_arena_create(int64_t capacity, int64_t alignment) {
  if (capacity <= 0) return nullptr;
  auto* a = new Arena();
  a->align = alignment > 0 ? alignment : 256;
  a->capacity = capacity / a->align * a->align;
  a->add_free(0, a->capacity);
  return a;
}

PHA_API void pha_arena_destroy(void* h) { delete static_cast<Arena*>(h); }

// Returns the offset of a block of at least `size` bytes, or -1 when no free block fits.
PHA_API int64_t pha_arena_alloc(void* h, int64_t size) {
  auto* a = static_cast<Arena*>(h);
  size = round_up(std::max<int64_t>(size, 1), a->align);
  auto it = a->free_set.lower_bound({size, -1});
  if (it == a->free_set.end()) return -1;
  const int64_t bsize = it->first, off = it->second;
  a->del_free(a->free_by_off.find(off));
  if (bsize > size) a->add_free(off + size, bsize - size);
  a->live[off] = size;
  a->used += size;
  a->peak = std::max(a->peak, a->used);
  return off;
}

// Frees the block at `offset`, merging with free neighbours. Returns 0, or -1 if unknown.
PHA_API int pha_arena_free(void* h, int64_t offset) {
  auto* a = static_cast<Arena*>(h);
  auto lv = a->live.find(offset);
  if (lv == a->live.end()) return -1;
  int64_t off = offset, size = lv->second;
  a->live.erase(lv);
  a->used -= size;
  auto next = a->free_by_off.lower_bound(off);
  if (next != a->free_by_off.end() && next->first == off + size) {
    size += next->second;
    a->del_free(next);
  }
  auto prev = a->free_by_off.lower_bound(off);
  if (prev != a->free_by_off.begin()) {
    --prev;
    if (prev->first + prev->second == off) {
      off = prev->first;
      size += prev->second;
      a->del_free(prev);
    }
  }
  a->add_free(off, size);
  return 0;
}

PHA_API int64_t pha_arena_used(void* h) { return static_cast<Arena*>(h)->used; }
PHA_API int64_t pha_arena_peak(void* h) { return static_cast<Arena*>(h)->peak; }
PHA_API int64_t pha_arena_capacity(void* h) { return static_cast<Arena*>(h)->capacity; }
PHA_API int64_t pha_arena_largest_free(void* h) {
  auto* a = static_cast<Arena*>(h);
  return a->free_set.empty() ? 0 : a->free_set.rbegin()->first;
}
PHA_API int64_t pha_arena_num_free_blocks(void* h) { return static_cast<int64_t>(static_cast<Arena*>(h)->free_by_off.size()); }

// Offline planner: tensor i is live over op steps [first_use[i], last_use[i]] (inclusive).
// Assigns offsets so tensors with overlapping lifetimes never overlap in memory, placing
// larger tensors first (greedy by size, best-fit against already-placed conflicts).
// Returns the total arena bytes needed (the plan's peak).
PHA_API int64_t pha_plan_memory(int64_t n, const int64_t* sizes, const int64_t* first_use, const int64_t* last_use,
                                int64_t alignment, int64_t* out_offsets) {
  if (alignment <= 0) alignment = 256;
  std::vector<int64_t> order(n);
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](int64_t x, int64_t y) { return sizes[x] > sizes[y]; });
  std::vector<int64_t> placed;
  int64_t total = 0;
  for (int64_t i : order) {
    const int64_t sz = round_up(std::max<int64_t>(sizes[i], 1), alignment);
    std::vector<std::pair<int64_t, int64_t>> busy;  // [off, end) of lifetime-overlapping placed tensors
    for (int64_t j : placed)
      if (!(last_use[j] < first_use[i] || last_use[i] < first_use[j]))
        busy.push_back({out_offsets[j], out_offsets[j] + round_up(std::max<int64_t>(sizes[j], 1), alignment)});
    std::sort(busy.begin(), busy.end());
    int64_t best = -1, best_gap = INT64_MAX, cursor = 0;
    for (auto& b : busy) {
      if (b.first > cursor) {
        const int64_t gap = b.first - cursor;
        if (gap >= sz && gap < best_gap) {
          best = cursor;
          best_gap = gap;
        }
      }
      cursor = std::max(cursor, b.second);
    }
    if (best < 0) best = cursor;
    out_offsets[i] = best;
    total = std::max(total, best + sz);
    placed.push_back(i);
  }
  return total;
}
