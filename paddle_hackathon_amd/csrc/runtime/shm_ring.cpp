// Shared-memory slot ring for multi-process DataLoader workers.
//
// Workers (forked processes) collate a batch and write it straight into a slot of a POSIX
// shared-memory segment; the trainer process consumes slots strictly in batch order and
// copies them into pinned staging memory for an async H2D DMA. This replaces pickling whole
// batches through a pipe (reference behaviour: python/paddle/fluid/dataloader/worker.py +
// dataloader_iter.py with use_shared_memory=True, and the C++ LoDTensorBlockingQueue in
// paddle/fluid/operators/reader/lod_tensor_blocking_queue.h).
//
// Slot life cycle: FREE -> WRITING (producer CAS) -> READY (commit, seq published)
//                  -> READING (consumer CAS on the wanted seq) -> FREE (release).
// Waiting uses shared (non-private) futexes on two epoch counters, so blocked producers and
// the consumer sleep in the kernel instead of spinning. Deadlock freedom requires the
// trainer to keep at most `nslots` batches outstanding, which the Python side enforces.
#include <fcntl.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <climits>
#include <cstring>
#include <ctime>
#include <new>
#include <string>

#include "runtime.h"

namespace {

constexpr uint32_t kMagic = 0x50484152;  // "PHAR"
enum SlotState : uint32_t { FREE = 0, WRITING = 1, READY = 2, READING = 3 };

struct alignas(64) RingHeader {
  uint32_t magic;
  uint32_t nslots;
  uint64_t slot_bytes;
  std::atomic<uint32_t> closed;
  std::atomic<uint32_t> free_epoch;   // bumped on release  (producers wait here)
  std::atomic<uint32_t> ready_epoch;  // bumped on commit   (consumer waits here)
};

struct alignas(64) SlotHeader {
  std::atomic<uint32_t> state;
  uint32_t pad;
  std::atomic<int64_t> seq;
  uint64_t nbytes;
};

struct Ring {
  void* base;
  size_t map_bytes;
  std::string name;
  bool owner;
  RingHeader* hdr() const { return static_cast<RingHeader*>(base); }
  SlotHeader* slot(uint32_t i) const {
    return reinterpret_cast<SlotHeader*>(static_cast<char*>(base) + sizeof(RingHeader)) + i;
  }
  char* data(uint32_t i) const {
    char* d0 = static_cast<char*>(base) + sizeof(RingHeader) + sizeof(SlotHeader) * hdr()->nslots;
    d0 = reinterpret_cast<char*>((reinterpret_cast<uintptr_t>(d0) + 4095) & ~uintptr_t(4095));
    return d0 + static_cast<size_t>(i) * hdr()->slot_bytes;
  }
};

size_t layout_bytes(uint32_t nslots, uint64_t slot_bytes) {
  size_t h = sizeof(RingHeader) + sizeof(SlotHeader) * nslots;
  h = (h + 4095) & ~size_t(4095);
  return h + nslots * slot_bytes;
}

int futex_wait(std::atomic<uint32_t>* addr, uint32_t expected, int timeout_ms) {
  struct timespec ts, *tsp = nullptr;
  if (timeout_ms >= 0) {
    ts.tv_sec = timeout_ms / 1000;
    ts.tv_nsec = (timeout_ms % 1000) * 1000000L;
    tsp = &ts;
  }
  return static_cast<int>(syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAIT, expected, tsp, nullptr, 0));
}

void futex_wake_all(std::atomic<uint32_t>* addr) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), FUTEX_WAKE, INT_MAX, nullptr, nullptr, 0);
}

int64_t now_ms() {
  using namespace std::chrono;
  return duration_cast<milliseconds>(steady_clock::now().time_since_epoch()).count();
}

Ring* map_ring(const char* name, bool create, uint32_t nslots, uint64_t slot_bytes) {
  int fd = shm_open(name, create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) return nullptr;
  size_t bytes;
  if (create) {
    bytes = layout_bytes(nslots, slot_bytes);
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      close(fd);
      shm_unlink(name);
      return nullptr;
    }
  } else {
    struct stat st;
    if (fstat(fd, &st) != 0) {
      close(fd);
      return nullptr;
    }
    bytes = static_cast<size_t>(st.st_size);
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    if (create) shm_unlink(name);
    return nullptr;
  }
  Ring* r = new Ring{p, bytes, name, create};
  if (create) {
    RingHeader* h = new (p) RingHeader();
    h->magic = kMagic;
    h->nslots = nslots;
    h->slot_bytes = slot_bytes;
    h->closed.store(0);
    h->free_epoch.store(0);
    h->ready_epoch.store(0);
    for (uint32_t i = 0; i < nslots; ++i) {
      SlotHeader* s = new (r->slot(i)) SlotHeader();
      s->state.store(FREE);
      s->seq.store(-1);
      s->nbytes = 0;
    }
  } else if (r->hdr()->magic != kMagic) {
    munmap(p, bytes);
    delete r;
    return nullptr;
  }
  return r;
}

}  // namespace

PHA_API void* pha_ring_create(const char* name, uint32_t nslots, uint64_t slot_bytes) {
  if (nslots == 0 || slot_bytes == 0) return nullptr;
  slot_bytes = (slot_bytes + 4095) & ~uint64_t(4095);
  return map_ring(name, true, nslots, slot_bytes);
}

PHA_API void* pha_ring_attach(const char* name) { return map_ring(name, false, 0, 0); }

PHA_API uint32_t pha_ring_nslots(void* h) { return static_cast<Ring*>(h)->hdr()->nslots; }
PHA_API uint64_t pha_ring_slot_bytes(void* h) { return static_cast<Ring*>(h)->hdr()->slot_bytes; }
PHA_API void* pha_ring_slot_ptr(void* h, uint32_t i) { return static_cast<Ring*>(h)->data(i); }
PHA_API uint64_t pha_ring_slot_nbytes(void* h, uint32_t i) { return static_cast<Ring*>(h)->slot(i)->nbytes; }

// Producer: claim a FREE slot. Returns slot index, -1 on timeout, -2 if the ring is closed.
PHA_API int pha_ring_acquire_write(void* h, int timeout_ms) {
  Ring* r = static_cast<Ring*>(h);
  RingHeader* hd = r->hdr();
  const int64_t deadline = timeout_ms < 0 ? -1 : now_ms() + timeout_ms;
  for (;;) {
    if (hd->closed.load(std::memory_order_acquire)) return -2;
    uint32_t epoch = hd->free_epoch.load(std::memory_order_acquire);
    for (uint32_t i = 0; i < hd->nslots; ++i) {
      uint32_t expect = FREE;
      if (r->slot(i)->state.compare_exchange_strong(expect, WRITING, std::memory_order_acq_rel)) return static_cast<int>(i);
    }
    int wait = -1;
    if (deadline >= 0) {
      int64_t left = deadline - now_ms();
      if (left <= 0) return -1;
      wait = static_cast<int>(left);
    }
    futex_wait(&hd->free_epoch, epoch, wait);
  }
}

// Producer: publish slot i as batch `seq` holding `nbytes` payload bytes.
PHA_API int pha_ring_commit(void* h, uint32_t i, int64_t seq, uint64_t nbytes) {
  Ring* r = static_cast<Ring*>(h);
  SlotHeader* s = r->slot(i);
  if (nbytes > r->hdr()->slot_bytes) return -1;
  s->nbytes = nbytes;
  s->seq.store(seq, std::memory_order_relaxed);
  s->state.store(READY, std::memory_order_release);
  r->hdr()->ready_epoch.fetch_add(1, std::memory_order_acq_rel);
  futex_wake_all(&r->hdr()->ready_epoch);
  return 0;
}

// Producer abort: hand a claimed slot back without publishing.
PHA_API void pha_ring_abort(void* h, uint32_t i) {
  Ring* r = static_cast<Ring*>(h);
  r->slot(i)->state.store(FREE, std::memory_order_release);
  r->hdr()->free_epoch.fetch_add(1, std::memory_order_acq_rel);
  futex_wake_all(&r->hdr()->free_epoch);
}

// Consumer: wait for batch `seq`. Returns slot index, -1 on timeout, -2 if closed.
PHA_API int pha_ring_acquire_read(void* h, int64_t seq, int timeout_ms) {
  Ring* r = static_cast<Ring*>(h);
  RingHeader* hd = r->hdr();
  const int64_t deadline = timeout_ms < 0 ? -1 : now_ms() + timeout_ms;
  for (;;) {
    uint32_t epoch = hd->ready_epoch.load(std::memory_order_acquire);
    for (uint32_t i = 0; i < hd->nslots; ++i) {
      SlotHeader* s = r->slot(i);
      if (s->state.load(std::memory_order_acquire) == READY && s->seq.load(std::memory_order_relaxed) == seq) {
        uint32_t expect = READY;
        if (s->state.compare_exchange_strong(expect, READING, std::memory_order_acq_rel)) return static_cast<int>(i);
      }
    }
    if (hd->closed.load(std::memory_order_acquire)) return -2;
    int wait = -1;
    if (deadline >= 0) {
      int64_t left = deadline - now_ms();
      if (left <= 0) return -1;
      wait = static_cast<int>(left);
    }
    futex_wait(&hd->ready_epoch, epoch, wait);
  }
}

PHA_API void pha_ring_release(void* h, uint32_t i) { pha_ring_abort(h, i); }

// Number of READY slots (diagnostics / tests).
PHA_API int pha_ring_ready_count(void* h) {
  Ring* r = static_cast<Ring*>(h);
  int n = 0;
  for (uint32_t i = 0; i < r->hdr()->nslots; ++i) n += r->slot(i)->state.load() == READY;
  return n;
}

// Wake every waiter and make further acquires fail (shutdown / worker death).
PHA_API void pha_ring_close(void* h) {
  Ring* r = static_cast<Ring*>(h);
  r->hdr()->closed.store(1, std::memory_order_release);
  r->hdr()->free_epoch.fetch_add(1);
  r->hdr()->ready_epoch.fetch_add(1);
  futex_wake_all(&r->hdr()->free_epoch);
  futex_wake_all(&r->hdr()->ready_epoch);
}

// Unmap (and unlink if this handle created the segment).
PHA_API void pha_ring_destroy(void* h) {
  Ring* r = static_cast<Ring*>(h);
  munmap(r->base, r->map_bytes);
  if (r->owner) shm_unlink(r->name.c_str());
  delete r;
}

// Unmap only, never unlink (used in forked children that inherited the creator's handle).
PHA_API void pha_ring_detach(void* h) {
  Ring* r = static_cast<Ring*>(h);
  munmap(r->base, r->map_bytes);
  delete r;
}
