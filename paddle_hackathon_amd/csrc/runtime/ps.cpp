// Parameter server: native dense/sparse tables with server-side optimizer rules, served over
// TCP to trainer processes (reference behaviour: paddle/fluid/distributed/ps/{service,table}
// — BrpcPsServer/BrpcPsClient, MemoryDenseTable, MemorySparseTable with its entry policies,
// SparseAccessor and the rules of table/sparse_sgd_rule.cc; python/paddle/distributed/ps/the_one_ps.py).
//
// Design for an MI355X node: trainers are GPU processes (one per GPU) that keep the dense
// model in HBM and page only the huge, sparsely touched embedding rows in and out of host
// memory; the server is a CPU process holding those tables in DRAM. So the server is plain
// C++: a thread per trainer connection, a length-prefixed binary protocol (no RPC framework),
// sparse tables split into 64 lock-striped hash shards so pushes from different trainers to
// different ids proceed in parallel, and dense tables guarded by one mutex each with an
// optional synchronous-merge mode (the grads of all trainers averaged and applied once,
// version bumped; pulls may wait for a version).
//
// Round 2 depth (reference paddle/fluid/distributed/ps/table/): a CTR accessor rule
// (ctr_accessor.cc: show/click statistics per feature, embedding + lazily created embedx with
// their own AdaGrad state, score-based embedx creation, decay/delete shrink and base-threshold
// save), a spill-to-disk mode of the sparse table (ssd_sparse_table.cc: a bounded in-memory row
// cache per shard, the coldest rows appended to a per-shard file and read back on access), and a
// graph table (common_graph_table.cc: weighted adjacency lists + node features, uniform or
// weighted neighbour sampling without replacement, random node sampling).
//
// Wire format (little endian): request  = {u32 magic, u32 cmd, u32 table, u32 arg, u64 n, u64 nbytes} + payload
//                              response = {i32 status, u32 pad, u64 nbytes} + payload
#include <arpa/inet.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "runtime.h"

namespace {

constexpr uint32_t kMagic = 0x50484153;  // "PHAS"
constexpr int kShards = 64;

enum Cmd : uint32_t {
  CREATE_DENSE = 1, CREATE_SPARSE = 2, PULL_DENSE = 3, PUSH_DENSE = 4, SET_DENSE = 5, PULL_SPARSE = 6,
  PUSH_SPARSE = 7, BARRIER = 8, SAVE = 9, LOAD = 10, TABLE_SIZE = 11, SHRINK = 12, STOP = 13,
  PUSH_SPARSE_DELTA = 14, PING = 15, SET_SPILL = 16,
  GRAPH_ADD_EDGES = 20, GRAPH_SAMPLE = 21, GRAPH_SET_FEAT = 22, GRAPH_GET_FEAT = 23, GRAPH_RANDOM_NODES = 24,
  GRAPH_NODE_COUNT = 25,
};

// optimizer rules applied on the server (sparse_sgd_rule.cc: Naive / AdaGrad (one g2sum per
// row) / StdAdaGrad (per element) / Adam; SUM = geo-SGD delta accumulation)
enum Rule : int32_t { SGD = 0, ADAGRAD = 1, STD_ADAGRAD = 2, ADAM = 3, SUM = 4, CTR = 5 };

#pragma pack(push, 1)
struct ReqHdr { uint32_t magic, cmd, table, arg; uint64_t n, nbytes; };
struct RespHdr { int32_t status; uint32_t pad; uint64_t nbytes; };
struct TableCfg {
  int32_t rule, dim, sync_trainers, entry_kind;   // entry: 0 always, 1 probability, 2 count filter
  float lr, beta1, beta2, eps, initial_g2sum, initial_range, min_bound, max_bound, entry_value;
  uint64_t seed;
  // CTR accessor (ctr_accessor.h CtrCommonAccessor parameters)
  float nonclk_coeff, click_coeff, embedx_threshold, show_click_decay, delete_threshold, delete_after_unseen_days,
      base_threshold;
  uint64_t cache_rows;   // spill mode: resident rows per table (0 = unbounded)
};
#pragma pack(pop)

bool read_full(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    const ssize_t r = ::recv(fd, c, n, 0);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    c += r;
    n -= (size_t)r;
  }
  return true;
}

bool write_full(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    const ssize_t r = ::send(fd, c, n, MSG_NOSIGNAL);
    if (r <= 0) {
      if (r < 0 && errno == EINTR) continue;
      return false;
    }
    c += r;
    n -= (size_t)r;
  }
  return true;
}

// optimizer-state floats kept after the weights of one row (sparse) / per table (dense)
int state_width(int rule, int dim) {
  switch (rule) {
    case ADAGRAD: return 1;
    case STD_ADAGRAD: return dim;
    case ADAM: return 2 * dim + 2;   // m, v, beta1^t, beta2^t
    case CTR: return 6;              // show, click, unseen_days, embed_g2sum, embedx_g2sum, has_embedx
    default: return 0;
  }
}

void apply_rule(const TableCfg& c, int rule, float* w, float* st, const float* g, int dim, float scale) {
  switch (rule) {
    case SGD:
      for (int i = 0; i < dim; ++i) w[i] -= c.lr * g[i] * scale;
      break;
    case SUM:
      for (int i = 0; i < dim; ++i) w[i] += g[i] * scale;
      break;
    case ADAGRAD: {
      const float ratio = c.lr * std::sqrt(c.initial_g2sum / (c.initial_g2sum + st[0]));
      double add = 0;
      for (int i = 0; i < dim; ++i) {
        const float gi = g[i] * scale;
        w[i] -= ratio * gi;
        add += (double)gi * gi;
      }
      st[0] += (float)(add / dim);
      break;
    }
    case STD_ADAGRAD:
      for (int i = 0; i < dim; ++i) {
        const float gi = g[i] * scale;
        w[i] -= c.lr * gi * std::sqrt(c.initial_g2sum / (c.initial_g2sum + st[i]));
        st[i] += gi * gi;
      }
      break;
    case ADAM: {
      float* m = st;
      float* v = st + dim;
      float& b1p = st[2 * dim];
      float& b2p = st[2 * dim + 1];
      if (b1p == 0.f) b1p = b2p = 1.f;
      b1p *= c.beta1;
      b2p *= c.beta2;
      const float lr = c.lr * std::sqrt(1.f - b2p) / (1.f - b1p);
      for (int i = 0; i < dim; ++i) {
        const float gi = g[i] * scale;
        m[i] = c.beta1 * m[i] + (1.f - c.beta1) * gi;
        v[i] = c.beta2 * v[i] + (1.f - c.beta2) * gi * gi;
        w[i] -= lr * m[i] / (std::sqrt(v[i]) + c.eps);
      }
      break;
    }
  }
  if (rule != SUM)
    for (int i = 0; i < dim; ++i) w[i] = std::min(std::max(w[i], c.min_bound), c.max_bound);
}

inline float ctr_score(const TableCfg& c, const float* st) {
  return (st[0] - st[1]) * c.nonclk_coeff + st[1] * c.click_coeff;
}

// one CTR push: p = [show, click, g_embed, g_embedx(dim-1)]; row = [embed_w, embedx | state]
void apply_ctr(const TableCfg& c, float* w, float* st, const float* p, int dim, std::mt19937_64& rng) {
  st[0] += p[0];
  st[1] += p[1];
  st[2] = 0.f;
  const float* g = p + 2;
  float r = c.lr * std::sqrt(c.initial_g2sum / (c.initial_g2sum + st[3]));
  w[0] -= r * g[0];
  st[3] += g[0] * g[0];
  if (st[5] > 0.f) {
    r = c.lr * std::sqrt(c.initial_g2sum / (c.initial_g2sum + st[4]));
    double add = 0;
    for (int i = 1; i < dim; ++i) {
      w[i] -= r * g[i];
      add += (double)g[i] * g[i];
    }
    st[4] += dim > 1 ? (float)(add / (dim - 1)) : 0.f;
  } else if (ctr_score(c, st) >= c.embedx_threshold) {   // feature became frequent: create embedx
    std::uniform_real_distribution<float> u(-c.initial_range, c.initial_range);
    for (int i = 1; i < dim; ++i) w[i] = c.initial_range > 0.f ? u(rng) : 0.f;
    st[5] = 1.f;
  }
  for (int i = 0; i < dim; ++i) w[i] = std::min(std::max(w[i], c.min_bound), c.max_bound);
}

struct DenseTable {
  TableCfg cfg;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<float> w, st, acc;
  int acc_count = 0;
  uint64_t version = 0;
};

struct SparseRow {
  std::vector<float> v;   // [dim weights | optimizer state]
  uint32_t seen = 0;      // training pulls (count-filter entry)
  uint32_t idle = 0;      // shrink passes since the last pull
  bool live = false;      // materialised (admitted by the entry policy)
  uint64_t last = 0;      // access tick (spill mode: coldest rows leave first)
};

struct SparseShard {
  std::mutex mu;
  std::unordered_map<uint64_t, SparseRow> rows;
  std::mt19937_64 rng;
  // spill mode (ssd_sparse_table): rows evicted to an append-only file, id -> byte offset
  std::unordered_map<uint64_t, uint64_t> disk;
  FILE* f = nullptr;
  uint64_t tick = 0;
  ~SparseShard() {
    if (f) fclose(f);
  }
};

struct SparseTable {
  TableCfg cfg;
  int sw = 0;
  SparseShard shards[kShards];
  size_t cap_per_shard() const { return cfg.cache_rows ? std::max<size_t>(1, cfg.cache_rows / kShards) : 0; }
};

// row record in a spill file: u32 seen | f32 v[dim + sw]
bool spill_read(SparseTable* t, SparseShard& sh, uint64_t id, SparseRow& r) {
  auto it = sh.disk.find(id);
  if (it == sh.disk.end() || !sh.f) return false;
  const size_t w = (size_t)t->cfg.dim + t->sw;
  r.v.assign(w, 0.f);
  uint32_t seen = 0;
  if (fseeko(sh.f, (off_t)it->second, SEEK_SET) != 0 || fread(&seen, 4, 1, sh.f) != 1 ||
      fread(r.v.data(), 4, w, sh.f) != w)
    return false;
  r.seen = seen;
  r.live = true;
  sh.disk.erase(it);
  return true;
}

void spill_evict(SparseTable* t, SparseShard& sh) {   // keep the hottest 3/4 of the cap resident
  const size_t cap = t->cap_per_shard();
  if (!cap || !sh.f || sh.rows.size() <= cap) return;
  std::vector<std::pair<uint64_t, uint64_t>> age;   // (last access, id)
  age.reserve(sh.rows.size());
  for (auto& kv : sh.rows)
    if (kv.second.live) age.emplace_back(kv.second.last, kv.first);
  const size_t keep = cap * 3 / 4;
  if (age.size() <= keep) return;
  std::nth_element(age.begin(), age.begin() + (age.size() - keep), age.end());
  fseeko(sh.f, 0, SEEK_END);
  const size_t w = (size_t)t->cfg.dim + t->sw;
  for (size_t i = 0; i < age.size() - keep; ++i) {
    auto it = sh.rows.find(age[i].second);
    const uint64_t off = (uint64_t)ftello(sh.f);
    const uint32_t seen = it->second.seen;
    fwrite(&seen, 4, 1, sh.f);
    fwrite(it->second.v.data(), 4, w, sh.f);
    sh.disk[it->first] = off;
    sh.rows.erase(it);
  }
  fflush(sh.f);
}

// resident row of ``id`` (read back from the spill file if it was evicted); nullptr if unknown
SparseRow* resident(SparseTable* t, SparseShard& sh, uint64_t id, bool create) {
  auto it = sh.rows.find(id);
  if (it == sh.rows.end()) {
    SparseRow r;
    const bool from_disk = spill_read(t, sh, id, r);
    if (!from_disk && !create) return nullptr;
    it = sh.rows.emplace(id, std::move(r)).first;
  }
  it->second.last = ++sh.tick;
  return &it->second;
}

struct GNode {
  std::vector<uint64_t> nbr;
  std::vector<float> w;
  std::vector<float> feat;
};

struct GraphTable {
  std::mutex mu[kShards];
  std::unordered_map<uint64_t, GNode> nodes[kShards];
  std::mt19937_64 rng[kShards];
  GraphTable() {
    for (int i = 0; i < kShards; ++i) rng[i].seed(0x9e3779b97f4a7c15ULL * (i + 1));
  }
};

struct Server {
  int listen_fd = -1, port = 0;
  std::atomic<bool> stopping{false};
  std::atomic<int> busy{0};   // requests read and not yet answered
  std::thread accept_thr;
  std::mutex conn_mu;
  std::vector<std::thread> conns;
  std::vector<int> conn_fds;
  std::mutex tab_mu;
  std::map<uint32_t, std::unique_ptr<DenseTable>> dense;
  std::map<uint32_t, std::unique_ptr<SparseTable>> sparse;
  std::map<uint32_t, std::unique_ptr<GraphTable>> graph;
  std::mutex bar_mu;
  std::condition_variable bar_cv;
  std::map<uint32_t, std::pair<uint64_t, uint64_t>> bar;   // tag -> (arrived, generation)
  std::mutex stop_mu;
  std::condition_variable stop_cv;

  DenseTable* get_dense(uint32_t t) {
    std::lock_guard<std::mutex> g(tab_mu);
    auto it = dense.find(t);
    return it == dense.end() ? nullptr : it->second.get();
  }
  SparseTable* get_sparse(uint32_t t) {
    std::lock_guard<std::mutex> g(tab_mu);
    auto it = sparse.find(t);
    return it == sparse.end() ? nullptr : it->second.get();
  }
  GraphTable* get_graph(uint32_t t) {
    std::lock_guard<std::mutex> g(tab_mu);
    auto& p = graph[t];
    if (!p) p = std::make_unique<GraphTable>();
    return p.get();
  }
  void wake_all() {
    bar_cv.notify_all();
    std::lock_guard<std::mutex> g(tab_mu);
    for (auto& kv : dense) {
      std::lock_guard<std::mutex> lk(kv.second->mu);
      kv.second->cv.notify_all();
    }
  }
};

inline uint64_t mix(uint64_t x) {  // shard selector (splitmix64 finaliser)
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

void init_row(const TableCfg& c, SparseShard& sh, SparseRow& r, int sw) {
  r.v.assign((size_t)c.dim + sw, 0.f);
  if (c.initial_range > 0.f) {
    std::uniform_real_distribution<float> u(-c.initial_range, c.initial_range);
    // CTR: only the 1-d embed starts random; embedx appears once the feature is frequent
    const int n = c.rule == CTR ? 1 : c.dim;
    for (int i = 0; i < n; ++i) r.v[i] = u(sh.rng);
  }
  r.live = true;
}

bool entry_admits(const TableCfg& c, SparseShard& sh, const SparseRow& r) {
  if (c.entry_kind == 1) return std::uniform_real_distribution<float>(0.f, 1.f)(sh.rng) < c.entry_value;
  if (c.entry_kind == 2) return (float)r.seen >= c.entry_value;
  return true;
}

int32_t save_or_load(Server* s, const ReqHdr& h, const std::string& path) {
  if (SparseTable* t = s->get_sparse(h.table)) {
    const int dim = t->cfg.dim;
    if (h.cmd == SAVE) {   // arg 1: weights only (inference); arg 2: CTR base save (score >= base_threshold)
      const int w = h.arg >= 1 ? dim : dim + t->sw;
      const bool base = h.arg == 2 && t->cfg.rule == CTR;
      FILE* f = fopen(path.c_str(), "wb");
      if (!f) return -4;
      const int32_t hdr[2] = {dim, w};
      fwrite(hdr, 4, 2, f);
      auto emit = [&](uint64_t id, const SparseRow& r) {
        if (!r.live || (base && ctr_score(t->cfg, r.v.data() + dim) < t->cfg.base_threshold)) return;
        fwrite(&id, 8, 1, f);
        fwrite(r.v.data(), 4, w, f);
      };
      for (auto& sh : t->shards) {
        std::lock_guard<std::mutex> g(sh.mu);
        for (auto& kv : sh.rows) emit(kv.first, kv.second);
        std::vector<std::pair<uint64_t, uint64_t>> spilled(sh.disk.begin(), sh.disk.end());
        const size_t rw = (size_t)dim + t->sw;
        SparseRow r;
        r.v.assign(rw, 0.f);
        r.live = true;
        for (auto& kv : spilled) {   // rows living in the spill file
          uint32_t seen;
          if (fseeko(sh.f, (off_t)kv.second, SEEK_SET) == 0 && fread(&seen, 4, 1, sh.f) == 1 &&
              fread(r.v.data(), 4, rw, sh.f) == rw)
            emit(kv.first, r);
        }
      }
      fclose(f);
      return 0;
    }
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return -4;
    int32_t hdr[2];
    if (fread(hdr, 4, 2, f) != 2 || hdr[0] != dim || hdr[1] < dim) {
      fclose(f);
      return -5;
    }
    std::vector<float> buf(hdr[1]);
    uint64_t id;
    while (fread(&id, 8, 1, f) == 1 && fread(buf.data(), 4, hdr[1], f) == (size_t)hdr[1]) {
      SparseShard& sh = t->shards[mix(id) % kShards];
      std::lock_guard<std::mutex> g(sh.mu);
      SparseRow& r = sh.rows[id];
      r.v.assign((size_t)dim + t->sw, 0.f);
      memcpy(r.v.data(), buf.data(), 4 * std::min<size_t>(buf.size(), r.v.size()));
      r.live = true;
    }
    fclose(f);
    return 0;
  }
  if (DenseTable* d = s->get_dense(h.table)) {
    std::lock_guard<std::mutex> g(d->mu);
    FILE* f = fopen(path.c_str(), h.cmd == SAVE ? "wb" : "rb");
    if (!f) return -4;
    const uint64_t n = d->w.size();
    int32_t st = 0;
    if (h.cmd == SAVE) {
      fwrite(&n, 8, 1, f);
      fwrite(d->w.data(), 4, n, f);
    } else {
      uint64_t m = 0;
      if (fread(&m, 8, 1, f) != 1 || m != n || fread(d->w.data(), 4, n, f) != n) st = -5;
    }
    fclose(f);
    return st;
  }
  return -1;
}

void handle(Server* s, int fd) {
  std::vector<char> in, out;
  for (;;) {
    ReqHdr h;
    if (!read_full(fd, &h, sizeof(h)) || h.magic != kMagic) break;
    in.resize(h.nbytes);
    if (h.nbytes && !read_full(fd, in.data(), h.nbytes)) break;
    out.clear();
    int32_t status = 0;
    ++s->busy;
    switch (h.cmd) {
      case PING:
        break;
      case CREATE_DENSE: {   // idempotent: every trainer may declare the table; n = numel
        if (h.nbytes < sizeof(TableCfg)) { status = -2; break; }
        TableCfg c;
        memcpy(&c, in.data(), sizeof(c));
        std::lock_guard<std::mutex> g(s->tab_mu);
        auto it = s->dense.find(h.table);
        if (it == s->dense.end()) {
          auto t = std::make_unique<DenseTable>();
          t->cfg = c;
          t->w.assign(h.n, 0.f);
          // dense state: per-element g2sum for both adagrads, m/v/pows for adam
          t->st.assign(c.rule == ADAM ? 2 * h.n + 2 : (c.rule == ADAGRAD || c.rule == STD_ADAGRAD) ? h.n : 0, 0.f);
          if (h.nbytes >= sizeof(TableCfg) + h.n * 4) memcpy(t->w.data(), in.data() + sizeof(TableCfg), h.n * 4);
          s->dense[h.table] = std::move(t);
        } else if (it->second->w.size() != h.n) {
          status = -3;
        }
        break;
      }
      case CREATE_SPARSE: {
        if (h.nbytes < sizeof(TableCfg)) { status = -2; break; }
        TableCfg c;
        memcpy(&c, in.data(), sizeof(c));
        std::lock_guard<std::mutex> g(s->tab_mu);
        auto it = s->sparse.find(h.table);
        if (it == s->sparse.end()) {
          auto t = std::make_unique<SparseTable>();
          t->cfg = c;
          t->sw = state_width(c.rule, c.dim);
          for (int i = 0; i < kShards; ++i) t->shards[i].rng.seed(c.seed * 1315423911ULL + i);
          s->sparse[h.table] = std::move(t);
        } else if (it->second->cfg.dim != c.dim) {
          status = -3;
        }
        break;
      }
      case SET_DENSE: {
        DenseTable* t = s->get_dense(h.table);
        if (!t || h.nbytes != t->w.size() * 4) { status = -1; break; }
        std::lock_guard<std::mutex> g(t->mu);
        memcpy(t->w.data(), in.data(), h.nbytes);
        break;
      }
      case PULL_DENSE: {   // arg = minimum version to wait for (synchronous training)
        DenseTable* t = s->get_dense(h.table);
        if (!t) { status = -1; break; }
        std::unique_lock<std::mutex> g(t->mu);
        t->cv.wait(g, [&] { return t->version >= h.arg || s->stopping.load(); });
        out.resize(t->w.size() * 4);
        memcpy(out.data(), t->w.data(), out.size());
        status = (int32_t)t->version;
        break;
      }
      case PUSH_DENSE: {
        DenseTable* t = s->get_dense(h.table);
        if (!t || h.nbytes != t->w.size() * 4) { status = -1; break; }
        const float* g = reinterpret_cast<const float*>(in.data());
        std::lock_guard<std::mutex> lk(t->mu);
        const int n = (int)t->w.size();
        const int sync = t->cfg.sync_trainers;
        if (sync > 1) {   // merge every trainer's grad, apply the mean once
          if (t->acc.empty()) t->acc.assign(n, 0.f);
          for (int i = 0; i < n; ++i) t->acc[i] += g[i];
          if (++t->acc_count < sync) {
            status = (int32_t)t->version;
            break;
          }
          g = t->acc.data();
        }
        const int rule = t->cfg.rule == ADAGRAD ? STD_ADAGRAD : t->cfg.rule;
        apply_rule(t->cfg, rule, t->w.data(), t->st.data(), g, n, sync > 1 ? 1.f / sync : 1.f);
        if (sync > 1) {
          std::fill(t->acc.begin(), t->acc.end(), 0.f);
          t->acc_count = 0;
        }
        ++t->version;
        t->cv.notify_all();
        status = (int32_t)t->version;
        break;
      }
      case PULL_SPARSE: {   // n ids -> n x dim rows; arg 1 = training pull (counts towards the entry policy)
        SparseTable* t = s->get_sparse(h.table);
        if (!t || h.nbytes != h.n * 8) { status = -1; break; }
        const int dim = t->cfg.dim;
        const uint64_t* ids = reinterpret_cast<const uint64_t*>(in.data());
        out.resize(h.n * (size_t)dim * 4);
        float* o = reinterpret_cast<float*>(out.data());
        for (uint64_t i = 0; i < h.n; ++i) {
          SparseShard& sh = t->shards[mix(ids[i]) % kShards];
          std::lock_guard<std::mutex> g(sh.mu);
          if (!h.arg) {   // inference pull: never creates rows
            SparseRow* r = resident(t, sh, ids[i], false);
            if (r && r->live) memcpy(o + i * dim, r->v.data(), dim * 4);
            else memset(o + i * dim, 0, dim * 4);
            spill_evict(t, sh);
            continue;
          }
          SparseRow& r = *resident(t, sh, ids[i], true);
          ++r.seen;
          r.idle = 0;
          if (!r.live && entry_admits(t->cfg, sh, r)) init_row(t->cfg, sh, r, t->sw);
          if (r.live) memcpy(o + i * dim, r.v.data(), dim * 4);
          else memset(o + i * dim, 0, dim * 4);
          spill_evict(t, sh);
        }
        break;
      }
      case PUSH_SPARSE:
      case PUSH_SPARSE_DELTA: {   // n ids + n x dim grads (or geo-SGD deltas)
        SparseTable* t = s->get_sparse(h.table);
        const int dim = t ? t->cfg.dim : 0;
        const int rule = h.cmd == PUSH_SPARSE_DELTA ? SUM : (t ? t->cfg.rule : 0);
        const int pw = rule == CTR ? dim + 2 : dim;   // CTR pushes carry show and click
        if (!t || h.nbytes != h.n * 8 + h.n * (size_t)pw * 4) { status = -1; break; }
        const uint64_t* ids = reinterpret_cast<const uint64_t*>(in.data());
        const float* g = reinterpret_cast<const float*>(in.data() + h.n * 8);
        for (uint64_t i = 0; i < h.n; ++i) {
          SparseShard& sh = t->shards[mix(ids[i]) % kShards];
          std::lock_guard<std::mutex> lk(sh.mu);
          SparseRow* r = resident(t, sh, ids[i], false);
          if (!r || !r->live) continue;   // not admitted: gradient dropped
          if (rule == CTR) apply_ctr(t->cfg, r->v.data(), r->v.data() + dim, g + i * pw, dim, sh.rng);
          else apply_rule(t->cfg, rule, r->v.data(), r->v.data() + dim, g + i * dim, dim, 1.f);
          spill_evict(t, sh);
        }
        break;
      }
      case BARRIER: {   // table = tag, n = participants
        std::unique_lock<std::mutex> g(s->bar_mu);
        auto& b = s->bar[h.table];
        const uint64_t gen = b.second;
        if (++b.first >= h.n) {
          b.first = 0;
          ++b.second;
          s->bar_cv.notify_all();
        } else {
          s->bar_cv.wait(g, [&] { return s->bar[h.table].second != gen || s->stopping.load(); });
        }
        break;
      }
      case TABLE_SIZE: {
        uint64_t n = 0;
        if (SparseTable* t = s->get_sparse(h.table)) {
          for (auto& sh : t->shards) {
            std::lock_guard<std::mutex> g(sh.mu);
            for (auto& kv : sh.rows) n += kv.second.live ? 1 : 0;
            n += sh.disk.size();
          }
        } else if (DenseTable* d = s->get_dense(h.table)) {
          n = d->w.size();
        } else {
          status = -1;
        }
        out.resize(8);
        memcpy(out.data(), &n, 8);
        break;
      }
      case SHRINK: {   // drop rows not pulled during the last `arg` shrink passes
        SparseTable* t = s->get_sparse(h.table);
        if (!t) { status = -1; break; }
        uint64_t dropped = 0;
        if (t->cfg.rule == CTR) {   // ctr_accessor Shrink: decay show/click, age, delete weak / stale
          const int dim = t->cfg.dim;
          for (auto& sh : t->shards) {
            std::lock_guard<std::mutex> g(sh.mu);
            for (auto it = sh.rows.begin(); it != sh.rows.end();) {
              float* st = it->second.v.data() + dim;
              if (it->second.live) {
                st[0] *= t->cfg.show_click_decay;
                st[1] *= t->cfg.show_click_decay;
                st[2] += 1.f;
              }
              if (!it->second.live || ctr_score(t->cfg, st) < t->cfg.delete_threshold ||
                  st[2] > t->cfg.delete_after_unseen_days) {
                it = sh.rows.erase(it);
                ++dropped;
              } else {
                ++it;
              }
            }
          }
          out.resize(8);
          memcpy(out.data(), &dropped, 8);
          break;
        }
        for (auto& sh : t->shards) {
          std::lock_guard<std::mutex> g(sh.mu);
          for (auto it = sh.rows.begin(); it != sh.rows.end();) {
            if (++it->second.idle > h.arg) {
              it = sh.rows.erase(it);
              ++dropped;
            } else {
              ++it;
            }
          }
        }
        out.resize(8);
        memcpy(out.data(), &dropped, 8);
        break;
      }
      case SAVE:
      case LOAD:
        status = save_or_load(s, h, std::string(in.data(), in.size()));
        break;
      case SET_SPILL: {   // payload = directory; per-shard append-only spill files
        SparseTable* t = s->get_sparse(h.table);
        if (!t || !t->cfg.cache_rows) { status = -1; break; }
        const std::string dir(in.data(), in.size());
        for (int k = 0; k < kShards; ++k) {
          SparseShard& sh = t->shards[k];
          std::lock_guard<std::mutex> g(sh.mu);
          if (sh.f) continue;
          const std::string path = dir + "/table" + std::to_string(h.table) + "_shard" + std::to_string(k) + ".spill";
          sh.f = fopen(path.c_str(), "w+b");
          if (!sh.f) { status = -4; break; }
        }
        break;
      }
      case GRAPH_ADD_EDGES: {   // n edges: src[n] u64, dst[n] u64, w[n] f32; arg 1 = also the reverse edges;
                                // arg 2: payload = n node ids to register (no edges)
        GraphTable* gt = s->get_graph(h.table);
        if (h.arg == 2) {
          if (h.nbytes != h.n * 8) { status = -1; break; }
          const uint64_t* ids = reinterpret_cast<const uint64_t*>(in.data());
          for (uint64_t i = 0; i < h.n; ++i) {
            const int k = (int)(mix(ids[i]) % kShards);
            std::lock_guard<std::mutex> g(gt->mu[k]);
            gt->nodes[k].emplace(ids[i], GNode());
          }
          break;
        }
        if (h.nbytes != h.n * 20) { status = -1; break; }
        const uint64_t* src = reinterpret_cast<const uint64_t*>(in.data());
        const uint64_t* dst = src + h.n;
        const float* w = reinterpret_cast<const float*>(dst + h.n);
        for (int pass = 0; pass < (h.arg ? 2 : 1); ++pass)
          for (uint64_t i = 0; i < h.n; ++i) {
            const uint64_t a = pass ? dst[i] : src[i], b = pass ? src[i] : dst[i];
            const int k = (int)(mix(a) % kShards);
            std::lock_guard<std::mutex> g(gt->mu[k]);
            GNode& nd = gt->nodes[k][a];
            nd.nbr.push_back(b);
            nd.w.push_back(w[i]);
          }
        break;
      }
      case GRAPH_SAMPLE: {   // n node ids -> counts u32[n] + sampled ids; arg = k | (weighted << 31)
        if (h.nbytes != h.n * 8) { status = -1; break; }
        GraphTable* gt = s->get_graph(h.table);
        const uint64_t* ids = reinterpret_cast<const uint64_t*>(in.data());
        const uint32_t k = h.arg & 0x7fffffffu;
        const bool weighted = (h.arg >> 31) != 0;
        std::vector<uint32_t> counts(h.n);
        std::vector<uint64_t> picked;
        for (uint64_t i = 0; i < h.n; ++i) {
          const int sk = (int)(mix(ids[i]) % kShards);
          std::lock_guard<std::mutex> g(gt->mu[sk]);
          auto it = gt->nodes[sk].find(ids[i]);
          if (it == gt->nodes[sk].end()) continue;
          const GNode& nd = it->second;
          const size_t deg = nd.nbr.size();
          std::mt19937_64& rng = gt->rng[sk];
          if (deg <= k) {
            picked.insert(picked.end(), nd.nbr.begin(), nd.nbr.end());
            counts[i] = (uint32_t)deg;
          } else if (!weighted) {   // k distinct positions (partial Fisher-Yates)
            std::vector<uint32_t> pos(deg);
            for (size_t j = 0; j < deg; ++j) pos[j] = (uint32_t)j;
            for (uint32_t j = 0; j < k; ++j) {
              const size_t r = j + std::uniform_int_distribution<size_t>(0, deg - 1 - j)(rng);
              std::swap(pos[j], pos[r]);
              picked.push_back(nd.nbr[pos[j]]);
            }
            counts[i] = k;
          } else {   // weighted without replacement: the k largest keys u^(1/w) (Efraimidis-Spirakis)
            std::vector<std::pair<double, uint32_t>> key(deg);
            std::uniform_real_distribution<double> u(1e-12, 1.0);
            for (size_t j = 0; j < deg; ++j)
              key[j] = {std::log(u(rng)) / std::max(1e-12, (double)nd.w[j]), (uint32_t)j};
            std::partial_sort(key.begin(), key.begin() + k, key.end(),
                              [](const auto& a, const auto& b) { return a.first > b.first; });
            for (uint32_t j = 0; j < k; ++j) picked.push_back(nd.nbr[key[j].second]);
            counts[i] = k;
          }
        }
        out.resize(h.n * 4 + picked.size() * 8);
        memcpy(out.data(), counts.data(), h.n * 4);
        if (!picked.empty()) memcpy(out.data() + h.n * 4, picked.data(), picked.size() * 8);
        break;
      }
      case GRAPH_SET_FEAT:
      case GRAPH_GET_FEAT: {   // n ids (+ n x arg floats for SET)
        GraphTable* gt = s->get_graph(h.table);
        const uint32_t dim = h.arg;
        const bool set = h.cmd == GRAPH_SET_FEAT;
        if (h.nbytes != h.n * 8 + (set ? h.n * (size_t)dim * 4 : 0)) { status = -1; break; }
        const uint64_t* ids = reinterpret_cast<const uint64_t*>(in.data());
        const float* fv = reinterpret_cast<const float*>(in.data() + h.n * 8);
        if (!set) out.assign(h.n * (size_t)dim * 4, 0);
        float* o = reinterpret_cast<float*>(out.data());
        for (uint64_t i = 0; i < h.n; ++i) {
          const int sk = (int)(mix(ids[i]) % kShards);
          std::lock_guard<std::mutex> g(gt->mu[sk]);
          if (set) {
            GNode& nd = gt->nodes[sk][ids[i]];
            nd.feat.assign(fv + i * dim, fv + (i + 1) * dim);
          } else {
            auto it = gt->nodes[sk].find(ids[i]);
            if (it != gt->nodes[sk].end())
              memcpy(o + i * dim, it->second.feat.data(), 4 * std::min<size_t>(dim, it->second.feat.size()));
          }
        }
        break;
      }
      case GRAPH_RANDOM_NODES:
      case GRAPH_NODE_COUNT: {   // arg = how many (uniform, without replacement) / node count
        GraphTable* gt = s->get_graph(h.table);
        std::vector<uint64_t> all;
        for (int k = 0; k < kShards; ++k) {
          std::lock_guard<std::mutex> g(gt->mu[k]);
          for (auto& kv : gt->nodes[k]) all.push_back(kv.first);
        }
        if (h.cmd == GRAPH_NODE_COUNT) {
          const uint64_t n = all.size();
          out.resize(8);
          memcpy(out.data(), &n, 8);
          break;
        }
        std::sort(all.begin(), all.end());
        std::mt19937_64 rng(h.n);   // n = seed
        const size_t k = std::min<size_t>(h.arg, all.size());
        for (size_t j = 0; j < k; ++j) std::swap(all[j], all[j + std::uniform_int_distribution<size_t>(0, all.size() - 1 - j)(rng)]);
        out.resize(k * 8);
        if (k) memcpy(out.data(), all.data(), k * 8);
        break;
      }
      case STOP: {
        // let the other connections' in-flight requests answer first (a trainer released from the
        // final barrier may not have its reply yet; the stop shuts every connection down), bounded
        // so a trainer stuck in a barrier that can never complete does not hold the server
        for (int i = 0; i < 10000 && s->busy.load() > 1; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        s->stopping = true;
        s->wake_all();
        if (s->listen_fd >= 0) ::shutdown(s->listen_fd, SHUT_RDWR);
        std::lock_guard<std::mutex> g(s->stop_mu);
        s->stop_cv.notify_all();
        break;
      }
      default:
        status = -100;
    }
    const RespHdr r{status, 0, out.size()};
    const bool sent = write_full(fd, &r, sizeof(r)) && (out.empty() || write_full(fd, out.data(), out.size()));
    --s->busy;
    if (!sent) break;
  }
  ::close(fd);
}

void accept_loop(Server* s) {
  while (!s->stopping.load()) {
    sockaddr_in a{};
    socklen_t al = sizeof(a);
    const int fd = ::accept(s->listen_fd, reinterpret_cast<sockaddr*>(&a), &al);
    if (fd < 0) {
      if (s->stopping.load()) break;
      if (errno == EINTR || errno == ECONNABORTED) continue;
      break;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(s->conn_mu);
    s->conn_fds.push_back(fd);
    s->conns.emplace_back(handle, s, fd);
  }
}

struct Client {
  int fd = -1;
  std::mutex mu;
};

int64_t call(Client* c, uint32_t cmd, uint32_t table, uint32_t arg, uint64_t n, const void* p1, size_t b1,
             const void* p2, size_t b2, void* out, size_t out_cap, uint64_t* out_bytes) {
  std::lock_guard<std::mutex> g(c->mu);
  const ReqHdr h{kMagic, cmd, table, arg, n, (uint64_t)(b1 + b2)};
  if (!write_full(c->fd, &h, sizeof(h))) return -1000;
  if (b1 && !write_full(c->fd, p1, b1)) return -1000;
  if (b2 && !write_full(c->fd, p2, b2)) return -1000;
  RespHdr r;
  if (!read_full(c->fd, &r, sizeof(r))) return -1001;
  if (out_bytes) *out_bytes = r.nbytes;
  if (r.nbytes) {
    if (!out || r.nbytes > out_cap) {   // drain what the caller has no room for
      std::vector<char> sink(r.nbytes);
      if (!read_full(c->fd, sink.data(), r.nbytes)) return -1001;
      return r.status < 0 ? r.status : -1002;
    }
    if (!read_full(c->fd, out, r.nbytes)) return -1001;
  }
  return r.status;
}

TableCfg make_cfg(const int32_t* iv, const float* fv, uint64_t seed) {
  TableCfg c;
  c.rule = iv[0];
  c.dim = iv[1];
  c.sync_trainers = iv[2];
  c.entry_kind = iv[3];
  c.lr = fv[0];
  c.beta1 = fv[1];
  c.beta2 = fv[2];
  c.eps = fv[3];
  c.initial_g2sum = fv[4];
  c.initial_range = fv[5];
  c.min_bound = fv[6];
  c.max_bound = fv[7];
  c.entry_value = fv[8];
  c.seed = seed;
  c.nonclk_coeff = fv[9];
  c.click_coeff = fv[10];
  c.embedx_threshold = fv[11];
  c.show_click_decay = fv[12];
  c.delete_threshold = fv[13];
  c.delete_after_unseen_days = fv[14];
  c.base_threshold = fv[15];
  c.cache_rows = (uint64_t)(uint32_t)iv[4];
  return c;
}

}  // namespace

// ------------------------------------------------------------------------------- server ABI
PHA_API void* pha_ps_server_start(const char* host, int port) {
  auto* s = new Server();
  s->listen_fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (s->listen_fd < 0) {
    delete s;
    return nullptr;
  }
  int one = 1;
  setsockopt(s->listen_fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons((uint16_t)port);
  a.sin_addr.s_addr = (host && *host) ? inet_addr(host) : htonl(INADDR_ANY);
  if (::bind(s->listen_fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(s->listen_fd, 128) != 0) {
    ::close(s->listen_fd);
    delete s;
    return nullptr;
  }
  socklen_t al = sizeof(a);
  getsockname(s->listen_fd, reinterpret_cast<sockaddr*>(&a), &al);
  s->port = ntohs(a.sin_port);
  s->accept_thr = std::thread(accept_loop, s);
  return s;
}

PHA_API int pha_ps_server_port(void* h) { return static_cast<Server*>(h)->port; }

// block until a trainer sends STOP (or timeout_ms elapses; < 0 = forever); 1 = stopped
PHA_API int pha_ps_server_wait(void* h, int64_t timeout_ms) {
  auto* s = static_cast<Server*>(h);
  std::unique_lock<std::mutex> g(s->stop_mu);
  auto pred = [&] { return s->stopping.load(); };
  if (timeout_ms < 0) s->stop_cv.wait(g, pred);
  else s->stop_cv.wait_for(g, std::chrono::milliseconds(timeout_ms), pred);
  return s->stopping.load() ? 1 : 0;
}

PHA_API void pha_ps_server_destroy(void* h) {
  auto* s = static_cast<Server*>(h);
  s->stopping = true;
  s->wake_all();
  if (s->listen_fd >= 0) {
    ::shutdown(s->listen_fd, SHUT_RDWR);
    ::close(s->listen_fd);
  }
  if (s->accept_thr.joinable()) s->accept_thr.join();
  {
    std::lock_guard<std::mutex> g(s->conn_mu);
    for (int fd : s->conn_fds) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : s->conns)
    if (t.joinable()) t.join();
  delete s;
}

// ------------------------------------------------------------------------------- client ABI
PHA_API void* pha_ps_client_connect(const char* host, int port, int64_t timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    sockaddr_in a{};
    a.sin_family = AF_INET;
    a.sin_port = htons((uint16_t)port);
    a.sin_addr.s_addr = inet_addr(host);
    if (::connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
      int one = 1;
      setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
      auto* c = new Client();
      c->fd = fd;
      return c;
    }
    ::close(fd);
    const auto ms =
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    if (timeout_ms >= 0 && ms >= timeout_ms) return nullptr;
    std::this_thread::sleep_for(std::chrono::milliseconds(50));   // server not up yet
  }
}

PHA_API void pha_ps_client_close(void* h) {
  auto* c = static_cast<Client*>(h);
  if (c->fd >= 0) ::close(c->fd);
  delete c;
}

// iv = {rule, dim, sync_trainers, entry_kind, cache_rows}
// fv = {lr, beta1, beta2, eps, initial_g2sum, initial_range, min_bound, max_bound, entry_value,
//       nonclk_coeff, click_coeff, embedx_threshold, show_click_decay, delete_threshold,
//       delete_after_unseen_days, base_threshold}
PHA_API int64_t pha_ps_create_dense(void* h, uint32_t table, uint64_t numel, const int32_t* iv, const float* fv,
                                    const float* init) {
  const TableCfg c = make_cfg(iv, fv, 0);
  return call(static_cast<Client*>(h), CREATE_DENSE, table, 0, numel, &c, sizeof(c), init, init ? numel * 4 : 0,
              nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_create_sparse(void* h, uint32_t table, const int32_t* iv, const float* fv, uint64_t seed) {
  const TableCfg c = make_cfg(iv, fv, seed);
  return call(static_cast<Client*>(h), CREATE_SPARSE, table, 0, 0, &c, sizeof(c), nullptr, 0, nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_set_dense(void* h, uint32_t table, const float* w, uint64_t numel) {
  return call(static_cast<Client*>(h), SET_DENSE, table, 0, numel, w, numel * 4, nullptr, 0, nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_pull_dense(void* h, uint32_t table, float* out, uint64_t numel, uint32_t min_version) {
  uint64_t nb = 0;
  const int64_t st = call(static_cast<Client*>(h), PULL_DENSE, table, min_version, 0, nullptr, 0, nullptr, 0, out,
                          numel * 4, &nb);
  return (st >= 0 && nb != numel * 4) ? -1003 : st;
}

PHA_API int64_t pha_ps_push_dense(void* h, uint32_t table, const float* g, uint64_t numel) {
  return call(static_cast<Client*>(h), PUSH_DENSE, table, 0, numel, g, numel * 4, nullptr, 0, nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_pull_sparse(void* h, uint32_t table, const uint64_t* ids, uint64_t n, int dim, float* out,
                                   int training) {
  uint64_t nb = 0;
  const int64_t st = call(static_cast<Client*>(h), PULL_SPARSE, table, training ? 1 : 0, n, ids, n * 8, nullptr, 0,
                          out, n * (size_t)dim * 4, &nb);
  return (st >= 0 && nb != n * (size_t)dim * 4) ? -1003 : st;
}

PHA_API int64_t pha_ps_push_sparse(void* h, uint32_t table, const uint64_t* ids, uint64_t n, int dim, const float* g,
                                   int delta) {
  return call(static_cast<Client*>(h), delta ? PUSH_SPARSE_DELTA : PUSH_SPARSE, table, 0, n, ids, n * 8, g,
              n * (size_t)dim * 4, nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_barrier(void* h, uint32_t tag, uint64_t n) {
  return call(static_cast<Client*>(h), BARRIER, tag, 0, n, nullptr, 0, nullptr, 0, nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_table_size(void* h, uint32_t table) {
  uint64_t v = 0;
  const int64_t st = call(static_cast<Client*>(h), TABLE_SIZE, table, 0, 0, nullptr, 0, nullptr, 0, &v, 8, nullptr);
  return st < 0 ? st : (int64_t)v;
}

PHA_API int64_t pha_ps_shrink(void* h, uint32_t table, uint32_t max_idle) {
  uint64_t v = 0;
  const int64_t st = call(static_cast<Client*>(h), SHRINK, table, max_idle, 0, nullptr, 0, nullptr, 0, &v, 8, nullptr);
  return st < 0 ? st : (int64_t)v;
}

PHA_API int64_t pha_ps_save(void* h, uint32_t table, const char* path, int mode, int load) {
  return call(static_cast<Client*>(h), load ? LOAD : SAVE, table, (uint32_t)mode, 0, path, strlen(path), nullptr, 0,
              nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_stop_server(void* h) {
  return call(static_cast<Client*>(h), STOP, 0, 0, 0, nullptr, 0, nullptr, 0, nullptr, 0, nullptr);
}

PHA_API int64_t pha_ps_set_spill(void* h, uint32_t table, const char* dir) {
  return call(static_cast<Client*>(h), SET_SPILL, table, 0, 0, dir, strlen(dir), nullptr, 0, nullptr, 0, nullptr);
}

// ------------------------------------------------------------------------------- graph ABI
PHA_API int64_t pha_ps_graph_add_edges(void* h, uint32_t table, const uint64_t* src, const uint64_t* dst,
                                       const float* w, uint64_t n, int bidirectional) {
  if (bidirectional == 2)   // register the n node ids in ``src``
    return call(static_cast<Client*>(h), GRAPH_ADD_EDGES, table, 2, n, src, n * 8, nullptr, 0, nullptr, 0, nullptr);
  std::vector<char> buf(n * 20);
  memcpy(buf.data(), src, n * 8);
  memcpy(buf.data() + n * 8, dst, n * 8);
  memcpy(buf.data() + n * 16, w, n * 4);
  return call(static_cast<Client*>(h), GRAPH_ADD_EDGES, table, bidirectional ? 1 : 0, n, buf.data(), buf.size(),
              nullptr, 0, nullptr, 0, nullptr);
}

// out: u32 counts[n] followed by the sampled u64 ids (capacity out_cap bytes); returns bytes written
PHA_API int64_t pha_ps_graph_sample(void* h, uint32_t table, const uint64_t* ids, uint64_t n, uint32_t k,
                                    int weighted, void* out, uint64_t out_cap) {
  uint64_t nb = 0;
  const uint32_t arg = (k & 0x7fffffffu) | (weighted ? 0x80000000u : 0u);
  const int64_t st = call(static_cast<Client*>(h), GRAPH_SAMPLE, table, arg, n, ids, n * 8, nullptr, 0, out, out_cap,
                          &nb);
  return st < 0 ? st : (int64_t)nb;
}

PHA_API int64_t pha_ps_graph_feat(void* h, uint32_t table, const uint64_t* ids, uint64_t n, uint32_t dim, float* feat,
                                  int set) {
  if (set)
    return call(static_cast<Client*>(h), GRAPH_SET_FEAT, table, dim, n, ids, n * 8, feat, n * (size_t)dim * 4, nullptr,
                0, nullptr);
  return call(static_cast<Client*>(h), GRAPH_GET_FEAT, table, dim, n, ids, n * 8, nullptr, 0, feat,
              n * (size_t)dim * 4, nullptr);
}

PHA_API int64_t pha_ps_graph_random_nodes(void* h, uint32_t table, uint32_t k, uint64_t seed, uint64_t* out) {
  uint64_t nb = 0;
  const int64_t st = call(static_cast<Client*>(h), GRAPH_RANDOM_NODES, table, k, seed, nullptr, 0, nullptr, 0, out,
                          (size_t)k * 8, &nb);
  return st < 0 ? st : (int64_t)(nb / 8);
}

PHA_API int64_t pha_ps_graph_node_count(void* h, uint32_t table) {
  uint64_t v = 0;
  const int64_t st = call(static_cast<Client*>(h), GRAPH_NODE_COUNT, table, 0, 0, nullptr, 0, nullptr, 0, &v, 8,
                          nullptr);
  return st < 0 ? st : (int64_t)v;
}
