// MultiSlot text parser for InMemoryDataset / QueueDataset (reference behaviour:
// paddle/fluid/framework/data_feed.cc MultiSlotDataFeed::ParseOneInstance).
//
// Each line is one instance: for every slot, "<n> v1 ... vn". Slots are float or uint64
// feasigns (int64). Parsing is a single pass over the buffer with strtof/strtoull, split
// into chunks of lines handled by the runtime thread pool; per-slot values are written
// into flat arrays with per-instance offsets (LoD), ready to become tensors.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "runtime.h"

namespace {

struct SlotData {
  std::vector<float> f;
  std::vector<int64_t> i;
  std::vector<int64_t> lod{0};
};

struct Parsed {
  int nslots = 0;
  std::vector<uint8_t> is_float;
  std::vector<SlotData> slots;
  int64_t ninst = 0;
  int64_t nbad = 0;
};

// Parse [b, e) lines into `out`. Returns false on malformed instance (skipped, counted).
void parse_range(const char* b, const char* e, Parsed& out) {
  const char* p = b;
  std::vector<size_t> mark_f(out.nslots), mark_i(out.nslots), mark_l(out.nslots);
  while (p < e) {
    const char* eol = static_cast<const char*>(memchr(p, '\n', e - p));
    if (!eol) eol = e;
    // skip blank lines
    const char* q = p;
    while (q < eol && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
    if (q == eol) {
      p = eol + 1;
      continue;
    }
    for (int s = 0; s < out.nslots; ++s) {
      mark_f[s] = out.slots[s].f.size();
      mark_i[s] = out.slots[s].i.size();
      mark_l[s] = out.slots[s].lod.size();
    }
    bool ok = true;
    const char* c = q;
    for (int s = 0; s < out.nslots && ok; ++s) {
      char* endp;
      long n = strtol(c, &endp, 10);
      if (endp == c || n < 0 || endp > eol) {
        ok = false;
        break;
      }
      c = endp;
      SlotData& sd = out.slots[s];
      for (long k = 0; k < n; ++k) {
        if (out.is_float[s]) {
          float v = strtof(c, &endp);
          if (endp == c || endp > eol) {
            ok = false;
            break;
          }
          sd.f.push_back(v);
        } else {
          unsigned long long v = strtoull(c, &endp, 10);
          if (endp == c || endp > eol) {
            ok = false;
            break;
          }
          sd.i.push_back(static_cast<int64_t>(v));
        }
        c = endp;
      }
      if (ok) sd.lod.push_back(static_cast<int64_t>(out.is_float[s] ? sd.f.size() : sd.i.size()));
    }
    if (ok) {
      ++out.ninst;
    } else {
      for (int s = 0; s < out.nslots; ++s) {  // roll back the partial instance
        out.slots[s].f.resize(mark_f[s]);
        out.slots[s].i.resize(mark_i[s]);
        out.slots[s].lod.resize(mark_l[s]);
      }
      ++out.nbad;
    }
    p = eol + 1;
  }
}

}  // namespace

PHA_API void* pha_ms_parse(const char* buf, size_t len, int nslots, const uint8_t* is_float, int nthreads) {
  auto* res = new Parsed();
  res->nslots = nslots;
  res->is_float.assign(is_float, is_float + nslots);
  res->slots.resize(nslots);
  // split on line boundaries into chunks, parse in parallel, then concatenate
  int chunks = nthreads > 0 ? nthreads : 8;
  if (len < (1u << 20)) chunks = 1;
  std::vector<const char*> cuts{buf};
  for (int k = 1; k < chunks; ++k) {
    const char* target = buf + len * k / chunks;
    if (target <= cuts.back()) continue;
    const char* nl = static_cast<const char*>(memchr(target, '\n', buf + len - target));
    if (!nl) break;
    cuts.push_back(nl + 1);
  }
  cuts.push_back(buf + len);
  const int nc = static_cast<int>(cuts.size()) - 1;
  std::vector<Parsed> parts(nc);
  for (auto& pp : parts) {
    pp.nslots = nslots;
    pp.is_float = res->is_float;
    pp.slots.resize(nslots);
  }
  struct Ctx {
    std::vector<const char*>* cuts;
    std::vector<Parsed>* parts;
  } ctx{&cuts, &parts};
  pha::parallel_for(nc, nc, [](int64_t b, int64_t e, void* v) {
    auto* c = static_cast<Ctx*>(v);
    for (int64_t k = b; k < e; ++k) parse_range((*c->cuts)[k], (*c->cuts)[k + 1], (*c->parts)[k]);
  }, &ctx);
  for (auto& pp : parts) {
    res->ninst += pp.ninst;
    res->nbad += pp.nbad;
    for (int s = 0; s < nslots; ++s) {
      SlotData& dst = res->slots[s];
      SlotData& src = pp.slots[s];
      const int64_t base = static_cast<int64_t>(res->is_float[s] ? dst.f.size() : dst.i.size());
      dst.f.insert(dst.f.end(), src.f.begin(), src.f.end());
      dst.i.insert(dst.i.end(), src.i.begin(), src.i.end());
      for (size_t k = 1; k < src.lod.size(); ++k) dst.lod.push_back(base + src.lod[k]);
    }
  }
  return res;
}

PHA_API int64_t pha_ms_ninst(void* h) { return static_cast<Parsed*>(h)->ninst; }
PHA_API int64_t pha_ms_nbad(void* h) { return static_cast<Parsed*>(h)->nbad; }
PHA_API int64_t pha_ms_slot_numel(void* h, int s) {
  auto* p = static_cast<Parsed*>(h);
  return static_cast<int64_t>(p->is_float[s] ? p->slots[s].f.size() : p->slots[s].i.size());
}
// Copy slot `s` values (float32 or int64 per slot type) and its ninst+1 offsets.
PHA_API void pha_ms_copy(void* h, int s, void* vals, int64_t* lod) {
  auto* p = static_cast<Parsed*>(h);
  SlotData& sd = p->slots[s];
  if (p->is_float[s]) {
    if (!sd.f.empty()) memcpy(vals, sd.f.data(), sd.f.size() * sizeof(float));
  } else if (!sd.i.empty()) {
    memcpy(vals, sd.i.data(), sd.i.size() * sizeof(int64_t));
  }
  memcpy(lod, sd.lod.data(), sd.lod.size() * sizeof(int64_t));
}
PHA_API void pha_ms_free(void* h) { delete static_cast<Parsed*>(h); }
