// Native inference engine: ProgramDesc / save_combine readers, the op set, the graph walker and the
// C APIs of pha_infer.h.
//
// Reference: paddle/fluid/inference/api/analysis_predictor.cc (load program + params, feed / fetch
// by the feed / fetch ops' `col`, run block 0 with the naive executor), capi_exp/pd_predictor.cc,
// pd_tensor.cc, pd_config.cc (the C surface), framework/framework.proto (wire format),
// framework/lod_tensor.cc:205 + tensor_util.cc:1046 (the params stream) and the op definitions in
// paddle/fluid/operators/*_op.cc + paddle/phi/infermeta for the shape rules of each op below.
//
// Design: one pass over block 0 in program order (the saved inference program is already
// topologically ordered), values in a name -> Tensor map, each intermediate freed after its last
// reader (liveness computed once at load). Reshape-like ops are views (shared buffer). Host
// (device -1) kernels are plain loops split over threads; device kernels live in gpu.hip.
#include "engine.h"
#include "pha_infer.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <numeric>
#include <set>
#include <sstream>
#include <thread>

namespace pha_infer {

// ==================================================================== protobuf wire decoding
namespace {
struct Wire {
  const uint8_t* p;
  const uint8_t* e;
  Wire(const void* b, size_t n) : p(static_cast<const uint8_t*>(b)), e(static_cast<const uint8_t*>(b) + n) {}
  bool done() const { return p >= e; }
  uint64_t varint() {
    uint64_t v = 0;
    for (int s = 0; s < 64; s += 7) {
      if (p >= e) throw Error("protobuf: truncated varint");
      const uint8_t b = *p++;
      v |= (uint64_t)(b & 0x7f) << s;
      if (!(b & 0x80)) return v;
    }
    throw Error("protobuf: varint too long");
  }
  void tag(int& field, int& wt) {
    const uint64_t t = varint();
    field = (int)(t >> 3);
    wt = (int)(t & 7);
  }
  Wire sub() {
    const uint64_t n = varint();
    if ((uint64_t)(e - p) < n) throw Error("protobuf: truncated field");
    Wire w(p, n);
    p += n;
    return w;
  }
  std::string str() {
    Wire w = sub();
    return std::string(reinterpret_cast<const char*>(w.p), w.e - w.p);
  }
  uint32_t f32() {
    if (e - p < 4) throw Error("protobuf: truncated fixed32");
    uint32_t v;
    std::memcpy(&v, p, 4);
    p += 4;
    return v;
  }
  uint64_t f64() {
    if (e - p < 8) throw Error("protobuf: truncated fixed64");
    uint64_t v;
    std::memcpy(&v, p, 8);
    p += 8;
    return v;
  }
  void skip(int wt) {
    if (wt == 0) varint();
    else if (wt == 1) f64();
    else if (wt == 2) sub();
    else if (wt == 5) f32();
    else throw Error("protobuf: unsupported wire type " + std::to_string(wt));
  }
  // a repeated varint field, packed (wt 2) or one element (wt 0)
  void ints(int wt, std::vector<int64_t>& out) {
    if (wt == 2) {
      Wire w = sub();
      while (!w.done()) out.push_back((int64_t)w.varint());
    } else {
      out.push_back((int64_t)varint());
    }
  }
};

float as_float(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
double as_double(uint64_t u) {
  double d;
  std::memcpy(&d, &u, 8);
  return d;
}

void parse_tensor_desc(Wire w, int& dtype, std::vector<int64_t>& dims) {
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    if (f == 1) dtype = (int)w.varint();
    else if (f == 2) w.ints(wt, dims);
    else w.skip(wt);
  }
}

VarDesc parse_var(Wire w) {
  VarDesc v;
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    if (f == 1) v.name = w.str();
    else if (f == 3) v.persistable = w.varint() != 0;
    else if (f == 2) {
      Wire t = w.sub();
      while (!t.done()) {
        int g, gt;
        t.tag(g, gt);
        if (g == 1) v.type = (int)t.varint();
        else if (g == 3 || g == 4) {   // lod_tensor / tensor_array: {tensor = 1, lod_level = 2}
          Wire l = t.sub();
          while (!l.done()) {
            int h, ht;
            l.tag(h, ht);
            if (h == 1) parse_tensor_desc(l.sub(), v.dtype, v.dims);
            else l.skip(ht);
          }
        } else if (g == 2) {
          parse_tensor_desc(t.sub(), v.dtype, v.dims);
        } else {
          t.skip(gt);
        }
      }
    } else {
      w.skip(wt);
    }
  }
  return v;
}

void parse_slot(Wire w, std::map<std::string, std::vector<std::string>>& m) {
  std::string name;
  std::vector<std::string> args;
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    if (f == 1) name = w.str();
    else if (f == 2) args.push_back(w.str());
    else w.skip(wt);
  }
  m[name] = args;
}

std::pair<std::string, Attr> parse_attr(Wire w) {
  std::string name;
  Attr a;
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    switch (f) {
      case 1: name = w.str(); break;
      case 2: a.type = (int)w.varint(); break;
      case 3: a.i = (int32_t)(uint32_t)w.varint(); break;
      case 4: a.f = as_float(w.f32()); break;
      case 5: a.s = w.str(); break;
      case 6: {   // int32 elements: sign from the low 32 bits
        std::vector<int64_t> v;
        w.ints(wt, v);
        for (auto x : v) a.ints.push_back((int32_t)(uint32_t)x);
        break;
      }
      case 7:
        if (wt == 2) {
          Wire s = w.sub();
          while (!s.done()) a.floats.push_back(as_float(s.f32()));
        } else {
          a.floats.push_back(as_float(w.f32()));
        }
        break;
      case 8: a.strings.push_back(w.str()); break;
      case 10: a.b = w.varint() != 0; break;
      case 11: case 14: case 15: w.ints(wt, a.ints); break;
      case 12: a.i = (int64_t)w.varint(); break;
      case 13: a.i = (int64_t)w.varint(); break;
      case 16:
        if (wt == 2) {
          Wire s = w.sub();
          while (!s.done()) a.floats.push_back(as_double(s.f64()));
        } else {
          a.floats.push_back(as_double(w.f64()));
        }
        break;
      default: w.skip(wt);
    }
  }
  return {name, a};
}

OpDesc parse_op(Wire w) {
  OpDesc op;
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    if (f == 3) op.type = w.str();
    else if (f == 1) parse_slot(w.sub(), op.inputs);
    else if (f == 2) parse_slot(w.sub(), op.outputs);
    else if (f == 4) op.attrs.insert(parse_attr(w.sub()));
    else w.skip(wt);
  }
  return op;
}

Block parse_block(Wire w) {
  Block b;
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    if (f == 3) b.vars.push_back(parse_var(w.sub()));
    else if (f == 4) b.ops.push_back(parse_op(w.sub()));
    else w.skip(wt);
  }
  return b;
}
}  // namespace

Program parse_program(const std::string& bytes) {
  Program prog;
  Wire w(bytes.data(), bytes.size());
  while (!w.done()) {
    int f, wt;
    w.tag(f, wt);
    if (f == 1) prog.blocks.push_back(parse_block(w.sub()));
    else w.skip(wt);
  }
  if (prog.blocks.empty()) throw Error("program has no blocks (not a ProgramDesc?)");
  return prog;
}

int64_t OpDesc::geti(const std::string& k, int64_t d) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) return d;
  const Attr& a = it->second;
  if (a.type == 6) return a.b;
  if (a.type == 1) return (int64_t)a.f;
  if (a.type == 3 || a.type == 11) return a.ints.empty() ? d : a.ints[0];
  return a.i;
}
double OpDesc::getf(const std::string& k, double d) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) return d;
  const Attr& a = it->second;
  if (a.type == 1) return a.f;
  if (a.type == 0 || a.type == 9) return (double)a.i;
  if (a.type == 4 || a.type == 12) return a.floats.empty() ? d : a.floats[0];
  return d;
}
bool OpDesc::getb(const std::string& k, bool d) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) return d;
  const Attr& a = it->second;
  if (a.type == 6) return a.b;
  if (a.type == 0 || a.type == 9) return a.i != 0;
  return d;
}
std::string OpDesc::gets(const std::string& k, const std::string& d) const {
  auto it = attrs.find(k);
  return it == attrs.end() || it->second.type != 2 ? d : it->second.s;
}
std::vector<int64_t> OpDesc::getints(const std::string& k, std::vector<int64_t> d) const {
  auto it = attrs.find(k);
  if (it == attrs.end()) return d;
  const Attr& a = it->second;
  if (a.type == 0 || a.type == 9) return {a.i};   // a scalar where the reference writes a list
  return a.ints;
}
std::string OpDesc::in(const std::string& slot) const {
  auto it = inputs.find(slot);
  return it == inputs.end() || it->second.empty() ? "" : it->second[0];
}
std::string OpDesc::out(const std::string& slot) const {
  auto it = outputs.find(slot);
  return it == outputs.end() || it->second.empty() ? "" : it->second[0];
}

// ==================================================================== tensors
size_t dtype_size(int dt) {
  switch (dt) {
    case BOOL: case U8: case I8: return 1;
    case I16: case F16: return 2;
    case I32: case F32: return 4;
    case I64: case F64: return 8;
  }
  throw Error("unsupported element type " + std::to_string(dt));
}

Buffer::Buffer(size_t bytes, int d) : n(bytes), dev(d) {
  if (dev >= 0) {
    ctx = gpu::current();
    p = gpu::alloc(bytes);
  } else {
    p = ::operator new(bytes ? bytes : 16);
  }
}
Buffer::~Buffer() {
  if (dev >= 0) gpu::release(ctx, p, n);
  else ::operator delete(p);
}

Tensor make_tensor(std::vector<int64_t> shape, int dtype, int dev) {
  Tensor t;
  t.shape = std::move(shape);
  t.dtype = dtype;
  t.buf = std::make_shared<Buffer>(t.bytes(), dev);
  return t;
}

Tensor to_device(const Tensor& t, int dev) {
  Tensor o = make_tensor(t.shape, t.dtype, dev);
  const int src = t.buf->dev;
  if (src < 0 && dev < 0) std::memcpy(o.raw(), t.raw(), t.bytes());
  else if (src < 0) gpu::h2d(o.raw(), t.raw(), t.bytes());
  else if (dev < 0) gpu::d2h(o.raw(), t.raw(), t.bytes());
  else gpu::d2d(o.raw(), t.raw(), t.bytes());
  return o;
}

namespace {
// ---- the params stream ---------------------------------------------------------------------------
Tensor read_lod_tensor(const std::string& buf, size_t& off) {
  // every length read from the file is checked against the bytes left before it is used
  // (n > size - off cannot wrap, unlike off + n > size)
  auto need = [&](uint64_t n) {
    if (off > buf.size() || n > buf.size() - off) throw Error("params stream truncated");
  };
  uint32_t ver;
  need(4);
  std::memcpy(&ver, buf.data() + off, 4);
  off += 4;
  if (ver != 0) throw Error("unsupported LoDTensor version " + std::to_string(ver));
  uint64_t nlod;
  need(8);
  std::memcpy(&nlod, buf.data() + off, 8);
  off += 8;
  if (nlod > 8) throw Error("params stream: " + std::to_string(nlod) + " LoD levels");
  for (uint64_t i = 0; i < nlod; ++i) {
    uint64_t nb;
    need(8);
    std::memcpy(&nb, buf.data() + off, 8);
    off += 8;
    need(nb);
    off += nb;
  }
  need(8);
  std::memcpy(&ver, buf.data() + off, 4);
  off += 4;
  if (ver != 0) throw Error("unsupported Tensor version " + std::to_string(ver));
  int32_t dsz;
  std::memcpy(&dsz, buf.data() + off, 4);
  off += 4;
  if (dsz < 0) throw Error("params stream: negative tensor desc size");
  need((uint64_t)dsz);
  int dtype = F32;
  std::vector<int64_t> dims;
  parse_tensor_desc(Wire(buf.data() + off, (size_t)dsz), dtype, dims);
  off += (size_t)dsz;
  uint64_t elems = 1;
  for (auto d : dims) {
    if (d < 0) throw Error("params stream: negative dim in a persistable's shape");
    if (d && elems > (uint64_t)INT64_MAX / (uint64_t)d) throw Error("params stream: tensor size overflows");
    elems *= (uint64_t)d;
  }
  if (elems > (uint64_t)INT64_MAX / 8) throw Error("params stream: tensor size overflows");
  need(elems * dtype_size(dtype));   // before allocating it
  Tensor t = make_tensor(dims, dtype, -1);
  need(t.bytes());
  std::memcpy(t.raw(), buf.data() + off, t.bytes());
  off += t.bytes();
  return t;
}

std::string read_file(const std::string& path) {
  std::ifstream f(path, std::ios::binary);
  if (!f) throw Error("cannot open " + path);
  std::ostringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

// ---- host threading ---------------------------------------------------------------------------
void parallel_for(int64_t n, const std::function<void(int64_t, int64_t)>& fn) {
  const int64_t nt = std::min<int64_t>(std::max(1u, std::min(8u, std::thread::hardware_concurrency())),
                                       std::max<int64_t>(1, n / 64));
  if (nt <= 1) {
    fn(0, n);
    return;
  }
  std::vector<std::thread> th;
  const int64_t chunk = (n + nt - 1) / nt;
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a < b) th.emplace_back(fn, a, b);
  }
  for (auto& x : th) x.join();
}

std::vector<int64_t> contiguous_strides(const std::vector<int64_t>& shape) {
  std::vector<int64_t> s(shape.size(), 1);
  for (int k = (int)shape.size() - 2; k >= 0; --k) s[k] = s[k + 1] * shape[k + 1];
  return s;
}

std::string shape_str(const std::vector<int64_t>& s) {
  std::string r = "[";
  for (size_t i = 0; i < s.size(); ++i) r += (i ? ", " : "") + std::to_string(s[i]);
  return r + "]";
}
}  // namespace

// ==================================================================== op kernels (host + device)
namespace {
struct Ctx {
  int dev;
  std::map<std::string, Tensor>& env;
  bool bf16 = false;   // GEMM-class ops (mul / matmul / fc / conv via im2col) on bf16 MFMA
  Tensor& get(const std::string& n) {
    auto it = env.find(n);
    if (it == env.end()) throw Error("variable " + n + " has no value");
    return it->second;
  }
  bool has(const std::string& n) const { return !n.empty() && env.count(n); }
  Tensor alloc(std::vector<int64_t> shape, int dtype = F32) { return make_tensor(std::move(shape), dtype, dev); }
  void set(const std::string& n, Tensor t) {
    if (!n.empty()) env[n] = std::move(t);
  }
  bool gpu() const { return dev >= 0; }
};

void need_f32(const Tensor& t, const char* op) {
  if (t.dtype != F32) throw Error(std::string(op) + ": float32 input expected, got type " + std::to_string(t.dtype));
}

// ---- strided copy: out (contiguous, `shape`) <- in viewed with element `strides` -------------------
void strided_copy(Ctx& c, const Tensor& in, const void* in_ptr, Tensor& out, const std::vector<int64_t>& shape,
                  const std::vector<int64_t>& strides) {
  const int es = (int)dtype_size(in.dtype);
  const int nd = (int)shape.size();
  if (c.gpu()) {
    gpu::strided_copy(in_ptr, out.raw(), es, nd, shape.data(), strides.data());
    return;
  }
  const int64_t total = out.numel();
  const char* src = static_cast<const char*>(in_ptr);
  char* dst = static_cast<char*>(out.raw());
  parallel_for(total, [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      int64_t rem = i, off = 0;
      for (int k = nd - 1; k >= 0; --k) {
        off += (rem % shape[k]) * strides[k];
        rem /= shape[k];
      }
      std::memcpy(dst + i * es, src + off * es, es);
    }
  });
}

// ---- GEMM: C[b] = alpha A[b] B[b] (+ bias) (relu) -----------------------------------------------
struct GemmArgs {
  const float* A;
  const float* B;
  float* C;
  const float* bias = nullptr;
  int batch = 1, M = 0, N = 0, K = 0;
  int64_t sAb = 0, sAm = 0, sAk = 0, sBb = 0, sBk = 0, sBn = 0, sCb = 0, sCm = 0;
  float alpha = 1.f;
  bool relu = false;
};

void gemm(Ctx& c, const GemmArgs& g) {
  if (c.gpu() && c.bf16 &&
      gpu::gemm_bf16(g.A, g.B, g.C, g.bias, g.batch, g.M, g.N, g.K, g.sAb, g.sAm, g.sAk, g.sBb, g.sBk, g.sBn, g.sCb,
                     g.sCm, g.alpha, g.relu))
    return;
  if (c.gpu()) {
    gpu::gemm(g.A, g.B, g.C, g.bias, g.batch, g.M, g.N, g.K, g.sAb, g.sAm, g.sAk, g.sBb, g.sBk, g.sBn, g.sCb, g.sCm,
              g.alpha, g.relu);
    return;
  }
  parallel_for((int64_t)g.batch * g.M, [&](int64_t a, int64_t b) {
    std::vector<float> row(g.N);
    for (int64_t r = a; r < b; ++r) {
      const int64_t bi = r / g.M, m = r % g.M;
      std::fill(row.begin(), row.end(), 0.f);
      const float* A = g.A + bi * g.sAb + m * g.sAm;
      const float* B = g.B + bi * g.sBb;
      for (int k = 0; k < g.K; ++k) {
        const float av = A[k * g.sAk];
        if (av == 0.f) continue;
        const float* Bk = B + k * g.sBk;
        if (g.sBn == 1)
          for (int n = 0; n < g.N; ++n) row[n] += av * Bk[n];
        else
          for (int n = 0; n < g.N; ++n) row[n] += av * Bk[n * g.sBn];
      }
      float* C = g.C + bi * g.sCb + m * g.sCm;
      for (int n = 0; n < g.N; ++n) {
        float v = g.alpha * row[n];
        if (g.bias) v += g.bias[n];
        if (g.relu && v < 0.f) v = 0.f;
        C[n] = v;
      }
    }
  });
}

// ---- conv2d (NCHW) --------------------------------------------------------------------------------
struct Pads {
  int t = 0, b = 0, l = 0, r = 0;
};

Pads conv_pads(const OpDesc& op, int H, int W, int KH, int KW, int sh, int sw, int dh, int dw) {
  Pads p;
  const std::string algo = op.gets("padding_algorithm", "EXPLICIT");
  auto pads = op.getints("paddings", {0, 0});
  if (algo == "VALID") return p;
  if (algo == "SAME") {
    auto same = [](int in, int k, int s, int d, int& lo, int& hi) {
      const int out = (in + s - 1) / s;
      const int tot = std::max((out - 1) * s + d * (k - 1) + 1 - in, 0);
      lo = tot / 2;
      hi = tot - lo;
    };
    same(H, KH, sh, dh, p.t, p.b);
    same(W, KW, sw, dw, p.l, p.r);
    return p;
  }
  if (pads.size() == 4) {
    p.t = (int)pads[0]; p.b = (int)pads[1]; p.l = (int)pads[2]; p.r = (int)pads[3];
  } else if (pads.size() == 2) {
    p.t = p.b = (int)pads[0]; p.l = p.r = (int)pads[1];
  } else if (pads.size() == 1) {
    p.t = p.b = p.l = p.r = (int)pads[0];
  }
  return p;
}

std::pair<int, int> pair2(const OpDesc& op, const std::string& k, int d) {
  auto v = op.getints(k, {d, d});
  if (v.size() == 1) return {(int)v[0], (int)v[0]};
  if (v.size() < 2) return {d, d};
  return {(int)v[0], (int)v[1]};
}

void op_conv2d(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("Input"));
  Tensor& w = c.get(op.in("Filter"));
  need_f32(x, "conv2d");
  const std::string fmt = op.gets("data_format", "NCHW");
  if (fmt == "NHWC") throw Error("conv2d: NHWC models are not supported by the native engine");
  if (x.ndim() != 4 || w.ndim() != 4) throw Error("conv2d: 4-D input and filter expected");
  const int N = (int)x.shape[0], C = (int)x.shape[1], H = (int)x.shape[2], W = (int)x.shape[3];
  const int Co = (int)w.shape[0], Cg = (int)w.shape[1], KH = (int)w.shape[2], KW = (int)w.shape[3];
  int groups = (int)op.geti("groups", 1);
  if (groups < 1) groups = 1;
  auto [sh, sw] = pair2(op, "strides", 1);
  auto [dh, dw] = pair2(op, "dilations", 1);
  const Pads p = conv_pads(op, H, W, KH, KW, sh, sw, dh, dw);
  const int OH = (H + p.t + p.b - (dh * (KH - 1) + 1)) / sh + 1;
  const int OW = (W + p.l + p.r - (dw * (KW - 1) + 1)) / sw + 1;
  if (Cg * groups != C) throw Error("conv2d: filter channels " + std::to_string(Cg) + " x groups != input channels");
  Tensor y = c.alloc({N, Co, OH, OW});
  const float* bias = c.has(op.in("Bias")) ? c.get(op.in("Bias")).data<float>() : nullptr;
  if (groups == C && Cg == 1) {   // depthwise (channel multiplier Co / C)
    const int mult = Co / C;
    if (c.gpu()) {
      gpu::depthwise_conv(x.data<float>(), w.data<float>(), y.data<float>(), N, C, H, W, KH, KW, OH, OW, sh, sw, p.t,
                          p.l, dh, dw, mult);
    } else {
      const float* xp = x.data<float>();
      const float* wp = w.data<float>();
      float* yp = y.data<float>();
      parallel_for((int64_t)N * Co, [&](int64_t a, int64_t b) {
        for (int64_t nc = a; nc < b; ++nc) {
          const int co = nc % Co, n = (int)(nc / Co), ci = co / mult;
          for (int oh = 0; oh < OH; ++oh)
            for (int ow = 0; ow < OW; ++ow) {
              float s = 0.f;
              for (int kh = 0; kh < KH; ++kh) {
                const int ih = oh * sh - p.t + kh * dh;
                if (ih < 0 || ih >= H) continue;
                for (int kw = 0; kw < KW; ++kw) {
                  const int iw = ow * sw - p.l + kw * dw;
                  if (iw < 0 || iw >= W) continue;
                  s += xp[(((int64_t)n * C + ci) * H + ih) * W + iw] * wp[((int64_t)co * KH + kh) * KW + kw];
                }
              }
              yp[nc * OH * OW + oh * OW + ow] = s;
            }
        }
      });
    }
  } else if (c.gpu()) {
    // the whole batch per launch: out[n][co][p] = sum_k W[co][k] col[n][k][p] as one batched GEMM
    // per group (A shared across images); a 1x1 / stride-1 / unpadded conv multiplies x in place
    const int Kg = Cg * KH * KW, P = OH * OW, Cog = Co / groups;
    const bool direct = KH == 1 && KW == 1 && sh == 1 && sw == 1 && p.t == 0 && p.l == 0 && p.b == 0 && p.r == 0 &&
                        OH == H && OW == W;
    Tensor col;
    const float* src = x.data<float>();
    int64_t sbb = (int64_t)C * H * W;
    if (!direct) {
      col = c.alloc({(int64_t)N * C * KH * KW, P});
      gpu::im2col(x.data<float>(), col.data<float>(), C, H, W, KH, KW, OH, OW, sh, sw, p.t, p.l, dh, dw, N);
      src = col.data<float>();
      sbb = (int64_t)C * KH * KW * P;
    }
    for (int g = 0; g < groups; ++g) {
      GemmArgs ga;
      ga.A = w.data<float>() + (int64_t)g * Cog * Kg;
      ga.B = src + (int64_t)g * Kg * P;
      ga.C = y.data<float>() + (int64_t)g * Cog * P;
      ga.batch = N;
      ga.M = Cog; ga.N = P; ga.K = Kg;
      ga.sAb = 0; ga.sAm = Kg; ga.sAk = 1;
      ga.sBb = sbb; ga.sBk = P; ga.sBn = 1;
      ga.sCb = (int64_t)Co * P; ga.sCm = P;
      gemm(c, ga);
    }
    if (bias) gpu::row_bias_act(y.data<float>(), bias, Co, P, N, false);
    bias = nullptr;
  } else {
    // im2col per image + GEMM per group: out[co, p] = sum_k W[co, k] col[k, p]
    const int Kg = Cg * KH * KW, P = OH * OW, Cog = Co / groups;
    Tensor col = c.alloc({(int64_t)C * KH * KW, P});
    for (int n = 0; n < N; ++n) {
      const float* xn = x.data<float>() + (int64_t)n * C * H * W;
      {
        float* cp = col.data<float>();
        parallel_for((int64_t)C * KH * KW, [&](int64_t a, int64_t b) {
          for (int64_t r = a; r < b; ++r) {
            const int kw = r % KW, kh = (r / KW) % KH, ci = (int)(r / (KW * KH));
            for (int oh = 0; oh < OH; ++oh)
              for (int ow = 0; ow < OW; ++ow) {
                const int ih = oh * sh - p.t + kh * dh, iw = ow * sw - p.l + kw * dw;
                cp[r * P + oh * OW + ow] =
                    (ih >= 0 && ih < H && iw >= 0 && iw < W) ? xn[((int64_t)ci * H + ih) * W + iw] : 0.f;
              }
          }
        });
      }
      for (int g = 0; g < groups; ++g) {
        GemmArgs ga;
        ga.A = w.data<float>() + (int64_t)g * Cog * Kg;
        ga.B = col.data<float>() + (int64_t)g * Kg * P;
        ga.C = y.data<float>() + ((int64_t)n * Co + (int64_t)g * Cog) * P;
        ga.M = Cog; ga.N = P; ga.K = Kg;
        ga.sAm = Kg; ga.sAk = 1; ga.sBk = P; ga.sBn = 1; ga.sCm = P;
        gemm(c, ga);
      }
    }
  }
  if (bias) {   // conv_op.cc's (MKLDNN-only) Bias input: + bias[co]
    const int64_t inner = (int64_t)OH * OW;
    std::vector<int64_t> shp = {N, Co, inner}, sx = {(int64_t)Co * inner, inner, 1}, sy = {0, 1, 0};
    if (c.gpu()) {
      gpu::binary(y.data<float>(), bias, y.data<float>(), gpu::ADD, 3, shp.data(), sx.data(), sy.data());
    } else {
      float* yp = y.data<float>();
      for (int64_t i = 0; i < y.numel(); ++i) yp[i] += bias[(i / inner) % Co];
    }
  }
  c.set(op.out("Output"), y);
}

// ---- elementwise --------------------------------------------------------------------------------
float host_binary(int op, float a, float b) {
  switch (op) {
    case gpu::ADD: return a + b;
    case gpu::SUB: return a - b;
    case gpu::MUL: return a * b;
    case gpu::DIV: return a / b;
    case gpu::MAX: return std::max(a, b);
    case gpu::MIN: return std::min(a, b);
    default: return std::pow(a, b);
  }
}

// out = x op y with the reference's broadcast: axis == -1 numpy (right-aligned), else Y's dims
// aligned with X's starting at `axis`
void binary(Ctx& c, const Tensor& x, const Tensor& y, int op, int axis, Tensor& out_t, bool alloc_out = true) {
  std::vector<int64_t> xs = x.shape, ys = y.shape;
  if (axis >= 0 && ys.size() < xs.size()) {
    std::vector<int64_t> t(axis, 1);
    t.insert(t.end(), ys.begin(), ys.end());
    while (t.size() < xs.size()) t.push_back(1);
    ys = t;
  }
  const size_t nd = std::max(xs.size(), ys.size());
  while (xs.size() < nd) xs.insert(xs.begin(), 1);
  while (ys.size() < nd) ys.insert(ys.begin(), 1);
  std::vector<int64_t> os(nd), sx(nd), sy(nd);
  const auto cx = contiguous_strides(xs), cy = contiguous_strides(ys);
  for (size_t k = 0; k < nd; ++k) {
    if (xs[k] != ys[k] && xs[k] != 1 && ys[k] != 1)
      throw Error("elementwise: shapes " + shape_str(x.shape) + " and " + shape_str(y.shape) + " do not broadcast");
    os[k] = std::max(xs[k], ys[k]);
    sx[k] = xs[k] == 1 ? 0 : cx[k];
    sy[k] = ys[k] == 1 ? 0 : cy[k];
  }
  if (alloc_out) out_t = c.alloc(os);
  if (nd == 0) {
    os = {1}; sx = {0}; sy = {0};
  }
  if (c.gpu()) {
    gpu::binary(x.data<float>(), y.data<float>(), out_t.data<float>(), op, (int)os.size(), os.data(), sx.data(),
                sy.data());
    return;
  }
  const float* xp = x.data<float>();
  const float* yp = y.data<float>();
  float* op_ = out_t.data<float>();
  const int n = (int)os.size();
  parallel_for(out_t.numel(), [&](int64_t a, int64_t b) {
    for (int64_t i = a; i < b; ++i) {
      int64_t rem = i, ox = 0, oy = 0;
      for (int k = n - 1; k >= 0; --k) {
        const int64_t q = rem % os[k];
        rem /= os[k];
        ox += q * sx[k];
        oy += q * sy[k];
      }
      op_[i] = host_binary(op, xp[ox], yp[oy]);
    }
  });
}

std::function<void(Ctx&, const OpDesc&)> op_elementwise(int which) {
  return [which](Ctx& c, const OpDesc& op) {
    Tensor& x = c.get(op.in("X"));
    Tensor& y = c.get(op.in("Y"));
    need_f32(x, "elementwise");
    need_f32(y, "elementwise");
    Tensor out;
    binary(c, x, y, which, (int)op.geti("axis", -1), out);
    c.set(op.out("Out"), out);
  };
}

float host_unary(int op, float v, float a, float b) {
  switch (op) {
    case gpu::RELU: return v > 0.f ? v : 0.f;
    case gpu::RELU6: return std::min(std::max(v, 0.f), a);
    case gpu::SIGMOID: return 1.f / (1.f + std::exp(-v));
    case gpu::TANH: return std::tanh(v);
    case gpu::GELU: return 0.5f * v * (1.f + std::erf(v * 0.70710678118654752f));
    case gpu::GELU_TANH: return 0.5f * v * (1.f + std::tanh(0.7978845608028654f * (v + 0.044715f * v * v * v)));
    case gpu::SILU: return v / (1.f + std::exp(-a * v));
    case gpu::HARD_SWISH: return v * std::min(std::max(v + 3.f, 0.f), 6.f) / 6.f;
    case gpu::HARD_SIGMOID: return std::min(std::max(a * v + b, 0.f), 1.f);
    case gpu::LEAKY_RELU: return v > 0.f ? v : a * v;
    case gpu::EXP: return std::exp(v);
    case gpu::SQRT: return std::sqrt(v);
    case gpu::ABS: return std::fabs(v);
    case gpu::SCALE: return a * v + b;
    case gpu::SQUARE: return v * v;
    case gpu::RSQRT: return 1.f / std::sqrt(v);
  }
  return v;
}

void unary(Ctx& c, const Tensor& x, Tensor& y, int which, float a, float b) {
  if (c.gpu()) {
    gpu::unary(x.data<float>(), y.data<float>(), x.numel(), which, a, b);
    return;
  }
  const float* xp = x.data<float>();
  float* yp = y.data<float>();
  parallel_for(x.numel(), [&](int64_t s, int64_t e) {
    for (int64_t i = s; i < e; ++i) yp[i] = host_unary(which, xp[i], a, b);
  });
}

std::function<void(Ctx&, const OpDesc&)> op_unary(int which, std::function<std::pair<float, float>(const OpDesc&)> ab) {
  return [which, ab](Ctx& c, const OpDesc& op) {
    Tensor& x = c.get(op.in("X"));
    need_f32(x, op.type.c_str());
    int w = which;
    if (w == gpu::GELU && op.getb("approximate", false)) w = gpu::GELU_TANH;
    const auto [a, b] = ab ? ab(op) : std::pair<float, float>{0.f, 0.f};
    Tensor y = c.alloc(x.shape);
    unary(c, x, y, w, a, b);
    c.set(op.out("Out"), y);
  };
}

void op_scale(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  need_f32(x, "scale");
  const float s = (float)op.getf("scale", 1.0), bias = (float)op.getf("bias", 0.0);
  const bool after = op.getb("bias_after_scale", true);
  Tensor y = c.alloc(x.shape);
  unary(c, x, y, gpu::SCALE, s, after ? bias : s * bias);
  c.set(op.out("Out"), y);
}

void op_dropout(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  if (op.gets("dropout_implementation", "downgrade_in_infer") == "upscale_in_train") {
    c.set(op.out("Out"), x);   // inference: identity
    return;
  }
  const float p = (float)op.getf("dropout_prob", 0.5);
  Tensor y = c.alloc(x.shape);
  unary(c, x, y, gpu::SCALE, 1.f - p, 0.f);
  c.set(op.out("Out"), y);
}

// ---- batch_norm (inference statistics) -----------------------------------------------------------
void op_batch_norm(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  need_f32(x, "batch_norm");
  if (op.gets("data_layout", "NCHW") == "NHWC") throw Error("batch_norm: NHWC is not supported by the native engine");
  const int64_t N = x.shape[0], C = x.ndim() > 1 ? x.shape[1] : 1;
  const int64_t inner = x.numel() / std::max<int64_t>(1, N * C);
  const float eps = (float)op.getf("epsilon", 1e-5);
  const float* sc = c.get(op.in("Scale")).data<float>();
  const float* bi = c.get(op.in("Bias")).data<float>();
  const float* mu = c.get(op.in("Mean")).data<float>();
  const float* va = c.get(op.in("Variance")).data<float>();
  Tensor y = c.alloc(x.shape);
  if (c.gpu()) {
    gpu::batch_norm(x.data<float>(), y.data<float>(), sc, bi, mu, va, eps, N, C, inner);
  } else {
    const float* xp = x.data<float>();
    float* yp = y.data<float>();
    parallel_for(N * C, [&](int64_t a, int64_t b) {
      for (int64_t nc = a; nc < b; ++nc) {
        const int64_t ch = nc % C;
        const float inv = 1.f / std::sqrt(va[ch] + eps);
        for (int64_t i = 0; i < inner; ++i) yp[nc * inner + i] = (xp[nc * inner + i] - mu[ch]) * inv * sc[ch] + bi[ch];
      }
    });
  }
  c.set(op.out("Y"), y);
}

// ---- pool2d ----------------------------------------------------------------------------------------
void op_pool2d(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  need_f32(x, "pool2d");
  if (op.gets("data_format", "NCHW") == "NHWC") throw Error("pool2d: NHWC is not supported by the native engine");
  const int N = (int)x.shape[0], C = (int)x.shape[1], H = (int)x.shape[2], W = (int)x.shape[3];
  const bool maxp = op.gets("pooling_type", "max") == "max";
  const bool global = op.getb("global_pooling", false), adaptive = op.getb("adaptive", false);
  auto [KH, KW] = pair2(op, "ksize", 1);
  auto [sh, sw] = pair2(op, "strides", 1);
  Pads p;
  int OH, OW;
  if (global) {
    KH = H; KW = W; OH = OW = 1; sh = sw = 1;
  } else if (adaptive) {
    OH = KH; OW = KW;
  } else {
    p = conv_pads(op, H, W, KH, KW, sh, sw, 1, 1);
    const bool ceil = op.getb("ceil_mode", false);
    auto outdim = [&](int in, int k, int s, int lo, int hi) {
      const int span = in + lo + hi - k;
      return (ceil ? (span + s - 1) / s : span / s) + 1;
    };
    OH = outdim(H, KH, sh, p.t, p.b);
    OW = outdim(W, KW, sw, p.l, p.r);
  }
  const bool excl = op.getb("exclusive", true);
  Tensor y = c.alloc({N, C, OH, OW});
  if (c.gpu()) {
    gpu::pool2d(x.data<float>(), y.data<float>(), N, C, H, W, OH, OW, KH, KW, sh, sw, p.t, p.l, maxp, excl,
                adaptive && !global);
  } else {
    const float* xp = x.data<float>();
    float* yp = y.data<float>();
    const bool ad = adaptive && !global;
    parallel_for((int64_t)N * C, [&](int64_t a, int64_t b) {
      for (int64_t nc = a; nc < b; ++nc)
        for (int oh = 0; oh < OH; ++oh)
          for (int ow = 0; ow < OW; ++ow) {
            int h0, h1, w0, w1;
            if (ad) {
              h0 = oh * H / OH; h1 = ((oh + 1) * H + OH - 1) / OH;
              w0 = ow * W / OW; w1 = ((ow + 1) * W + OW - 1) / OW;
            } else {
              h0 = oh * sh - p.t; w0 = ow * sw - p.l; h1 = h0 + KH; w1 = w0 + KW;
            }
            const int ch0 = std::max(h0, 0), cw0 = std::max(w0, 0), ch1 = std::min(h1, H), cw1 = std::min(w1, W);
            float acc = maxp ? -INFINITY : 0.f;
            for (int h = ch0; h < ch1; ++h)
              for (int w = cw0; w < cw1; ++w) {
                const float v = xp[nc * H * W + h * W + w];
                acc = maxp ? std::max(acc, v) : acc + v;
              }
            if (!maxp) {
              const int cnt = (excl || ad) ? (ch1 - ch0) * (cw1 - cw0) : KH * KW;
              acc = cnt > 0 ? acc / cnt : 0.f;
            }
            yp[nc * OH * OW + oh * OW + ow] = acc;
          }
    });
  }
  c.set(op.out("Out"), y);
}

// ---- shape ops (views) --------------------------------------------------------------------------
Tensor view(const Tensor& x, std::vector<int64_t> shape) {
  Tensor t = x;
  t.shape = std::move(shape);
  if (t.numel() != x.numel())
    throw Error("reshape: " + shape_str(x.shape) + " cannot be viewed as " + shape_str(t.shape));
  return t;
}

void op_reshape2(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  auto sh = op.getints("shape");
  std::vector<int64_t> out(sh.size());
  int64_t known = 1;
  int neg = -1;
  for (size_t i = 0; i < sh.size(); ++i) {
    out[i] = sh[i] == 0 ? x.shape.at(i) : sh[i];
    if (out[i] == -1) neg = (int)i;
    else known *= out[i];
  }
  if (neg >= 0) out[neg] = known ? x.numel() / known : 0;
  c.set(op.out("Out"), view(x, out));
}

void op_flatten_range(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  const int nd = x.ndim();
  int s = (int)op.geti("start_axis", 1), e = (int)op.geti("stop_axis", -1);
  if (nd == 0) {
    c.set(op.out("Out"), view(x, {1}));
    return;
  }
  if (s < 0) s += nd;
  if (e < 0) e += nd;
  std::vector<int64_t> out(x.shape.begin(), x.shape.begin() + s);
  int64_t m = 1;
  for (int k = s; k <= e; ++k) m *= x.shape[k];
  out.push_back(m);
  out.insert(out.end(), x.shape.begin() + e + 1, x.shape.end());
  c.set(op.out("Out"), view(x, out));
}

void op_flatten2(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  const int axis = (int)op.geti("axis", 1);
  int64_t a = 1, b = 1;
  for (int k = 0; k < x.ndim(); ++k) (k < axis ? a : b) *= x.shape[k];
  c.set(op.out("Out"), view(x, {a, b}));
}

void op_squeeze2(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  auto axes = op.getints("axes");
  std::set<int> drop;
  for (auto a : axes) drop.insert((int)(a < 0 ? a + x.ndim() : a));
  std::vector<int64_t> out;
  for (int k = 0; k < x.ndim(); ++k) {
    const bool d = axes.empty() ? x.shape[k] == 1 : (drop.count(k) && x.shape[k] == 1);
    if (!d) out.push_back(x.shape[k]);
  }
  c.set(op.out("Out"), view(x, out));
}

void op_unsqueeze2(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  std::vector<int64_t> out = x.shape;
  for (auto a : op.getints("axes")) {
    int k = (int)(a < 0 ? a + (int64_t)out.size() + 1 : a);
    out.insert(out.begin() + k, 1);
  }
  c.set(op.out("Out"), view(x, out));
}

void op_assign(Ctx& c, const OpDesc& op) { c.set(op.out("Out"), c.get(op.in("X"))); }

void op_transpose2(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  auto perm = op.getints("axis");
  const auto st = contiguous_strides(x.shape);
  std::vector<int64_t> shape(perm.size()), strides(perm.size());
  for (size_t k = 0; k < perm.size(); ++k) {
    shape[k] = x.shape.at(perm[k]);
    strides[k] = st.at(perm[k]);
  }
  Tensor y = c.alloc(shape, x.dtype);
  strided_copy(c, x, x.raw(), y, shape, strides);
  c.set(op.out("Out"), y);
}

void op_slice(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("Input"));
  auto axes = op.getints("axes"), starts = op.getints("starts"), ends = op.getints("ends");
  auto dec = op.getints("decrease_axis");
  std::vector<int64_t> shape = x.shape, begin(x.ndim(), 0);
  for (size_t i = 0; i < axes.size(); ++i) {
    const int a = (int)(axes[i] < 0 ? axes[i] + x.ndim() : axes[i]);
    const int64_t d = x.shape[a];
    int64_t s = starts[i] < 0 ? starts[i] + d : starts[i];
    int64_t e = ends[i] < 0 ? ends[i] + d : ends[i];
    s = std::min(std::max<int64_t>(s, 0), d);
    e = std::min(std::max<int64_t>(e, 0), d);
    begin[a] = s;
    shape[a] = std::max<int64_t>(e - s, 0);
  }
  const auto st = contiguous_strides(x.shape);
  int64_t off = 0;
  for (int k = 0; k < x.ndim(); ++k) off += begin[k] * st[k];
  Tensor y = c.alloc(shape, x.dtype);
  strided_copy(c, x, static_cast<const char*>(x.raw()) + off * dtype_size(x.dtype), y, shape, st);
  if (!dec.empty()) {
    std::set<int> d;
    for (auto a : dec) d.insert((int)(a < 0 ? a + x.ndim() : a));
    std::vector<int64_t> o;
    for (int k = 0; k < x.ndim(); ++k)
      if (!d.count(k)) o.push_back(shape[k]);
    if (o.empty()) o.push_back(1);
    y = view(y, o);
  }
  c.set(op.out("Out"), y);
}

void op_concat(Ctx& c, const OpDesc& op) {
  const auto& names = op.inputs.at("X");
  std::vector<Tensor*> xs;
  for (auto& n : names) xs.push_back(&c.get(n));
  const int nd = xs[0]->ndim();
  int axis = (int)op.geti("axis", 0);
  if (axis < 0) axis += nd;
  std::vector<int64_t> shape = xs[0]->shape;
  shape[axis] = 0;
  for (auto* t : xs) shape[axis] += t->shape[axis];
  Tensor y = c.alloc(shape, xs[0]->dtype);
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < axis; ++k) outer *= shape[k];
  for (int k = axis + 1; k < nd; ++k) inner *= shape[k];
  const size_t es = dtype_size(y.dtype);
  const size_t row = (size_t)shape[axis] * inner * es;
  size_t at = 0;
  for (auto* t : xs) {
    const size_t w = (size_t)t->shape[axis] * inner * es;
    char* dst = static_cast<char*>(y.raw()) + at;
    const char* src = static_cast<const char*>(t->raw());
    if (c.gpu()) {
      for (int64_t o = 0; o < outer; ++o) gpu::d2d(dst + o * row, src + o * w, w);
    } else {
      for (int64_t o = 0; o < outer; ++o) std::memcpy(dst + o * row, src + o * w, w);
    }
    at += w;
  }
  c.set(op.out("Out"), y);
}

// ---- matmul family ----------------------------------------------------------------------------------
// out = alpha * op(X) op(Y) with batch broadcasting over the leading dims
void matmul(Ctx& c, const Tensor& x0, const Tensor& y0, bool tx, bool ty, float alpha, Tensor& out) {
  need_f32(x0, "matmul");
  need_f32(y0, "matmul");
  Tensor x = x0, y = y0;
  bool sx_vec = false, sy_vec = false;
  if (x.ndim() == 1) { x = view(x, {1, x.shape[0]}); tx = false; sx_vec = true; }
  if (y.ndim() == 1) { y = view(y, {y.shape[0], 1}); ty = false; sy_vec = true; }
  const int xr = x.ndim(), yr = y.ndim();
  const int64_t M = tx ? x.shape[xr - 1] : x.shape[xr - 2], Kx = tx ? x.shape[xr - 2] : x.shape[xr - 1];
  const int64_t Ky = ty ? y.shape[yr - 1] : y.shape[yr - 2], N = ty ? y.shape[yr - 2] : y.shape[yr - 1];
  if (Kx != Ky) throw Error("matmul: inner dims " + shape_str(x0.shape) + " x " + shape_str(y0.shape));
  std::vector<int64_t> bx(x.shape.begin(), x.shape.end() - 2), by(y.shape.begin(), y.shape.end() - 2);
  const size_t nb = std::max(bx.size(), by.size());
  while (bx.size() < nb) bx.insert(bx.begin(), 1);
  while (by.size() < nb) by.insert(by.begin(), 1);
  std::vector<int64_t> bo(nb);
  int64_t batch = 1;
  for (size_t k = 0; k < nb; ++k) {
    if (bx[k] != by[k] && bx[k] != 1 && by[k] != 1) throw Error("matmul: batch dims do not broadcast");
    bo[k] = std::max(bx[k], by[k]);
    batch *= bo[k];
  }
  // an operand whose batch dims are neither the output's nor all ones is expanded to the output's
  auto batch_stride = [&](Tensor& t, std::vector<int64_t>& bt, int64_t r, int64_t cdim) -> int64_t {
    int64_t prod = 1;
    for (auto v : bt) prod *= v;
    if (prod == 1) return 0;
    if (bt == bo) return r * cdim;
    std::vector<int64_t> shape = bo, st(nb + 2);
    shape.push_back(r);
    shape.push_back(cdim);
    const auto cs = contiguous_strides([&] { auto s = bt; s.push_back(r); s.push_back(cdim); return s; }());
    for (size_t k = 0; k < nb; ++k) st[k] = bt[k] == 1 ? 0 : cs[k];
    st[nb] = cdim;
    st[nb + 1] = 1;
    Tensor e = c.alloc(shape, t.dtype);
    strided_copy(c, t, t.raw(), e, shape, st);
    t = e;
    return r * cdim;
  };
  const int64_t xrows = x.shape[xr - 2], xcols = x.shape[xr - 1], yrows = y.shape[yr - 2], ycols = y.shape[yr - 1];
  GemmArgs g;
  g.sAb = batch_stride(x, bx, xrows, xcols);
  g.sBb = batch_stride(y, by, yrows, ycols);
  std::vector<int64_t> oshape = bo;
  if (!sx_vec) oshape.push_back(M);
  if (!sy_vec) oshape.push_back(N);
  out = c.alloc(oshape);
  g.A = x.data<float>();
  g.B = y.data<float>();
  g.C = out.data<float>();
  g.batch = (int)batch;
  g.M = (int)M; g.N = (int)N; g.K = (int)Kx;
  g.sAm = tx ? 1 : xcols; g.sAk = tx ? xcols : 1;
  g.sBk = ty ? 1 : ycols; g.sBn = ty ? ycols : 1;
  g.sCb = M * N; g.sCm = N;
  g.alpha = alpha;
  gemm(c, g);
}

void op_matmul_v2(Ctx& c, const OpDesc& op) {
  Tensor out;
  matmul(c, c.get(op.in("X")), c.get(op.in("Y")), op.getb("trans_x", false), op.getb("trans_y", false), 1.f, out);
  c.set(op.out("Out"), out);
}

void op_matmul(Ctx& c, const OpDesc& op) {
  Tensor out;
  matmul(c, c.get(op.in("X")), c.get(op.in("Y")), op.getb("transpose_X", false), op.getb("transpose_Y", false),
         (float)op.getf("alpha", 1.0), out);
  c.set(op.out("Out"), out);
}

void op_mul(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  Tensor& y = c.get(op.in("Y"));
  const int xn = (int)op.geti("x_num_col_dims", 1), yn = (int)op.geti("y_num_col_dims", 1);
  int64_t m = 1, k = 1, k2 = 1, n = 1;
  for (int i = 0; i < x.ndim(); ++i) (i < xn ? m : k) *= x.shape[i];
  for (int i = 0; i < y.ndim(); ++i) (i < yn ? k2 : n) *= y.shape[i];
  Tensor out;
  matmul(c, view(x, {m, k}), view(y, {k2, n}), false, false, 1.f, out);
  std::vector<int64_t> os(x.shape.begin(), x.shape.begin() + xn);
  os.insert(os.end(), y.shape.begin() + yn, y.shape.end());
  c.set(op.out("Out"), view(out, os));
}

void op_fc(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("Input"));
  Tensor& w = c.get(op.in("W"));
  need_f32(x, "fc");
  const int nc = (int)op.geti("in_num_col_dims", 1);
  int64_t m = 1, k = 1;
  for (int i = 0; i < x.ndim(); ++i) (i < nc ? m : k) *= x.shape[i];
  if (w.ndim() != 2 || w.shape[0] != k) throw Error("fc: input " + shape_str(x.shape) + " vs W " + shape_str(w.shape));
  const int64_t N = w.shape[1];
  std::vector<int64_t> os(x.shape.begin(), x.shape.begin() + nc);
  os.push_back(N);
  Tensor out = c.alloc(os);
  GemmArgs g;
  g.A = x.data<float>(); g.B = w.data<float>(); g.C = out.data<float>();
  g.bias = c.has(op.in("Bias")) ? c.get(op.in("Bias")).data<float>() : nullptr;
  g.M = (int)m; g.N = (int)N; g.K = (int)k;
  g.sAm = k; g.sAk = 1; g.sBk = N; g.sBn = 1; g.sCm = N;
  g.relu = op.gets("activation_type", "") == "relu";
  gemm(c, g);
  c.set(op.out("Out"), out);
}

// ---- softmax / layer_norm ---------------------------------------------------------------------------
void op_softmax(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  need_f32(x, "softmax");
  int axis = (int)op.geti("axis", -1);
  if (axis < 0) axis += x.ndim();
  int64_t outer = 1, inner = 1;
  for (int k = 0; k < axis; ++k) outer *= x.shape[k];
  for (int k = axis + 1; k < x.ndim(); ++k) inner *= x.shape[k];
  const int64_t n = x.ndim() ? x.shape[axis] : 1;
  Tensor y = c.alloc(x.shape);
  if (c.gpu()) {
    gpu::softmax(x.data<float>(), y.data<float>(), outer, n, inner);
  } else {
    const float* xp = x.data<float>();
    float* yp = y.data<float>();
    parallel_for(outer * inner, [&](int64_t a, int64_t b) {
      for (int64_t r = a; r < b; ++r) {
        const int64_t o = r / inner, in = r % inner;
        const float* px = xp + o * n * inner + in;
        float* py = yp + o * n * inner + in;
        float m = -INFINITY, s = 0.f;
        for (int64_t j = 0; j < n; ++j) m = std::max(m, px[j * inner]);
        for (int64_t j = 0; j < n; ++j) s += std::exp(px[j * inner] - m);
        for (int64_t j = 0; j < n; ++j) py[j * inner] = std::exp(px[j * inner] - m) / s;
      }
    });
  }
  c.set(op.out("Out"), y);
}

void op_layer_norm(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  need_f32(x, "layer_norm");
  const int bna = (int)op.geti("begin_norm_axis", 1);
  int64_t rows = 1, cols = 1;
  for (int k = 0; k < x.ndim(); ++k) (k < bna ? rows : cols) *= x.shape[k];
  const float eps = (float)op.getf("epsilon", 1e-5);
  const float* sc = c.has(op.in("Scale")) ? c.get(op.in("Scale")).data<float>() : nullptr;
  const float* bi = c.has(op.in("Bias")) ? c.get(op.in("Bias")).data<float>() : nullptr;
  Tensor y = c.alloc(x.shape);
  if (c.gpu()) {
    gpu::layer_norm(x.data<float>(), y.data<float>(), sc, bi, rows, cols, eps);
  } else {
    const float* xp = x.data<float>();
    float* yp = y.data<float>();
    parallel_for(rows, [&](int64_t a, int64_t b) {
      for (int64_t r = a; r < b; ++r) {
        const float* px = xp + r * cols;
        float* py = yp + r * cols;
        double mean = 0, var = 0;
        for (int64_t j = 0; j < cols; ++j) mean += px[j];
        mean /= cols;
        for (int64_t j = 0; j < cols; ++j) var += (px[j] - mean) * (px[j] - mean);
        const float inv = 1.f / std::sqrt((float)(var / cols) + eps);
        for (int64_t j = 0; j < cols; ++j) {
          float o = (float)(px[j] - mean) * inv;
          if (sc) o *= sc[j];
          if (bi) o += bi[j];
          py[j] = o;
        }
      }
    });
  }
  c.set(op.out("Y"), y);
}

// ---- embedding / cast / fill / shape ----------------------------------------------------------------
void op_lookup(Ctx& c, const OpDesc& op, bool v1) {
  Tensor& ids = c.get(op.in("Ids"));
  Tensor& w = c.get(op.in("W"));
  if (ids.dtype != I64) throw Error("lookup_table: int64 ids expected");
  const int64_t V = w.shape[0], H = w.shape[1], pad = op.geti("padding_idx", -1);
  std::vector<int64_t> os = ids.shape;
  if (v1 && !os.empty() && os.back() == 1) os.pop_back();
  os.push_back(H);
  Tensor out = c.alloc(os);
  const int64_t n = ids.numel();
  if (c.gpu()) {
    gpu::embedding(ids.data<int64_t>(), w.data<float>(), out.data<float>(), n, H, V, pad);
  } else {
    const int64_t* ip = ids.data<int64_t>();
    const float* wp = w.data<float>();
    float* op_ = out.data<float>();
    for (int64_t r = 0; r < n; ++r) {
      const int64_t id = ip[r];
      if (id == pad || id < 0 || id >= V) std::fill(op_ + r * H, op_ + (r + 1) * H, 0.f);
      else std::memcpy(op_ + r * H, wp + id * H, H * sizeof(float));
    }
  }
  c.set(op.out("Out"), out);
}

void op_cast(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("X"));
  const int od = (int)op.geti("out_dtype", F32);
  Tensor y = c.alloc(x.shape, od);
  if (c.gpu()) {
    gpu::cast(x.raw(), x.dtype, y.raw(), od, x.numel());
  } else {
    auto rd = [&](int64_t i) -> double {
      switch (x.dtype) {
        case F32: return x.data<float>()[i];
        case I64: return (double)x.data<int64_t>()[i];
        case I32: return x.data<int32_t>()[i];
        case F64: return x.data<double>()[i];
        case BOOL: case U8: return x.data<uint8_t>()[i];
      }
      throw Error("cast: unsupported input type");
    };
    for (int64_t i = 0; i < x.numel(); ++i) {
      const double v = rd(i);
      switch (od) {
        case F32: y.data<float>()[i] = (float)v; break;
        case I64: y.data<int64_t>()[i] = (int64_t)v; break;
        case I32: y.data<int32_t>()[i] = (int32_t)v; break;
        case F64: y.data<double>()[i] = v; break;
        case BOOL: case U8: y.data<uint8_t>()[i] = (uint8_t)(v != 0); break;
        default: throw Error("cast: unsupported output type");
      }
    }
  }
  c.set(op.out("Out"), y);
}

void op_fill_constant(Ctx& c, const OpDesc& op) {
  auto shape = op.getints("shape");
  const int dt = (int)op.geti("dtype", F32);
  float v = (float)op.getf("value", 0.0);
  const std::string sv = op.gets("str_value", "");
  if (!sv.empty()) v = std::stof(sv);
  Tensor host = make_tensor(shape, dt, -1);
  for (int64_t i = 0; i < host.numel(); ++i) {
    if (dt == F32) host.data<float>()[i] = v;
    else if (dt == I64) host.data<int64_t>()[i] = (int64_t)v;
    else if (dt == I32) host.data<int32_t>()[i] = (int32_t)v;
    else throw Error("fill_constant: unsupported dtype");
  }
  c.set(op.out("Out"), c.gpu() ? to_device(host, c.dev) : host);
}

void op_shape(Ctx& c, const OpDesc& op) {
  Tensor& x = c.get(op.in("Input"));
  Tensor host = make_tensor({(int64_t)x.ndim()}, I32, -1);
  for (int k = 0; k < x.ndim(); ++k) host.data<int32_t>()[k] = (int32_t)x.shape[k];
  c.set(op.out("Out"), c.gpu() ? to_device(host, c.dev) : host);
}

using OpFn = std::function<void(Ctx&, const OpDesc&)>;

const std::map<std::string, OpFn>& registry() {
  static const std::map<std::string, OpFn> r = [] {
    std::map<std::string, OpFn> m;
    m["conv2d"] = op_conv2d;
    m["depthwise_conv2d"] = op_conv2d;
    m["batch_norm"] = op_batch_norm;
    m["pool2d"] = op_pool2d;
    m["elementwise_add"] = op_elementwise(gpu::ADD);
    m["elementwise_sub"] = op_elementwise(gpu::SUB);
    m["elementwise_mul"] = op_elementwise(gpu::MUL);
    m["elementwise_div"] = op_elementwise(gpu::DIV);
    m["elementwise_max"] = op_elementwise(gpu::MAX);
    m["elementwise_min"] = op_elementwise(gpu::MIN);
    m["elementwise_pow"] = op_elementwise(gpu::POW);
    m["relu"] = op_unary(gpu::RELU, nullptr);
    m["relu6"] = op_unary(gpu::RELU6, [](const OpDesc& o) { return std::pair<float, float>{(float)o.getf("threshold", 6.0), 0.f}; });
    m["sigmoid"] = op_unary(gpu::SIGMOID, nullptr);
    m["tanh"] = op_unary(gpu::TANH, nullptr);
    m["gelu"] = op_unary(gpu::GELU, nullptr);
    m["silu"] = op_unary(gpu::SILU, [](const OpDesc&) { return std::pair<float, float>{1.f, 0.f}; });
    m["swish"] = op_unary(gpu::SILU, [](const OpDesc& o) { return std::pair<float, float>{(float)o.getf("beta", 1.0), 0.f}; });
    m["hard_swish"] = op_unary(gpu::HARD_SWISH, nullptr);
    m["hard_sigmoid"] = op_unary(gpu::HARD_SIGMOID, [](const OpDesc& o) {
      return std::pair<float, float>{(float)o.getf("slope", 0.2), (float)o.getf("offset", 0.5)};
    });
    m["leaky_relu"] = op_unary(gpu::LEAKY_RELU, [](const OpDesc& o) { return std::pair<float, float>{(float)o.getf("alpha", 0.02), 0.f}; });
    m["exp"] = op_unary(gpu::EXP, nullptr);
    m["sqrt"] = op_unary(gpu::SQRT, nullptr);
    m["rsqrt"] = op_unary(gpu::RSQRT, nullptr);
    m["abs"] = op_unary(gpu::ABS, nullptr);
    m["square"] = op_unary(gpu::SQUARE, nullptr);
    m["scale"] = op_scale;
    m["dropout"] = op_dropout;
    m["reshape2"] = op_reshape2;
    m["reshape"] = op_reshape2;
    m["flatten_contiguous_range"] = op_flatten_range;
    m["flatten2"] = op_flatten2;
    m["flatten"] = op_flatten2;
    m["squeeze2"] = op_squeeze2;
    m["unsqueeze2"] = op_unsqueeze2;
    m["assign"] = op_assign;
    m["transpose2"] = op_transpose2;
    m["transpose"] = op_transpose2;
    m["slice"] = op_slice;
    m["concat"] = op_concat;
    m["matmul_v2"] = op_matmul_v2;
    m["matmul"] = op_matmul;
    m["mul"] = op_mul;
    m["fc"] = op_fc;
    m["softmax"] = op_softmax;
    m["layer_norm"] = op_layer_norm;
    m["lookup_table_v2"] = [](Ctx& c, const OpDesc& o) { op_lookup(c, o, false); };
    m["lookup_table"] = [](Ctx& c, const OpDesc& o) { op_lookup(c, o, true); };
    m["cast"] = op_cast;
    m["fill_constant"] = op_fill_constant;
    m["shape"] = op_shape;
    return m;
  }();
  return r;
}
}  // namespace

// ==================================================================== the predictor
struct Predictor {
  Program prog;
  int dev = -1;
  gpu::Context* gctx = nullptr;   // this predictor's device, stream and block pool
  std::map<std::string, Tensor> params;   // persistables, on the device
  std::vector<std::string> in_names, out_names;
  std::map<std::string, Tensor> inputs;   // set_input values (device)
  std::vector<Tensor> outputs;            // last run's fetch values (host)
  std::vector<std::vector<std::string>> release;   // per op: intermediates dead after it
  std::string unsupported;
  std::vector<std::string> applied_passes;

  bool bf16 = false;   // Config.EnableMkldnnBfloat16 (reference AnalysisConfig): bf16 matrix products

  Predictor(const std::string& model_file, const std::string& params_file, int device, bool ir_optim = true,
            bool bf16_ = false)
      : dev(device), bf16(bf16_) {
    prog = parse_program(read_file(model_file));
    if (dev >= 0) gctx = gpu::create_context(dev);
    gpu::Bind bind(gctx);
    Block& b = prog.blocks[0];
    // persistables in name order (save_combine writes them sorted by name), read on the host
    std::vector<std::string> pnames;
    for (auto& v : b.vars)
      if (v.persistable && v.type == 7 && v.name != "feed" && v.name != "fetch") pnames.push_back(v.name);
    std::sort(pnames.begin(), pnames.end());
    std::map<std::string, Tensor> host;
    if (!pnames.empty()) {
      const std::string pb = read_file(params_file);
      size_t off = 0;
      for (auto& n : pnames) host[n] = read_lod_tensor(pb, off);
      if (off != pb.size()) throw Error("params file has trailing bytes (program / params mismatch)");
    }
    if (ir_optim) run_passes(b, host);
    for (auto& kv : host) params[kv.first] = dev >= 0 ? to_device(kv.second, dev) : kv.second;
    std::map<int, std::string> ins, outs;
    std::set<std::string> missing;
    for (auto& op : b.ops) {
      if (op.type == "feed") ins[(int)op.geti("col", 0)] = op.out("Out");
      else if (op.type == "fetch") outs[(int)op.geti("col", 0)] = op.in("X");
      else if (!registry().count(op.type)) missing.insert(op.type);
    }
    for (auto& kv : ins) in_names.push_back(kv.second);
    for (auto& kv : outs) out_names.push_back(kv.second);
    for (auto& m : missing) unsupported += (unsupported.empty() ? "" : ",") + m;
    // liveness: the last op reading each non-persistable value
    std::map<std::string, size_t> last;
    for (size_t i = 0; i < b.ops.size(); ++i)
      for (auto& kv : b.ops[i].inputs)
        for (auto& n : kv.second) last[n] = i;
    std::set<std::string> keep(out_names.begin(), out_names.end());
    release.assign(b.ops.size(), {});
    for (auto& kv : last)
      if (!params.count(kv.first) && !keep.count(kv.first)) release[kv.second].push_back(kv.first);
  }

  ~Predictor() {
    {
      gpu::Bind bind(gctx);
      params.clear();
      inputs.clear();
      outputs.clear();
    }
    gpu::destroy_context(gctx);
  }

  // ---- IR passes on the host copies of the persistables (reference paddle_pass_builder.cc:108:
  // conv_bn_fuse_pass, conv_eltwiseadd_bn_fuse_pass, conv_elementwise_add_fuse_pass) -------------
  static std::map<std::string, int> consumers(const Block& b) {
    std::map<std::string, int> n;
    for (auto& op : b.ops)
      for (auto& kv : op.inputs)
        for (auto& v : kv.second) ++n[v];
    return n;
  }
  static const OpDesc* sole_consumer(const Block& b, const std::string& v, size_t after) {
    const OpDesc* hit = nullptr;
    for (size_t i = after; i < b.ops.size(); ++i)
      for (auto& kv : b.ops[i].inputs)
        for (auto& n : kv.second)
          if (n == v) {
            if (hit) return nullptr;
            hit = &b.ops[i];
          }
    return hit;
  }
  void run_passes(Block& b, std::map<std::string, Tensor>& host) {
    int add_fused = 0, bn_fused = 0;
    auto is_conv = [](const OpDesc& o) { return o.type == "conv2d" || o.type == "depthwise_conv2d"; };
    auto f32_param = [&](const std::string& n) { return host.count(n) && host[n].dtype == F32; };
    for (size_t i = 0; i < b.ops.size(); ++i) {
      OpDesc& conv = b.ops[i];
      if (!is_conv(conv) || conv.gets("data_format", "NCHW") == "NHWC" || !f32_param(conv.in("Filter"))) continue;
      // conv + elementwise_add(per-channel persistable, axis 1) -> conv with Bias
      if (conv.in("Bias").empty()) {
        const OpDesc* add = sole_consumer(b, conv.out("Output"), i + 1);
        if (add && add->type == "elementwise_add" && add->in("X") == conv.out("Output") && add->geti("axis", -1) == 1 &&
            f32_param(add->in("Y")) && host[add->in("Y")].numel() == host[conv.in("Filter")].shape[0]) {
          conv.inputs["Bias"] = {add->in("Y")};
          const std::string out = add->out("Out");
          b.ops.erase(b.ops.begin() + (add - &b.ops[0]));
          conv.outputs["Output"] = {out};
          ++add_fused;
        }
      }
      // conv (+ Bias) + batch_norm (inference statistics) -> conv with folded filter and bias
      const OpDesc* bn = sole_consumer(b, conv.out("Output"), i + 1);
      if (!bn || bn->type != "batch_norm" || bn->in("X") != conv.out("Output")) continue;
      if (!(bn->getb("is_test", false) || bn->getb("use_global_stats", false))) continue;
      if (bn->gets("data_layout", "NCHW") != "NCHW") continue;
      const std::string sn = bn->in("Scale"), bnb = bn->in("Bias"), mn = bn->in("Mean"), vn = bn->in("Variance");
      if (!f32_param(sn) || !f32_param(bnb) || !f32_param(mn) || !f32_param(vn)) continue;
      const Tensor& w = host[conv.in("Filter")];
      const int64_t Co = w.shape[0], per = w.numel() / Co;
      const float eps = (float)bn->getf("epsilon", 1e-5);
      Tensor nw = make_tensor(w.shape, F32, -1), nb = make_tensor({Co}, F32, -1);
      const float* cb = conv.in("Bias").empty() ? nullptr : host[conv.in("Bias")].data<float>();
      for (int64_t c = 0; c < Co; ++c) {
        const float k = host[sn].data<float>()[c] / std::sqrt(host[vn].data<float>()[c] + eps);
        for (int64_t e = 0; e < per; ++e) nw.data<float>()[c * per + e] = w.data<float>()[c * per + e] * k;
        nb.data<float>()[c] = ((cb ? cb[c] : 0.f) - host[mn].data<float>()[c]) * k + host[bnb].data<float>()[c];
      }
      const std::string base = conv.out("Output");
      host[base + "@bn_folded_filter"] = nw;
      host[base + "@bn_folded_bias"] = nb;
      conv.inputs["Filter"] = {base + "@bn_folded_filter"};
      conv.inputs["Bias"] = {base + "@bn_folded_bias"};
      const std::string out = bn->out("Y");
      b.ops.erase(b.ops.begin() + (bn - &b.ops[0]));
      conv.outputs["Output"] = {out};
      ++bn_fused;
    }
    // persistables no op reads any more (the original filters / BN statistics) are dropped
    const auto uses = consumers(b);
    for (auto it = host.begin(); it != host.end();) {
      if (!uses.count(it->first)) it = host.erase(it);
      else ++it;
    }
    if (add_fused) applied_passes.push_back("conv_elementwise_add_fuse_pass x" + std::to_string(add_fused));
    if (bn_fused) applied_passes.push_back("conv_bn_fuse_pass x" + std::to_string(bn_fused));
  }

  void set_input(const std::string& name, const Tensor& host_t) {
    gpu::Bind bind(gctx);
    inputs[name] = dev >= 0 ? to_device(host_t, dev) : host_t;
  }

  void run() {
    if (!unsupported.empty()) throw Error("the program has ops the native engine does not run: " + unsupported);
    gpu::Bind bind(gctx);
    const Block& b = prog.blocks[0];
    std::map<std::string, Tensor> env = params;
    for (auto& n : in_names) {
      auto it = inputs.find(n);
      if (it == inputs.end()) throw Error("input " + n + " was not set");
      env[n] = it->second;
    }
    Ctx c{dev, env, bf16};
    for (size_t i = 0; i < b.ops.size(); ++i) {
      const OpDesc& op = b.ops[i];
      if (op.type == "feed" || op.type == "fetch") continue;
      try {
        registry().at(op.type)(c, op);
      } catch (const std::exception& e) {
        throw Error("op #" + std::to_string(i) + " (" + op.type + "): " + e.what());
      }
      for (auto& n : release[i]) env.erase(n);
    }
    outputs.clear();
    for (auto& n : out_names) outputs.push_back(to_device(c.get(n), -1));
    if (dev >= 0) gpu::sync();
  }
};

}  // namespace pha_infer

// ==================================================================== C APIs
using pha_infer::Error;
using pha_infer::Predictor;
using pha_infer::Tensor;

struct PhaPredictor {
  Predictor* p;
  std::string passes;
};

namespace {
thread_local std::string g_err;

template <typename F>
int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}
}  // namespace

extern "C" {

PhaPredictor* pha_infer_create3(const char* model_file, const char* params_file, int device, int ir_optim,
                                int bf16) {
  PhaPredictor* out = nullptr;
  guard([&] {
    auto* pr = new Predictor(model_file, params_file ? params_file : "", device, ir_optim != 0, bf16 != 0);
    std::string s;
    for (auto& x : pr->applied_passes) s += (s.empty() ? "" : ";") + x;
    out = new PhaPredictor{pr, s};
  });
  return out;
}
PhaPredictor* pha_infer_create2(const char* model_file, const char* params_file, int device, int ir_optim) {
  return pha_infer_create3(model_file, params_file, device, ir_optim, 0);
}
PhaPredictor* pha_infer_create(const char* model_file, const char* params_file, int device) {
  return pha_infer_create2(model_file, params_file, device, 1);
}
const char* pha_infer_applied_passes(const PhaPredictor* p) { return p->passes.c_str(); }
size_t pha_infer_pooled_bytes(const PhaPredictor* p) {
  return p->p->gctx ? pha_infer::gpu::pooled_bytes(p->p->gctx) : 0;
}
const char* pha_infer_last_error(void) { return g_err.c_str(); }
int pha_infer_num_inputs(const PhaPredictor* p) { return (int)p->p->in_names.size(); }
const char* pha_infer_input_name(const PhaPredictor* p, int i) { return p->p->in_names.at(i).c_str(); }
int pha_infer_num_outputs(const PhaPredictor* p) { return (int)p->p->out_names.size(); }
const char* pha_infer_output_name(const PhaPredictor* p, int i) { return p->p->out_names.at(i).c_str(); }
const char* pha_infer_unsupported_ops(const PhaPredictor* p) { return p->p->unsupported.c_str(); }

int pha_infer_set_input(PhaPredictor* p, const char* name, int dtype, const int64_t* shape, int ndim,
                        const void* data) {
  return guard([&] {
    Tensor host = pha_infer::make_tensor(std::vector<int64_t>(shape, shape + ndim), dtype, -1);
    std::memcpy(host.raw(), data, host.bytes());
    p->p->set_input(name, host);
  });
}
int pha_infer_run(PhaPredictor* p) { return guard([&] { p->p->run(); }); }
int pha_infer_output_shape(const PhaPredictor* p, int i, int64_t* shape, int* ndim, int* dtype) {
  return guard([&] {
    const Tensor& t = p->p->outputs.at(i);
    if (t.ndim() > 8) throw Error("output has more than 8 dims");
    for (int k = 0; k < t.ndim(); ++k) shape[k] = t.shape[k];
    *ndim = t.ndim();
    *dtype = t.dtype;
  });
}
int pha_infer_copy_output(const PhaPredictor* p, int i, void* dst, size_t bytes) {
  return guard([&] {
    const Tensor& t = p->p->outputs.at(i);
    if (bytes < t.bytes()) throw Error("output buffer too small");
    std::memcpy(dst, t.raw(), t.bytes());
  });
}
void pha_infer_destroy(PhaPredictor* p) {
  if (!p) return;
  delete p->p;
  delete p;
}

// ---- reference C API subset ---------------------------------------------------------------------
struct PD_Config {
  std::string prog, params;
  bool gpu = false;
  int dev = 0;
  bool ir_optim = true;
  bool bf16 = false;
};
struct PD_Predictor {
  PhaPredictor* p;
};
struct PD_Tensor {
  PD_Predictor* owner;
  std::string name;
  bool input;
  std::vector<int64_t> shape;
};

PD_Config* PD_ConfigCreate(void) { return new PD_Config(); }
void PD_ConfigSwitchIrOptim(PD_Config* c, PD_Bool x) { c->ir_optim = x != 0; }
PD_Bool PD_ConfigIrOptim(PD_Config* c) { return c->ir_optim; }
// reference: AnalysisConfig::EnableMkldnnBfloat16 — here the GPU device path's matrix products
// (mul / matmul / fc / convolutions) run with bf16 operands on the MFMA GEMM of libpha_kernels.so
void PD_ConfigEnableMkldnnBfloat16(PD_Config* c) { c->bf16 = true; }
PD_Bool PD_ConfigMkldnnBfloat16Enabled(PD_Config* c) { return c->bf16; }
void PD_ConfigDestroy(PD_Config* c) { delete c; }
void PD_ConfigSetModel(PD_Config* c, const char* prog, const char* params) {
  c->prog = prog;
  c->params = params ? params : "";
}
const char* PD_ConfigGetProgFile(PD_Config* c) { return c->prog.c_str(); }
const char* PD_ConfigGetParamsFile(PD_Config* c) { return c->params.c_str(); }
void PD_ConfigEnableUseGpu(PD_Config* c, uint64_t, int32_t device_id) {
  c->gpu = true;
  c->dev = device_id;
}
void PD_ConfigDisableGpu(PD_Config* c) { c->gpu = false; }
PD_Bool PD_ConfigUseGpu(PD_Config* c) { return c->gpu; }
int32_t PD_ConfigGpuDeviceId(PD_Config* c) { return c->dev; }

PD_Predictor* PD_PredictorCreate(PD_Config* c) {
  PhaPredictor* p = pha_infer_create3(c->prog.c_str(), c->params.c_str(), c->gpu ? c->dev : -1, c->ir_optim, c->bf16);
  delete c;
  if (!p) {
    std::fprintf(stderr, "PD_PredictorCreate: %s\n", g_err.c_str());
    return nullptr;
  }
  return new PD_Predictor{p};
}
void PD_PredictorDestroy(PD_Predictor* p) {
  if (!p) return;
  pha_infer_destroy(p->p);
  delete p;
}
size_t PD_PredictorGetInputNum(PD_Predictor* p) { return p->p->p->in_names.size(); }
size_t PD_PredictorGetOutputNum(PD_Predictor* p) { return p->p->p->out_names.size(); }

static PD_OneDimArrayCstr* cstr_array(const std::vector<std::string>& v) {
  auto* a = new PD_OneDimArrayCstr{v.size(), new char*[v.size()]};
  for (size_t i = 0; i < v.size(); ++i) {
    a->data[i] = new char[v[i].size() + 1];
    std::memcpy(a->data[i], v[i].c_str(), v[i].size() + 1);
  }
  return a;
}
PD_OneDimArrayCstr* PD_PredictorGetInputNames(PD_Predictor* p) { return cstr_array(p->p->p->in_names); }
PD_OneDimArrayCstr* PD_PredictorGetOutputNames(PD_Predictor* p) { return cstr_array(p->p->p->out_names); }
void PD_OneDimArrayCstrDestroy(PD_OneDimArrayCstr* a) {
  if (!a) return;
  for (size_t i = 0; i < a->size; ++i) delete[] a->data[i];
  delete[] a->data;
  delete a;
}
void PD_OneDimArrayInt32Destroy(PD_OneDimArrayInt32* a) {
  if (!a) return;
  delete[] a->data;
  delete a;
}
PD_Tensor* PD_PredictorGetInputHandle(PD_Predictor* p, const char* name) { return new PD_Tensor{p, name, true, {}}; }
PD_Tensor* PD_PredictorGetOutputHandle(PD_Predictor* p, const char* name) { return new PD_Tensor{p, name, false, {}}; }
PD_Bool PD_PredictorRun(PD_Predictor* p) {
  if (pha_infer_run(p->p) != 0) {
    std::fprintf(stderr, "PD_PredictorRun: %s\n", g_err.c_str());
    return 0;
  }
  return 1;
}
void PD_TensorDestroy(PD_Tensor* t) { delete t; }
void PD_TensorReshape(PD_Tensor* t, size_t n, int32_t* shape) { t->shape.assign(shape, shape + n); }
static void copy_from(PD_Tensor* t, int dt, const void* data) {
  if (pha_infer_set_input(t->owner->p, t->name.c_str(), dt, t->shape.data(), (int)t->shape.size(), data) != 0)
    std::fprintf(stderr, "PD_TensorCopyFromCpu: %s\n", g_err.c_str());
}
void PD_TensorCopyFromCpuFloat(PD_Tensor* t, const float* d) { copy_from(t, PHA_FLOAT32, d); }
void PD_TensorCopyFromCpuInt64(PD_Tensor* t, const int64_t* d) { copy_from(t, PHA_INT64, d); }
void PD_TensorCopyFromCpuInt32(PD_Tensor* t, const int32_t* d) { copy_from(t, PHA_INT32, d); }
static const Tensor* out_tensor(PD_Tensor* t) {
  const auto& names = t->owner->p->p->out_names;
  for (size_t i = 0; i < names.size(); ++i)
    if (names[i] == t->name && i < t->owner->p->p->outputs.size()) return &t->owner->p->p->outputs[i];
  return nullptr;
}
static void copy_to(PD_Tensor* t, int dt, void* d) {
  const Tensor* o = out_tensor(t);
  if (!o || o->dtype != dt) {
    std::fprintf(stderr, "PD_TensorCopyToCpu: no output %s of that type\n", t->name.c_str());
    return;
  }
  std::memcpy(d, o->raw(), o->bytes());
}
void PD_TensorCopyToCpuFloat(PD_Tensor* t, float* d) { copy_to(t, PHA_FLOAT32, d); }
void PD_TensorCopyToCpuInt64(PD_Tensor* t, int64_t* d) { copy_to(t, PHA_INT64, d); }
void PD_TensorCopyToCpuInt32(PD_Tensor* t, int32_t* d) { copy_to(t, PHA_INT32, d); }
PD_OneDimArrayInt32* PD_TensorGetShape(PD_Tensor* t) {
  std::vector<int64_t> s = t->shape;
  if (!t->input) {
    const Tensor* o = out_tensor(t);
    if (o) s = o->shape;
  }
  auto* a = new PD_OneDimArrayInt32{s.size(), new int32_t[s.size() ? s.size() : 1]};
  for (size_t i = 0; i < s.size(); ++i) a->data[i] = (int32_t)s[i];
  return a;
}
const char* PD_TensorGetName(PD_Tensor* t) { return t->name.c_str(); }

}  // extern "C"
