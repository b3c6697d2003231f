// Internal types of the native inference engine (see pha_infer.h).
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

namespace pha_infer {

// ---- ProgramDesc (framework.proto subset the engine reads) -------------------------------------
struct Attr {
  int type = -1;   // AttrType: 0 INT 1 FLOAT 2 STRING 3 INTS 4 FLOATS 5 STRINGS 6 BOOLEAN 7 BOOLEANS
                   // 8 BLOCK 9 LONG 10 BLOCKS 11 LONGS 12 FLOAT64S
  int64_t i = 0;
  float f = 0.f;
  bool b = false;
  std::string s;
  std::vector<int64_t> ints;   // INTS, LONGS, BOOLEANS, BLOCKS
  std::vector<double> floats;  // FLOATS, FLOAT64S
  std::vector<std::string> strings;
};

struct OpDesc {
  std::string type;
  std::map<std::string, std::vector<std::string>> inputs, outputs;
  std::map<std::string, Attr> attrs;

  bool has(const std::string& k) const { return attrs.count(k) != 0; }
  int64_t geti(const std::string& k, int64_t d) const;
  double getf(const std::string& k, double d) const;
  bool getb(const std::string& k, bool d) const;
  std::string gets(const std::string& k, const std::string& d) const;
  std::vector<int64_t> getints(const std::string& k, std::vector<int64_t> d = {}) const;
  // the first argument of a slot ("" when absent)
  std::string in(const std::string& slot) const;
  std::string out(const std::string& slot) const;
};

struct VarDesc {
  std::string name;
  int type = 7;    // VarType.Type of the variable (7 LOD_TENSOR, 9 FEED_MINIBATCH, 10 FETCH_LIST)
  int dtype = 5;   // element type of a LOD_TENSOR
  std::vector<int64_t> dims;
  bool persistable = false;
};

struct Block {
  std::vector<VarDesc> vars;
  std::vector<OpDesc> ops;
};

struct Program {
  std::vector<Block> blocks;
};

Program parse_program(const std::string& bytes);

// ---- tensors ------------------------------------------------------------------------------------
enum DType { BOOL = 0, I16 = 1, I32 = 2, I64 = 3, F16 = 4, F32 = 5, F64 = 6, U8 = 20, I8 = 21 };
size_t dtype_size(int dt);

namespace gpu {
struct Context;
}

struct Buffer {
  void* p = nullptr;
  size_t n = 0;
  int dev = -1;   // -1 host
  gpu::Context* ctx = nullptr;   // device blocks: the pool they return to
  Buffer(size_t bytes, int dev);
  ~Buffer();
  Buffer(const Buffer&) = delete;
  Buffer& operator=(const Buffer&) = delete;
};

struct Tensor {
  std::vector<int64_t> shape;
  int dtype = F32;
  std::shared_ptr<Buffer> buf;
  size_t offset = 0;   // bytes into buf (views)

  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
  size_t bytes() const { return (size_t)numel() * dtype_size(dtype); }
  int ndim() const { return (int)shape.size(); }
  template <typename T>
  T* data() const { return reinterpret_cast<T*>(static_cast<char*>(buf->p) + offset); }
  void* raw() const { return static_cast<char*>(buf->p) + offset; }
};

Tensor make_tensor(std::vector<int64_t> shape, int dtype, int dev);
Tensor to_device(const Tensor& t, int dev);   // copy (host <-> device), same shape / dtype

struct Error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

// ---- GPU entry points (gpu.hip). All fp32 unless noted; stream = the engine's stream. ------------
namespace gpu {
// a predictor's device, stream and block pool; GPU calls run on the context bound to the thread
Context* create_context(int dev);
void destroy_context(Context* c);
struct Bind {   // RAII: hipSetDevice(c->dev) + bind c to this thread; restores both on exit
  explicit Bind(Context* c);
  ~Bind();
  Bind(const Bind&) = delete;
  Bind& operator=(const Bind&) = delete;
  void* prev_ctx;
  Context* ctx;
  int prev_dev = 0;
};
Context* current();
size_t pooled_bytes(Context* c);
void* stream();
void sync();
void* alloc(size_t n);                       // from the bound context's pool
void release(Context* c, void* p, size_t n); // back to c's pool
void h2d(void* dst, const void* src, size_t n);
void d2h(void* dst, const void* src, size_t n);
void d2d(void* dst, const void* src, size_t n);

// C[b] (M x N) = alpha * A[b] (M x K) . B[b] (K x N) (+ bias[n]) (relu); element (m, k) of A at
// A + b * sAb + m * sAm + k * sAk (likewise B, C: sCm row stride, unit column stride)
void gemm(const float* A, const float* B, float* C, const float* bias, int batch, int M, int N, int K,
          int64_t sAb, int64_t sAm, int64_t sAk, int64_t sBb, int64_t sBk, int64_t sBn, int64_t sCb, int64_t sCm,
          float alpha, bool relu);
// the same product with bf16 operands on the kernel library's persistent MFMA GEMM (libpha_kernels.so
// pha_gemm4p_batched, resolved next to this library): A / B converted to zero-padded bf16 images
// (B as B^T [N][K], the NT layout), fp32 accumulation, bf16 result widened into C with alpha / bias
// / ReLU. Returns false (nothing done) when the kernel library cannot be loaded.
bool gemm_bf16(const float* A, const float* B, float* C, const float* bias, int batch, int M, int N, int K,
               int64_t sAb, int64_t sAm, int64_t sAk, int64_t sBb, int64_t sBk, int64_t sBn, int64_t sCb,
               int64_t sCm, float alpha, bool relu);
// col [N][C*KH*KW][OH*OW] of N NCHW images
void im2col(const float* x, float* col, int C, int H, int W, int KH, int KW, int OH, int OW, int sh, int sw, int pt,
            int pl, int dh, int dw, int N);
// y[b][r][i] += bias[r] (then ReLU) over batch x rows x inner
void row_bias_act(float* y, const float* bias, int64_t rows, int64_t inner, int64_t batch, bool relu);
void depthwise_conv(const float* x, const float* w, float* y, int N, int C, int H, int W, int KH, int KW, int OH,
                    int OW, int sh, int sw, int pt, int pl, int dh, int dw, int mult);
enum Unary { RELU, RELU6, SIGMOID, TANH, GELU, GELU_TANH, SILU, HARD_SWISH, HARD_SIGMOID, LEAKY_RELU, EXP, SQRT,
             ABS, SCALE, SQUARE, RSQRT };
void unary(const float* x, float* y, int64_t n, int op, float a, float b);
enum Binary { ADD, SUB, MUL, DIV, MAX, MIN, POW };
// out[i] = x[ix] op y[iy] over an up-to-8-dim output; strides of x / y per output dim (0: broadcast)
void binary(const float* x, const float* y, float* out, int op, int nd, const int64_t* shape, const int64_t* sx,
            const int64_t* sy);
void batch_norm(const float* x, float* y, const float* scale, const float* bias, const float* mean,
                const float* var, float eps, int64_t N, int64_t C, int64_t inner);
void pool2d(const float* x, float* y, int N, int C, int H, int W, int OH, int OW, int KH, int KW, int sh, int sw,
            int pt, int pl, bool maxp, bool exclusive, bool adaptive);
// out = in viewed with per-dim element strides (permute / slice / broadcast), nd <= 8, any dtype size
void strided_copy(const void* in, void* out, int esize, int nd, const int64_t* shape, const int64_t* strides);
void softmax(const float* x, float* y, int64_t outer, int64_t n, int64_t inner);
void layer_norm(const float* x, float* y, const float* scale, const float* bias, int64_t rows, int64_t cols,
                float eps);
void embedding(const int64_t* ids, const float* w, float* out, int64_t n, int64_t H, int64_t V, int64_t pad);
void cast(const void* x, int xdt, void* y, int ydt, int64_t n);
void fill(float* y, int64_t n, float v);
}  // namespace gpu

}  // namespace pha_infer
