// GPU kernels of the native inference engine (gfx950). fp32 end to end, so a predictor matches
// the host path to fp32 rounding: the matrix products run on the fp32 matrix cores
// (v_mfma_f32_16x16x4_f32, 64 x 64 tiles of four 32 x 32 wave tiles staged through LDS); the
// rest are one-pass grid-stride kernels. Reference: the phi GPU kernels the reference's
// AnalysisPredictor dispatches (conv2d via cuDNN, matmul via cuBLAS, batch_norm / pool2d /
// softmax / layer_norm / elementwise in phi/kernels/gpu).
#include <hip/hip_runtime.h>

#include <dlfcn.h>

#include <cmath>
#include <cstdio>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "engine.h"

namespace pha_infer {
namespace gpu {

// Per-predictor device context: device id, its own non-blocking stream and a caching pool of
// device blocks (exact-size free lists, rounded to 256 B). Every entry point below runs on the
// context bound to the calling thread (``Bind``), so two predictors on different devices, or a
// predictor driven from a thread whose current HIP device was changed by someone else, each use
// their own device and stream (reference: Config.EnableUseGpu(mem, dev_id) per predictor, the
// pooled allocator of analysis_predictor.cc:398-406).
struct Context {
  int dev = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::map<size_t, std::vector<void*>> free_blocks;
  std::vector<void*> all_blocks;
  size_t pooled_bytes = 0;
};

namespace {
thread_local Context* tl_ctx = nullptr;

void ck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw Error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}
void ck_launch(const char* what) { ck(hipGetLastError(), what); }

unsigned blocks_for(int64_t n, int per = 256) {
  int64_t b = (n + per - 1) / per;
  return (unsigned)(b < 1 ? 1 : (b > 65535 * 16 ? 65535 * 16 : b));
}

typedef float f4 __attribute__((ext_vector_type(4)));

// ---- fp32 MFMA GEMM -----------------------------------------------------------------------------
constexpr int BM = 64, BN = 64, BK = 16, PAD = 4;

__global__ __launch_bounds__(256) void gemm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                   float* __restrict__ C, const float* __restrict__ bias, int M,
                                                   int N, int K, int64_t sAb, int64_t sAm, int64_t sAk, int64_t sBb,
                                                   int64_t sBk, int64_t sBn, int64_t sCb, int64_t sCm, float alpha,
                                                   int relu) {
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int64_t b = blockIdx.z;
  A += b * sAb;
  B += b * sBb;
  C += b * sCb;
  const bool a_kfast = sAk == 1, b_nfast = sBn == 1;
  f4 acc[2][2];
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < K; k0 += BK) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int e = tid + 256 * r;
      int m, k;
      if (a_kfast) { m = e >> 4; k = e & 15; } else { m = e & 63; k = e >> 6; }
      const int gm = m0 + m, gk = k0 + k;
      As[k][m] = (gm < M && gk < K) ? A[gm * sAm + gk * sAk] : 0.f;
      int n, kb;
      if (b_nfast) { n = e & 63; kb = e >> 6; } else { n = e >> 4; kb = e & 15; }
      const int gn = n0 + n, gkb = k0 + kb;
      Bs[kb][n] = (gn < N && gkb < K) ? B[gkb * sBk + gn * sBn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 4) {
      const int kr = kk + (lane >> 4), c = lane & 15;
      float a0 = As[kr][wm * 32 + c], a1 = As[kr][wm * 32 + 16 + c];
      float b0 = Bs[kr][wn * 32 + c], b1 = Bs[kr][wn * 32 + 16 + c];
      acc[0][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    __syncthreads();
  }
  // D[i][j]: column j = lane % 16, rows 4 * (lane / 16) + r
  for (int mi = 0; mi < 2; ++mi)
    for (int ni = 0; ni < 2; ++ni)
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 32 + mi * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 32 + ni * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = alpha * acc[mi][ni][r];
          if (bias) v += bias[n];
          if (relu) v = v > 0.f ? v : 0.f;
          C[m * sCm + n] = v;
        }
      }
}

// 128 x 128 x 16 fp32 MFMA GEMM: 4 waves (2 x 2) of 64 x 64, 16 accumulators per wave; the next
// K-tile is loaded into registers (16-B loads along the contiguous dimension when the layout
// allows) while the current one multiplies, then written to the other LDS buffer: one barrier per
// K-tile. LDS rows are padded to 144 floats so the four 16-lane rows of a fragment read hit four
// disjoint bank groups.
constexpr int TB = 128, TK = 16, TPAD = 16;

template <bool AV, bool BV>
__global__ __launch_bounds__(256) void gemm128_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                      float* __restrict__ C, const float* __restrict__ bias, int M,
                                                      int N, int K, int64_t sAb, int64_t sAm, int64_t sAk,
                                                      int64_t sBb, int64_t sBk, int64_t sBn, int64_t sCb,
                                                      int64_t sCm, float alpha, int relu) {
  __shared__ float As[2][TK][TB + TPAD];
  __shared__ float Bs[2][TK][TB + TPAD];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int m0 = blockIdx.y * TB, n0 = blockIdx.x * TB;
  const int64_t bz = blockIdx.z;
  A += bz * sAb;
  B += bz * sBb;
  C += bz * sCb;
  // per-thread staging registers: 8 A values and 8 B values per K-tile
  float ra[8], rb[8];
  auto load = [&](int k0) {
    if constexpr (AV) {   // A[m][k] with k contiguous: thread -> (row m, 4-wide k chunk), 2 passes
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int e = tid + 256 * r, m = e >> 2, kq = (e & 3) * 4;
        const int gm = m0 + m, gk = k0 + kq;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (gm < M && gk < K) v = *reinterpret_cast<const f4*>(A + gm * sAm + gk);
        ra[4 * r] = v[0]; ra[4 * r + 1] = v[1]; ra[4 * r + 2] = v[2]; ra[4 * r + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = tid + 256 * r;
        int m, k;
        if (sAk == 1) { m = e >> 4; k = e & 15; } else { m = e & 127; k = e >> 7; }
        const int gm = m0 + m, gk = k0 + k;
        ra[r] = (gm < M && gk < K) ? A[gm * sAm + gk * sAk] : 0.f;
      }
    }
    if constexpr (BV) {   // B[k][n] with n contiguous: thread -> (k row, 4-wide n chunk), 2 passes
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int e = tid + 256 * r, k = e >> 5, nq = (e & 31) * 4;
        const int gk = k0 + k, gn = n0 + nq;
        f4 v = {0.f, 0.f, 0.f, 0.f};
        if (gk < K && gn < N) v = *reinterpret_cast<const f4*>(B + gk * sBk + gn);
        rb[4 * r] = v[0]; rb[4 * r + 1] = v[1]; rb[4 * r + 2] = v[2]; rb[4 * r + 3] = v[3];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = tid + 256 * r;
        int n, k;
        if (sBn == 1) { n = e & 127; k = e >> 7; } else { n = e >> 4; k = e & 15; }
        const int gn = n0 + n, gk = k0 + k;
        rb[r] = (gn < N && gk < K) ? B[gk * sBk + gn * sBn] : 0.f;
      }
    }
  };
  auto store = [&](int buf) {
    if constexpr (AV) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int e = tid + 256 * r, m = e >> 2, kq = (e & 3) * 4;
#pragma unroll
        for (int q = 0; q < 4; ++q) As[buf][kq + q][m] = ra[4 * r + q];
      }
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = tid + 256 * r;
        int m, k;
        if (sAk == 1) { m = e >> 4; k = e & 15; } else { m = e & 127; k = e >> 7; }
        As[buf][k][m] = ra[r];
      }
    }
    if constexpr (BV) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int e = tid + 256 * r, k = e >> 5, nq = (e & 31) * 4;
        *reinterpret_cast<f4*>(&Bs[buf][k][nq]) = f4{rb[4 * r], rb[4 * r + 1], rb[4 * r + 2], rb[4 * r + 3]};
      }
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int e = tid + 256 * r;
        int n, k;
        if (sBn == 1) { n = e & 127; k = e >> 7; } else { n = e >> 4; k = e & 15; }
        Bs[buf][k][n] = rb[r];
      }
    }
  };
  f4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < K; k0 += TK) {
    const bool more = k0 + TK < K;
    if (more) load(k0 + TK);
#pragma unroll
    for (int kk = 0; kk < TK; kk += 4) {
      const int kr = kk + (lane >> 4), c = lane & 15;
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[cur][kr][wm * 64 + i * 16 + c];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[cur][kr][wn * 64 + j * 16 + c];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }
  // D[i][j]: column = lane % 16, rows 4 * (lane / 16) + r
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * 64 + i * 16 + 4 * (lane >> 4) + r;
        const int n = n0 + wn * 64 + j * 16 + (lane & 15);
        if (m < M && n < N) {
          float v = alpha * acc[i][j][r];
          if (bias) v += bias[n];
          if (relu) v = v > 0.f ? v : 0.f;
          C[m * sCm + n] = v;
        }
      }
}

// bias along the GEMM's rows (conv: one value per output channel = row)
__global__ void row_bias_act_kernel(float* __restrict__ y, const float* __restrict__ bias, int64_t rows,
                                    int64_t inner, int64_t batch, int relu) {
  const int64_t total = batch * rows * inner;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    float v = y[i] + (bias ? bias[(i / inner) % rows] : 0.f);
    y[i] = relu && v < 0.f ? 0.f : v;
  }
}

__global__ void im2col_kernel(const float* __restrict__ x, float* __restrict__ col, int C, int H, int W, int KH,
                              int KW, int OH, int OW, int sh, int sw, int pt, int pl, int dh, int dw, int N) {
  // col[n][c * KH * KW + kh * KW + kw][oh * OW + ow] for every image n of the batch
  const int64_t per = (int64_t)C * KH * KW * OH * OW, total = per * N;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ow = i % OW;
    int64_t t = i / OW;
    const int oh = t % OH;
    t /= OH;
    const int kw = t % KW;
    t /= KW;
    const int kh = t % KH;
    t /= KH;
    const int c = (int)(t % C);
    const int64_t n = t / C;
    const int ih = oh * sh - pt + kh * dh, iw = ow * sw - pl + kw * dw;
    col[i] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? x[((n * C + c) * H + ih) * W + iw] : 0.f;
  }
}

__global__ void dwconv_kernel(const float* __restrict__ x, const float* __restrict__ w, float* __restrict__ y, int N,
                              int C, int H, int W, int KH, int KW, int OH, int OW, int sh, int sw, int pt, int pl,
                              int dh, int dw, int mult) {
  const int Co = C * mult;
  const int64_t total = (int64_t)N * Co * OH * OW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ow = i % OW;
    int64_t t = i / OW;
    const int oh = t % OH;
    t /= OH;
    const int co = t % Co;
    const int n = (int)(t / Co);
    const int c = co / mult;
    float s = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int ih = oh * sh - pt + kh * dh;
      if (ih < 0 || ih >= H) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int iw = ow * sw - pl + kw * dw;
        if (iw < 0 || iw >= W) continue;
        s += x[(((int64_t)n * C + c) * H + ih) * W + iw] * w[((int64_t)co * KH + kh) * KW + kw];
      }
    }
    y[i] = s;
  }
}

__device__ __forceinline__ float apply_unary(float v, int op, float a, float b) {
  switch (op) {
    case RELU: return v > 0.f ? v : 0.f;
    case RELU6: return fminf(fmaxf(v, 0.f), a);
    case SIGMOID: return 1.f / (1.f + expf(-v));
    case TANH: return tanhf(v);
    case GELU: return 0.5f * v * (1.f + erff(v * 0.70710678118654752f));
    case GELU_TANH: return 0.5f * v * (1.f + tanhf(0.7978845608028654f * (v + 0.044715f * v * v * v)));
    case SILU: return v / (1.f + expf(-a * v));
    case HARD_SWISH: return v * fminf(fmaxf(v + 3.f, 0.f), 6.f) / 6.f;
    case HARD_SIGMOID: return fminf(fmaxf(a * v + b, 0.f), 1.f);
    case LEAKY_RELU: return v > 0.f ? v : a * v;
    case EXP: return expf(v);
    case SQRT: return sqrtf(v);
    case ABS: return fabsf(v);
    case SCALE: return a * v + b;
    case SQUARE: return v * v;
    case RSQRT: return rsqrtf(v);
  }
  return v;
}

__global__ void unary_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int op, float a, float b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = apply_unary(x[i], op, a, b);
}

struct Dims8 {
  int64_t shape[8], sx[8], sy[8];
};

__global__ void binary_kernel(const float* __restrict__ x, const float* __restrict__ y, float* __restrict__ out,
                              int op, int nd, Dims8 d, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t rem = i, ox = 0, oy = 0;
    for (int k = nd - 1; k >= 0; --k) {
      const int64_t c = rem % d.shape[k];
      rem /= d.shape[k];
      ox += c * d.sx[k];
      oy += c * d.sy[k];
    }
    const float a = x[ox], b = y[oy];
    float v;
    switch (op) {
      case ADD: v = a + b; break;
      case SUB: v = a - b; break;
      case MUL: v = a * b; break;
      case DIV: v = a / b; break;
      case MAX: v = fmaxf(a, b); break;
      case MIN: v = fminf(a, b); break;
      default: v = powf(a, b); break;
    }
    out[i] = v;
  }
}

__global__ void bn_kernel(const float* __restrict__ x, float* __restrict__ y, const float* __restrict__ scale,
                          const float* __restrict__ bias, const float* __restrict__ mean,
                          const float* __restrict__ var, float eps, int64_t C, int64_t inner, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = (i / inner) % C;
    const float inv = rsqrtf(var[c] + eps);
    y[i] = (x[i] - mean[c]) * inv * scale[c] + bias[c];
  }
}

__global__ void pool_kernel(const float* __restrict__ x, float* __restrict__ y, int N, int C, int H, int W, int OH,
                            int OW, int KH, int KW, int sh, int sw, int pt, int pl, int maxp, int exclusive,
                            int adaptive) {
  const int64_t total = (int64_t)N * C * OH * OW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int ow = i % OW;
    int64_t t = i / OW;
    const int oh = t % OH;
    const int64_t nc = t / OH;
    int h0, h1, w0, w1;
    if (adaptive) {
      h0 = (oh * H) / OH;
      h1 = ((oh + 1) * H + OH - 1) / OH;
      w0 = (ow * W) / OW;
      w1 = ((ow + 1) * W + OW - 1) / OW;
    } else {
      h0 = oh * sh - pt;
      w0 = ow * sw - pl;
      h1 = h0 + KH;
      w1 = w0 + KW;
    }
    const int ch0 = h0 < 0 ? 0 : h0, cw0 = w0 < 0 ? 0 : w0;
    const int ch1 = h1 > H ? H : h1, cw1 = w1 > W ? W : w1;
    const float* p = x + nc * H * W;
    float acc = maxp ? -INFINITY : 0.f;
    for (int h = ch0; h < ch1; ++h)
      for (int w = cw0; w < cw1; ++w) {
        const float v = p[h * W + w];
        acc = maxp ? fmaxf(acc, v) : acc + v;
      }
    if (!maxp) {
      const int cnt = (exclusive || adaptive) ? (ch1 - ch0) * (cw1 - cw0) : KH * KW;
      acc = cnt > 0 ? acc / cnt : 0.f;
    }
    y[i] = acc;
  }
}

template <typename E>
__global__ void strided_kernel(const E* __restrict__ in, E* __restrict__ out, int nd, Dims8 d, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t rem = i, off = 0;
    for (int k = nd - 1; k >= 0; --k) {
      off += (rem % d.shape[k]) * d.sx[k];
      rem /= d.shape[k];
    }
    out[i] = in[off];
  }
}

// one 256-thread block per row of `n` elements (stride `inner` between them)
__global__ __launch_bounds__(256) void softmax_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n,
                                                      int64_t inner) {
  __shared__ float red[256];
  const int64_t row = blockIdx.x;
  const int64_t o = row / inner, in = row % inner;
  const float* px = x + o * n * inner + in;
  float* py = y + o * n * inner + in;
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < n; j += 256) m = fmaxf(m, px[j * inner]);
  red[threadIdx.x] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  m = red[0];
  __syncthreads();
  float sum = 0.f;
  for (int64_t j = threadIdx.x; j < n; j += 256) sum += expf(px[j * inner] - m);
  red[threadIdx.x] = sum;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  const float inv = 1.f / red[0];
  for (int64_t j = threadIdx.x; j < n; j += 256) py[j * inner] = expf(px[j * inner] - m) * inv;
}

__global__ __launch_bounds__(256) void layer_norm_kernel(const float* __restrict__ x, float* __restrict__ y,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ bias, int64_t cols, float eps) {
  __shared__ float r1[256], r2[256];
  const float* px = x + blockIdx.x * cols;
  float* py = y + blockIdx.x * cols;
  float s = 0.f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) s += px[j];
  r1[threadIdx.x] = s;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) r1[threadIdx.x] += r1[threadIdx.x + k];
    __syncthreads();
  }
  const float mean = r1[0] / cols;
  float v = 0.f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) {
    const float d = px[j] - mean;
    v += d * d;
  }
  r2[threadIdx.x] = v;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) r2[threadIdx.x] += r2[threadIdx.x + k];
    __syncthreads();
  }
  const float inv = rsqrtf(r2[0] / cols + eps);
  for (int64_t j = threadIdx.x; j < cols; j += 256) {
    float o = (px[j] - mean) * inv;
    if (scale) o *= scale[j];
    if (bias) o += bias[j];
    py[j] = o;
  }
}

__global__ void embedding_kernel(const int64_t* __restrict__ ids, const float* __restrict__ w, float* __restrict__ out,
                                 int64_t n, int64_t H, int64_t V, int64_t pad) {
  const int64_t total = n * H;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / H, h = i % H;
    const int64_t id = ids[r];
    out[i] = (id == pad || id < 0 || id >= V) ? 0.f : w[id * H + h];
  }
}

template <typename X, typename Y>
__global__ void cast_kernel(const X* __restrict__ x, Y* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (Y)x[i];
}

__global__ void fill_kernel(float* y, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) y[i] = v;
}

Dims8 dims(int nd, const int64_t* shape, const int64_t* sx, const int64_t* sy) {
  if (nd > 8) throw Error("more than 8 dims");
  Dims8 d{};
  for (int k = 0; k < nd; ++k) {
    d.shape[k] = shape[k];
    d.sx[k] = sx[k];
    d.sy[k] = sy ? sy[k] : 0;
  }
  return d;
}
}  // namespace

Context* create_context(int dev) {
  ck(hipSetDevice(dev), "hipSetDevice");
  auto* c = new Context();
  c->dev = dev;
  ck(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
  return c;
}
void destroy_context(Context* c) {
  if (!c) return;
  int prev = 0;
  (void)hipGetDevice(&prev);
  (void)hipSetDevice(c->dev);
  (void)hipStreamSynchronize(c->stream);
  for (void* p : c->all_blocks) (void)hipFree(p);
  (void)hipStreamDestroy(c->stream);
  (void)hipSetDevice(prev);
  delete c;
}
Bind::Bind(Context* c) : prev_ctx(tl_ctx), ctx(c) {
  if (!c) return;
  (void)hipGetDevice(&prev_dev);
  ck(hipSetDevice(c->dev), "hipSetDevice");
  tl_ctx = c;
}
Bind::~Bind() {
  if (!ctx) return;
  tl_ctx = static_cast<Context*>(prev_ctx);
  (void)hipSetDevice(prev_dev);
}
Context* current() {
  if (!tl_ctx) throw Error("native engine: GPU call outside a predictor's device context");
  return tl_ctx;
}
static hipStream_t cur_stream() { return current()->stream; }
void* stream() { return cur_stream(); }
void sync() { ck(hipStreamSynchronize(cur_stream()), "hipStreamSynchronize"); }
void* alloc(size_t n) {
  Context* c = current();
  const size_t sz = ((n ? n : 16) + 255) & ~(size_t)255;
  {
    std::lock_guard<std::mutex> g(c->mu);
    auto it = c->free_blocks.find(sz);
    if (it != c->free_blocks.end() && !it->second.empty()) {
      void* p = it->second.back();
      it->second.pop_back();
      return p;
    }
  }
  void* p = nullptr;
  ck(hipMalloc(&p, sz), "hipMalloc");
  std::lock_guard<std::mutex> g(c->mu);
  c->all_blocks.push_back(p);
  c->pooled_bytes += sz;
  return p;
}
// a block back into its context's pool: reused by later allocations of the same size, which are
// ordered after every use of the block on the context's single stream; freed with the context
void release(Context* c, void* p, size_t n) {
  if (!p || !c) return;
  const size_t sz = ((n ? n : 16) + 255) & ~(size_t)255;
  std::lock_guard<std::mutex> g(c->mu);
  c->free_blocks[sz].push_back(p);
}
size_t pooled_bytes(Context* c) {
  std::lock_guard<std::mutex> g(c->mu);
  return c->pooled_bytes;
}
void h2d(void* dst, const void* src, size_t n) {
  ck(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, cur_stream()), "h2d");
  sync();
}
void d2h(void* dst, const void* src, size_t n) {
  ck(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, cur_stream()), "d2h");
  sync();
}
void d2d(void* dst, const void* src, size_t n) {
  ck(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, cur_stream()), "d2d");
}

void gemm(const float* A, const float* B, float* C, const float* bias, int batch, int M, int N, int K, int64_t sAb,
          int64_t sAm, int64_t sAk, int64_t sBb, int64_t sBk, int64_t sBn, int64_t sCb, int64_t sCm, float alpha,
          bool relu) {
  if (M <= 0 || N <= 0 || batch <= 0) return;
  if (batch > 65535) throw Error("gemm: batch > 65535");
  if ((int64_t)M * N >= 64 * 64 * 8) {   // the 128-tile kernel, 16-B loads where the layout allows
    const bool av = sAk == 1 && K % 4 == 0 && sAm % 4 == 0 && sAb % 4 == 0 && ((size_t)A & 15) == 0;
    const bool bv = sBn == 1 && N % 4 == 0 && sBk % 4 == 0 && sBb % 4 == 0 && ((size_t)B & 15) == 0;
    dim3 grid((N + TB - 1) / TB, (M + TB - 1) / TB, batch);
#define PHA_G128(X, Y)                                                                                        \
  hipLaunchKernelGGL((gemm128_kernel<X, Y>), grid, dim3(256), 0, cur_stream(), A, B, C, bias, M, N, K, sAb, sAm, sAk, \
                     sBb, sBk, sBn, sCb, sCm, alpha, relu ? 1 : 0)
    if (av && bv) PHA_G128(true, true);
    else if (av) PHA_G128(true, false);
    else if (bv) PHA_G128(false, true);
    else PHA_G128(false, false);
#undef PHA_G128
    ck_launch("gemm128");
    return;
  }
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch);
  hipLaunchKernelGGL(gemm_kernel, grid, dim3(256), 0, cur_stream(), A, B, C, bias, M, N, K, sAb, sAm, sAk, sBb, sBk, sBn,
                     sCb, sCm, alpha, relu ? 1 : 0);
  ck_launch("gemm");
}

// ---- bf16 GEMM on the kernel library ---------------------------------------------------------------
namespace {
typedef int (*Gemm4pBatched)(int, const void*, const void*, void*, long, long, long, long, long, long, int, int, int,
                             int, const float*, int, int, float*, int, hipStream_t, void*, int, long, long, long);

Gemm4pBatched g4p_entry() {
  static Gemm4pBatched fn = []() -> Gemm4pBatched {
    Dl_info info{};
    if (!dladdr(reinterpret_cast<void*>(&g4p_entry), &info) || !info.dli_fname) return nullptr;
    std::string dir(info.dli_fname);
    dir = dir.substr(0, dir.find_last_of('/') + 1);
    void* h = dlopen((dir + "libpha_kernels.so").c_str(), RTLD_NOW | RTLD_GLOBAL);
    return h ? reinterpret_cast<Gemm4pBatched>(dlsym(h, "pha_gemm4p_batched")) : nullptr;
  }();
  return fn;
}

// dst[b][r][c] (rows_p x cols_p, zero outside rows x cols) = bf16(src[b * sb + r * sr + c * sc])
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                      int rows, int cols, int rows_p, int cols_p, int64_t sb,
                                                      int64_t sr, int64_t sc, int64_t total) {
  for (int64_t i = blockIdx.x * 256L + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t per = (int64_t)rows_p * cols_p;
    const int64_t b = i / per, rc = i - b * per;
    const int r = (int)(rc / cols_p), c = (int)(rc - (int64_t)r * cols_p);
    float v = 0.f;
    if (r < rows && c < cols) v = src[b * sb + r * sr + c * sc];
    uint32_t u = __float_as_uint(v);
    u += 0x7fffu + ((u >> 16) & 1u);   // round to nearest even (finite inputs)
    dst[i] = (uint16_t)(u >> 16);
  }
}

// the same conversion when the source's unit stride runs along r (a B [K][N] operand turned into the
// NT layout's B^T, or a transposed A): 64 x 64 tiles through LDS, so both the fp32 reads (along r)
// and the bf16 writes (along c) are coalesced
__global__ __launch_bounds__(256) void to_bf16_t_kernel(const float* __restrict__ src, uint16_t* __restrict__ dst,
                                                        int rows, int cols, int rows_p, int cols_p, int64_t sb,
                                                        int64_t sc) {
  __shared__ float tile[64][65];
  const int64_t b = blockIdx.z;
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int j = ty; j < 64; j += 4) {
    const int r = r0 + tx, c = c0 + j;
    tile[j][tx] = (r < rows && c < cols) ? src[b * sb + (int64_t)c * sc + r] : 0.f;
  }
  __syncthreads();
  for (int j = ty; j < 64; j += 4) {
    const int r = r0 + j, c = c0 + tx;
    if (r < rows_p && c < cols_p) {
      uint32_t u = __float_as_uint(tile[tx][j]);
      u += 0x7fffu + ((u >> 16) & 1u);
      dst[(b * rows_p + r) * cols_p + c] = (uint16_t)(u >> 16);
    }
  }
}

void convert_bf16(const float* src, uint16_t* dst, int nbatch, int rows, int cols, int rows_p, int cols_p, int64_t sb,
                  int64_t sr, int64_t sc) {
  if (sr == 1 && sc != 1) {
    hipLaunchKernelGGL(to_bf16_t_kernel, dim3((rows_p + 63) / 64, (cols_p + 63) / 64, nbatch), dim3(256), 0,
                       cur_stream(), src, dst, rows, cols, rows_p, cols_p, sb, sc);
  } else {
    const int64_t n = (int64_t)nbatch * rows_p * cols_p;
    hipLaunchKernelGGL(to_bf16_kernel, dim3(blocks_for(n)), dim3(256), 0, cur_stream(), src, dst, rows, cols, rows_p,
                       cols_p, sb, sr, sc, n);
  }
}

// C[b][m][n] = relu(alpha * c16[b][m][n] + bias[n]) over the unpadded M x N
__global__ __launch_bounds__(256) void from_bf16_kernel(const uint16_t* __restrict__ c16, float* __restrict__ C,
                                                        const float* __restrict__ bias, int M, int N, int ldc,
                                                        int64_t sb16, int64_t sCb, int64_t sCm, float alpha, int relu,
                                                        int64_t total) {
  for (int64_t i = blockIdx.x * 256L + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t per = (int64_t)M * N;
    const int64_t b = i / per, mn = i - b * per;
    const int m = (int)(mn / N), n = (int)(mn - (int64_t)m * N);
    float v = alpha * __uint_as_float((uint32_t)c16[b * sb16 + (int64_t)m * ldc + n] << 16);
    if (bias) v += bias[n];
    if (relu && v < 0.f) v = 0.f;
    C[b * sCb + (int64_t)m * sCm + n] = v;
  }
}
}  // namespace

bool gemm_bf16(const float* A, const float* B, float* C, const float* bias, int batch, int M, int N, int K,
               int64_t sAb, int64_t sAm, int64_t sAk, int64_t sBb, int64_t sBk, int64_t sBn, int64_t sCb,
               int64_t sCm, float alpha, bool relu) {
  Gemm4pBatched fn = g4p_entry();
  if (!fn || M <= 0 || N <= 0 || K <= 0 || batch <= 0) return false;
  const int Mp = (M + 7) / 8 * 8, Np = (N + 7) / 8 * 8, Kp = (K + 63) / 64 * 64;
  const int ba = sAb ? batch : 1, bb = sBb ? batch : 1;
  const size_t na = (size_t)ba * Mp * Kp, nb = (size_t)bb * Np * Kp, nc = (size_t)batch * Mp * Np;
  Context* cx = current();
  if (ba > 65535 || bb > 65535) return false;
  auto* a16 = static_cast<uint16_t*>(alloc(na * 2));
  auto* b16 = static_cast<uint16_t*>(alloc(nb * 2));
  auto* c16 = static_cast<uint16_t*>(alloc(nc * 2));
  convert_bf16(A, a16, ba, M, K, Mp, Kp, sAb, sAm, sAk);
  convert_bf16(B, b16, bb, N, K, Np, Kp, sBb, sBn, sBk);
  ck_launch("to_bf16");
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, cx->dev);
  // NT (A [M][K], B^T [N][K]) with the early-release schedule, PIN + SPREAD DMA placement (LV 40, the
  // training path's default: ops/gemm.py _epi_default)
  const int epi = 65536 | (8 << 17) | (1 << 28);
  const int rc = fn(1, a16, b16, c16, Mp, Np, Kp, Kp, Kp, Np, 0, 0, 0, epi, nullptr, cus, 0, nullptr, 1, cx->stream,
                    nullptr, batch, ba > 1 ? (long)Mp * Kp : 0, bb > 1 ? (long)Np * Kp : 0, (long)Mp * Np);
  if (rc != 0) throw Error("pha_gemm4p_batched failed (" + std::to_string(rc) + ")");
  const int64_t tot = (int64_t)batch * M * N;
  hipLaunchKernelGGL(from_bf16_kernel, dim3(blocks_for(tot)), dim3(256), 0, cur_stream(), c16, C, bias, M, N, Np,
                     (int64_t)Mp * Np, sCb, sCm, alpha, relu ? 1 : 0, tot);
  ck_launch("from_bf16");
  release(cx, a16, na * 2);
  release(cx, b16, nb * 2);
  release(cx, c16, nc * 2);
  return true;
}

void im2col(const float* x, float* col, int C, int H, int W, int KH, int KW, int OH, int OW, int sh, int sw, int pt,
            int pl, int dh, int dw, int N) {
  hipLaunchKernelGGL(im2col_kernel, dim3(blocks_for((int64_t)N * C * KH * KW * OH * OW)), dim3(256), 0, cur_stream(), x,
                     col, C, H, W, KH, KW, OH, OW, sh, sw, pt, pl, dh, dw, N);
  ck_launch("im2col");
}
void row_bias_act(float* y, const float* bias, int64_t rows, int64_t inner, int64_t batch, bool relu) {
  hipLaunchKernelGGL(row_bias_act_kernel, dim3(blocks_for(batch * rows * inner)), dim3(256), 0, cur_stream(), y, bias,
                     rows, inner, batch, relu ? 1 : 0);
  ck_launch("row_bias_act");
}

void depthwise_conv(const float* x, const float* w, float* y, int N, int C, int H, int W, int KH, int KW, int OH,
                    int OW, int sh, int sw, int pt, int pl, int dh, int dw, int mult) {
  hipLaunchKernelGGL(dwconv_kernel, dim3(blocks_for((int64_t)N * C * mult * OH * OW)), dim3(256), 0, cur_stream(), x, w, y,
                     N, C, H, W, KH, KW, OH, OW, sh, sw, pt, pl, dh, dw, mult);
  ck_launch("depthwise_conv");
}

void unary(const float* x, float* y, int64_t n, int op, float a, float b) {
  hipLaunchKernelGGL(unary_kernel, dim3(blocks_for(n)), dim3(256), 0, cur_stream(), x, y, n, op, a, b);
  ck_launch("unary");
}

void binary(const float* x, const float* y, float* out, int op, int nd, const int64_t* shape, const int64_t* sx,
            const int64_t* sy) {
  int64_t total = 1;
  for (int k = 0; k < nd; ++k) total *= shape[k];
  if (!total) return;
  hipLaunchKernelGGL(binary_kernel, dim3(blocks_for(total)), dim3(256), 0, cur_stream(), x, y, out, op, nd,
                     dims(nd, shape, sx, sy), total);
  ck_launch("binary");
}

void batch_norm(const float* x, float* y, const float* scale, const float* bias, const float* mean,
                const float* var, float eps, int64_t N, int64_t C, int64_t inner) {
  const int64_t total = N * C * inner;
  hipLaunchKernelGGL(bn_kernel, dim3(blocks_for(total)), dim3(256), 0, cur_stream(), x, y, scale, bias, mean, var, eps, C,
                     inner, total);
  ck_launch("batch_norm");
}

void pool2d(const float* x, float* y, int N, int C, int H, int W, int OH, int OW, int KH, int KW, int sh, int sw,
            int pt, int pl, bool maxp, bool exclusive, bool adaptive) {
  hipLaunchKernelGGL(pool_kernel, dim3(blocks_for((int64_t)N * C * OH * OW)), dim3(256), 0, cur_stream(), x, y, N, C, H, W,
                     OH, OW, KH, KW, sh, sw, pt, pl, maxp ? 1 : 0, exclusive ? 1 : 0, adaptive ? 1 : 0);
  ck_launch("pool2d");
}

void strided_copy(const void* in, void* out, int esize, int nd, const int64_t* shape, const int64_t* strides) {
  int64_t total = 1;
  for (int k = 0; k < nd; ++k) total *= shape[k];
  if (!total) return;
  const Dims8 d = dims(nd, shape, strides, nullptr);
  const dim3 g(blocks_for(total));
  if (esize == 4)
    hipLaunchKernelGGL(strided_kernel<uint32_t>, g, dim3(256), 0, cur_stream(), (const uint32_t*)in, (uint32_t*)out, nd, d, total);
  else if (esize == 8)
    hipLaunchKernelGGL(strided_kernel<uint64_t>, g, dim3(256), 0, cur_stream(), (const uint64_t*)in, (uint64_t*)out, nd, d, total);
  else if (esize == 2)
    hipLaunchKernelGGL(strided_kernel<uint16_t>, g, dim3(256), 0, cur_stream(), (const uint16_t*)in, (uint16_t*)out, nd, d, total);
  else
    hipLaunchKernelGGL(strided_kernel<uint8_t>, g, dim3(256), 0, cur_stream(), (const uint8_t*)in, (uint8_t*)out, nd, d, total);
  ck_launch("strided_copy");
}

void softmax(const float* x, float* y, int64_t outer, int64_t n, int64_t inner) {
  const int64_t rows = outer * inner;
  if (rows > 2147483647) throw Error("softmax: too many rows");
  hipLaunchKernelGGL(softmax_kernel, dim3((unsigned)rows), dim3(256), 0, cur_stream(), x, y, n, inner);
  ck_launch("softmax");
}

void layer_norm(const float* x, float* y, const float* scale, const float* bias, int64_t rows, int64_t cols,
                float eps) {
  hipLaunchKernelGGL(layer_norm_kernel, dim3((unsigned)rows), dim3(256), 0, cur_stream(), x, y, scale, bias, cols, eps);
  ck_launch("layer_norm");
}

void embedding(const int64_t* ids, const float* w, float* out, int64_t n, int64_t H, int64_t V, int64_t pad) {
  hipLaunchKernelGGL(embedding_kernel, dim3(blocks_for(n * H)), dim3(256), 0, cur_stream(), ids, w, out, n, H, V, pad);
  ck_launch("embedding");
}

void cast(const void* x, int xdt, void* y, int ydt, int64_t n) {
  const dim3 g(blocks_for(n));
#define PHA_CAST(XT, XC, YT, YC)                                                                              \
  if (xdt == XC && ydt == YC) {                                                                               \
    hipLaunchKernelGGL((cast_kernel<XT, YT>), g, dim3(256), 0, cur_stream(), (const XT*)x, (YT*)y, n);            \
    ck_launch("cast");                                                                                        \
    return;                                                                                                   \
  }
  PHA_CAST(float, F32, int64_t, I64)
  PHA_CAST(float, F32, int32_t, I32)
  PHA_CAST(int64_t, I64, float, F32)
  PHA_CAST(int32_t, I32, float, F32)
  PHA_CAST(int64_t, I64, int32_t, I32)
  PHA_CAST(int32_t, I32, int64_t, I64)
  PHA_CAST(float, F32, float, F32)
  PHA_CAST(int64_t, I64, int64_t, I64)
#undef PHA_CAST
  throw Error("cast: unsupported dtype pair " + std::to_string(xdt) + " -> " + std::to_string(ydt));
}

void fill(float* y, int64_t n, float v) {
  hipLaunchKernelGGL(fill_kernel, dim3(blocks_for(n)), dim3(256), 0, cur_stream(), y, n, v);
  ck_launch("fill");
}

}  // namespace gpu
}  // namespace pha_infer
