// Softmax-cross-entropy (hard labels), bias+GELU, and embedding gather for gfx950.
//
// softmax_ce: one 256-thread block per row, single pass with an online
//   (max, sum-exp) pair per thread merged across the block — the logits row is
//   read once in forward; backward re-reads it once and writes dlogits once.
//   Reference: paddle/phi/kernels/gpu/cross_entropy_kernel.cu (hard-label path).
// bias_gelu: 8-wide vectorised elementwise, exact erf GELU (or tanh approx).
//   Reference: phi/kernels/gpu/gelu_kernel.cu, operators/fused/fused_dropout_act_bias.h.
// embedding: one wave per output row, 16-byte vector row copies.
//   Reference: phi/kernels/gpu/embedding_kernel.cu.
#include "common.h"
#include <algorithm>

using namespace pha;

namespace {

// VEC: V % 8 == 0 (16-B row loads); else one element per lane-iteration (vocabularies like
// BERT's 30522: the rows are not 16-B aligned, and the fp32 torch fallback cost ~0.6 ms per step)
template <typename T, bool VEC = true>
__global__ __launch_bounds__(256) void softmax_ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                             float* __restrict__ loss, float* __restrict__ lse_out,
                                                             int V, int ignore_index) {
  const long row = blockIdx.x;
  const T* xr = logits + row * (long)V;
  float m = -INFINITY, s = 0.f;
  if constexpr (VEC) {
    for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
      float v[8];
      Vec8<T>::ld(xr + c, v);
      float vm = v[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) vm = fmaxf(vm, v[i]);
      const float nm = fmaxf(m, vm);
      float acc = s * __expf(m - nm);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += __expf(v[i] - nm);
      m = nm;
      s = acc;
    }
  } else {
    for (int c0 = 0; c0 < V; c0 += 256 * 8) {   // 8 strided elements per thread, then one update
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = c0 + i * 256 + (int)threadIdx.x;
        v[i] = c < V ? Cvt<T>::ld(xr, c) : -INFINITY;
      }
      float vm = v[0];
#pragma unroll
      for (int i = 1; i < 8; ++i) vm = fmaxf(vm, v[i]);
      const float nm = fmaxf(m, vm);
      if (nm == -INFINITY) continue;
      float acc = s * __expf(m - nm);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc += __expf(v[i] - nm);
      m = nm;
      s = acc;
    }
  }
  // merge (m, s) pairs across the wave, then across waves
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    const float nm = fmaxf(m, om);
    s = (nm == -INFINITY) ? 0.f : s * __expf(m - nm) + os * __expf(om - nm);
    m = nm;
  }
  __shared__ float sm[4], ss[4];
  if (lane == 0) { sm[wid] = m; ss[wid] = s; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) {
      const float nm = fmaxf(M, sm[i]);
      S = S * __expf(M - nm) + ss[i] * __expf(sm[i] - nm);
      M = nm;
    }
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const long lab = labels[row];
    if (lab == ignore_index || lab < 0 || lab >= V) {
      loss[row] = 0.f;
    } else {
      loss[row] = lse - Cvt<T>::ld(xr, lab);
    }
  }
}

template <typename T, bool VEC = true>
__global__ __launch_bounds__(256) void softmax_ce_bwd_kernel(const float* __restrict__ gloss, const T* __restrict__ logits,
                                                             const int64_t* __restrict__ labels, const float* __restrict__ lse,
                                                             T* __restrict__ dx, int V, int ignore_index) {
  const long row = blockIdx.x;
  const long lab = labels[row];
  const bool ign = (lab == ignore_index || lab < 0 || lab >= V);
  const float g = ign ? 0.f : gloss[row];
  const float l = lse[row];
  const T* xr = logits + row * (long)V;
  T* dr = dx + row * (long)V;
  if constexpr (!VEC) {
    for (int c = threadIdx.x; c < V; c += 256) {
      const float p = __expf(Cvt<T>::ld(xr, c) - l);
      Cvt<T>::st(dr, c, g * (p - (c == lab ? 1.f : 0.f)));
    }
    return;
  }
  for (int c = threadIdx.x * 8; c < V; c += 256 * 8) {
    float v[8], o[8];
    Vec8<T>::ld(xr + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float p = __expf(v[i] - l);
      o[i] = g * (p - ((c + i) == lab ? 1.f : 0.f));
    }
    Vec8<T>::st(dr + c, o);
  }
}

// tanh(u) = 1 - 2 / (exp(2u) + 1) on v_exp_f32 + v_rcp_f32 (a few instructions; libm tanhf is a
// long branchy sequence that made the bias+GELU passes VALU-bound); saturates to +-1, error ~1e-7
__device__ __forceinline__ float fast_tanh(float u) {
  const float e = __expf(2.f * u);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

__device__ __forceinline__ float gelu_f(float x, bool approx) {
  if (approx) {
    const float k = 0.7978845608028654f;  // sqrt(2/pi)
    const float u = k * (x + 0.044715f * x * x * x);
    return 0.5f * x * (1.f + fast_tanh(u));
  }
  return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
}

__device__ __forceinline__ float gelu_grad(float x, bool approx) {
  if (approx) {
    // tanh-GELU = x s, s = sigmoid(2u), u = k (x + c x^3): d/dx = s + x s (1 - s) 2k (1 + 3c x^2) —
    // 9 VALU + exp2 + rcp (log2(e) folded into the polynomial) instead of ~15 + exp + rcp: the
    // dGELU pass over the GPT MLP's [tokens, 4H] pre-activation is memory-bound only when its VALU
    // work stays well under the HBM time
    constexpr float k = 0.7978845608028654f, c = 0.044715f;
    constexpr float c0 = -2.f * k * 1.4426950408889634f, c1 = c0 * c;
    const float x2 = x * x;
    const float sg = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(x * __builtin_fmaf(x2, c1, c0)));
    const float q = x * __builtin_fmaf(x2, 6.f * k * c, 2.f * k) * (1.f - sg);
    return __builtin_fmaf(q, sg, sg);
  }
  const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_fwd_kernel(const T* __restrict__ x, const T* __restrict__ b, T* __restrict__ y,
                                                            long n8, int H, bool approx) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8], o[8];
    Vec8<T>::ld(x + i * 8, v);
    if (b) {
      float bv[8];
      Vec8<T>::ld(b + (int)((unsigned)i % (unsigned)(H / 8)) * 8, bv);   // n8 < 2^32 (host check)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += bv[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = gelu_f(v[k], approx);
    Vec8<T>::st(y + i * 8, o);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_kernel(const T* __restrict__ gy, const T* __restrict__ x, const T* __restrict__ b,
                                                            T* __restrict__ gx, long n8, int H, bool approx) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    float v[8], g[8], o[8];
    Vec8<T>::ld(x + i * 8, v);
    Vec8<T>::ld(gy + i * 8, g);
    if (b) {
      float bv[8];
      Vec8<T>::ld(b + (int)((unsigned)i % (unsigned)(H / 8)) * 8, bv);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += bv[k];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * gelu_grad(v[k], approx);
    Vec8<T>::st(gx + i * 8, o);
  }
}

// bias-GELU backward over a [rows, H] activation (bias gradient taken elsewhere — the next
// weight-gradient GEMM sums it, ops/gemm.mm_tn_db): thread = one 8-column chunk over a block of
// rows, bias in registers, 4 rows of loads in flight, no per-element index arithmetic
template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_rows_kernel(const T* __restrict__ gy, const T* __restrict__ x,
                                                                 const T* __restrict__ b, T* __restrict__ gx, int rows,
                                                                 int H, int rows_per_block, bool approx) {
  const int c8 = blockIdx.x * 256 + threadIdx.x;
  if (c8 * 8 >= H) return;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  float bv[8];
  Vec8<T>::ld(b + c8 * 8, bv);
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    const long off = (long)r * H + c8 * 8;
    float v[8], g[8], o[8];
    Vec8<T>::ld(x + off, v);
    Vec8<T>::ld(gy + off, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = g[k] * gelu_grad(v[k] + bv[k], approx);
    Vec8<T>::st(gx + off, o);
  }
}

// bias-GELU backward that also forms the bias gradient: thread = one 8-column chunk, block row
// y = a contiguous range of rows; the column sums of gx over that range go to part[y][H] (fp32),
// so db needs no second pass over gx (reference: fused_gemm_epilogue / fused_feedforward's
// bias grad reduction).
template <typename T>
__global__ __launch_bounds__(256) void bias_gelu_bwd_db_kernel(const T* __restrict__ gy, const T* __restrict__ x,
                                                               const T* __restrict__ b, T* __restrict__ gx,
                                                               float* __restrict__ part, int rows, int H,
                                                               int rows_per_block, bool approx) {
  const int c8 = blockIdx.x * 256 + threadIdx.x;   // chunk of 8 columns
  if (c8 * 8 >= H) return;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  float bv[8], acc[8];
  Vec8<T>::ld(b + c8 * 8, bv);
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0.f;
#pragma unroll 4
  for (int r = r0; r < r1; ++r) {
    const long off = (long)r * H + c8 * 8;
    float v[8], g[8], o[8];
    Vec8<T>::ld(x + off, v);
    Vec8<T>::ld(gy + off, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = g[k] * gelu_grad(v[k] + bv[k], approx);
      acc[k] += round_to<T>(o[k]);   // the bias gradient of the stored (rounded) gx
    }
    Vec8<T>::st(gx + off, o);
  }
  Vec8<float>::st(part + (long)blockIdx.y * H + c8 * 8, acc);
}

// bias gradient of a linear layer: per-row-block column sums of gy [rows, H] (thread = 8-column
// chunk, 16-B loads, fp32 accumulation); part[blockIdx.y] is summed by the caller
template <typename T>
__global__ __launch_bounds__(256) void col_sum_partial_kernel(const T* __restrict__ gy, float* __restrict__ part,
                                                              int rows, int H, int rows_per_block) {
  const int c8 = blockIdx.x * 256 + threadIdx.x;
  if (c8 * 8 >= H) return;
  const int r0 = blockIdx.y * rows_per_block, r1 = min(rows, r0 + rows_per_block);
  float acc[8], acc2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = acc2[k] = 0.f;
  int r = r0;
  for (; r + 1 < r1; r += 2) {   // two rows in flight per iteration
    float g[8], h[8];
    Vec8<T>::ld(gy + (long)r * H + c8 * 8, g);
    Vec8<T>::ld(gy + (long)(r + 1) * H + c8 * 8, h);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      acc[k] += g[k];
      acc2[k] += h[k];
    }
  }
  if (r < r1) {
    float g[8];
    Vec8<T>::ld(gy + (long)r * H + c8 * 8, g);
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] += g[k];
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] += acc2[k];
  Vec8<float>::st(part + (long)blockIdx.y * H + c8 * 8, acc);
}

// dst[C][R] = src[R][C]^T for 2-byte elements: 64 x 64 tiles through LDS (rows padded by 2
// elements), 16-B loads and stores on both sides (R, C % 8 == 0)
__global__ __launch_bounds__(256) void transpose16_kernel(const uint16_t* __restrict__ src, uint16_t* __restrict__ dst,
                                                          int R, int C) {
  __shared__ uint16_t tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j;       // 64 rows x 8 chunks
    const int rr = idx >> 3, cc = (idx & 7) * 8;
    if (r0 + rr < R && c0 + cc < C) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + (long)(r0 + rr) * C + c0 + cc);
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) tile[rr][cc + k] = e[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j;       // 64 output rows (input columns) x 8 chunks
    const int oc = idx >> 3, orr = (idx & 7) * 8;
    if (c0 + oc < C && r0 + orr < R) {
      uint4 v;
      uint16_t* e = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[k] = tile[orr + k][oc];
      *reinterpret_cast<uint4*>(dst + (long)(c0 + oc) * R + r0 + orr) = v;
    }
  }
}

// NHWC max pooling (reference: phi/kernels/funcs/pooling.cu, max_pool2d_with_index): a thread
// owns 8 channels (16 B) of one output pixel; the window position of the max (kh * KW + kw, first
// max wins like the reference) is kept as one byte per element for the backward.
struct PoolGeo {
  int N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw;
};

// I: index type of the element walk — unsigned 32-bit whenever the tensor allows (a 64-bit
// division / modulo is a long software sequence on CDNA; four per element made both kernels
// VALU-bound at ~40-60 % of the HBM rate on ResNet-50's 112x112x64 pooling)
template <typename T, typename I>
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeo g) {
  const I cv = (I)(g.C / 8);
  const I total = (I)g.N * (I)g.OH * (I)g.OW * cv;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const int c8 = (int)(i % cv);
    const I pix = i / cv, prow = pix / (I)g.OW;
    const int ow = (int)(pix - prow * (I)g.OW), n = (int)(prow / (I)g.OH), oh = (int)(prow - (I)n * (I)g.OH);
    float best[8];
    uint8_t bi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; bi[k] = 0; }
    for (int kh = 0; kh < g.KH; ++kh) {
      const int ih = oh * g.sh - g.ph + kh;
      if ((unsigned)ih >= (unsigned)g.H) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int iw = ow * g.sw - g.pw + kw;
        if ((unsigned)iw >= (unsigned)g.W) continue;
        float v[8];
        Vec8<T>::ld(x + (((long)n * g.H + ih) * g.W + iw) * g.C + c8 * 8, v);
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (v[k] > best[k] || (v[k] != v[k] && best[k] == best[k])) {   // NaN propagates
            best[k] = v[k];
            bi[k] = (uint8_t)(kh * g.KW + kw);
          }
      }
    }
    Vec8<T>::st(y + (long)i * 8, best);
    uint2 packed;
    packed.x = bi[0] | (bi[1] << 8) | (bi[2] << 16) | ((uint32_t)bi[3] << 24);
    packed.y = bi[4] | (bi[5] << 8) | (bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + (long)i * 8) = packed;
  }
}

// gather form (no atomics): an input pixel sums the gradients of the <= ceil(K/s)^2 windows that
// cover it and chose it
template <typename T, typename I>
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const T* __restrict__ gy, const uint8_t* __restrict__ idx,
                                                          T* __restrict__ gx, PoolGeo g) {
  const I cv = (I)(g.C / 8);
  const I total = (I)g.N * (I)g.H * (I)g.W * cv;
  for (I i = (I)blockIdx.x * 256 + threadIdx.x; i < total; i += (I)gridDim.x * 256) {
    const int c8 = (int)(i % cv);
    const I pix = i / cv, prow = pix / (I)g.W;
    const int iw = (int)(pix - prow * (I)g.W), n = (int)(prow / (I)g.H), ih = (int)(prow - (I)n * (I)g.H);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    // windows oh with oh*sh - ph <= ih <= oh*sh - ph + KH - 1
    const int oh_lo = max(0, (ih + g.ph - g.KH + g.sh) / g.sh), oh_hi = min(g.OH - 1, (ih + g.ph) / g.sh);
    const int ow_lo = max(0, (iw + g.pw - g.KW + g.sw) / g.sw), ow_hi = min(g.OW - 1, (iw + g.pw) / g.sw);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = ih - (oh * g.sh - g.ph);
      if (kh < 0 || kh >= g.KH) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = iw - (ow * g.sw - g.pw);
        if (kw < 0 || kw >= g.KW) continue;
        const long o = (((long)n * g.OH + oh) * g.OW + ow) * g.C + c8 * 8;
        const uint2 packed = *reinterpret_cast<const uint2*>(idx + o);
        float d[8];
        Vec8<T>::ld(gy + o, d);
        const uint8_t me = (uint8_t)(kh * g.KW + kw);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t w = k < 4 ? packed.x : packed.y;
          if (((w >> (8 * (k & 3))) & 0xff) == me) acc[k] += d[k];
        }
      }
    }
    Vec8<T>::st(gx + (long)i * 8, acc);
  }
}

// one wave per output row; row bytes multiple of 16
__global__ __launch_bounds__(256) void embedding_fwd_kernel(const int64_t* __restrict__ ids, const uint4* __restrict__ w,
                                                            uint4* __restrict__ out, long rows, int row_vecs, long vocab) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  if (r >= rows) return;
  const int lane = threadIdx.x & 63;
  long id = ids[r];
  uint4* dst = out + r * row_vecs;
  if (id < 0 || id >= vocab) {
    for (int c = lane; c < row_vecs; c += 64) dst[c] = make_uint4(0, 0, 0, 0);
    return;
  }
  const uint4* src = w + id * row_vecs;
  for (int c = lane; c < row_vecs; c += 64) dst[c] = src[c];
}

// Embedding backward, deterministic and sort-free (reference: phi/kernels/gpu/embedding_grad_kernel.cu:246,
// whose default path is an atomicAdd scatter and whose deterministic path sorts the ids):
//   gw[v][:] = sum of gy[r][:] over tokens r with ids[r] == v, in increasing r
// One workgroup owns an output block of EB_ROWS vocabulary rows x EB_DCH columns, accumulated in
// fp32 in LDS (128 KB). It scans the whole id vector (4 bytes per token per block, L2-resident),
// compacts the matching token positions into an LDS list in token order (wave ballots + ordered
// wave offsets), and adds those gradient rows in list order: every output element is summed in
// token order by one thread, so results are bitwise reproducible, with no atomics and no sort.
// Rows nobody looked up (and padding_idx) come out zero; the block writes its whole region.
constexpr int EB_ROWS = 32, EB_DCH = 1024, EB_CAP = 4096;

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float (&o)[4]);
template <> __device__ __forceinline__ void ld4<bf16_t>(const bf16_t* p, float (&o)[4]) {
  const uint2 r = *reinterpret_cast<const uint2*>(p);
  o[0] = __uint_as_float(r.x << 16); o[1] = __uint_as_float(r.x & 0xffff0000u);
  o[2] = __uint_as_float(r.y << 16); o[3] = __uint_as_float(r.y & 0xffff0000u);
}
template <> __device__ __forceinline__ void ld4<half_t>(const half_t* p, float (&o)[4]) {
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const h4 r = *reinterpret_cast<const h4*>(p);
  for (int e = 0; e < 4; ++e) o[e] = (float)r[e];
}
template <> __device__ __forceinline__ void ld4<float>(const float* p, float (&o)[4]) {
  const float4 r = *reinterpret_cast<const float4*>(p);
  o[0] = r.x; o[1] = r.y; o[2] = r.z; o[3] = r.w;
}

template <typename T>
// Token chunks (grid.z, `chunk` tokens each, ws != null): a small vocabulary (token types, positions)
// leaves too few (row, column) blocks to fill the chip — each chunk then writes fp32 partial rows to
// ws[z] and chunk_sum_kernel adds the chunks in order (still deterministic).
__global__ __launch_bounds__(256) void embedding_bwd_kernel(const int64_t* __restrict__ ids, const T* __restrict__ gy,
                                                            T* __restrict__ gw, long n, int D, long V, long pad,
                                                            long chunk, float* __restrict__ ws) {
  extern __shared__ __attribute__((aligned(16))) unsigned char eb_smem[];
  float* acc = reinterpret_cast<float*>(eb_smem);                       // [EB_ROWS][EB_DCH]
  int* list = reinterpret_cast<int*>(eb_smem + EB_ROWS * EB_DCH * 4);   // [EB_CAP]
  int* wcnt = list + EB_CAP;                                            // [4]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const long v0 = (long)blockIdx.x * EB_ROWS;
  const int d0 = blockIdx.y * EB_DCH;
  const int dn = min(EB_DCH, D - d0);
  for (int i = tid; i < EB_ROWS * EB_DCH / 4; i += 256) reinterpret_cast<float4*>(acc)[i] = make_float4(0, 0, 0, 0);
  int cnt = 0;
  auto flush = [&]() {   // add the listed gradient rows, in list (= token) order
    __syncthreads();
    const int c = tid * 4;
    if (c < dn) {
      int k = 0;
      // 8 gradient rows in flight per step (loads first, then the adds in list order: the same
      // summation order as one row at a time — a serial load -> add chain cost ~1 HBM latency per row)
      for (; k + 8 <= cnt; k += 8) {
        float g[8][4];
        int ee[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          ee[u] = list[k + u];
          ld4<T>(gy + (long)(ee[u] >> 5) * D + d0 + c, g[u]);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          float* a = acc + (ee[u] & 31) * EB_DCH + c;
#pragma unroll
          for (int q = 0; q < 4; ++q) a[q] += g[u][q];
        }
      }
      for (; k < cnt; ++k) {
        const int e = list[k];
        const long r = e >> 5;
        float g[4];
        ld4<T>(gy + r * D + d0 + c, g);
        float* a = acc + (e & 31) * EB_DCH + c;
#pragma unroll
        for (int q = 0; q < 4; ++q) a[q] += g[q];
      }
    }
    __syncthreads();
    cnt = 0;
  };
  const long t0 = (long)blockIdx.z * chunk, t1 = min(n, t0 + chunk);
  long idn = t0 + tid < t1 ? ids[t0 + tid] : -1;   // the next 256 ids load during this batch's compaction
  for (long base = t0; base < t1; base += 256) {
    const long r = base + tid;
    const long id = idn;
    idn = r + 256 < t1 ? ids[r + 256] : -1;
    const bool m = id >= v0 && id < v0 + EB_ROWS && id < V && id != pad;
    const unsigned long long bal = __ballot(m);
    const int pre = __popcll(bal & ((1ULL << lane) - 1ULL));
    if (lane == 0) wcnt[wid] = __popcll(bal);
    __syncthreads();
    int off = cnt, tot = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const int cw = wcnt[w];
      if (w < wid) off += cw;
      tot += cw;
    }
    if (m) list[off + pre] = (int)(r << 5) | (int)(id - v0);
    cnt += tot;
    __syncthreads();
    if (cnt > EB_CAP - 256) flush();
  }
  flush();
  const int c = tid * 4;
  if (c < dn) {
    for (int row = 0; row < EB_ROWS; ++row) {
      const long v = v0 + row;
      if (v >= V) break;
      const float* a = acc + row * EB_DCH + c;
      if (ws) {
        *reinterpret_cast<float4*>(ws + ((long)blockIdx.z * V + v) * D + d0 + c) = make_float4(a[0], a[1], a[2], a[3]);
        continue;
      }
      T* o = gw + v * D + d0 + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) Cvt<T>::st(o, q, a[q]);
    }
  }
}

inline int grid_for(long n, int per_block) {
  long g = (n + per_block - 1) / per_block;
  if (g > 256L * 16) g = 256L * 16;   // grid-stride beyond ~16 blocks per CU
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace

PHA_API int pha_softmax_ce_fwd(int dt, const void* logits, const int64_t* labels, float* loss, float* lse,
                               long rows, int V, int ignore_index, hipStream_t stream) {
  if (V <= 0) return (int)hipErrorInvalidValue;
  PHA_DISPATCH_T(dt, T, {
    if (V % 8 == 0)
      hipLaunchKernelGGL((softmax_ce_fwd_kernel<T, true>), dim3(rows), dim3(256), 0, stream, (const T*)logits, labels, loss, lse, V, ignore_index);
    else
      hipLaunchKernelGGL((softmax_ce_fwd_kernel<T, false>), dim3(rows), dim3(256), 0, stream, (const T*)logits, labels, loss, lse, V, ignore_index);
  });
  return (int)hipGetLastError();
}

PHA_API int pha_softmax_ce_bwd(int dt, const float* gloss, const void* logits, const int64_t* labels, const float* lse,
                               void* dx, long rows, int V, int ignore_index, hipStream_t stream) {
  if (V <= 0) return (int)hipErrorInvalidValue;
  PHA_DISPATCH_T(dt, T, {
    if (V % 8 == 0)
      hipLaunchKernelGGL((softmax_ce_bwd_kernel<T, true>), dim3(rows), dim3(256), 0, stream, gloss, (const T*)logits, labels, lse, (T*)dx, V, ignore_index);
    else
      hipLaunchKernelGGL((softmax_ce_bwd_kernel<T, false>), dim3(rows), dim3(256), 0, stream, gloss, (const T*)logits, labels, lse, (T*)dx, V, ignore_index);
  });
  return (int)hipGetLastError();
}

PHA_API int pha_bias_gelu_fwd(int dt, const void* x, const void* b, void* y, long n, int H, int approx, hipStream_t stream) {
  if (n % 8 || (b && H % 8) || n / 8 >= (1L << 32)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  PHA_DISPATCH_T(dt, T, {
    hipLaunchKernelGGL((bias_gelu_fwd_kernel<T>), dim3(grid_for(n8, 256)), dim3(256), 0, stream, (const T*)x, (const T*)b, (T*)y, n8, H, approx != 0);
  });
  return (int)hipGetLastError();
}

PHA_API int pha_bias_gelu_bwd(int dt, const void* gy, const void* x, const void* b, void* gx, long n, int H, int approx, hipStream_t stream) {
  if (n % 8 || (b && H % 8) || n / 8 >= (1L << 32)) return (int)hipErrorInvalidValue;
  const long n8 = n / 8;
  PHA_DISPATCH_T(dt, T, {
    hipLaunchKernelGGL((bias_gelu_bwd_kernel<T>), dim3(grid_for(n8, 256)), dim3(256), 0, stream, (const T*)gy, (const T*)x, (const T*)b, (T*)gx, n8, H, approx != 0);
  });
  return (int)hipGetLastError();
}

PHA_API int pha_bias_gelu_bwd_rows(int dt, const void* gy, const void* x, const void* b, void* gx, int rows, int H,
                                   int rows_per_block, int approx, hipStream_t stream) {
  if (H % 8 || rows <= 0 || rows_per_block <= 0 || !b) return (int)hipErrorInvalidValue;
  const dim3 grid((H / 8 + 255) / 256, (rows + rows_per_block - 1) / rows_per_block);
  PHA_DISPATCH_T(dt, T, {
    hipLaunchKernelGGL((bias_gelu_bwd_rows_kernel<T>), grid, dim3(256), 0, stream, (const T*)gy, (const T*)x,
                       (const T*)b, (T*)gx, rows, H, rows_per_block, approx != 0);
  });
  return (int)hipGetLastError();
}

// part: [ceil(rows / rows_per_block), H] fp32 workspace; db = part.sum(0) (done by the caller)
PHA_API int pha_bias_gelu_bwd_db(int dt, const void* gy, const void* x, const void* b, void* gx, float* part, int rows,
                                 int H, int rows_per_block, int approx, hipStream_t stream) {
  if (H % 8 || rows <= 0 || rows_per_block <= 0 || !b) return (int)hipErrorInvalidValue;
  const dim3 grid((H / 8 + 255) / 256, (rows + rows_per_block - 1) / rows_per_block);
  PHA_DISPATCH_T(dt, T, {
    hipLaunchKernelGGL((bias_gelu_bwd_db_kernel<T>), grid, dim3(256), 0, stream, (const T*)gy, (const T*)x,
                       (const T*)b, (T*)gx, part, rows, H, rows_per_block, approx != 0);
  });
  return (int)hipGetLastError();
}

// part: [ceil(rows / rows_per_block), H] fp32; column sums of gy = part.sum(0) (done by the caller)
PHA_API int pha_col_sum_partial(int dt, const void* gy, float* part, int rows, int H, int rows_per_block,
                                hipStream_t stream) {
  if (H % 8 || rows <= 0 || rows_per_block <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((H / 8 + 255) / 256, (rows + rows_per_block - 1) / rows_per_block);
  PHA_DISPATCH_T(dt, T, {
    hipLaunchKernelGGL((col_sum_partial_kernel<T>), grid, dim3(256), 0, stream, (const T*)gy, part, rows, H,
                       rows_per_block);
  });
  return (int)hipGetLastError();
}

// many weight transposes in ONE launch (the cached [out][in] copies of all linear weights an
// optimizer step updated: 50 launches of ~5.5 us per BERT-base step before): block b takes global
// tile b, its matrix found by a scan of the tile offsets (at most kTr16Batch, scalar loads)
constexpr int kTr16Batch = 64;
struct Tr16Batch {
  const uint16_t* src[kTr16Batch];
  uint16_t* dst[kTr16Batch];
  int R[kTr16Batch], C[kTr16Batch];
  int tile0[kTr16Batch + 1];   // first global tile of each matrix; tile0[n] = total
  int n;
};
__global__ __launch_bounds__(256) void transpose16_batch_kernel(Tr16Batch bt) {
  __shared__ uint16_t tile[64][66];
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < bt.n && bt.tile0[e + 1] <= b) ++e;
  const int R = bt.R[e], C = bt.C[e];
  const int t = b - bt.tile0[e], ct = (C + 63) / 64;
  const int r0 = (t / ct) * 64, c0 = (t % ct) * 64;
  const uint16_t* __restrict__ src = bt.src[e];
  uint16_t* __restrict__ dst = bt.dst[e];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j;
    const int rr = idx >> 3, cc = (idx & 7) * 8;
    if (r0 + rr < R && c0 + cc < C) {
      const uint4 v = *reinterpret_cast<const uint4*>(src + (long)(r0 + rr) * C + c0 + cc);
      const uint16_t* el = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) tile[rr][cc + k] = el[k];
    }
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int idx = threadIdx.x + 256 * j;
    const int oc = idx >> 3, orr = (idx & 7) * 8;
    if (c0 + oc < C && r0 + orr < R) {
      uint4 v;
      uint16_t* el = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int k = 0; k < 8; ++k) el[k] = tile[orr + k][oc];
      *reinterpret_cast<uint4*>(dst + (long)(c0 + oc) * R + r0 + orr) = v;
    }
  }
}

// dst_i [C_i][R_i] = src_i [R_i][C_i]^T for n <= 64 matrices of 2-byte elements (R_i, C_i % 8 == 0)
PHA_API int pha_transpose16_batch(int n, const void* const* src, void* const* dst, const int* R, const int* C,
                                  hipStream_t stream) {
  if (n <= 0 || n > kTr16Batch) return (int)hipErrorInvalidValue;
  Tr16Batch bt{};
  bt.n = n;
  long tiles = 0;
  for (int i = 0; i < n; ++i) {
    if (R[i] % 8 || C[i] % 8 || R[i] <= 0 || C[i] <= 0 || !src[i] || !dst[i]) return (int)hipErrorInvalidValue;
    bt.src[i] = (const uint16_t*)src[i];
    bt.dst[i] = (uint16_t*)dst[i];
    bt.R[i] = R[i];
    bt.C[i] = C[i];
    bt.tile0[i] = (int)tiles;
    tiles += (long)((R[i] + 63) / 64) * ((C[i] + 63) / 64);
  }
  if (tiles > 0x7fffffff) return (int)hipErrorInvalidValue;
  bt.tile0[n] = (int)tiles;
  hipLaunchKernelGGL(transpose16_batch_kernel, dim3((unsigned)tiles), dim3(256), 0, stream, bt);
  return (int)hipGetLastError();
}

// dst [C][R] = src [R][C]^T, 2-byte elements, R % 8 == C % 8 == 0
PHA_API int pha_transpose16(const void* src, void* dst, int R, int C, hipStream_t stream) {
  if (R % 8 || C % 8 || R <= 0 || C <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose16_kernel, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, stream,
                     (const uint16_t*)src, (uint16_t*)dst, R, C);
  return (int)hipGetLastError();
}

// NHWC max pool forward (idx: one byte per output element, the window position of the max)
PHA_API int pha_maxpool2d_nhwc_fwd(int dt, const void* x, void* y, uint8_t* idx, int N, int H, int W, int C, int OH,
                                   int OW, int KH, int KW, int sh, int sw, int ph, int pw, hipStream_t stream) {
  if (C % 8 || KH * KW > 256 || ph >= KH || pw >= KW) return (int)hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw};
  const long total = (long)N * OH * OW * (C / 8);
  const unsigned grid = (unsigned)std::min((total + 255) / 256, 8192L);
  PHA_DISPATCH_T(dt, T, {
    if (total * 8 < (1L << 31))   // 32-bit walk (element offsets i * 8 included)
      hipLaunchKernelGGL((maxpool_fwd_kernel<T, unsigned>), dim3(grid), dim3(256), 0, stream, (const T*)x, (T*)y, idx, g);
    else
      hipLaunchKernelGGL((maxpool_fwd_kernel<T, long>), dim3(grid), dim3(256), 0, stream, (const T*)x, (T*)y, idx, g);
  });
  return (int)hipGetLastError();
}

PHA_API int pha_maxpool2d_nhwc_bwd(int dt, const void* gy, const uint8_t* idx, void* gx, int N, int H, int W, int C,
                                   int OH, int OW, int KH, int KW, int sh, int sw, int ph, int pw, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  PoolGeo g{N, H, W, C, OH, OW, KH, KW, sh, sw, ph, pw};
  const long total = (long)N * H * W * (C / 8);
  const unsigned grid = (unsigned)std::min((total + 255) / 256, 8192L);
  PHA_DISPATCH_T(dt, T, {
    if (total * 8 < (1L << 31))
      hipLaunchKernelGGL((maxpool_bwd_kernel<T, unsigned>), dim3(grid), dim3(256), 0, stream, (const T*)gy, idx, (T*)gx, g);
    else
      hipLaunchKernelGGL((maxpool_bwd_kernel<T, long>), dim3(grid), dim3(256), 0, stream, (const T*)gy, idx, (T*)gx, g);
  });
  return (int)hipGetLastError();
}

// out[i] = sum_z ws[z][i] in chunk order (4 per thread)
template <typename T>
__global__ __launch_bounds__(256) void chunk_sum_kernel(const float* __restrict__ ws, T* __restrict__ out, int Z, long len) {
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i < len; i += (long)gridDim.x * 1024) {
    float4 s = *reinterpret_cast<const float4*>(ws + i);
    for (int z = 1; z < Z; ++z) {
      const float4 v = *reinterpret_cast<const float4*>(ws + (long)z * len + i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    Cvt<T>::st(out + i, 0, s.x);
    Cvt<T>::st(out + i, 1, s.y);
    Cvt<T>::st(out + i, 2, s.z);
    Cvt<T>::st(out + i, 3, s.w);
  }
}

// gw [V][D] (T) = embedding gradient of gy [n][D] (T) for ids [n] (int64); padding row pad (or -1).
// chunks > 1: token ranges of ceil(n / chunks) per grid.z slice with fp32 partials in ws
// ([chunks][V][D] floats), summed in order into gw.
PHA_API int pha_embedding_bwd(int dt, const int64_t* ids, const void* gy, void* gw, long n, int D, long V, long pad,
                              hipStream_t stream, int chunks, float* ws) {
  if (n <= 0 || D <= 0 || V <= 0) return (int)hipErrorInvalidValue;
  if (D % 4 || n >= (1L << 26)) return (int)hipErrorInvalidValue;
  if (chunks < 1 || (chunks > 1 && !ws) || chunks > 65535) return (int)hipErrorInvalidValue;
  const long chunk = (n + chunks - 1) / chunks;
  const dim3 grid((unsigned)((V + EB_ROWS - 1) / EB_ROWS), (unsigned)((D + EB_DCH - 1) / EB_DCH), (unsigned)chunks);
  const size_t lds = (size_t)EB_ROWS * EB_DCH * 4 + EB_CAP * 4 + 16;
  PHA_DISPATCH_T(dt, T, {
    static bool attr = false;
    if (!attr) {
      hipFuncSetAttribute((const void*)embedding_bwd_kernel<T>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    hipLaunchKernelGGL(embedding_bwd_kernel<T>, grid, dim3(256), lds, stream, ids, (const T*)gy, (T*)gw, n, D, V, pad,
                       chunk, chunks > 1 ? ws : nullptr);
    if (chunks > 1) {
      const long len = V * (long)D;
      const unsigned g = (unsigned)std::min((len / 4 + 255) / 256, 8192L);
      hipLaunchKernelGGL(chunk_sum_kernel<T>, dim3(g), dim3(256), 0, stream, ws, (T*)gw, chunks, len);
    }
  });
  return (int)hipGetLastError();
}

PHA_API int pha_embedding_fwd(const int64_t* ids, const void* w, void* out, long rows, int row_bytes, long vocab, hipStream_t stream) {
  if (row_bytes % 16) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, ids, (const uint4*)w, (uint4*)out, rows, row_bytes / 16, vocab);
  return (int)hipGetLastError();
}

// hipGraph-safe dropout seeds (ops/hip.dropout_seed): ++counter and a copy of the new value for one
// dropout site in ONE launch (was an in-place add plus a clone: two tiny kernels per site and
// replay, ~10 us of a BERT-base step each)
namespace {
__global__ void seed_bump_kernel(int* __restrict__ counter, int* __restrict__ out) {
  if (threadIdx.x == 0) {
    const int v = counter[0] + 1;
    counter[0] = v;
    out[0] = v;
  }
}
}  // namespace

PHA_API int pha_seed_bump(int* counter, int* out, hipStream_t stream) {
  if (!counter || !out) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(seed_bump_kernel, dim3(1), dim3(64), 0, stream, counter, out);
  return (int)hipGetLastError();
}
