// LayerNorm (fwd/bwd) and row softmax (fwd/bwd) for gfx950.
//
// Design: one wave64 per row. A row of H elements is split into NCH chunks of
// 512 (64 lanes x 8 elements, one 16-byte vector per lane per chunk), held in
// registers between the statistics pass and the output pass, so every element
// is read from HBM exactly once and written once (memory-bound ops: the roof is
// HBM bandwidth, Appendix B of the CDNA guide). 4 waves (4 rows) per 256-thread
// block. Statistics in fp32, two-pass (exact) mean/variance from registers.
//
// Reference behaviour: paddle/phi/kernels/gpu/layer_norm_kernel.cu,
// layer_norm_grad_kernel.cu, softmax_kernel.cu / gpudnn/softmax_gpudnn.h.
#include <stdlib.h>
#include <type_traits>

#include "common.h"

using namespace pha;

namespace {

constexpr int kWaves = 4;

// counter-based dropout mask of the fused bias-dropout-residual-LN (fused_bias_dropout_residual_
// layer_norm): element idx = row * H + col keeps iff a 16-bit hash of (seed, idx) >= thresh, so the
// backward regenerates exactly the forward's mask and no mask tensor is stored.
// keep bits (bit i: element idx0 + i) of the 8 elements idx0 .. idx0 + 7 (idx0 % 8 == 0) that one
// lane's 16-B vector covers: ONE murmur finalizer per element pair, the low / high 16 bits are the
// even / odd element's draw. Two 32-bit multiplies per pair instead of four per element (a
// wave64 v_mul_lo_u32 is 16 cycles: the per-element double hash made the BDRLN passes VALU-bound)
__device__ __forceinline__ unsigned bd_keep8(unsigned seed, long idx0, unsigned thresh) {
  const unsigned s = seed ^ ((unsigned)(idx0 >> 33) * 0x85ebca6bU);
  const unsigned p0 = (unsigned)(idx0 >> 1) * 0x9e3779b1U;
  unsigned bits = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    unsigned x = s ^ (p0 + (unsigned)j * 0x9e3779b1U);
    x ^= x >> 16;
    x *= 0x85ebca6bU;
    x ^= x >> 13;
    x *= 0xc2b2ae35U;
    x ^= x >> 16;
    bits |= ((x & 0xffffU) >= thresh ? 1u : 0u) << (2 * j);
    bits |= ((x >> 16) >= thresh ? 1u : 0u) << (2 * j + 1);
  }
  return bits;
}

struct BdArgs {            // x -> dropout(x + xb) before the residual add (thresh 0: no dropout)
  const void* xb;          // [H] bias of x (fp32 when xb_f32, else type T), may be null
  unsigned seed, thresh;
  float kscale;
  int xb_f32;
  const unsigned* seedp;   // hipGraph replays: device word xor-ed into seed (null: seed alone)
};

__device__ __forceinline__ unsigned bd_seed(const BdArgs& bd) { return bd.seedp ? bd.seed ^ *bd.seedp : bd.seed; }

template <typename T, typename W, int NCH>
// With `r` set: the pre-LN residual add is fused in — hs = x + r (rounded to T, exactly what
// a separate add would store) is written out and normalised, saving one full read+write pass.
__global__ __launch_bounds__(256) void ln_fwd_kernel(const T* __restrict__ x, const W* __restrict__ w,
                                                     const W* __restrict__ b, T* __restrict__ y,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                     int rows, int H, float eps, const T* __restrict__ r = nullptr,
                                                     T* __restrict__ hs = nullptr, BdArgs bd = BdArgs{nullptr, 0u, 0u, 1.f, 0}) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (long)row * H;
  float v[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
      Vec8<T>::ld(xr + col, v[c]);
      if (r) {
        float rv[8];
        Vec8<T>::ld(r + (long)row * H + col, rv);
        if (bd.xb || bd.thresh) {   // fused bias + dropout of x (rounded to T as a separate op would store)
          float bv[8];
          if (bd.xb) {
            if (bd.xb_f32) Vec8<float>::ld((const float*)bd.xb + col, bv);
            else Vec8<T>::ld((const T*)bd.xb + col, bv);
          }
          const unsigned kb = bd.thresh ? bd_keep8(bd_seed(bd), (long)row * H + col, bd.thresh) : 0xffu;
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            float z = round_to<T>(v[c][i] + (bd.xb ? bv[i] : 0.f));
            if (bd.thresh) z = ((kb >> i) & 1u) ? round_to<T>(z * bd.kscale) : 0.f;
            v[c][i] = z;
          }
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) v[c][i] = round_to<T>(v[c][i] + rv[i]);  // stats on the stored sum
        Vec8<T>::st(hs + (long)row * H + col, v[c]);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = 0.f;
    }
  }
  const float mu = wave_sum(s) / H;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { float d = v[c][i] - mu; ss += d * d; }
    }
  }
  const float rs = rsqrtf(wave_sum(ss) / H + eps);
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
  T* yr = y + (long)row * H;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
      float wv[8], bv[8], o[8];
      Vec8<W>::ld(w + col, wv);
      if (b) Vec8<W>::ld(b + col, bv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * rs * wv[i] + (b ? bv[i] : 0.f);
      Vec8<T>::st(yr + col, o);
    }
  }
}

// dx per row + per-block partial column sums of dy*xhat (dw) and dy (db).
// 8 elements held as their raw vector(s) (16 B for bf16 / fp16, 32 B for fp32), unpacked on use
template <typename T>
struct Raw8 {
  uint4 v;
  __device__ __forceinline__ void ld(const T* p) { v = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void unpack(float (&o)[8]) const { Vec8<T>::unpack(v, o); }
};
template <>
struct Raw8<float> {
  float4 a, b;
  __device__ __forceinline__ void ld(const float* p) {
    a = *reinterpret_cast<const float4*>(p);
    b = *reinterpret_cast<const float4*>(p + 4);
  }
  __device__ __forceinline__ void unpack(float (&o)[8]) const {
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
};

// BW waves per block (16 -> 1024 threads): a grid of one block per CU then still gives 4
// waves per SIMD to hide HBM latency, while the dw/db partials stay one [H] row per block.
// XS: also per-block partial column sums of the final dx (part_x) — the bias gradient of a linear
// layer whose output entered the residual sum (its bias folded into the add-LN forward), so that
// layer's backward needs no separate column-sum pass over the same gradient
// DRP: the fused bias-dropout-residual-LN backward in one pass — besides dx (= d residual) it writes
// dxd = dropout'(dx): the regenerated keep mask (bd_keep) times kscale on dx rounded to T, exactly
// what dropout_bias_bwd_kernel computes from the stored dx, without re-reading it
template <typename T, typename W, int NCH, int BW, bool XS = false, bool DRP = false>
__global__ __launch_bounds__(BW * 64) __attribute__((amdgpu_waves_per_eu(NCH <= 3 ? 4 : NCH <= 4 ? 2 : 1))) void ln_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const W* __restrict__ w, const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, T* __restrict__ dx,
                                                         float* __restrict__ part_w, float* __restrict__ part_b,
                                                         int rows, int H, const T* __restrict__ dres,
                                                         float* __restrict__ part_x = nullptr,
                                                         T* __restrict__ dxd = nullptr,
                                                         BdArgs bd = BdArgs{nullptr, 0u, 0u, 1.f, 0}) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const unsigned dseed = DRP ? bd_seed(bd) : 0u;
  // dropout' of the finished dx of (row, col .. col + 7)
  auto drop_store = [&](int row, int col, const float (&o)[8]) {
    float g[8];
    const unsigned kb = bd_keep8(dseed, (long)row * H + col, bd.thresh);
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = ((kb >> i) & 1u) ? round_to<T>(o[i]) * bd.kscale : 0.f;
    Vec8<T>::st(dxd + (long)row * H + col, g);
  };
  float aw[NCH][8], ab[NCH][8], ax[XS ? NCH : 1][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      aw[c][i] = 0.f;
      ab[c][i] = 0.f;
      if constexpr (XS) ax[c][i] = 0.f;
    }

  // H = 1537..2048 (NCH 4, the GPT-1.3B width): one HBM round trip per row with x / dy / dres held
  // raw in registers (2 waves per SIMD, no spills); other widths re-read x and dy in pass 2
  if constexpr (NCH == 4) {
  for (int row = blockIdx.x * BW + wid; row < rows; row += gridDim.x * BW) {
    const float mu = mean[row], rs = rstd[row];
    const T* xr = x + (long)row * H;
    const T* gr = dy + (long)row * H;
    // one HBM round trip per row: x, dy (and the residual gradient) are loaded once, kept as raw
    // 16-B vectors and unpacked again for pass 2 (no second read, no dependent dres load)
    Raw8<T> rx[NCH], rg[NCH], rr[NCH];
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < H) {
        rx[c].ld(xr + col);
        rg[c].ld(gr + col);
        if (!XS && dres) rr[c].ld(dres + (long)row * H + col);   // XS: re-read in pass 2 (registers)
      }
    }
    // pass 1: row statistics of g = dy*w
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < H) {
        float xv[8], gv[8], wv[8];
        rx[c].unpack(xv);
        rg[c].unpack(gv);
        Vec8<W>::ld(w + col, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float g = gv[i] * wv[i];
          s1 += g * (xv[i] - mu) * rs;
          s2 += g;
        }
      }
    }
    const float c1 = wave_sum(s1) / H, c2 = wave_sum(s2) / H;
    T* dr = dx + (long)row * H;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < H) {
        float xv[8], gv[8], wv[8], o[8];
        rx[c].unpack(xv);
        rg[c].unpack(gv);
        Vec8<W>::ld(w + col, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xh = (xv[i] - mu) * rs;
          o[i] = rs * (gv[i] * wv[i] - xh * c1 - c2);
          aw[c][i] += gv[i] * xh;
          ab[c][i] += gv[i];
        }
        if (dres) {  // fused residual branch: dx += d(sum output)
          float rv[8];
          if constexpr (XS) Vec8<T>::ld(dres + (long)row * H + col, rv);
          else rr[c].unpack(rv);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += rv[i];
        }
        if constexpr (XS) {
#pragma unroll
          for (int i = 0; i < 8; ++i) ax[c][i] += round_to<T>(o[i]);   // the stored gradient's sum
        }
        if constexpr (DRP) drop_store(row, col, o);
        Vec8<T>::st(dr + col, o);
      }
    }
  }
  } else {
  for (int row = blockIdx.x * BW + wid; row < rows; row += gridDim.x * BW) {
    const float mu = mean[row], rs = rstd[row];
    const T* xr = x + (long)row * H;
    const T* gr = dy + (long)row * H;
    // pass 1: row statistics of g = dy*w (re-read in pass 2 from L1/L2 instead of
    // holding x and g in registers: keeps VGPRs for the dw/db accumulators)
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < H) {
        float xv[8], gv[8], wv[8];
        Vec8<T>::ld(xr + col, xv);
        Vec8<T>::ld(gr + col, gv);
        Vec8<W>::ld(w + col, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float g = gv[i] * wv[i];
          s1 += g * (xv[i] - mu) * rs;
          s2 += g;
        }
      }
    }
    const float c1 = wave_sum(s1) / H, c2 = wave_sum(s2) / H;
    T* dr = dx + (long)row * H;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < H) {
        float xv[8], gv[8], wv[8], o[8];
        Vec8<T>::ld(xr + col, xv);
        Vec8<T>::ld(gr + col, gv);
        Vec8<W>::ld(w + col, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xh = (xv[i] - mu) * rs;
          o[i] = rs * (gv[i] * wv[i] - xh * c1 - c2);
          aw[c][i] += gv[i] * xh;
          ab[c][i] += gv[i];
        }
        if (dres) {  // fused residual branch: dx += d(sum output)
          float rv[8];
          Vec8<T>::ld(dres + (long)row * H + col, rv);
#pragma unroll
          for (int i = 0; i < 8; ++i) o[i] += rv[i];
        }
        if constexpr (XS) {
#pragma unroll
          for (int i = 0; i < 8; ++i) ax[c][i] += round_to<T>(o[i]);   // the stored gradient's sum
        }
        if constexpr (DRP) drop_store(row, col, o);
        Vec8<T>::st(dr + col, o);
      }
    }
  }
  }
  // block reduction of the BW waves' partial column sums through LDS, one column chunk at a time
  __shared__ float red[BW][512];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    for (int pass = 0; pass < (XS ? 3 : 2); ++pass) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        float v = pass == 0 ? aw[c][i] : ab[c][i];
        if constexpr (XS) v = pass == 2 ? ax[c][i] : v;
        red[wid][lane * 8 + i] = v;
      }
      __syncthreads();
      for (int k = threadIdx.x; k < 512; k += BW * 64) {
        const int cc = c * 512 + k;
        if (cc < H) {
          float t = 0.f;
#pragma unroll
          for (int q = 0; q < BW; ++q) t += red[q][k];
          float* dst = pass == 0 ? part_w : pass == 1 ? part_b : part_x;
          dst[(long)blockIdx.x * H + cc] = t;
        }
      }
      __syncthreads();
    }
  }
}

// sum partials [P, H] over P -> out [H] (cast to W). 64 columns per block (one per lane, so
// every row read is a coalesced 256-B segment), the 4 waves split the P rows.
// first stage of the [P, H] column sum: grid (H/64, kColSplit) so the whole chip streams the
// partials (one 64-column stripe per block would leave 224 of 256 CUs idle at H = 2048)
constexpr int kColSplit = 8;
__global__ __launch_bounds__(256) void col_partial_kernel(const float* __restrict__ part, float* __restrict__ out,
                                                          int P, int H) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int chunk = (P + kColSplit - 1) / kColSplit;
  const int p0 = blockIdx.y * chunk, p1 = min(P, p0 + chunk);
  float s = 0.f;
  if (col < H)
#pragma unroll 4
    for (int p = p0 + w; p < p1; p += 4) s += part[(long)p * H + col];
  __shared__ float red[4][64];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < H) out[(long)blockIdx.y * H + col] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

template <typename W>
__global__ __launch_bounds__(256) void col_reduce_kernel(const float* __restrict__ part, W* __restrict__ out, int P, int H) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < H)
    for (int p = w; p < P; p += 4) s += part[(long)p * H + col];
  __shared__ float red[4][64];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < H) Cvt<W>::st(out, col, red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

// backward of x -> dropout(x + xb): dx = dh * keep * kscale (the regenerated mask), per-block
// partial column sums of dx (the bias gradient) as in ln_bwd_kernel. BW waves per block.
template <typename T, int NCH, int BW>
__global__ __launch_bounds__(BW * 64) void dropout_bias_bwd_kernel(const T* __restrict__ dh, T* __restrict__ dx,
                                                                   float* __restrict__ part, int rows, int H,
                                                                   unsigned seed, unsigned thresh, float kscale,
                                                                   const unsigned* __restrict__ seedp) {
  if (seedp) seed ^= *seedp;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float acc[NCH][8];
#pragma unroll
  for (int c = 0; c < NCH; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[c][i] = 0.f;
  // rows strided over the grid, the next row's loads issued before this row's hash / store work
  // (one HBM round trip per row in flight behind the VALU instead of a stall per row)
  const int stride = gridDim.x * BW;
  int row = blockIdx.x * BW + wid;
  Raw8<T> cur[NCH];
  auto load = [&](int r, Raw8<T>(&dst)[NCH]) {
#pragma unroll
    for (int c = 0; c < NCH; ++c)
      if (c * 512 + lane * 8 < H) dst[c].ld(dh + (long)r * H + c * 512 + lane * 8);
  };
  if (row < rows) load(row, cur);
  for (; row < rows; row += stride) {
    Raw8<T> nxt[NCH];
    if (row + stride < rows) load(row + stride, nxt);
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int col = c * 512 + lane * 8;
      if (col < H) {
        float g[8];
        cur[c].unpack(g);
        const unsigned kb = thresh ? bd_keep8(seed, (long)row * H + col, thresh) : 0xffu;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          g[i] = ((kb >> i) & 1u) ? g[i] * kscale : 0.f;
          acc[c][i] += round_to<T>(g[i]);
        }
        Vec8<T>::st(dx + (long)row * H + col, g);
      }
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) cur[c] = nxt[c];
  }
  __shared__ float red[BW][512];
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[wid][lane * 8 + i] = acc[c][i];
    __syncthreads();
    for (int k = threadIdx.x; k < 512; k += BW * 64) {
      const int cc = c * 512 + k;
      if (cc < H) {
        float t = 0.f;
#pragma unroll
        for (int q = 0; q < BW; ++q) t += red[q][k];
        part[(long)blockIdx.x * H + cc] = t;
      }
    }
    __syncthreads();
  }
}

template <typename T, int NCH>
__global__ __launch_bounds__(256) void softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int rows, int H) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (long)row * H;
  float v[NCH][8];
  float m = -INFINITY;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
      Vec8<T>::ld(xr + col, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) m = fmaxf(m, v[c][i]);
    }
  }
  m = wave_max(m);
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
#pragma unroll
      for (int i = 0; i < 8; ++i) { v[c][i] = __expf(v[c][i] - m); s += v[c][i]; }
    }
  }
  const float inv = 1.f / wave_sum(s);
  T* yr = y + (long)row * H;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[c][i] * inv;
      Vec8<T>::st(yr + col, o);
    }
  }
}

template <typename T, int NCH>
__global__ __launch_bounds__(256) void softmax_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ y, T* __restrict__ dx, int rows, int H) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (row >= rows) return;
  float yv[NCH][8], gv[NCH][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
      Vec8<T>::ld(y + (long)row * H + col, yv[c]);
      Vec8<T>::ld(dy + (long)row * H + col, gv[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += yv[c][i] * gv[c][i];
    }
  }
  s = wave_sum(s);
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const int col = c * 512 + lane * 8;
    if (col < H) {
      float o[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = yv[c][i] * (gv[c][i] - s);
      Vec8<T>::st(dx + (long)row * H + col, o);
    }
  }
}

template <typename F>
int dispatch_nch_small(int H, F&& f) {
  const int n = (H + 511) / 512;
  switch (n) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: case 6: f(std::integral_constant<int, 6>{}); break;
    case 7: case 8: f(std::integral_constant<int, 8>{}); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

template <typename F>
int dispatch_nch(int H, F&& f) {
  const int n = (H + 511) / 512;
  switch (n) {
    case 1: f(std::integral_constant<int, 1>{}); break;
    case 2: f(std::integral_constant<int, 2>{}); break;
    case 3: f(std::integral_constant<int, 3>{}); break;
    case 4: f(std::integral_constant<int, 4>{}); break;
    case 5: case 6: f(std::integral_constant<int, 6>{}); break;
    case 7: case 8: f(std::integral_constant<int, 8>{}); break;
    case 9: case 10: case 11: case 12: f(std::integral_constant<int, 12>{}); break;
    case 13: case 14: case 15: case 16: f(std::integral_constant<int, 16>{}); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace

// r / hs (optional, both or neither): fused residual add, hs = x + r is normalised and stored.
PHA_API int pha_layer_norm_fwd2(int dt, int wdt, const void* x, const void* r, void* hs, const void* w, const void* b,
                                void* y, float* mean, float* rstd, int rows, int H, float eps, hipStream_t stream) {
  if (H % 8 || rows <= 0 || (!r) != (!hs)) return (int)hipErrorInvalidValue;
  const dim3 grid((rows + kWaves - 1) / kWaves), block(256);
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    if (wdt == kF32) {
      rc = dispatch_nch(H, [&](auto nch) {
        hipLaunchKernelGGL((ln_fwd_kernel<T, float, decltype(nch)::value>), grid, block, 0, stream,
                           (const T*)x, (const float*)w, (const float*)b, (T*)y, mean, rstd, rows, H, eps,
                           (const T*)r, (T*)hs);
      });
    } else {
      rc = dispatch_nch(H, [&](auto nch) {
        hipLaunchKernelGGL((ln_fwd_kernel<T, T, decltype(nch)::value>), grid, block, 0, stream,
                           (const T*)x, (const T*)w, (const T*)b, (T*)y, mean, rstd, rows, H, eps,
                           (const T*)r, (T*)hs);
      });
    }
  });
  return rc;
}

// waves per block of the LN backward: 16 while the dw/db accumulators fit the 128-VGPR
// budget of 4 waves/SIMD (H <= 1536), 8 above (two blocks per CU).
constexpr int bwd_waves(int nch) { return nch <= 3 ? 16 : 8; }

PHA_API int pha_layer_norm_bwd_nblocks(int rows, int H) {
  const int bw = bwd_waves((H + 511) / 512);
  const int cap = bw == 16 ? 256 : 512;
  const int need = (rows + bw - 1) / bw;
  return need < cap ? need : cap;
}

// fused_bias_dropout_residual_layer_norm forward: hs = r + dropout(x + xb) (stored), y = LN(hs).
// thresh = round(p * 65536) (0: no dropout), kscale = 1 / (1 - p).
// xbdt: dtype of xb (fp32 or the activation type)
PHA_API int pha_bdrln_fwd2(int dt, int wdt, int xbdt, const void* x, const void* xb, const void* r, void* hs,
                           const void* w, const void* b, void* y, float* mean, float* rstd, int rows, int H, float eps,
                           unsigned seed, unsigned thresh, float kscale, hipStream_t stream, const unsigned* seedp) {
  if (H % 8 || rows <= 0 || !r || !hs) return (int)hipErrorInvalidValue;
  if (xb && xbdt != kF32 && xbdt != dt) return (int)hipErrorInvalidValue;
  const dim3 grid((rows + kWaves - 1) / kWaves), block(256);
  const BdArgs bd{xb, seed, thresh, kscale, xbdt == kF32 ? 1 : 0, seedp};
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    if (wdt == kF32) {
      rc = dispatch_nch(H, [&](auto nch) {
        hipLaunchKernelGGL((ln_fwd_kernel<T, float, decltype(nch)::value>), grid, block, 0, stream,
                           (const T*)x, (const float*)w, (const float*)b, (T*)y, mean, rstd, rows, H, eps,
                           (const T*)r, (T*)hs, bd);
      });
    } else {
      rc = dispatch_nch(H, [&](auto nch) {
        hipLaunchKernelGGL((ln_fwd_kernel<T, T, decltype(nch)::value>), grid, block, 0, stream,
                           (const T*)x, (const T*)w, (const T*)b, (T*)y, mean, rstd, rows, H, eps,
                           (const T*)r, (T*)hs, bd);
      });
    }
  });
  return rc;
}

PHA_API int pha_bdrln_fwd(int dt, int wdt, const void* x, const void* xb, const void* r, void* hs, const void* w,
                          const void* b, void* y, float* mean, float* rstd, int rows, int H, float eps, unsigned seed,
                          unsigned thresh, float kscale, hipStream_t stream) {
  return pha_bdrln_fwd2(dt, wdt, wdt, x, xb, r, hs, w, b, y, mean, rstd, rows, H, eps, seed, thresh, kscale, stream,
                        nullptr);
}

PHA_API int pha_layer_norm_fwd(int dt, int wdt, const void* x, const void* w, const void* b, void* y,
                               float* mean, float* rstd, int rows, int H, float eps, hipStream_t stream) {
  return pha_layer_norm_fwd2(dt, wdt, x, nullptr, nullptr, w, b, y, mean, rstd, rows, H, eps, stream);
}

// single-launch column sums of up to three [P, H] fp32 partial arrays (blockIdx.y picks the array):
// 16 waves per 64-column stripe split the P rows, so each wave has at most P / 16 independent
// loads in flight (one HBM / L2 round trip or two at P = 256) and a backward's weight, bias and
// residual-bias gradients finish in ONE short launch instead of two per array (each tiny launch
// costs ~4.5 us of the BERT-base step, 17 of them per layer)
struct ColSumJob {
  const float* part[3];
  void* out[3];
  int f32[3];   // output fp32 (else the activation type T)
};
constexpr int kColSum1MaxP = 1024;
// PHA_COLSUM1=0: the two-launch-per-array path (A/B switch), read once
inline bool colsum1_on() {
  static const bool on = [] {
    const char* e = getenv("PHA_COLSUM1");
    return !(e && e[0] == '0');
  }();
  return on;
}
template <typename T>
__global__ __launch_bounds__(1024) void col_sum_n_kernel(ColSumJob job, int P, int H) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, j = blockIdx.y;
  const float* part = j == 0 ? job.part[0] : j == 1 ? job.part[1] : job.part[2];
  const int col = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (col < H)
#pragma unroll 8
    for (int p = w; p < P; p += 16) s += part[(long)p * H + col];
  __shared__ float red[16][64];
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && col < H) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][lane];
    void* out = j == 0 ? job.out[0] : j == 1 ? job.out[1] : job.out[2];
    const int f32 = j == 0 ? job.f32[0] : j == 1 ? job.f32[1] : job.f32[2];
    if (f32) static_cast<float*>(out)[col] = t;
    else Cvt<T>::st(static_cast<T*>(out), col, t);
  }
}
template <typename T>
void col_sum_n(const ColSumJob& job, int n, int P, int H, hipStream_t stream) {
  hipLaunchKernelGGL((col_sum_n_kernel<T>), dim3((H + 63) / 64, n), dim3(1024), 0, stream, job, P, H);
}

// column sums of the [P, H] partials into out: P <= kColSum1MaxP in one launch; larger P through
// the chip-wide first stage into rows [P, P + kColSplit) of the same workspace
template <typename W>
void col_sum(float* part, W* out, int P, int H, hipStream_t stream) {
  if (P <= kColSum1MaxP && colsum1_on()) {
    ColSumJob job{{part, nullptr, nullptr}, {out, nullptr, nullptr}, {std::is_same<W, float>::value ? 1 : 0, 0, 0}};
    col_sum_n<W>(job, 1, P, H, stream);
  } else if (P > 4 * kColSplit) {
    float* stage = part + (long)P * H;
    hipLaunchKernelGGL(col_partial_kernel, dim3((H + 63) / 64, kColSplit), dim3(256), 0, stream, part, stage, P, H);
    hipLaunchKernelGGL((col_reduce_kernel<W>), dim3((H + 63) / 64), dim3(256), 0, stream, stage, out, kColSplit, H);
  } else {
    hipLaunchKernelGGL((col_reduce_kernel<W>), dim3((H + 63) / 64), dim3(256), 0, stream, part, out, P, H);
  }
}

// the LN backward's dw (+ db, + dxs) column sums: one launch for all of them while P is small.
// wf32 / xf32: dw, db / dxs are fp32 (else T)
template <typename T>
void col_sum_wbx(float* pw, void* dw, float* pb, void* db, float* px, void* dxs, bool wf32, bool xf32, int P, int H,
                 hipStream_t stream) {
  if (P <= kColSum1MaxP && colsum1_on()) {
    ColSumJob job{{pw, nullptr, nullptr}, {dw, nullptr, nullptr}, {wf32, 0, 0}};
    int n = 1;
    if (db) { job.part[n] = pb; job.out[n] = db; job.f32[n] = wf32; ++n; }
    if (dxs) { job.part[n] = px; job.out[n] = dxs; job.f32[n] = xf32; ++n; }
    col_sum_n<T>(job, n, P, H, stream);
    return;
  }
  if (wf32) col_sum<float>(pw, (float*)dw, P, H, stream);
  else col_sum<T>(pw, (T*)dw, P, H, stream);
  if (db) {
    if (wf32) col_sum<float>(pb, (float*)db, P, H, stream);
    else col_sum<T>(pb, (T*)db, P, H, stream);
  }
  if (dxs) {
    if (xf32) col_sum<float>(px, (float*)dxs, P, H, stream);
    else col_sum<T>(px, (T*)dxs, P, H, stream);
  }
}

// [P, H] fp32 row partials -> [H] column sums in dt (a bias gradient's last step); part needs
// P + 8 rows (the chip-wide first stage writes rows [P, P + 8))
PHA_API int pha_col_sum_rows(int dt, float* part, void* out, int P, int H, hipStream_t stream) {
  if (P <= 0 || H <= 0) return (int)hipErrorInvalidValue;
  if (dt == kF32) col_sum<float>(part, (float*)out, P, H, stream);
  else if (dt == kBF16) col_sum<bf16_t>(part, (bf16_t*)out, P, H, stream);
  else if (dt == kF16) col_sum<half_t>(part, (half_t*)out, P, H, stream);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

// part_w / part_b: workspace [nblocks + 8, H] fp32 each (nblocks = pha_layer_norm_bwd_nblocks;
// the last 8 rows are the column-sum stage);
// dw/db outputs (may be null db); dres (optional): gradient of the fused residual sum, added to dx.
PHA_API int pha_layer_norm_bwd2(int dt, int wdt, const void* dy, const void* x, const void* w, const float* mean,
                                const float* rstd, const void* dres, void* dx, void* dw, void* db, float* part_w,
                                float* part_b, int nblocks, int rows, int H, hipStream_t stream) {
  if (H % 8 || rows <= 0 || nblocks <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid(nblocks);
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    if (wdt == kF32) {
      rc = dispatch_nch_small(H, [&](auto nch) {
        hipLaunchKernelGGL((ln_bwd_kernel<T, float, decltype(nch)::value, bwd_waves(decltype(nch)::value)>), grid, dim3(bwd_waves(decltype(nch)::value) * 64), 0, stream,
                           (const T*)dy, (const T*)x, (const float*)w, mean, rstd, (T*)dx, part_w, part_b, rows, H,
                           (const T*)dres);
      });
      if (rc) return rc;
      col_sum_wbx<T>(part_w, dw, part_b, db, nullptr, nullptr, true, true, nblocks, H, stream);
    } else {
      rc = dispatch_nch_small(H, [&](auto nch) {
        hipLaunchKernelGGL((ln_bwd_kernel<T, T, decltype(nch)::value, bwd_waves(decltype(nch)::value)>), grid, dim3(bwd_waves(decltype(nch)::value) * 64), 0, stream,
                           (const T*)dy, (const T*)x, (const T*)w, mean, rstd, (T*)dx, part_w, part_b, rows, H,
                           (const T*)dres);
      });
      if (rc) return rc;
      col_sum_wbx<T>(part_w, dw, part_b, db, nullptr, nullptr, false, false, nblocks, H, stream);
    }
  });
  return rc ? rc : (int)hipGetLastError();
}

// fused_bias_dropout_residual_layer_norm backward without the input bias: dx = LN'(dy) (the
// residual's gradient) and dxd = dropout'(dx) with the forward's mask (seed / thresh / kscale / seedp
// as pha_bdrln_fwd2) in one pass; dw / db as pha_layer_norm_bwd2
PHA_API int pha_layer_norm_dropout_bwd(int dt, int wdt, const void* dy, const void* x, const void* w,
                                       const float* mean, const float* rstd, void* dx, void* dxd, void* dw, void* db,
                                       float* part_w, float* part_b, int nblocks, int rows, int H, unsigned seed,
                                       unsigned thresh, float kscale, hipStream_t stream, const unsigned* seedp) {
  if (H % 8 || rows <= 0 || nblocks <= 0 || !dxd || thresh == 0) return (int)hipErrorInvalidValue;
  const dim3 grid(nblocks);
  const BdArgs bd{nullptr, seed, thresh, kscale, 0, seedp};
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    if (wdt == kF32) {
      rc = dispatch_nch_small(H, [&](auto nch) {
        constexpr int nc = decltype(nch)::value;
        hipLaunchKernelGGL((ln_bwd_kernel<T, float, nc, bwd_waves(nc), false, true>), grid, dim3(bwd_waves(nc) * 64),
                           0, stream, (const T*)dy, (const T*)x, (const float*)w, mean, rstd, (T*)dx, part_w, part_b,
                           rows, H, (const T*)nullptr, (float*)nullptr, (T*)dxd, bd);
      });
      if (rc) return rc;
      col_sum_wbx<T>(part_w, dw, part_b, db, nullptr, nullptr, true, true, nblocks, H, stream);
    } else {
      rc = dispatch_nch_small(H, [&](auto nch) {
        constexpr int nc = decltype(nch)::value;
        hipLaunchKernelGGL((ln_bwd_kernel<T, T, nc, bwd_waves(nc), false, true>), grid, dim3(bwd_waves(nc) * 64), 0,
                           stream, (const T*)dy, (const T*)x, (const T*)w, mean, rstd, (T*)dx, part_w, part_b, rows,
                           H, (const T*)nullptr, (float*)nullptr, (T*)dxd, bd);
      });
      if (rc) return rc;
      col_sum_wbx<T>(part_w, dw, part_b, db, nullptr, nullptr, false, false, nblocks, H, stream);
    }
  });
  return rc ? rc : (int)hipGetLastError();
}

// pha_layer_norm_bwd2 plus dxs = column sums of the final dx (type wdt; part_x: [nblocks + 8, H])
PHA_API int pha_layer_norm_bwd3(int dt, int wdt, int xsdt, const void* dy, const void* x, const void* w, const float* mean,
                                const float* rstd, const void* dres, void* dx, void* dw, void* db, void* dxs,
                                float* part_w, float* part_b, float* part_x, int nblocks, int rows, int H,
                                hipStream_t stream) {
  if (!dxs || !part_x)
    return pha_layer_norm_bwd2(dt, wdt, dy, x, w, mean, rstd, dres, dx, dw, db, part_w, part_b, nblocks, rows, H,
                               stream);
  if (H % 8 || rows <= 0 || nblocks <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid(nblocks);
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    if (wdt == kF32) {
      rc = dispatch_nch_small(H, [&](auto nch) {
        constexpr int N = decltype(nch)::value;
        hipLaunchKernelGGL((ln_bwd_kernel<T, float, N, bwd_waves(N), true>), grid, dim3(bwd_waves(N) * 64), 0, stream,
                           (const T*)dy, (const T*)x, (const float*)w, mean, rstd, (T*)dx, part_w, part_b, rows, H,
                           (const T*)dres, part_x);
      });
      if (rc) return rc;
      col_sum_wbx<T>(part_w, dw, part_b, db, part_x, dxs, true, xsdt == kF32, nblocks, H, stream);
    } else {
      rc = dispatch_nch_small(H, [&](auto nch) {
        constexpr int N = decltype(nch)::value;
        hipLaunchKernelGGL((ln_bwd_kernel<T, T, N, bwd_waves(N), true>), grid, dim3(bwd_waves(N) * 64), 0, stream,
                           (const T*)dy, (const T*)x, (const T*)w, mean, rstd, (T*)dx, part_w, part_b, rows, H,
                           (const T*)dres, part_x);
      });
      if (rc) return rc;
      col_sum_wbx<T>(part_w, dw, part_b, db, part_x, dxs, false, xsdt == kF32, nblocks, H, stream);
    }
  });
  return rc ? rc : (int)hipGetLastError();
}

PHA_API int pha_layer_norm_bwd(int dt, int wdt, const void* dy, const void* x, const void* w, const float* mean,
                               const float* rstd, void* dx, void* dw, void* db, float* part_w, float* part_b,
                               int nblocks, int rows, int H, hipStream_t stream) {
  return pha_layer_norm_bwd2(dt, wdt, dy, x, w, mean, rstd, nullptr, dx, dw, db, part_w, part_b, nblocks, rows, H,
                             stream);
}

// backward of the dropout(x + xb) branch: dx = dh * mask * kscale; dbias (type of wdt, may be null)
// = column sums of dx; part: workspace [nblocks + 8, H] fp32 (nblocks = pha_layer_norm_bwd_nblocks)
PHA_API int pha_dropout_bias_bwd(int dt, int wdt, const void* dh, void* dx, void* dbias, float* part, int nblocks,
                                 int rows, int H, unsigned seed, unsigned thresh, float kscale, hipStream_t stream,
                                 const unsigned* seedp) {
  if (H % 8 || rows <= 0 || nblocks <= 0) return (int)hipErrorInvalidValue;
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    rc = dispatch_nch_small(H, [&](auto nch) {
      constexpr int bw = bwd_waves(decltype(nch)::value);
      hipLaunchKernelGGL((dropout_bias_bwd_kernel<T, decltype(nch)::value, bw>), dim3(nblocks), dim3(bw * 64), 0,
                         stream, (const T*)dh, (T*)dx, part, rows, H, seed, thresh, kscale, seedp);
    });
    if (rc) return rc;
    if (dbias) {
      if (wdt == kF32) col_sum<float>(part, (float*)dbias, nblocks, H, stream);
      else col_sum<T>(part, (T*)dbias, nblocks, H, stream);
    }
  });
  return rc ? rc : (int)hipGetLastError();
}

PHA_API int pha_softmax_fwd(int dt, const void* x, void* y, int rows, int H, hipStream_t stream) {
  if (H % 8 || rows <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((rows + kWaves - 1) / kWaves), block(256);
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    rc = dispatch_nch(H, [&](auto nch) {
      hipLaunchKernelGGL((softmax_fwd_kernel<T, decltype(nch)::value>), grid, block, 0, stream, (const T*)x, (T*)y, rows, H);
    });
  });
  return rc;
}

PHA_API int pha_softmax_bwd(int dt, const void* dy, const void* y, void* dx, int rows, int H, hipStream_t stream) {
  if (H % 8 || rows <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((rows + kWaves - 1) / kWaves), block(256);
  int rc = 0;
  PHA_DISPATCH_T(dt, T, {
    rc = dispatch_nch(H, [&](auto nch) {
      hipLaunchKernelGGL((softmax_bwd_kernel<T, decltype(nch)::value>), grid, block, 0, stream, (const T*)dy, (const T*)y, (T*)dx, rows, H);
    });
  });
  return rc;
}
