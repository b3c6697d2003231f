// Fake-quantization kernels for quantization-aware training / post-training calibration on gfx950.
// Reference behaviour: paddle/fluid/operators/fake_quantize_op.cu.h (FindAbsMaxKernel,
// FindChannelAbsMaxKernelQuantAxis0/1, ClipAndQuant(Dequant)Kernel, ChannelClipAndQuantDequant
// KernelQuantAxis0/1, FindMovingAverageAbsMaxKernel) and fake_dequantize_op.cu.h.
//
//   scale      = max |x|                      (per tensor, or per channel of quant_axis)
//   bin        = 2^(bits-1) - 1
//   round_type 1 (default, TiesAwayFromZero):  q = round(bin * clip(x, -s, s) / s)
//   round_type 0 (TiesToEven):                 q = clip(rint(bin * x / s), -bin - 1, bin)
//   quant-dequant: out = q * s / bin;  quant only: out = q
//   1/s is inverse(s) = s <= 1e-30 ? 1 / (s + 1e-6) : 1 / s (all-zero input quantizes to 0)
//
// MI355X design. The reductions read 8 elements per lane in 16-B vectors (fp32: two), reduce a
// wave with DPP shuffles and a workgroup through LDS, and publish the maximum of non-negative
// floats with an integer atomic max on its bit pattern (order independent, so deterministic).
// Per-channel scales for a channel axis with unit inner stride (Linear weights [in, out] at
// quant_axis = 1) are column reductions: a lane owns one column and walks the rows, so the loads
// of a wave are 64 consecutive columns (coalesced) instead of one strided channel per workgroup.
// The elementwise pass is one streaming read + write (HBM-bound).
#include "common.h"
#include <type_traits>

namespace pha {
namespace {

__device__ __forceinline__ float inv_scale(float s) { return s <= 1e-30f ? 1.f / (s + 1e-6f) : 1.f / s; }

__device__ __forceinline__ float qfun(float x, float s, float inv_s, float bin, int round_type) {
  if (round_type == 0) {
    float v = rintf(bin * inv_s * x);
    return fminf(fmaxf(v, -bin - 1.f), bin);
  }
  float v = fminf(fmaxf(x, -s), s);
  return roundf(bin * inv_s * v);
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, long i, long n, float (&v)[8]) {
  if (i + 8 <= n) {
    if constexpr (sizeof(T) == 2) {
      Vec8<T>::ld(p + i, v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = Cvt<T>::ld(p, i + e);
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (i + e < n) ? Cvt<T>::ld(p, i + e) : 0.f;
  }
}

// per-tensor abs max -> *out (caller zeroes it); grid-stride, 8 elements per lane and step
template <typename T>
__global__ __launch_bounds__(256) void absmax_kernel(const T* __restrict__ x, long n, unsigned* __restrict__ out) {
  __shared__ float red[4];
  float m = 0.f;
  const long stride = (long)gridDim.x * 256 * 8;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    float v[8];
    ld8<T>(x, i, n, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(v[e]));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
    atomicMax(out, __float_as_uint(m));   // non-negative floats order like their bit patterns
  }
}

// channel abs max, x viewed as [outer, C, inner] (channel = quant axis): one workgroup per channel
template <typename T>
__global__ __launch_bounds__(256) void chmax_kernel(const T* __restrict__ x, long outer, long C, long inner,
                                                    float* __restrict__ out) {
  __shared__ float red[4];
  const long c = blockIdx.x;
  float m = 0.f;
  const long per = outer * inner;
  for (long t = threadIdx.x; t < per; t += 256) {
    const long o = t / inner, k = t - o * inner;
    m = fmaxf(m, fabsf(Cvt<T>::ld(x, (o * C + c) * inner + k)));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) out[c] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// inner == 1: column max of [outer, C]; a lane owns a column, a workgroup 256 columns x a row slab;
// slabs combine through the bit-pattern atomic max (caller zeroes out)
template <typename T>
__global__ __launch_bounds__(256) void colmax_kernel(const T* __restrict__ x, long rows, long C, long rows_per,
                                                     unsigned* __restrict__ out) {
  const long c = (long)blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  const long r0 = (long)blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  float m = 0.f;
  for (long r = r0; r < r1; ++r) m = fmaxf(m, fabsf(Cvt<T>::ld(x, r * C + c)));
  atomicMax(out + c, __float_as_uint(m));
}

// out = q(x) (DEQ: * s / bin); scale per tensor (C == 1) or per channel of [outer, C, inner]
template <typename T, typename O, bool DEQ>
__global__ __launch_bounds__(256) void qdq_kernel(const T* __restrict__ x, O* __restrict__ y, long n, long C,
                                                  long inner, const float* __restrict__ scale, float bin,
                                                  int round_type) {
  const long stride = (long)gridDim.x * 256 * 8;
  for (long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8; i < n; i += stride) {
    float v[8];
    ld8<T>(x, i, n, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const long idx = i + e;
      const float s = C == 1 ? scale[0] : scale[(idx / inner) % C];
      const float q = qfun(v[e], s, inv_scale(s), bin, round_type);
      v[e] = DEQ ? q * s / bin : q;
    }
    if (i + 8 <= n && sizeof(O) == 2) {
      Vec8<O>::st(y + i, v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (i + e < n) Cvt<O>::st(y, i + e, v[e]);
    }
  }
}

// moving-average scale: state = r*state + 1, accum = r*accum + cur, scale = accum / state
__global__ void moving_avg_kernel(const float* __restrict__ cur, float* state, float* accum, float* scale, float rate) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const float st = rate * state[0] + 1.f;
    const float ac = rate * accum[0] + cur[0];
    state[0] = st;
    accum[0] = ac;
    scale[0] = ac / st;
  }
}

int grid_for(long n) {
  long g = (n / 8 + 255) / 256;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

template <typename F>
int by_dtype(int dt, F&& f) {
  switch (dt) {
    case kF32: f((float*)nullptr); break;
    case kBF16: f((bf16_t*)nullptr); break;
    case kF16: f((half_t*)nullptr); break;
    default: return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

}  // namespace
}  // namespace pha

using namespace pha;

// per-tensor abs max of x[n] -> out[0] (fp32); out is zeroed here (same stream)
PHA_API int pha_quant_absmax(int dt, const void* x, long n, float* out, hipStream_t st) {
  if (n < 0 || !out) return (int)hipErrorInvalidValue;
  hipMemsetAsync(out, 0, sizeof(float), st);
  if (n == 0) return (int)hipGetLastError();
  return by_dtype(dt, [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    hipLaunchKernelGGL(absmax_kernel<T>, dim3(grid_for(n)), dim3(256), 0, st, static_cast<const T*>(x), n,
                       reinterpret_cast<unsigned*>(out));
  });
}

// per-channel abs max of x viewed as [outer, C, inner] -> out[C]
PHA_API int pha_quant_channel_absmax(int dt, const void* x, long outer, long C, long inner, float* out,
                                     hipStream_t st) {
  if (outer <= 0 || C <= 0 || inner <= 0 || !out) return (int)hipErrorInvalidValue;
  return by_dtype(dt, [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    if (inner == 1) {
      hipMemsetAsync(out, 0, sizeof(float) * C, st);
      const long rows_per = 64;
      const dim3 grid((unsigned)((C + 255) / 256), (unsigned)((outer + rows_per - 1) / rows_per));
      hipLaunchKernelGGL(colmax_kernel<T>, grid, dim3(256), 0, st, static_cast<const T*>(x), outer, C, rows_per,
                         reinterpret_cast<unsigned*>(out));
    } else {
      hipLaunchKernelGGL(chmax_kernel<T>, dim3((unsigned)C), dim3(256), 0, st, static_cast<const T*>(x), outer, C,
                         inner, out);
    }
  });
}

// y = quant(x) (dequant: * s / bin); C == 1: per-tensor scale[0], else scale[c] of [., C, inner].
// out_dt: the output dtype (x's dtype, or fp32 for integer levels)
PHA_API int pha_quant_dequant(int dt, int out_dt, const void* x, void* y, long n, long C, long inner,
                              const float* scale, int bits, int round_type, int dequant, hipStream_t st) {
  if (n < 0 || C <= 0 || inner <= 0 || bits < 2 || bits > 16 || !scale) return (int)hipErrorInvalidValue;
  if (out_dt != kF32 && out_dt != dt) return (int)hipErrorInvalidValue;
  if (n == 0) return 0;
  const float bin = (float)((1 << (bits - 1)) - 1);
  const int g = grid_for(n);
  return by_dtype(dt, [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    const T* xp = static_cast<const T*>(x);
    if (out_dt == kF32) {
      if (dequant) hipLaunchKernelGGL((qdq_kernel<T, float, true>), dim3(g), dim3(256), 0, st, xp, (float*)y, n, C, inner, scale, bin, round_type);
      else hipLaunchKernelGGL((qdq_kernel<T, float, false>), dim3(g), dim3(256), 0, st, xp, (float*)y, n, C, inner, scale, bin, round_type);
    } else if (out_dt == dt) {
      if (dequant) hipLaunchKernelGGL((qdq_kernel<T, T, true>), dim3(g), dim3(256), 0, st, xp, (T*)y, n, C, inner, scale, bin, round_type);
      else hipLaunchKernelGGL((qdq_kernel<T, T, false>), dim3(g), dim3(256), 0, st, xp, (T*)y, n, C, inner, scale, bin, round_type);
    }
  });
}

PHA_API int pha_quant_moving_avg(const float* cur, float* state, float* accum, float* scale, float rate, hipStream_t st) {
  if (!cur || !state || !accum || !scale) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(moving_avg_kernel, dim3(1), dim3(64), 0, st, cur, state, accum, scale, rate);
  return (int)hipGetLastError();
}
