// fp32 operands of the three-term split products (ops/conv_gemm.py split3, ops/gemm.py mm_f32):
//
//   x = hi + lo,  hi = bf16(x),  lo = bf16(x - hi)      (both round-to-nearest-even)
//   (finite x past the largest bf16: hi = x truncated to bf16; non-finite x: lo = 0)
//   out[o][p][i] = (bit p of lo_mask ? lo : hi)(x[o][i])      o < outer, p < 3, i < inner
//
// i.e. the concatenation of three parts along one dimension of a contiguous tensor (outer = the
// product of the dimensions before it, inner = that dimension and the ones after). One streaming
// pass — 4 B read and 6 B written per element, 8 elements per lane in 16-B vectors — where the
// torch expression takes five elementwise passes plus the concatenation copy.
#include "common.h"

namespace pha {
namespace {

__global__ __launch_bounds__(256) void split3_kernel(const float* __restrict__ x, uint4* __restrict__ out,
                                                     unsigned outer, unsigned inner8, int lo_mask) {
  const unsigned n = outer * inner8;
  for (unsigned v = blockIdx.x * 256u + threadIdx.x; v < n; v += gridDim.x * 256u) {
    const unsigned o = v / inner8, i8 = v - o * inner8;
    const float4 a = reinterpret_cast<const float4*>(x)[2 * (size_t)v];
    const float4 b = reinterpret_cast<const float4*>(x)[2 * (size_t)v + 1];
    const float f[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      uint16_t h[2], l[2];
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const float v = f[2 * k + e];
        h[e] = f32_to_bf16(v);
        // |v| above the largest bf16 rounds hi to inf: take the truncated hi instead (finite, and
        // lo stays exact); a non-finite v keeps lo = 0 so hi + lo is v itself (inf - inf = NaN
        // otherwise)
        if (!__builtin_isfinite(bf16_to_f32(h[e])) && __builtin_isfinite(v)) h[e] = (uint16_t)(__float_as_uint(v) >> 16);
        l[e] = __builtin_isfinite(v) ? f32_to_bf16(v - bf16_to_f32(h[e])) : (uint16_t)0;
      }
      hw[k] = (uint32_t)h[0] | ((uint32_t)h[1] << 16);
      lw[k] = (uint32_t)l[0] | ((uint32_t)l[1] << 16);
    }
    const uint4 H = {hw[0], hw[1], hw[2], hw[3]}, L = {lw[0], lw[1], lw[2], lw[3]};
    uint4* dst = out + (size_t)o * 3 * inner8 + i8;
#pragma unroll
    for (int p = 0; p < 3; ++p) dst[(size_t)p * inner8] = ((lo_mask >> p) & 1) ? L : H;
  }
}

}  // namespace
}  // namespace pha

using namespace pha;

// inner % 8 == 0, 16-B aligned x / out, outer * inner / 8 < 2^32
PHA_API int pha_split3_f32(const float* x, void* out, long outer, long inner, int lo_mask, hipStream_t st) {
  if (inner % 8 || outer <= 0 || inner <= 0 || ((size_t)x & 15) || ((size_t)out & 15)) return (int)hipErrorInvalidValue;
  const long n8 = outer * (inner / 8);
  if (n8 >= (1L << 32)) return (int)hipErrorInvalidValue;
  const long grid = n8 / 256 + 1 < 8192 ? n8 / 256 + 1 : 8192;
  hipLaunchKernelGGL(split3_kernel, dim3((unsigned)grid), dim3(256), 0, st, x, static_cast<uint4*>(out),
                     (unsigned)outer, (unsigned)(inner / 8), lo_mask);
  return (int)hipGetLastError();
}
