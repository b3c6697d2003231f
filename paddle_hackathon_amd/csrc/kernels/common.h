// Shared device helpers for the gfx950 (MI355X / CDNA4) kernel library.
//
// Conventions
//  * wave64 everywhere: lane = threadIdx.x & 63, reductions use __shfl_xor over 64 lanes.
//  * bf16/f16 tensors are moved in 16-byte vectors (8 elements / lane) — hipcc does not
//    auto-vectorize 2-byte loads (CDNA guide, Guideline 13).
//  * all math in fp32; storage dtype is a template parameter (float, bf16_t, half_t).
//  * every entry point takes the caller's hipStream_t (the current torch stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PHA_API extern "C" __attribute__((visibility("default")))

namespace pha {

enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

struct bf16_t { uint16_t v; };
struct half_t { _Float16 v; };

__device__ __forceinline__ float bf16_to_f32(uint16_t h) {
  return __uint_as_float(static_cast<uint32_t>(h) << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fc0;  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);                       // round-to-nearest-even
  return static_cast<uint16_t>(u >> 16);
}

// ---- scalar load/store as float -------------------------------------------------
template <typename T> struct Cvt;
template <> struct Cvt<float> {
  static __device__ __forceinline__ float ld(const float* p, long i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, long i, float v) { p[i] = v; }
};
template <> struct Cvt<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p, long i) { return bf16_to_f32(p[i].v); }
  static __device__ __forceinline__ void st(bf16_t* p, long i, float v) { p[i].v = f32_to_bf16(v); }
};
template <> struct Cvt<half_t> {
  static __device__ __forceinline__ float ld(const half_t* p, long i) { return (float)p[i].v; }
  static __device__ __forceinline__ void st(half_t* p, long i, float v) { p[i].v = (_Float16)v; }
};

// round a float to T's precision and back (what storing to T and reloading would give)
template <typename T> __device__ __forceinline__ float round_to(float v);
template <> __device__ __forceinline__ float round_to<float>(float v) { return v; }
template <> __device__ __forceinline__ float round_to<bf16_t>(float v) { return bf16_to_f32(f32_to_bf16(v)); }
template <> __device__ __forceinline__ float round_to<half_t>(float v) { return (float)(_Float16)v; }

// ---- 8-wide vector load/store (16 B for 2-byte types, 2x16 B for fp32) -----------
template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
  static __device__ __forceinline__ void unpack(const uint4& r, float (&o)[8]) {
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = __uint_as_float(w[i] << 16);
      o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void ld(const bf16_t* p, float (&o)[8]) {
    uint4 r = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = __uint_as_float(w[i] << 16);
      o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void st(bf16_t* p, const float (&o)[8]) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = static_cast<uint32_t>(f32_to_bf16(o[2 * i])) | (static_cast<uint32_t>(f32_to_bf16(o[2 * i + 1])) << 16);
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
  }
};
template <> struct Vec8<half_t> {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  static __device__ __forceinline__ void unpack(const uint4& r, float (&o)[8]) {
    const h8 v = __builtin_bit_cast(h8, r);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)v[i];
  }
  static __device__ __forceinline__ void ld(const half_t* p, float (&o)[8]) {
    h8 r = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = (float)r[i];
  }
  static __device__ __forceinline__ void st(half_t* p, const float (&o)[8]) {
    h8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (_Float16)o[i];
    *reinterpret_cast<h8*>(p) = r;
  }
};
template <> struct Vec8<float> {
  static __device__ __forceinline__ void ld(const float* p, float (&o)[8]) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w;
    o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  static __device__ __forceinline__ void st(float* p, const float (&o)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(o[0], o[1], o[2], o[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(o[4], o[5], o[6], o[7]);
  }
};

// ---- wave64 / block reductions ------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide reduction; `red` must hold >= blockDim/64 floats; returns result to all threads.
template <bool kMax>
__device__ __forceinline__ float block_reduce(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = kMax ? wave_max(v) : wave_sum(v);
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < nw; ++i) r = kMax ? fmaxf(r, red[i]) : r + red[i];
  __syncthreads();
  return r;
}

}  // namespace pha

#define PHA_DISPATCH_T(dt, T, ...)                  \
  switch (dt) {                                     \
    case pha::kF32: { typedef float T; __VA_ARGS__; break; }      \
    case pha::kBF16: { typedef pha::bf16_t T; __VA_ARGS__; break; } \
    case pha::kF16: { typedef pha::half_t T; __VA_ARGS__; break; }  \
    default: return (int)hipErrorInvalidValue;      \
  }
