// MFMA tile building blocks shared by the large-tile GEMM / convolution kernels (gemm256.hip,
// gemm8p.hip): 16x16x32 MFMA wrappers, the LDS image swizzles for row (ds_read_b128) and
// transposed (ds_read_b64_tr_b16) fragment reads, and the 16-B global->LDS DMA.
#pragma once
#include "common.h"

namespace pha {
namespace g256 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

template <typename T> struct Mf;
template <> struct Mf<bf16_t> {
  static __device__ __forceinline__ f32x4 mma(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c,
                                                   0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t cvt(float v) {
    return __builtin_bit_cast(uint16_t, (__bf16)v);
  }
};
template <> struct Mf<half_t> {
  static __device__ __forceinline__ f32x4 mma(uint4 a, uint4 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c,
                                                  0, 0, 0);
  }
  static __device__ __forceinline__ uint16_t cvt(float v) {
    return __builtin_bit_cast(uint16_t, (_Float16)v);
  }
};

// byte offset in a [rows][BK] bf16 image. BK = 64: 128-B rows, 16-B chunk ^= row & 7; BK = 32:
// 64-B rows, chunk ^= (row >> 2) & 3 — either way the 16 rows of a fragment read cover all 16
// chunk slots of a 256-B bank row (SQ_LDS_BANK_CONFLICT = 0 measured)
template <int BK>
__device__ __forceinline__ int img_off(int row, int chunk) {
  if constexpr (BK == 64) return row * 128 + ((chunk ^ (row & 7)) << 4);
  // BK 32 (64-B rows): XOR of the 4-row block's entry in f = {0, 2, 3, 1}. ds_read_b128 serves
  // lanes {0-3, 12-15, 20-27} (and three more such groups) in one LDS cycle, i.e. fragment rows
  // 0-3 and 12-15 of chunk k with rows 4-11 of chunk k + 1; the plain (row >> 2) & 3 put rows
  // 0-3 / k and 4-7 / k + 1 on the same 16-B slots — a 2-way conflict in every group (37-47 %
  // SQ_LDS_BANK_CONFLICT, profiles/resnet_pmc_r5/). f makes all four groups conflict-free.
  else return row * 64 + ((chunk ^ ((0x78 >> (((row >> 2) & 3) << 1)) & 3)) << 4);
}

// 16-B global -> LDS DMA (global_load_lds_dwordx4; M0 = the wave's LDS destination, lane-linear).
// Issued from inline asm on purpose: hipcc's waitcnt pass treats every LDS DMA it can see as a
// pending write to ALL of LDS and puts s_waitcnt vmcnt(0) in front of the next ds_read, which
// drains the prefetch pipeline each k-step. Invisible to it, the DMAs are ordered only by the
// kernels' own counted s_waitcnt vmcnt(N) + s_barrier (and the "memory" clobber keeps LDS
// accesses from moving across the issue).
__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_wave_base) {
  const unsigned lds = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)lds_wave_base;
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :: "v"(src), "s"(__builtin_amdgcn_readfirstlane(lds)) : "memory", "m0");
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

__device__ __forceinline__ int tn_mask(int row, int row_bytes) {
  if (row_bytes >= 256) return ((row & 3) | (((row >> 3) & 1) << 2)) << 1;
  return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 1;   // 128-B rows: two rows per bank row
}

typedef short tn_v4i16 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint2 tr16(const unsigned char* ptr) {
  const tn_v4i16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) tn_v4i16*)(ptr));
  return __builtin_bit_cast(uint2, r);
}

// 8-k operand of a 16-column block starting at column c0 (multiple of 16), k-rows r0 .. r0+7 of
// the group (the caller passes r0 = kbase + 8 * (lane >> 4))
template <int ROWB>
__device__ __forceinline__ uint4 tn_frag(const unsigned char* img, int r0, int c0, int q, int pp) {
  const int ch = (c0 >> 3) + (pp >> 1);
  const int ra = r0 + q, rb = r0 + 4 + q;
  const uint2 lo = tr16(img + ra * ROWB + ((ch ^ tn_mask(ra, ROWB)) << 4) + 8 * (pp & 1));
  const uint2 hi = tr16(img + rb * ROWB + ((ch ^ tn_mask(rb, ROWB)) << 4) + 8 * (pp & 1));
  return uint4{lo.x, lo.y, hi.x, hi.y};
}

}  // namespace g256
}  // namespace pha
