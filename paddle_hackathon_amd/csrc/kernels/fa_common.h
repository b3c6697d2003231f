// Shared pieces of the flash-attention kernels (flash_attn.hip: forward + two-kernel backward,
// flash_attn_bwd.hip: single-kernel backward): MFMA fragment types, the 32x32x16 accumulator
// row map, the dual-use LDS image (row reads + ds_read_b64_tr_b16 transposed reads) and the
// per-operand (token, head) strides that let packed [B, S, H, 3D] QKV be read in place.
#pragma once
#include "common.h"

using namespace pha;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

constexpr float kLog2e = 1.4426950408889634f;

// 2^x as the bare v_exp_f32. exp2f() wraps it in a denormal-range fixup (compare, scale by 2^64,
// v_ldexp, select: 4 extra VALU ops per element, 128 per backward tile at one wave per SIMD);
// softmax probabilities below 2^-126 are zero for every use here (-inf masks give exactly 0)
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
constexpr float kLn2 = 0.6931471805599453f;

template <typename T> struct MF;
template <> struct MF<bf16_t> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
    // plain conversions: hipcc lowers the pair to one v_cvt_pk_bf16_f32 (RNE) on gfx950
    typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
    const bf16x2 v = {(__bf16)lo, (__bf16)hi};
    return __builtin_bit_cast(uint32_t, v);
  }
};
template <> struct MF<half_t> {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
    typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;
    const f16x2 v = {(_Float16)lo, (_Float16)hi};
    return __builtin_bit_cast(uint32_t, v);
  }
};

template <typename F>
__device__ __forceinline__ F as_frag(u32x4 v) { return __builtin_bit_cast(F, v); }

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// row of the 32x32 accumulator held in register r by lane-half h
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

struct FaStrides {
  long q_tok, kv_tok, o_tok, dq_tok, dkv_tok;
  int q_head, kv_head, o_head, dq_head, dkv_head;
  int order_g;   // key/query blocks of one (b, h) kept together on an XCD (see fa_block)
  int prio = 0;  // 8-wave kernels' wave priorities: 0 none, 1 waves 0-3 high, 2 high while issuing MFMAs
};

__device__ __forceinline__ int v_lds_off(int row, int chunk) {  // 256-B rows, tr-read friendly XOR
  return row * 256 + 16 * (chunk ^ (((row & 3) << 2) | ((row >> 2) & 3)));
}

typedef short v4i16 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x2 ds_read_tr16(const unsigned char* lds_ptr) {
  const v4i16 r = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) v4i16*)(lds_ptr));
  return __builtin_bit_cast(u32x2, r);
}

__device__ __forceinline__ int dual_off(int row, int chunk) { return v_lds_off(row, chunk); }

// 8 elements of a transposed operand: rows r0+{0..3} and r0+8+{0..3} of a dual image, the
// lane's 32-column block (column block cb = 32-wide d block index)
__device__ __forceinline__ u32x4 tr_frag(const unsigned char* img, int r0, int db, int g, int tq, int tp) {
  const int chunk = 4 * db + 2 * (g & 1) + (tp >> 1);
  const u32x2 lo = ds_read_tr16(img + dual_off(r0 + tq, chunk) + 8 * (tp & 1));
  const u32x2 hi = ds_read_tr16(img + dual_off(r0 + 8 + tq, chunk) + 8 * (tp & 1));
  return u32x4{lo[0], lo[1], hi[0], hi[1]};
}

FaStrides dense_strides(int H, int Hk, int D) {
  FaStrides f;
  f.order_g = 0;
  f.q_tok = f.o_tok = f.dq_tok = f.dkv_tok = (long)H * D;
  f.kv_tok = (long)Hk * D;
  f.q_head = f.kv_head = f.o_head = f.dq_head = f.dkv_head = D;
  return f;
}

// Workgroup id -> ((b, h) index, block rank), block rank 0 = the heaviest causal block.
// Workgroups are dispatched round-robin over the 8 XCDs (CDNA guide T1), so XCD x runs the ids
// x, x+8, ...: give each XCD its own (b, h) pairs (bh = x mod 8), walk them heaviest block group
// first (longest-processing-time order, no tail of long workgroups), and keep the G blocks of a
// group of one pair consecutive on that XCD so they stream the same Q/dO or K/V tiles through its
// L2. Falls back to plain (b, h)-fastest order when the shape does not split evenly.
__device__ __forceinline__ void fa_block(int BH, int nblk, int G, int& bh, int& blk) {
  const int id = blockIdx.x + gridDim.x * blockIdx.y;
  if (G <= 0 || BH % 8 || nblk % G) {
    bh = id % BH;
    blk = id / BH;
    return;
  }
  const int xcd = id & 7, slot = id >> 3, nbx = BH >> 3;
  const int grp = slot / (nbx * G), rem = slot - grp * (nbx * G);
  bh = (rem / G) * 8 + xcd;
  blk = grp * G + rem % G;
}

}  // namespace

namespace pha {
// Extensions of the 4-wave flash-attention kernels (template bit EXT): an additive score bias
// (EXT & 1: key-padding mask [B,1,1,Sk] or full [B|1, H|1, S, Sk], fp32, natural-log units,
// key stride 1) and in-kernel dropout of the attention probabilities (EXT & 2), regenerated bit
// for bit in the backward from (seed, b*H+h, query, key) — reference: fmha_ref.h:87-172 (src_mask +
// dropout) and fused_attention_op.cu.
struct FaExt {
  const float* bias;
  long sb, sh, sq;       // bias element strides of batch, head, query (0 = broadcast)
  unsigned seed;         // dropout stream
  unsigned thresh;       // drop when the element's 16-bit random < thresh  (thresh = rate * 65536)
  float keep_scale;      // 1 / (1 - rate)
  // gradient outputs' element strides (0: dense [B, S, H, D]): token and head strides of dQ and of
  // dK / dV, so a packed [B, S, H, 3D] QKV gradient is written in place (no concatenation pass)
  long gq_tok = 0, gkv_tok = 0;
  int gq_head = 0, gkv_head = 0;
  // hipGraph replays: a device word xor-ed into seed (bumped by a captured kernel every replay, so
  // each replay draws a new mask; the backward reads the forward's copy). null: seed alone
  const unsigned* seedp = nullptr;
  // head-dim-64 kernels: the forward's keep mask as bits [B*H][dmask_w][S up to 64] (word w: keys
  // 32w .. 32w + 31), read by the backward instead of re-hashing; null: the backward regenerates it
  unsigned* dmask = nullptr;
  int dmask_w = 0;
};

__device__ __forceinline__ unsigned fa_seed(const FaExt& ex) { return ex.seedp ? ex.seed ^ *ex.seedp : ex.seed; }

__device__ __forceinline__ unsigned fa_mix(unsigned x) {   // lowbias32 finaliser
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}
// per-(b, h) stream, then per query row, then one 32-bit draw per key pair (16 bits per key)
__device__ __forceinline__ unsigned fa_stream(unsigned seed, int bh) { return fa_mix(seed ^ ((unsigned)bh * 0x85ebca77U)); }
__device__ __forceinline__ unsigned fa_row(unsigned sbh, int q) { return fa_mix(sbh + (unsigned)q * 0x9e3779b1U); }
__device__ __forceinline__ bool fa_keep(unsigned row, int key, unsigned thresh) {
  const unsigned r = fa_mix(row ^ (unsigned)(key >> 1));
  return ((key & 1) ? (r >> 16) : (r & 0xffffU)) >= thresh;
}
}  // namespace pha

