// Flash attention (forward + backward) for gfx950 / MI355X, bf16 & f16, head_dim 64/128.
//
// Layout: q [B, S, H, D], k/v [B, Sk, Hk, D] (GQA: Hk | H), o like q, lse [B, H, S] fp32.
// Replaces the reference's fused_attention_op.cu / fmha_ref.h (which materialise the
// S x S score matrix) with an online-softmax kernel that never leaves registers/LDS.
//
// Forward structure (CDNA guide §3 / Appendix B "swapped QK^T"):
//  * workgroup = 4 waves = 128 query rows of one (batch, head); each wave owns 32 rows.
//  * per 64-key tile: K staged in LDS (row-major, 16-B chunks XOR-swizzled by row so the
//    ds_read_b128 A-fragment reads are conflict-free), V staged transposed (V^T[d][key],
//    row padded to 136 B) for the PV A-operand.
//  * S^T = K . Q^T with v_mfma_f32_32x32x16_bf16: the query sits on the lane, its 32 key
//    scores in 16 regs of this lane + 16 of lane^32, so the row max/sum are register
//    reductions plus ONE cross-half swap; the S^T accumulator, packed to bf16, is
//    directly the B operand of O^T += V^T . P^T (no LDS round trip for P), and O^T keeps
//    the query on the lane so the online-softmax rescale is lane-local.
//  * exp2 with log2(e)*scale folded into one multiply; fp32 statistics; LSE saved for bwd.
//
// Backward: a key-parallel dK/dV kernel and a query-parallel dQ kernel (see below) — no
// atomics and no cross-workgroup reduction; both prefetch their next tile into registers.
#include "fa_common.h"
#include <type_traits>
#include <cstdlib>

using namespace pha;

namespace {


constexpr int BM = 128;   // query rows per workgroup (4 waves x 32)
constexpr int BN = 64;    // keys per tile
constexpr int VT_PAD = 4; // keys of padding per V^T row (row = 136 B)

// K tile: BN rows x D, 16-B chunks swizzled by (row & (CH-1)), CH = D/8 chunks per row
template <int D>
__device__ __forceinline__ int k_lds_off(int row, int chunk) {
  constexpr int CH = D / 8;
  return row * (D * 2) + ((chunk ^ (row & (CH - 1))) * 16);
}

template <typename T, int D, bool CAUSAL, int EXT = 0>
__global__ __launch_bounds__(256) void fa_fwd_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                     const T* __restrict__ V, T* __restrict__ O,
                                                     float* __restrict__ LSE, int S, int Sk, int H, int Hk,
                                                     float scale_log2, FaExt ex) {
  typedef typename MF<T>::frag frag;
  constexpr int CH = D / 8;
  constexpr int ND = D / 32;            // 32-wide d blocks of O^T
  constexpr int NK = D / 16;            // k-steps over d for S
  constexpr int VT_STRIDE = (BN + VT_PAD) * 2;  // bytes per V^T row
  __shared__ __attribute__((aligned(16))) unsigned char smem[BN * D * 2 + D * VT_STRIDE];
  unsigned char* k_lds = smem;
  unsigned char* vt_lds = smem + BN * D * 2;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int nqb = (S + BM - 1) / BM;
  const int qb = CAUSAL ? (nqb - 1 - (int)blockIdx.x) : (int)blockIdx.x;  // heavy blocks first
  const int head = blockIdx.y, b = blockIdx.z;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM;
  const int q = q0 + wid * 32 + lr;        // this lane's query row
  const long qstride = (long)H * D, kstride = (long)Hk * D;
  const T* Qb = Q + ((long)b * S) * qstride + (long)head * D;
  const T* Kb = K + ((long)b * Sk) * kstride + (long)hk * D;
  const T* Vb = V + ((long)b * Sk) * kstride + (long)hk * D;
  // extensions: this lane's bias row and dropout stream (query on the lane)
  const float* brow = ((EXT & 1) && q < S) ? ex.bias + (long)b * ex.sb + (long)head * ex.sh + (long)q * ex.sq : nullptr;
  const unsigned drow = (EXT & 2) ? fa_row(fa_stream(fa_seed(ex), b * H + head), q) : 0u;

  // Q fragments (B operand of S^T = K Q^T): Q[q][16kk + 8h + j]
  frag qf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 v = {0, 0, 0, 0};
    if (q < S) v = *reinterpret_cast<const u32x4*>(Qb + (long)q * qstride + 16 * kk + 8 * h);
    qf[kk] = as_frag<frag>(v);
  }
  f32x16 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = zero16();
  float m_run = -INFINITY, l_run = 0.f;

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM);
  const int wave_qmax = q0 + wid * 32 + 31;

  // ---- register-staged K/V pipeline (T14): tile t+1 is loaded into VGPRs while tile t is
  // computed, and written to LDS after the next barrier.
  //   K: 4 x 16-B chunks per thread (row-major, swizzled into LDS).
  //   V: thread owns 4 consecutive keys x one 8-wide d chunk, so the transposed V^T image is
  //      written with 8 ds_write_b64 (4 keys each) instead of 32 ds_write_b16.
  constexpr int KCH = (BN * CH) / 256;          // K chunks per thread
  constexpr int VITEMS = (BN / 4) * CH;          // (4-key group, d chunk) items
  constexpr int VIT = (VITEMS + 255) / 256;      // V items per thread (2 at D = 256)
  u32x4 kreg[KCH];
  u32x4 vreg[VIT][4];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + 256 * i;
      const int row = c / CH, ch = c % CH;
      const int key = k0 + row;
      kreg[i] = (key < Sk) ? *reinterpret_cast<const u32x4*>(Kb + (long)key * kstride + ch * 8) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int v_item = tid + 256 * it;
      if (v_item < VITEMS) {
        const int v_kg = v_item / CH, v_ch = v_item % CH;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int key = k0 + v_kg * 4 + j;
          vreg[it][j] = (key < Sk) ? *reinterpret_cast<const u32x4*>(Vb + (long)key * kstride + v_ch * 8) : u32x4{0, 0, 0, 0};
        }
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < KCH; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<u32x4*>(k_lds + k_lds_off<D>(c / CH, c % CH)) = kreg[i];
    }
#pragma unroll
    for (int it = 0; it < VIT; ++it) {
      const int v_item = tid + 256 * it;
      if (v_item < VITEMS) {
        const int v_kg = v_item / CH, v_ch = v_item % CH;
        const uint16_t* e0 = reinterpret_cast<const uint16_t*>(&vreg[it][0]);
        const uint16_t* e1 = reinterpret_cast<const uint16_t*>(&vreg[it][1]);
        const uint16_t* e2 = reinterpret_cast<const uint16_t*>(&vreg[it][2]);
        const uint16_t* e3 = reinterpret_cast<const uint16_t*>(&vreg[it][3]);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          u32x2 w;
          w[0] = (uint32_t)e0[e] | ((uint32_t)e1[e] << 16);
          w[1] = (uint32_t)e2[e] | ((uint32_t)e3[e] << 16);
          *reinterpret_cast<u32x2*>(vt_lds + (v_ch * 8 + e) * VT_STRIDE + v_kg * 8) = w;
        }
      }
    }
  };

  if (kend > 0) load_tile(0);
  for (int k0 = 0; k0 < kend; k0 += BN) {
    __syncthreads();  // previous tile fully consumed
    store_tile();
    __syncthreads();
    if (k0 + BN < kend) load_tile(k0 + BN);     // in flight during this tile's MFMAs
    if (CAUSAL && k0 > wave_qmax) continue;  // whole tile masked for this wave (barriers stay uniform)

    // ---- S^T = K . Q^T for two 32-key blocks ------------------------------------------
    f32x16 s[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = zero16();
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const u32x4 a = *reinterpret_cast<const u32x4*>(k_lds + k_lds_off<D>(kb * 32 + lr, 2 * kk + h));
        s[kb] = MF<T>::mma(as_frag<frag>(a), qf[kk], s[kb]);
      }
    }
    // ---- masking (only on diagonal / ragged tiles) + online softmax (query on the lane) ----
    const bool need_mask = (EXT & 1) || (k0 + BN > Sk) || (CAUSAL && k0 + BN - 1 > q0 + wid * 32);
    float tmax = -INFINITY;
    if (need_mask) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + kb * 32 + acc_row(r, h);
          const bool masked = (key >= Sk) || (CAUSAL && key > q);
          float v = masked ? -INFINITY : s[kb][r] * scale_log2;
          if constexpr (EXT & 1) {
            if (!masked && brow) v += brow[key] * kLog2e;
          }
          s[kb][r] = v;
          tmax = fmaxf(tmax, v);
        }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = s[kb][r] * scale_log2;
          s[kb][r] = v;
          tmax = fmaxf(tmax, v);
        }
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    // deferred rescale (CDNA guide T13): keep the running max unless some row grew by more
    // than kThr (log2 units) — P is then bounded by 2^kThr, harmless for bf16 P and fp32 l/O.
    constexpr float kThr = 8.f;
    if (!__all(tmax <= m_run + kThr)) {
      const float m_new = fmaxf(m_run, tmax);
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      const float alpha = fexp2(m_run - m_use);
      l_run *= alpha;
#pragma unroll
      for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
      m_run = m_new;
    }
    const float m_use = (m_run == -INFINITY) ? 0.f : m_run;
    float psum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(s[kb][r] - m_use);
        s[kb][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 32, 64);
    l_run += psum;
    if constexpr (EXT & 2) {   // dropout on P for the PV product only (the softmax sum is undropped)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + kb * 32 + acc_row(r, h);
          s[kb][r] = fa_keep(drow, key, ex.thresh) ? s[kb][r] * ex.keep_scale : 0.f;
        }
    }

    // ---- O^T += V^T . P^T ---------------------------------------------------------------
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const f32x16& sv = s[ks >> 1];
      const int s8 = (ks & 1) * 8;
      u32x4 pw;
      pw[0] = MF<T>::pack(sv[s8 + 0], sv[s8 + 1]);
      pw[1] = MF<T>::pack(sv[s8 + 2], sv[s8 + 3]);
      pw[2] = MF<T>::pack(sv[s8 + 4], sv[s8 + 5]);
      pw[3] = MF<T>::pack(sv[s8 + 6], sv[s8 + 7]);
      const frag pf = as_frag<frag>(pw);
      const int kbase = 16 * ks + 4 * h;
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        const unsigned char* row = vt_lds + (db * 32 + lr) * VT_STRIDE;
        const u32x2 lo = *reinterpret_cast<const u32x2*>(row + kbase * 2);
        const u32x2 hi = *reinterpret_cast<const u32x2*>(row + (kbase + 8) * 2);
        const u32x4 a = {lo[0], lo[1], hi[0], hi[1]};
        o[db] = MF<T>::mma(as_frag<frag>(a), pf, o[db]);
      }
    }
  }

  // ---- epilogue: normalise, store O and LSE ---------------------------------------------
  if (q < S) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    T* orow = O + ((long)b * S + q) * qstride + (long)head * D;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = db * 32 + 8 * g + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(o[db][4 * g + 0] * inv, o[db][4 * g + 1] * inv);
        w[1] = MF<T>::pack(o[db][4 * g + 2] * inv, o[db][4 * g + 3] * inv);
        *reinterpret_cast<u32x2*>(orow + d) = w;
      }
    if (h == 0) {
      const float lse = (l_run > 0.f) ? (m_run + log2f(l_run)) * kLn2 : INFINITY;
      LSE[((long)b * H + head) * S + q] = lse;
    }
  }
}

// ============================================================================================
// Forward v2 (D = 128): workgroup = 8 waves = 256 query rows, 64-key tiles.
//  * K and V staged row-major in a double-buffered LDS ring (one barrier per tile, tile t+1
//    fetched into registers during tile t's MFMAs and written after them — T14).
//  * V is never transposed in software: the PV A-operand (V^T[d][key]) is read with
//    ds_read_b64_tr_b16 straight from the row-major V image (T10); rows are 256 B with the
//    16-B chunk XOR (ch ^ ((row&3)<<2 | (row>>2)&3)) that makes those reads conflict-free.
//  * K rows XOR-swizzled by (row & 15) for the conflict-free ds_read_b128 S^T A-operand.
//  * everything else (swapped S^T = K Q^T, lane-local online softmax, deferred rescale,
//    accumulator-as-B-operand P^T) as in fa_fwd_kernel.
// ============================================================================================
// LDS-DMA 16 B per lane: global (sbase + voff) -> LDS m0 + lane * 16 (issued from asm so the
// compiler's waitcnt pass does not drain it at the first LDS read; the kernel waits explicitly)
__device__ __forceinline__ void fa_glds16(unsigned voff, const void* sbase, unsigned m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}

#ifndef PHA_FA_GROUPS
#define PHA_FA_GROUPS 7   // sched_group_barrier interleaves on: bit 0 dK/dV v3, bit 1 dQ v3, bit 2 forward v3
#endif
constexpr bool kFwdGroups = (PHA_FA_GROUPS >> 2) & 1;   // fa_fwd_v3_kernel's read-ahead interleave
#ifndef PHA_FWD_AHEAD
#define PHA_FWD_AHEAD 8
#endif
constexpr int kFwdAhead = PHA_FWD_AHEAD;
constexpr int BM2 = 256;
constexpr int NT2 = 512;

// element strides (token, head) of each operand, so packed [B, S, H, 3D] QKV projections and
// their packed gradient are read/written in place (no split copies, no concat of dq/dk/dv)

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(NT2) void fa_fwd_v2_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                        const T* __restrict__ V, T* __restrict__ O,
                                                        float* __restrict__ LSE, int S, int Sk, int H, int Hk,
                                                        float scale_log2, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int D = 128, CH = 16, ND = 4, NK = 8;
  constexpr int TILE = BN * D * 2;                   // 16 KiB per K or V tile
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int nqb = (S + BM2 - 1) / BM2;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / nqb, nqb, fs.order_g, bh, rank);
  const int qb = CAUSAL ? (nqb - 1 - rank) : rank;
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM2;
  const int q = q0 + wid * 32 + lr;
  const long qstride = fs.q_tok, kstride = fs.kv_tok;
  const T* Qb = Q + ((long)b * S) * qstride + (long)head * fs.q_head;
  const T* Kb = K + ((long)b * Sk) * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + ((long)b * Sk) * kstride + (long)hk * fs.kv_head;

  frag qf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 v = {0, 0, 0, 0};
    if (q < S) v = *reinterpret_cast<const u32x4*>(Qb + (long)q * qstride + 16 * kk + 8 * h);
    qf[kk] = as_frag<frag>(v);
  }
  f32x16 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = zero16();
  float m_run = -INFINITY, l_run = 0.f;

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM2);
  const int ntile = (kend + BN - 1) / BN;
  const int wave_q0 = q0 + wid * 32, wave_qmax = wave_q0 + 31;

  // 64 keys x 16 chunks = 1024 chunks per operand: 2 per thread each for K and V
  u32x4 kreg[2], vreg[2];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + NT2 * i;
      // keys past Sk read row Sk - 1 (finite; their scores are masked to -inf, P = 0): no exec
      // branch per load, no zero-fill of the prefetch registers
      const int key = min(k0 + (c >> 4), Sk - 1), ch = c & 15;
      kreg[i] = *reinterpret_cast<const u32x4*>(Kb + (long)key * kstride + ch * 8);
      vreg[i] = *reinterpret_cast<const u32x4*>(Vb + (long)key * kstride + ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    unsigned char* kl = smem + buf * 2 * TILE;
    unsigned char* vl = kl + TILE;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + NT2 * i;
      const int row = c >> 4, ch = c & 15;
      *reinterpret_cast<u32x4*>(kl + k_lds_off<D>(row, ch)) = kreg[i];
      *reinterpret_cast<u32x4*>(vl + v_lds_off(row, ch)) = vreg[i];
    }
  };

  // per-lane constant parts of the transposed V read address
  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;

  if (ntile > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
  }
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * BN;
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(k0 + BN);
    const unsigned char* kl = smem + cur * 2 * TILE;
    const unsigned char* vl = kl + TILE;
    if (!(CAUSAL && k0 > wave_qmax)) {
      f32x16 s[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        s[kb] = zero16();
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(kl + k_lds_off<D>(kb * 32 + lr, 2 * kk + h));
          s[kb] = MF<T>::mma(as_frag<frag>(a), qf[kk], s[kb]);
        }
      }
      const bool need_mask = (k0 + BN > Sk) || (CAUSAL && k0 + BN - 1 > wave_q0);
      // scores stay unscaled: max(c s) = c max(s) for c = scale * log2(e) > 0 (the launcher
      // requires scale > 0), and the exponent below is one fma(s, c, -m) per element
      float tmax = -INFINITY;
      if (need_mask) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = k0 + kb * 32 + acc_row(r, h);
            const bool masked = (key >= Sk) | (CAUSAL & (key > q));
            const float v = masked ? -INFINITY : s[kb][r];
            s[kb][r] = v;
            tmax = fmaxf(tmax, v);
          }
      } else {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb)
#pragma unroll
          for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, s[kb][r]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * scale_log2;
      constexpr float kThr = 8.f;
      if (!__all(tmax <= m_run + kThr)) {
        const float m_new = fmaxf(m_run, tmax);
        const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
        const float alpha = fexp2(m_run - m_use);
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < ND; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
        m_run = m_new;
      }
      const float m_use = (m_run == -INFINITY) ? 0.f : m_run;
      float psum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(s[kb][r], scale_log2, -m_use));
          s[kb][r] = p;
          psum += p;
        }
      psum += __shfl_xor(psum, 32, 64);
      l_run += psum;

      // O^T += V^T P^T : A = V^T via two transposed reads (keys 16ks+4h+{0..3}, +8)
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const f32x16& sv = s[ks >> 1];
        const int s8 = (ks & 1) * 8;
        u32x4 pw;
        pw[0] = MF<T>::pack(sv[s8 + 0], sv[s8 + 1]);
        pw[1] = MF<T>::pack(sv[s8 + 2], sv[s8 + 3]);
        pw[2] = MF<T>::pack(sv[s8 + 4], sv[s8 + 5]);
        pw[3] = MF<T>::pack(sv[s8 + 6], sv[s8 + 7]);
        const frag pf = as_frag<frag>(pw);
        const int row0 = 16 * ks + 4 * h + tq;
#pragma unroll
        for (int db = 0; db < ND; ++db) {
          const int chunk = 4 * db + 2 * (g & 1) + (tp >> 1);
          const u32x2 lo = ds_read_tr16(vl + v_lds_off(row0, chunk) + 8 * (tp & 1));
          const u32x2 hi = ds_read_tr16(vl + v_lds_off(row0 + 8, chunk) + 8 * (tp & 1));
          const u32x4 a = {lo[0], lo[1], hi[0], hi[1]};
          o[db] = MF<T>::mma(as_frag<frag>(a), pf, o[db]);
        }
      }
    }
    if (t + 1 < ntile) store_tile(cur ^ 1);
    __syncthreads();
  }

  if (q < S) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    T* orow = O + ((long)b * S + q) * fs.o_tok + (long)head * fs.o_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(o[db][4 * gg + 0] * inv, o[db][4 * gg + 1] * inv);
        w[1] = MF<T>::pack(o[db][4 * gg + 2] * inv, o[db][4 * gg + 3] * inv);
        *reinterpret_cast<u32x2*>(orow + d) = w;
      }
    if (h == 0) {
      const float lse = (l_run > 0.f) ? (m_run + log2f(l_run)) * kLn2 : INFINITY;
      LSE[((long)b * H + head) * S + q] = lse;
    }
  }
}

// Forward v3 (D = 128, default): fa_fwd_v2's geometry with K / V tiles by LDS-DMA (no staging
// registers, no ds_write), the mask folded into the score accumulators' initial values (-inf where
// masked: the max / exp loops have no selects), lane-offset + immediate LDS addressing and the
// K-row reads issued ahead of the QK^T MFMAs.
template <typename T, bool CAUSAL>
__global__ __launch_bounds__(NT2) void fa_fwd_v3_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                        const T* __restrict__ V, T* __restrict__ O,
                                                        float* __restrict__ LSE, int S, int Sk, int H, int Hk,
                                                        float scale_log2, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int ND = 4, NK = 8;
  constexpr int TILE = BN * 128 * 2;                 // 16 KiB per K or V tile
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * TILE];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            lr = lane & 31;
  const int nqb = (S + BM2 - 1) / BM2;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / nqb, nqb, fs.order_g, bh, rank);
  const int qb = CAUSAL ? (nqb - 1 - rank) : rank;
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM2;
  const int q = q0 + wid * 32 + lr;
  const long qstride = fs.q_tok, kstride = fs.kv_tok;
  const T* Qb = Q + ((long)b * S) * qstride + (long)head * fs.q_head;
  const T* Kb = K + ((long)b * Sk) * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + ((long)b * Sk) * kstride + (long)hk * fs.kv_head;

  frag qf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 v = {0, 0, 0, 0};
    if (q < S) v = *reinterpret_cast<const u32x4*>(Qb + (long)q * qstride + 16 * kk + 8 * h);
    qf[kk] = as_frag<frag>(v);
  }
  f32x16 o[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) o[i] = zero16();
  float m_run = -INFINITY, l_run = 0.f;

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM2);
  const int ntile = (kend + BN - 1) / BN;
  const int wave_q0 = q0 + wid * 32, wave_qmax = wave_q0 + 31;

  // K / V tile by LDS-DMA: 32 1-KiB pieces (4 rows of one operand), 4 per wave; K rows swizzled as
  // k_lds_off (chunk ^ row & 15), V rows as v_lds_off (the tr-read image)
  auto load_tile = [&](int k0, int buf) {
    const unsigned lds = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)(smem + buf * 2 * TILE);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gidx = wid * 4 + u, which = gidx >> 4;
      const int row = (gidx & 15) * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (which ? (((row & 3) << 2) | ((row >> 2) & 3)) : (row & 15));
      const T* base = (which ? Vb : Kb) + (long)k0 * kstride;
      const unsigned voff = (unsigned)(((long)(min(k0 + row, Sk - 1) - k0) * kstride + ch * 8) * 2);
      fa_glds16(voff, base, __builtin_amdgcn_readfirstlane(lds + which * TILE + (gidx & 15) * 1024));
    }
  };

  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  int koff[NK], troff[ND][2];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) koff[kk] = lr * 256 + 16 * ((2 * kk + h) ^ (lr & 15));
#pragma unroll
  for (int db = 0; db < ND; ++db)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi)
      troff[db][hi] = (4 * h + tq) * 256 + hi * 2048 +
                      16 * (4 * (db ^ tq) + ((2 * (g & 1) + (tp >> 1)) ^ ((h + 2 * hi) & 3))) + 8 * (tp & 1);

  if (ntile > 0) {
    load_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // wave priorities (fs.prio): the two waves of a SIMD (w, w + 4) otherwise reach their MFMA and
  // softmax phases together after every barrier; a priority skew lets one wave's exp / pack VALU
  // issue under the other's MFMAs
  if (fs.prio == 1 && wid < 4) __builtin_amdgcn_s_setprio(1);
  const bool dyn_prio = fs.prio == 2;
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * BN;
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(k0 + BN, cur ^ 1);
    const unsigned char* kl = smem + cur * 2 * TILE;
    const unsigned char* vl = kl + TILE;
    if (!(CAUSAL && k0 > wave_qmax)) {
      if (dyn_prio) __builtin_amdgcn_s_setprio(1);
      const bool need_mask = (k0 + BN > Sk) || (CAUSAL && k0 + BN - 1 > wave_q0);
      f32x16 s[2];
      s[0] = zero16();
      s[1] = zero16();
      if (need_mask) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int base = k0 + kb * 32 + 4 * h;
          const int lim1 = CAUSAL ? q - base : 1 << 20, lim2 = Sk - base;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rb = (r & 3) + 8 * (r >> 2);
            s[kb][r] = ((rb > lim1) | (rb >= lim2)) ? -INFINITY : 0.f;
          }
        }
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(kl + kb * 8192 + koff[kk]);
          s[kb] = MF<T>::mma(as_frag<frag>(a), qf[kk], s[kb]);
        }
      if constexpr (kFwdGroups) {
        __builtin_amdgcn_sched_group_barrier(0x100, kFwdAhead, 0);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (dyn_prio) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(0);
      }
      // scores unscaled (scale > 0: max(c s) = c max(s)); masked scores are -inf already
      float tmax = -INFINITY;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) tmax = fmaxf(tmax, s[kb][r]);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * scale_log2;
      constexpr float kThr = 8.f;
      if (!__all(tmax <= m_run + kThr)) {
        const float m_new = fmaxf(m_run, tmax);
        const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
        const float alpha = fexp2(m_run - m_use);
        l_run *= alpha;
#pragma unroll
        for (int i = 0; i < ND; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[i][r] *= alpha;
        m_run = m_new;
      }
      const float m_use = (m_run == -INFINITY) ? 0.f : m_run;
      float psum = 0.f;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(s[kb][r], scale_log2, -m_use));
          s[kb][r] = p;
          psum += p;
        }
      psum += __shfl_xor(psum, 32, 64);
      l_run += psum;
      if (dyn_prio) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const f32x16& sv = s[ks >> 1];
        const int s8 = (ks & 1) * 8;
        u32x4 pw;
        pw[0] = MF<T>::pack(sv[s8 + 0], sv[s8 + 1]);
        pw[1] = MF<T>::pack(sv[s8 + 2], sv[s8 + 3]);
        pw[2] = MF<T>::pack(sv[s8 + 4], sv[s8 + 5]);
        pw[3] = MF<T>::pack(sv[s8 + 6], sv[s8 + 7]);
        const frag pf = as_frag<frag>(pw);
#pragma unroll
        for (int db = 0; db < ND; ++db) {
          const u32x2 lo = ds_read_tr16(vl + ks * 4096 + troff[db][0]);
          const u32x2 hi = ds_read_tr16(vl + ks * 4096 + troff[db][1]);
          o[db] = MF<T>::mma(as_frag<frag>(u32x4{lo[0], lo[1], hi[0], hi[1]}), pf, o[db]);
        }
      }
      if (dyn_prio) {
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA'd tile has landed (asm: untracked)
    __syncthreads();
  }

  if (q < S) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    T* orow = O + ((long)b * S + q) * fs.o_tok + (long)head * fs.o_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(o[db][4 * gg + 0] * inv, o[db][4 * gg + 1] * inv);
        w[1] = MF<T>::pack(o[db][4 * gg + 2] * inv, o[db][4 * gg + 3] * inv);
        *reinterpret_cast<u32x2*>(orow + d) = w;
      }
    if (h == 0) {
      const float lse = (l_run > 0.f) ? (m_run + log2f(l_run)) * kLn2 : INFINITY;
      LSE[((long)b * H + head) * S + q] = lse;
    }
  }
}

// ============================================================================================
// Forward v4 (D = 128): 4 waves x 64 query rows — two 32-row blocks A, B per wave, one wave per
// SIMD with the whole 512-register file — and the softmax software-pipelined against the MFMAs
// INSIDE each wave (the 8-wave kernels rely on the two waves of a SIMD drifting apart, which the
// per-tile barrier prevents). The pipeline runs over 32-key sub-tiles u (half a 64-key DMA tile),
// which keeps the in-flight scores at 2 x 16 registers per block:
//   phase 1:  S(u) = K_u Q^T for A and B (16 MFMAs; each K fragment read once for both blocks)
//             || finish of u-1: second half of its exps, row sums, P(u-1) packed to bf16
//   phase 2:  O^T += V_{u-1}^T P(u-1)^T for A and B (16 MFMAs; each V fragment read once)
//             || start of u: row max, running-max update, first half of its exps
// The O rescale a raised running max needs (deferred by kThr as in v3) lands after phase 2's
// MFMAs, i.e. between P(u-1) V and P(u) V. K / V tiles arrive by LDS-DMA a whole tile ahead
// (K ring of 2, V ring of 3: V(t-1) is still read in tile t's first sub-tile), one barrier per
// 64-key tile.
// ============================================================================================
#ifndef PHA_FA4_GROUPS
#define PHA_FA4_GROUPS 1
#endif
#ifndef PHA_FA4_SLOTS
#define PHA_FA4_SLOTS 1   // hand-slotted steady sub-tiles (step_steady)
#endif

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fa_fwd_v4_kernel(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V, T* __restrict__ O,
                      float* __restrict__ LSE, int S, int Sk, int H, int Hk, float scale_log2, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int ND = 4, NK = 8;
  constexpr int TILE = BN * 128 * 2;   // 16 KiB per K or V tile
  __shared__ __attribute__((aligned(16))) unsigned char smem[5 * TILE];   // K ring [2] | V ring [3]

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            lr = lane & 31;
  const int nqb = (S + BM2 - 1) / BM2;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / nqb, nqb, fs.order_g, bh, rank);
  const int qb = CAUSAL ? (nqb - 1 - rank) : rank;
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM2;
  // block A rows rA0 + [0, 32) in the workgroup's lower half, block B rows rB0 + [0, 32) mirrored in
  // the upper half (wave 0: rows 0-31 and 224-255, wave 3: 96-127 and 128-159): under the causal
  // mask every wave then has the same work — A's keys end where B's are still running, and the
  // steps after A's last run B alone at half the cost
  const int rA0 = q0 + 32 * wid, rB0 = q0 + BM2 - 32 - 32 * wid;
  const int qa = rA0 + lr, qbq = rB0 + lr;
  const long qstride = fs.q_tok, kstride = fs.kv_tok;
  const T* Qb = Q + ((long)b * S) * qstride + (long)head * fs.q_head;
  const T* Kb = K + ((long)b * Sk) * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + ((long)b * Sk) * kstride + (long)hk * fs.kv_head;

  frag qA[NK], qB[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 va = {0, 0, 0, 0}, vb = {0, 0, 0, 0};
    if (qa < S) va = *reinterpret_cast<const u32x4*>(Qb + (long)qa * qstride + 16 * kk + 8 * h);
    if (qbq < S) vb = *reinterpret_cast<const u32x4*>(Qb + (long)qbq * qstride + 16 * kk + 8 * h);
    qA[kk] = as_frag<frag>(va);
    qB[kk] = as_frag<frag>(vb);
  }
  f32x16 oA[ND], oB[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { oA[i] = zero16(); oB[i] = zero16(); }
  float mA = -INFINITY, mB = -INFINITY, lA = 0.f, lB = 0.f, uA = 0.f, uB = 0.f, alA = 1.f, alB = 1.f;
  bool rsA = false, rsB = false;

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM2);
  const int ntile = (kend + BN - 1) / BN;
  const int nsub = (kend + 31) / 32;
  // last 32-key sub-tile with a visible key for block A / B (causal: keys <= the block's last row)
  const int uA_last = CAUSAL ? min(nsub - 1, (rA0 + 31) / 32) : nsub - 1;
  const int uB_last = CAUSAL ? min(nsub - 1, (rB0 + 31) / 32) : nsub - 1;

  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)smem;
  // 16 1-KiB LDS-DMA pieces per tile (4 rows each), 4 per wave; K rows swizzled as k_lds_off, V
  // rows as v_lds_off (the tr-read image)
  auto load_k = [&](int k0, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gidx = wid * 4 + u, row = gidx * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (row & 15);
      const unsigned voff = (unsigned)(((long)(min(k0 + row, Sk - 1) - k0) * kstride + ch * 8) * 2);
      fa_glds16(voff, Kb + (long)k0 * kstride, __builtin_amdgcn_readfirstlane(lds0 + slot * TILE + gidx * 1024));
    }
  };
  auto load_v = [&](int k0, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gidx = wid * 4 + u, row = gidx * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      const unsigned voff = (unsigned)(((long)(min(k0 + row, Sk - 1) - k0) * kstride + ch * 8) * 2);
      fa_glds16(voff, Vb + (long)k0 * kstride,
                __builtin_amdgcn_readfirstlane(lds0 + (2 + slot) * TILE + gidx * 1024));
    }
  };

  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  int koff[NK], troff[ND][2];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) koff[kk] = lr * 256 + 16 * ((2 * kk + h) ^ (lr & 15));
#pragma unroll
  for (int db = 0; db < ND; ++db)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi)
      troff[db][hi] = (4 * h + tq) * 256 + hi * 2048 +
                      16 * (4 * (db ^ tq) + ((2 * (g & 1) + (tp >> 1)) ^ ((h + 2 * hi) & 3))) + 8 * (tp & 1);

  // the previous sub-tile's scores per block: [0, 8) already exponentiated, [8, 16) raw
  float pvA[16], pvB[16];
  u32x4 pA[2], pB[2];
  constexpr float kThr = 8.f;
  // masked scores -> -inf (sub-tiles that straddle the causal diagonal or the key end)
  auto mask_s = [&](float (&sv)[16], int k0, int qrow) __attribute__((always_inline)) {
    const int base = k0 + 4 * h;
    const int lim1 = CAUSAL ? qrow - base : 1 << 20, lim2 = Sk - base;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rb = (r & 3) + 8 * (r >> 2);
      sv[r] = ((rb > lim1) | (rb >= lim2)) ? -INFINITY : sv[r];
    }
  };

  // top of tile t: K(t), V(t) landed, every wave done with K(t-1) and V(t-2); then issue K(t+1),
  // V(t+1) into the freed ring slots (every wave issues its share, active or not)
  int tsync = -1;
  auto sync_to = [&](int t) __attribute__((always_inline)) {
    while (tsync < t) {
      ++tsync;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // asm DMA: untracked by the compiler
      __syncthreads();
      if (tsync + 1 < ntile) {
        load_k((tsync + 1) * BN, (tsync + 1) & 1);
        load_v((tsync + 1) * BN, (tsync + 1) % 3);
      }
    }
  };
  u32x4 kf[NK], vf[2 * ND];   // fragments read one phase ahead (one wave per SIMD: no other wave
                              // hides an LDS read's latency)
  auto load_kf = [&](int u) __attribute__((always_inline)) {
    const unsigned char* kl = smem + ((u >> 1) & 1) * TILE + (u & 1) * 8192;
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) kf[kk] = *reinterpret_cast<const u32x4*>(kl + koff[kk]);
  };
  auto load_vf = [&](int u) __attribute__((always_inline)) {
    const unsigned char* vl = smem + (2 + ((u >> 1) % 3)) * TILE + (u & 1) * 8192;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        const u32x2 lo = ds_read_tr16(vl + ks * 4096 + troff[db][0]);
        const u32x2 hi = ds_read_tr16(vl + ks * 4096 + troff[db][1]);
        vf[ks * ND + db] = u32x4{lo[0], lo[1], hi[0], hi[1]};
      }
  };
  // one sub-tile step with per-block flags: CA / CB = sub-tile u has visible keys for block A / B,
  // PA / PB = sub-tile u - 1 had. The score accumulators start from an inline zero and are read out
  // once; everything the softmax touches lives in VGPRs (no accumulator-register round trips)
  auto step = [&](auto ca_c, auto pa_c, auto cb_c, auto pb_c, int u) __attribute__((always_inline)) {
    constexpr bool CA = decltype(ca_c)::value, PA = decltype(pa_c)::value;
    constexpr bool CB = decltype(cb_c)::value, PB = decltype(pb_c)::value;
    const int k0 = u * 32;
    f32x16 cA, cB;
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 1: QK^T of sub-tile u || finish of u - 1
    if constexpr (CA) cA = zero16();
    if constexpr (CB) cB = zero16();
    if constexpr (CA || CB) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        if constexpr (CA) cA = MF<T>::mma(as_frag<frag>(kf[kk]), qA[kk], cA);
        if constexpr (CB) cB = MF<T>::mma(as_frag<frag>(kf[kk]), qB[kk], cB);
      }
    }
    if constexpr (PA || PB) load_vf(u - 1);   // V fragments of P(u-1) V, read under the QK^T MFMAs
    auto finish = [&](float (&pv)[16], u32x4 (&pp)[2], float um, float& l) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 8; r < 16; ++r) pv[r] = fexp2(fmaf(pv[r], scale_log2, -um));
      float sm = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) sm += pv[r];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) pp[ks][jj] = MF<T>::pack(pv[8 * ks + 2 * jj], pv[8 * ks + 2 * jj + 1]);
      l += sm + __shfl_xor(sm, 32, 64);
    };
    if constexpr (PA) finish(pvA, pA, uA, lA);
    if constexpr (PB) finish(pvB, pB, uB, lB);
    __builtin_amdgcn_sched_barrier(0);
    // tile top of the next 64-key tile in the middle of an odd sub-tile, so the next sub-tile's K
    // fragments can be read under this one's P V MFMAs
    if ((u & 1) && ((u + 1) >> 1) < ntile) sync_to((u + 1) >> 1);
    float sA[16], sB[16];
    if constexpr (CA) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sA[r] = cA[r];
      if ((k0 + 32 > Sk) || (CAUSAL && k0 + 31 > rA0)) mask_s(sA, k0, qa);
    }
    if constexpr (CB) {
#pragma unroll
      for (int r = 0; r < 16; ++r) sB[r] = cB[r];
      if ((k0 + 32 > Sk) || (CAUSAL && k0 + 31 > rB0)) mask_s(sB, k0, qbq);
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 2: P(u-1) V of sub-tile u - 1 || start of u
    if constexpr (PA || PB) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int db = 0; db < ND; ++db) {
          if constexpr (PA) oA[db] = MF<T>::mma(as_frag<frag>(vf[ks * ND + db]), as_frag<frag>(pA[ks]), oA[db]);
          if constexpr (PB) oB[db] = MF<T>::mma(as_frag<frag>(vf[ks * ND + db]), as_frag<frag>(pB[ks]), oB[db]);
        }
    }
    if constexpr (CA || CB) load_kf(u + 1);   // next sub-tile's K fragments, read under the P V MFMAs
    auto start = [&](const float (&sv)[16], float (&pv)[16], float& m, float& um, float& al, bool& rs)
                     __attribute__((always_inline)) {
      float t = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) t = fmaxf(t, sv[r]);
      t = fmaxf(t, __shfl_xor(t, 32, 64)) * scale_log2;
      rs = !__all(t <= m + kThr);
      const float nm = rs ? fmaxf(m, t) : m;
      const float un = nm == -INFINITY ? 0.f : nm;
      al = rs ? fexp2(m - un) : 1.f;
      m = nm;
      um = un;
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        pv[r] = fexp2(fmaf(sv[r], scale_log2, -um));
        pv[8 + r] = sv[8 + r];
      }
    };
    if constexpr (CA) start(sA, pvA, mA, uA, alA, rsA);
    if constexpr (CB) start(sB, pvB, mB, uB, alB, rsB);
    __builtin_amdgcn_sched_barrier(0);
    // a raised running max rescales O after P(u-1) V, before P(u) V
    if constexpr (CA) {
      lA *= alA;
      if (rsA) {
        asm volatile("" ::: "memory");   // keep the (rare) rescale a branch, not a multiply per step
#pragma unroll
        for (int i = 0; i < ND; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) oA[i][r] *= alA;
      }
    }
    if constexpr (CB) {
      lB *= alB;
      if (rsB) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < ND; ++i)
#pragma unroll
          for (int r = 0; r < 16; ++r) oB[i][r] *= alB;
      }
    }
  };

  // steady sub-tile (CUR and PREV): MFMAs, LDS reads and softmax VALU placed slot by slot
  // behind sched_barrier fences (the compiler's own schedule issues the MFMAs as one burst and
  // the VALU after it — no overlap at one wave per SIMD): per slot the A and B MFMAs, one or two
  // operand reads for the next phase and ~10 VALU
  auto step_steady = [&](int u) __attribute__((always_inline)) {
    f32x16 cA = zero16(), cB = zero16();
    float sa = 0.f, sb = 0.f;
    const unsigned char* vl = smem + (2 + (((u - 1) >> 1) % 3)) * TILE + ((u - 1) & 1) * 8192;
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 1: QK^T of u || finish of u - 1 || V fragments of u - 1
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      cA = MF<T>::mma(as_frag<frag>(kf[j]), qA[j], cA);
      {
        const int ks = j >> 2, db = j & 3;
        const u32x2 lo = ds_read_tr16(vl + ks * 4096 + troff[db][0]);
        const u32x2 hi = ds_read_tr16(vl + ks * 4096 + troff[db][1]);
        vf[j] = u32x4{lo[0], lo[1], hi[0], hi[1]};
      }
      pvA[8 + j] = fexp2(fmaf(pvA[8 + j], scale_log2, -uA));
      sa += pvA[j];
      sa += pvA[8 + j];
      if (j & 1) {
        const int e = 2 * (j >> 1);   // pack units of elements e, e+1 (ready) and 8+e, 9+e (just done)
        pA[0][j >> 1] = MF<T>::pack(pvA[e], pvA[e + 1]);
        pA[1][j >> 1] = MF<T>::pack(pvA[8 + e], pvA[9 + e]);
      }
      cB = MF<T>::mma(as_frag<frag>(kf[j]), qB[j], cB);
      pvB[8 + j] = fexp2(fmaf(pvB[8 + j], scale_log2, -uB));
      sb += pvB[j];
      sb += pvB[8 + j];
      if (j & 1) {
        const int e = 2 * (j >> 1);
        pB[0][j >> 1] = MF<T>::pack(pvB[e], pvB[e + 1]);
        pB[1][j >> 1] = MF<T>::pack(pvB[8 + e], pvB[9 + e]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    sa += __shfl_xor(sa, 32, 64);
    sb += __shfl_xor(sb, 32, 64);
    lA += sa;
    lB += sb;
    if ((u & 1) && ((u + 1) >> 1) < ntile) sync_to((u + 1) >> 1);
    {   // sub-tiles straddling the causal diagonal or the key end (the last one or two per wave)
      const int k0 = u * 32;
      if ((k0 + 32 > Sk) || (CAUSAL && k0 + 31 > rA0)) {
        const int base = k0 + 4 * h;
        const int la = CAUSAL ? qa - base : 1 << 20, lb = CAUSAL ? qbq - base : 1 << 20, l2 = Sk - base;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rb = (r & 3) + 8 * (r >> 2);
          cA[r] = ((rb > la) | (rb >= l2)) ? -INFINITY : cA[r];
          cB[r] = ((rb > lb) | (rb >= l2)) ? -INFINITY : cB[r];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- phase 2: P(u-1) V || start of u || K fragments of u + 1
    const unsigned char* kl = smem + (((u + 1) >> 1) & 1) * TILE + ((u + 1) & 1) * 8192;
    float ta = -INFINITY, tb = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int ks = j >> 2, db = j & 3;
      oA[db] = MF<T>::mma(as_frag<frag>(vf[j]), as_frag<frag>(pA[ks]), oA[db]);
      kf[j] = *reinterpret_cast<const u32x4*>(kl + koff[j]);
      if (j < 4) {
        ta = fmaxf(ta, fmaxf(fmaxf(cA[4 * j], cA[4 * j + 1]), fmaxf(cA[4 * j + 2], cA[4 * j + 3])));
        tb = fmaxf(tb, fmaxf(fmaxf(cB[4 * j], cB[4 * j + 1]), fmaxf(cB[4 * j + 2], cB[4 * j + 3])));
      }
      if (j == 4) {
        ta = fmaxf(ta, __shfl_xor(ta, 32, 64)) * scale_log2;
        tb = fmaxf(tb, __shfl_xor(tb, 32, 64)) * scale_log2;
        rsA = !__all(ta <= mA + kThr);
        rsB = !__all(tb <= mB + kThr);
        const float nA = rsA ? fmaxf(mA, ta) : mA, nB = rsB ? fmaxf(mB, tb) : mB;
        const float unA = nA == -INFINITY ? 0.f : nA, unB = nB == -INFINITY ? 0.f : nB;
        alA = rsA ? fexp2(mA - unA) : 1.f;
        alB = rsB ? fexp2(mB - unB) : 1.f;
        mA = nA;
        mB = nB;
        uA = unA;
        uB = unB;
      }
      if (j >= 4) {
        const int r = 2 * (j - 4);
        pvA[r] = fexp2(fmaf(cA[r], scale_log2, -uA));
        pvA[r + 1] = fexp2(fmaf(cA[r + 1], scale_log2, -uA));
        pvA[8 + r] = cA[8 + r];
        pvA[9 + r] = cA[9 + r];
      }
      oB[db] = MF<T>::mma(as_frag<frag>(vf[j]), as_frag<frag>(pB[ks]), oB[db]);
      if (j >= 4) {
        const int r = 2 * (j - 4);
        pvB[r] = fexp2(fmaf(cB[r], scale_log2, -uB));
        pvB[r + 1] = fexp2(fmaf(cB[r + 1], scale_log2, -uB));
        pvB[8 + r] = cB[8 + r];
        pvB[9 + r] = cB[9 + r];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    lA *= alA;
    lB *= alB;
    if (rsA) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oA[i][r] *= alA;
    }
    if (rsB) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int i = 0; i < ND; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) oB[i][r] *= alB;
    }
  };

  using TT = std::true_type;
  using FF = std::false_type;

  if (ntile > 0) {
    load_k(0, 0);
    load_v(0, 0);
    // first sub-tile, the steady loop (a tile-top sync before every even sub-tile), the drain, then
    // the causal tail (barriers / DMAs only). Per-iteration variants inside the loop body make the
    // register allocator spill, hence the peeled first and last steps.
    sync_to(0);
    load_kf(0);
    step(TT{}, FF{}, TT{}, FF{}, 0);
    int u = 1;
    if (PHA_FA4_SLOTS)
      for (; u <= uA_last; ++u) step_steady(u);
    else
      for (; u <= uA_last; ++u) step(TT{}, TT{}, TT{}, TT{}, u);
    if (uA_last == uB_last) {
      step(FF{}, TT{}, FF{}, TT{}, u);   // both drain
    } else {
      step(FF{}, TT{}, TT{}, TT{}, u);   // A drains, B goes on
      for (++u; u <= uB_last; ++u) step(FF{}, FF{}, TT{}, TT{}, u);
      step(FF{}, FF{}, FF{}, TT{}, u);   // B drains
    }
    sync_to(ntile - 1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // no DMA left in flight at exit

  auto store = [&](const f32x16 (&o)[ND], float l, float m, int q) __attribute__((always_inline)) {
    if (q >= S) return;
    const float inv = l > 0.f ? 1.f / l : 0.f;
    T* orow = O + ((long)b * S + q) * fs.o_tok + (long)head * fs.o_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(o[db][4 * gg + 0] * inv, o[db][4 * gg + 1] * inv);
        w[1] = MF<T>::pack(o[db][4 * gg + 2] * inv, o[db][4 * gg + 3] * inv);
        *reinterpret_cast<u32x2*>(orow + d) = w;
      }
    if (h == 0) LSE[((long)b * H + head) * S + q] = (l > 0.f) ? (m + log2f(l)) * kLn2 : INFINITY;
  };
  store(oA, lA, mA, qa);
  store(oB, lB, mB, qbq);
}

// delta[b,h,q] = sum_d dO * O  (fp32)
template <typename T, int D>
__global__ __launch_bounds__(256) void fa_bwd_pre_kernel(const T* __restrict__ O, const T* __restrict__ dO,
                                                         float* __restrict__ delta, int B, int S, int H) {
  // D/8 lanes per (b, q, head) row, 8 elements each: every lane of the wave loads (a whole wave
  // per 128-element row would leave 3/4 of the lanes idle)
  constexpr int LPR = D / 8, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63;
  const long row = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool ok = row < (long)B * S * H;
  float s = 0.f;
  if (ok) {
    const long off = row * D + (lane % LPR) * 8;
    float a[8], g[8];
    Vec8<T>::ld(O + off, a);
    Vec8<T>::ld(dO + off, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] * g[i];
  }
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if (ok && lane % LPR == 0) {
    const int head = row % H;
    const long bq = row / H;
    const int q = bq % S;
    const int b = bq / S;
    delta[((long)b * H + head) * S + q] = s;
  }
}

// ============================================================================================
// Backward = two kernels (no atomics, no cross-workgroup reduction):
//
//  fa_bwd_dkdv_kernel — key-parallel. Workgroup = 4 waves = 128 keys, key on the MFMA lane;
//    each wave keeps its 32 keys' K/V fragments in registers and accumulates dK^T, dV^T over
//    all query tiles (32 rows each; Q/dO tile t+1 prefetched into registers during tile t):
//      S  = Q K^T, dP = dO V^T           C[q][key]  (A = Q / dO rows from LDS)
//      P  = exp2(S c - lse), dS = P (dP - delta)    (row constants broadcast from LDS)
//      dV^T += dO^T P, dK^T += Q^T dS    accumulator-as-B-operand; A = transposed images
//
//  fa_bwd_dq_kernel — query-parallel (the forward's structure). Workgroup = 4 waves = 128
//    queries, query on the lane, Q/dO fragments in registers; per 64-key tile:
//      S^T = K Q^T, dP^T = V dO^T        A = K / V rows (swizzled LDS)
//      dS^T lane-local (the lane's own lse/delta), dQ^T += K^T dS^T (A = K^T image)
// ============================================================================================

// transposed 4-row gather: 4 rows x one 8-wide chunk (4 x u32x4) -> 8 x u32x2 (4 rows each)
__device__ __forceinline__ void write_t4(unsigned char* img, int row_stride_bytes, int chunk, int row0,
                                         const u32x4 (&r)[4]) {
  const uint16_t* e0 = reinterpret_cast<const uint16_t*>(&r[0]);
  const uint16_t* e1 = reinterpret_cast<const uint16_t*>(&r[1]);
  const uint16_t* e2 = reinterpret_cast<const uint16_t*>(&r[2]);
  const uint16_t* e3 = reinterpret_cast<const uint16_t*>(&r[3]);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    u32x2 w;
    w[0] = (uint32_t)e0[e] | ((uint32_t)e1[e] << 16);
    w[1] = (uint32_t)e2[e] | ((uint32_t)e3[e] << 16);
    *reinterpret_cast<u32x2*>(img + (chunk * 8 + e) * row_stride_bytes + row0 * 2) = w;
  }
}

template <typename T, int D, bool CAUSAL, int EXT = 0>
__global__ __launch_bounds__(256) void fa_bwd_dkdv_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                          const T* __restrict__ V, const T* __restrict__ dO,
                                                          const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                          T* __restrict__ dK, T* __restrict__ dV,
                                                          int S, int Sk, int H, int Hk, float scale, FaExt ex) {
  typedef typename MF<T>::frag frag;
  constexpr int NK = D / 16;
  constexpr int ND = D / 32;
  constexpr int CH = D / 8;
  constexpr int BQ = 32;
  constexpr int ROWB = D * 2 + 16;            // [q][d] row images (16-B pad)
  constexpr int TB = (BQ + 4) * 2;            // [d][q] transposed images (row = 72 B)
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BQ * ROWB + 2 * D * TB + 2 * BQ * 4];
  unsigned char* q_lds = smem;
  unsigned char* do_lds = q_lds + BQ * ROWB;
  unsigned char* qt_lds = do_lds + BQ * ROWB;
  unsigned char* dot_lds = qt_lds + D * TB;
  float* lse_lds = reinterpret_cast<float*>(dot_lds + D * TB);
  float* del_lds = lse_lds + BQ;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int head = blockIdx.y, b = blockIdx.z;
  const int hk = head / (H / Hk);
  const int k0 = blockIdx.x * 128;
  const int key = k0 + wid * 32 + lr;
  const long qstride = (long)H * D, kstride = (long)Hk * D;
  const T* Qb = Q + (long)b * S * qstride + (long)head * D;
  const T* dOb = dO + (long)b * S * qstride + (long)head * D;
  const T* Kb = K + (long)b * Sk * kstride + (long)hk * D;
  const T* Vb = V + (long)b * Sk * kstride + (long)hk * D;
  const float* lse_b = LSE + ((long)b * H + head) * S;
  const float* del_b = DELTA + ((long)b * H + head) * S;
  const float scale_log2 = scale * kLog2e;
  // extensions (key on the lane): bias column of this key, dropout stream of the (b, h)
  const float* bcol = (EXT & 1) ? ex.bias + (long)b * ex.sb + (long)head * ex.sh + min(key, Sk - 1) : nullptr;
  const unsigned dstream = (EXT & 2) ? fa_stream(fa_seed(ex), b * H + head) : 0u;

  // keys past Sk read row Sk - 1 (finite; their P and dS are masked to 0 and their dK / dV rows
  // are not stored): unconditional loads, no exec branch per load
  const int keyc = min(key, Sk - 1);
  frag kf[NK], vf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    kf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Kb + (long)keyc * kstride + 16 * kk + 8 * h));
    vf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Vb + (long)keyc * kstride + 16 * kk + 8 * h));
  }
  // retire the fragment loads here, through the builtin (the waitcnt pass tracks it; inline asm
  // it does not): otherwise the loop's MFMAs carry counted waits for them that, in steady state,
  // drain most of the next tile's prefetch (vmcnt counts in issue order)
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt / lgkmcnt untouched
  f32x16 dvt[ND], dkt[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { dvt[i] = zero16(); dkt[i] = zero16(); }

  // staging items: [0, ITEMS) are (4-row group, chunk) of Q, [ITEMS, 2 ITEMS) of dO; thread tid owns
  // items tid + 256 i (one each up to D = 128, two at D = 256)
  constexpr int ITEMS = (BQ / 4) * CH;        // per tensor (D=128: 128, D=64: 64)
  constexpr int SIT = (2 * ITEMS + 255) / 256;
  u32x4 sreg[SIT][4];
  float srow = 0.f;
  auto load_tile = [&](int qt) {
#pragma unroll
    for (int i = 0; i < SIT; ++i) {
      const int item = tid + 256 * i;
      if (item < 2 * ITEMS) {
        const bool is_q = item < ITEMS;
        const int it = is_q ? item : item - ITEMS;
        const int rg = it / CH, ch = it % CH;
        const T* src = is_q ? Qb : dOb;
#pragma unroll
        for (int j = 0; j < 4; ++j) {   // rows past S read row S - 1 (finite, masked to P = 0)
          const int qq = min(qt + rg * 4 + j, S - 1);
          sreg[i][j] = *reinterpret_cast<const u32x4*>(src + (long)qq * qstride + ch * 8);
        }
      }
    }
    if (tid < 2 * BQ) srow = (tid < BQ ? lse_b : del_b)[min(qt + (tid & (BQ - 1)), S - 1)];
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < SIT; ++i) {
      const int item = tid + 256 * i;
      if (item < 2 * ITEMS) {
        const bool is_q = item < ITEMS;
        const int it = is_q ? item : item - ITEMS;
        const int rg = it / CH, ch = it % CH;
        unsigned char* rows = is_q ? q_lds : do_lds;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<u32x4*>(rows + (rg * 4 + j) * ROWB + ch * 16) = sreg[i][j];
        write_t4(is_q ? qt_lds : dot_lds, TB, ch, rg * 4, sreg[i]);
      }
    }
    if (tid < 2 * BQ) (tid < BQ ? lse_lds : del_lds)[tid & (BQ - 1)] = srow;
  };

  const int qstart = CAUSAL ? (k0 / BQ) * BQ : 0;
  if (qstart < S) load_tile(qstart);
  for (int qt = qstart; qt < S; qt += BQ) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (qt + BQ < S) load_tile(qt + BQ);
    if (CAUSAL && (k0 + wid * 32) > (qt + BQ - 1)) continue;   // no query of this tile sees these keys

    f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const u32x4 qa = *reinterpret_cast<const u32x4*>(q_lds + lr * ROWB + (2 * kk + h) * 16);
      const u32x4 ga = *reinterpret_cast<const u32x4*>(do_lds + lr * ROWB + (2 * kk + h) * 16);
      sacc = MF<T>::mma(as_frag<frag>(qa), kf[kk], sacc);
      dpacc = MF<T>::mma(as_frag<frag>(ga), vf[kk], dpacc);
    }
    const bool need_mask = EXT || (qt + BQ > S) || (k0 + 128 > Sk) || (CAUSAL && k0 + wid * 32 + 31 > qt);
    if (need_mask) {
      // branch-free: out-of-range / causal-masked elements become 2^-inf = 0 through a select on the
      // exponent, the bias read is clamped and unconditional (an exec branch per element around
      // it serialised its load latency)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = acc_row(r, h);
        const int qq = qt + ql;
        const bool valid = (qq < S) & (key < Sk) & !(CAUSAL & (key > qq));
        float sv = sacc[r] * scale_log2;
        if constexpr (EXT & 1) sv += bcol[(long)min(qq, S - 1) * ex.sq] * kLog2e;
        float p = fexp2(valid ? sv - lse_lds[ql] * kLog2e : -INFINITY), ds;
        float dpv = dpacc[r];
        if constexpr (EXT & 2) {   // dV sees the dropped P; dS = P (Z dP / (1-rate) - delta)
          const bool kp = fa_keep(fa_row(dstream, qq), key, ex.thresh);
          dpv = kp ? dpv * ex.keep_scale : 0.f;
          ds = p * (dpv - del_lds[ql]);
          p = kp ? p * ex.keep_scale : 0.f;
        } else {
          ds = p * (dpv - del_lds[ql]);
        }
        sacc[r] = p;
        dpacc[r] = ds;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int ql = acc_row(r, h);
        const float p = fexp2(sacc[r] * scale_log2 - lse_lds[ql] * kLog2e);
        sacc[r] = p;
        dpacc[r] = p * (dpacc[r] - del_lds[ql]);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      u32x4 pw, dw;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pw[j] = MF<T>::pack(sacc[8 * s2 + 2 * j], sacc[8 * s2 + 2 * j + 1]);
        dw[j] = MF<T>::pack(dpacc[8 * s2 + 2 * j], dpacc[8 * s2 + 2 * j + 1]);
      }
      const int qbase = 16 * s2 + 4 * h;
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        const unsigned char* r1 = dot_lds + (db * 32 + lr) * TB;
        const unsigned char* r2 = qt_lds + (db * 32 + lr) * TB;
        const u32x2 a0 = *reinterpret_cast<const u32x2*>(r1 + qbase * 2);
        const u32x2 a1 = *reinterpret_cast<const u32x2*>(r1 + (qbase + 8) * 2);
        const u32x2 b0 = *reinterpret_cast<const u32x2*>(r2 + qbase * 2);
        const u32x2 b1 = *reinterpret_cast<const u32x2*>(r2 + (qbase + 8) * 2);
        const u32x4 av = {a0[0], a0[1], a1[0], a1[1]};
        const u32x4 bv = {b0[0], b0[1], b1[0], b1[1]};
        dvt[db] = MF<T>::mma(as_frag<frag>(av), as_frag<frag>(pw), dvt[db]);
        dkt[db] = MF<T>::mma(as_frag<frag>(bv), as_frag<frag>(dw), dkt[db]);
      }
    }
  }
  if (key < Sk) {
    // dK/dV are [B, Sk, H, D] (or strided into a packed QKV gradient: ex.gkv_tok / gkv_head)
    const long gt = ex.gkv_tok ? ex.gkv_tok : (long)H * D;
    const long gh = ex.gkv_head ? ex.gkv_head : D;
    T* dkr = dK + ((long)b * Sk + key) * gt + (long)head * gh;
    T* dvr = dV + ((long)b * Sk + key) * gt + (long)head * gh;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int d = db * 32 + acc_row(r, h);
        Cvt<T>::st(dkr, d, dkt[db][r] * scale);
        Cvt<T>::st(dvr, d, dvt[db][r]);
      }
  }
}

template <typename T, int D, bool CAUSAL, int EXT = 0>
__global__ __launch_bounds__(256) void fa_bwd_dq_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                        const T* __restrict__ V, const T* __restrict__ dO,
                                                        const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                        T* __restrict__ dQ, int S, int Sk, int H, int Hk, float scale,
                                                        FaExt ex) {
  typedef typename MF<T>::frag frag;
  constexpr int CH = D / 8;
  constexpr int ND = D / 32;
  constexpr int NK = D / 16;
  constexpr int KT_STRIDE = (BN + VT_PAD) * 2;  // K^T image row bytes
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BN * D * 2 + D * KT_STRIDE];
  unsigned char* k_lds = smem;                  // K rows (swizzled)
  unsigned char* v_lds = smem + BN * D * 2;     // V rows (swizzled)
  unsigned char* kt_lds = v_lds + BN * D * 2;   // K^T [d][key]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int nqb = (S + BM - 1) / BM;
  const int qb = CAUSAL ? (nqb - 1 - (int)blockIdx.x) : (int)blockIdx.x;
  const int head = blockIdx.y, b = blockIdx.z;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM;
  const int q = q0 + wid * 32 + lr;
  const long qstride = (long)H * D, kstride = (long)Hk * D;
  const T* Qb = Q + (long)b * S * qstride + (long)head * D;
  const T* dOb = dO + (long)b * S * qstride + (long)head * D;
  const T* Kb = K + (long)b * Sk * kstride + (long)hk * D;
  const T* Vb = V + (long)b * Sk * kstride + (long)hk * D;
  const float scale_log2 = scale * kLog2e;
  const float lse2 = (q < S) ? LSE[((long)b * H + head) * S + q] * kLog2e : 0.f;
  const float dlt = (q < S) ? DELTA[((long)b * H + head) * S + q] : 0.f;
  // clamped row (q past S reads row S - 1; its probabilities are masked): read unconditionally
  const float* brow = (EXT & 1) ? ex.bias + (long)b * ex.sb + (long)head * ex.sh + (long)min(q, S - 1) * ex.sq : nullptr;
  const unsigned drow = (EXT & 2) ? fa_row(fa_stream(fa_seed(ex), b * H + head), q) : 0u;

  frag qf[NK], gf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 a = {0, 0, 0, 0}, g = {0, 0, 0, 0};
    if (q < S) {
      a = *reinterpret_cast<const u32x4*>(Qb + (long)q * qstride + 16 * kk + 8 * h);
      g = *reinterpret_cast<const u32x4*>(dOb + (long)q * qstride + 16 * kk + 8 * h);
    }
    qf[kk] = as_frag<frag>(a);
    gf[kk] = as_frag<frag>(g);
  }
  f32x16 dq[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dq[i] = zero16();

  // staging: K as (4-key group, chunk) items -> K rows + K^T image; V as 16-B row chunks
  constexpr int KITEMS = (BN / 4) * CH;
  constexpr int KIT = (KITEMS + 255) / 256;     // K items per thread (2 at D = 256)
  constexpr int VCH = (BN * CH) / 256;
  u32x4 kreg[KIT][4];
  u32x4 vreg[VCH];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < KIT; ++i) {
      const int item = tid + 256 * i;
      if (item < KITEMS) {
        const int kg = item / CH, kch = item % CH;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int kk = k0 + kg * 4 + j;
          kreg[i][j] = (kk < Sk) ? *reinterpret_cast<const u32x4*>(Kb + (long)kk * kstride + kch * 8) : u32x4{0, 0, 0, 0};
        }
      }
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + 256 * i;
      const int kk = k0 + c / CH;
      vreg[i] = (kk < Sk) ? *reinterpret_cast<const u32x4*>(Vb + (long)kk * kstride + (c % CH) * 8) : u32x4{0, 0, 0, 0};
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int i = 0; i < KIT; ++i) {
      const int item = tid + 256 * i;
      if (item < KITEMS) {
        const int kg = item / CH, kch = item % CH;
#pragma unroll
        for (int j = 0; j < 4; ++j) *reinterpret_cast<u32x4*>(k_lds + k_lds_off<D>(kg * 4 + j, kch)) = kreg[i][j];
        write_t4(kt_lds, KT_STRIDE, kch, kg * 4, kreg[i]);
      }
    }
#pragma unroll
    for (int i = 0; i < VCH; ++i) {
      const int c = tid + 256 * i;
      *reinterpret_cast<u32x4*>(v_lds + k_lds_off<D>(c / CH, c % CH)) = vreg[i];
    }
  };

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM);
  const int wave_qmax = q0 + wid * 32 + 31;
  if (kend > 0) load_tile(0);
  for (int k0 = 0; k0 < kend; k0 += BN) {
    __syncthreads();
    store_tile();
    __syncthreads();
    if (k0 + BN < kend) load_tile(k0 + BN);
    if (CAUSAL && k0 > wave_qmax) continue;
    f32x16 s[2], dp[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      s[kb] = zero16();
      dp[kb] = zero16();
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const u32x4 a = *reinterpret_cast<const u32x4*>(k_lds + k_lds_off<D>(kb * 32 + lr, 2 * kk + h));
        const u32x4 c = *reinterpret_cast<const u32x4*>(v_lds + k_lds_off<D>(kb * 32 + lr, 2 * kk + h));
        s[kb] = MF<T>::mma(as_frag<frag>(a), qf[kk], s[kb]);
        dp[kb] = MF<T>::mma(as_frag<frag>(c), gf[kk], dp[kb]);
      }
    }
    const bool need_mask = EXT || (k0 + BN > Sk) || (CAUSAL && k0 + BN - 1 > q0 + wid * 32);
    if (need_mask) {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kk = k0 + kb * 32 + acc_row(r, h);
          // branch-free (select on the exponent, clamped unconditional bias read)
          const bool ok = (kk < Sk) & !(CAUSAL & (kk > q));
          float sv = s[kb][r] * scale_log2;
          if constexpr (EXT & 1) sv += brow[min(kk, Sk - 1)] * kLog2e;
          const float p = fexp2(ok ? sv - lse2 : -INFINITY);
          float dpv = dp[kb][r];
          if constexpr (EXT & 2) dpv = fa_keep(drow, kk, ex.thresh) ? dpv * ex.keep_scale : 0.f;
          s[kb][r] = p * (dpv - dlt);   // dS^T
        }
    } else {
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) s[kb][r] = fexp2(s[kb][r] * scale_log2 - lse2) * (dp[kb][r] - dlt);
    }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const f32x16& sv = s[ks >> 1];
      const int s8 = (ks & 1) * 8;
      u32x4 pw;
      pw[0] = MF<T>::pack(sv[s8 + 0], sv[s8 + 1]);
      pw[1] = MF<T>::pack(sv[s8 + 2], sv[s8 + 3]);
      pw[2] = MF<T>::pack(sv[s8 + 4], sv[s8 + 5]);
      pw[3] = MF<T>::pack(sv[s8 + 6], sv[s8 + 7]);
      const frag pf = as_frag<frag>(pw);
      const int kbase = 16 * ks + 4 * h;
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        const unsigned char* row = kt_lds + (db * 32 + lr) * KT_STRIDE;
        const u32x2 lo = *reinterpret_cast<const u32x2*>(row + kbase * 2);
        const u32x2 hi = *reinterpret_cast<const u32x2*>(row + (kbase + 8) * 2);
        const u32x4 a = {lo[0], lo[1], hi[0], hi[1]};
        dq[db] = MF<T>::mma(as_frag<frag>(a), pf, dq[db]);
      }
    }
  }
  if (q < S) {
    T* qrow = dQ + ((long)b * S + q) * (ex.gq_tok ? ex.gq_tok : qstride) + (long)head * (ex.gq_head ? ex.gq_head : D);
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = db * 32 + 8 * g + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(dq[db][4 * g + 0] * scale, dq[db][4 * g + 1] * scale);
        w[1] = MF<T>::pack(dq[db][4 * g + 2] * scale, dq[db][4 * g + 3] * scale);
        *reinterpret_cast<u32x2*>(qrow + d) = w;
      }
  }
}

// ============================================================================================
// Backward v2 (D = 128): 8-wave workgroups, one row-major LDS image per operand tile read
// both by rows (ds_read_b128) and transposed (ds_read_b64_tr_b16) — the dual-use image of
// T10 (256-B rows, chunk ^ ((row&3)<<2 | (row>>2)&3)), double-buffered, one barrier per tile.
//
//  fa_bwd_dkdv_v2: 128 keys per workgroup (4 waves, 32 per wave, key on the lane, K/V fragments and
//    dK^T/dV^T accumulators in registers); 64-query tiles processed as two 32-row halves:
//      S = Q K^T, dP = dO V^T        A = Q / dO rows (row reads)
//      dV^T += dO^T P, dK^T += Q^T dS  A = dO^T / Q^T (transposed reads), B = accumulators
//  fa_bwd_dq_v2: 256 queries per workgroup (query on the lane, Q/dO fragments in registers);
//    64-key tiles:  S^T = K Q^T, dP^T = V dO^T (row reads), dQ^T += K^T dS^T (tr reads of K).
// ============================================================================================

// 4 waves (128 keys) with one wave per SIMD: the per-wave state (K/V fragments 64 regs, dK^T/dV^T
// 128, S/dP 32, staging 32) exceeds the 256-register share two waves per SIMD would leave.
constexpr int NTKV = 256;

// A/B-measured code-shape switches (tools/bench_fa.py, B=8 S=2048 H=16 D=128 causal, backward):
// a separate unmasked probability loop for the interior tiles pays in dK/dV (0.938 -> 0.811 ms with
// the bare exp) but not in dQ (0.945 -> 1.105 ms: the dQ loop's schedule degrades); the bare
// v_exp_f32 pays in dQ too (0.848 -> 0.811 ms). profiles/flash_attn_exp_mask_ab_r2.log
constexpr bool kSplitMaskDkdv = true;
constexpr bool kSplitMaskDq = false;
constexpr bool kDqBareExp = true;
constexpr bool kDkdvGroups = PHA_FA_GROUPS & 1;   // fa_bwd_dkdv_v3's sched_group_barrier interleave
#ifndef PHA_DKDV_AHEAD
#define PHA_DKDV_AHEAD 16
#endif
constexpr int kDkdvAhead = PHA_DKDV_AHEAD;   // operand reads issued before the first S / dP MFMA
#ifndef PHA_DKDV_ASM_SP
#define PHA_DKDV_ASM_SP 1
#endif
constexpr bool kDkdvAsmSP = PHA_DKDV_ASM_SP;   // fa_bwd_dkdv_v3: S / dP chains as asm MFMAs into VGPRs
constexpr bool kDqGroups = (PHA_FA_GROUPS >> 1) & 1;   // fa_bwd_dq_v3's read-ahead interleave
#ifndef PHA_DQ_AHEAD
#define PHA_DQ_AHEAD 8
#endif
constexpr int kDqAhead = PHA_DQ_AHEAD;

template <typename T, bool CAUSAL, bool ILP2>
__global__ __launch_bounds__(NTKV) __attribute__((amdgpu_waves_per_eu(1, 1))) void fa_bwd_dkdv_v2(const T* __restrict__ Q, const T* __restrict__ K,
                                                      const T* __restrict__ V, const T* __restrict__ dO,
                                                      const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                      T* __restrict__ dK, T* __restrict__ dV, int S, int Sk, int H,
                                                      int Hk, float scale, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int D = 128, NK = 8, ND = 4, BQ = 64;
  constexpr int IMG = BQ * 256;                         // 16 KiB per operand image
  constexpr int BUF = 2 * IMG + 2 * BQ * 4;             // Q, dO, lse, delta
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / ((Sk + NTKV / 2 - 1) / (NTKV / 2)), (Sk + NTKV / 2 - 1) / (NTKV / 2), fs.order_g, bh, rank);
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int k0 = rank * (NTKV / 2);
  const int wk0 = k0 + wid * 32;
  const int key = wk0 + lr;
  const long kstride = fs.kv_tok;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const float* lse_b = LSE + ((long)b * H + head) * S;
  const float* del_b = DELTA + ((long)b * H + head) * S;
  const float scale_log2 = scale * kLog2e;

  // keys past Sk read row Sk - 1 (finite; their P and dS are masked to 0 and their dK / dV rows
  // are not stored): unconditional loads, no exec branch per load
  const int keyc = min(key, Sk - 1);
  frag kf[NK], vf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    kf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Kb + (long)keyc * kstride + 16 * kk + 8 * h));
    vf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Vb + (long)keyc * kstride + 16 * kk + 8 * h));
  }
  // retire the fragment loads here, through the builtin (the waitcnt pass tracks it; inline asm
  // it does not): otherwise the loop's MFMAs carry counted waits for them that, in steady state,
  // drain most of the next tile's prefetch (vmcnt counts in issue order)
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt / lgkmcnt untouched
  f32x16 dvt[ND], dkt[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { dvt[i] = zero16(); dkt[i] = zero16(); }

  // staging: 64 rows x 16 chunks for Q and dO = 2048 chunks, 8 per thread; lse/delta 128 floats
  constexpr int SPT = 2048 / NTKV;
  u32x4 sreg[SPT];
  float srow = 0.f;
  auto load_tile = [&](int qt) {
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int c = tid + NTKV * i;              // [0, 2048): first 1024 Q, then dO
      const int which = c >> 10, cc = c & 1023;
      const int row = cc >> 4, ch = cc & 15;
      // rows past S read row S - 1 (finite, and masked to P = 0): no exec branch per load
      const int qq = min(qt + row, S - 1);
      const T* src = which ? dOb : Qb;
      const long rs = which ? fs.o_tok : fs.q_tok;
      sreg[i] = *reinterpret_cast<const u32x4*>(src + (long)qq * rs + ch * 8);
    }
    // raw value: any arithmetic on it here would wait (in-order vmcnt) for the whole prefetch
    // issued just above; the log2(e) scaling happens in store_tile, after the tile's MFMAs
    if (tid < 2 * BQ) srow = (tid < BQ ? lse_b : del_b)[min(qt + (tid & (BQ - 1)), S - 1)];
  };
  auto store_tile = [&](int buf) {
    unsigned char* base = smem + buf * BUF;
#pragma unroll
    for (int i = 0; i < SPT; ++i) {
      const int c = tid + NTKV * i;
      const int which = c >> 10, cc = c & 1023;
      *reinterpret_cast<u32x4*>(base + which * IMG + dual_off(cc >> 4, cc & 15)) = sreg[i];
    }
    if (tid < 2 * BQ) reinterpret_cast<float*>(base + 2 * IMG)[tid] = tid < BQ ? srow * kLog2e : srow;
  };

  const int qstart = CAUSAL ? (k0 / BQ) * BQ : 0;
  const int ntile = qstart < S ? (S - qstart + BQ - 1) / BQ : 0;
  if (ntile > 0) {
    load_tile(qstart);
    store_tile(0);
    __syncthreads();
  }
  for (int t = 0; t < ntile; ++t) {
    const int qt = qstart + t * BQ;
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(qt + BQ);
    const unsigned char* q_img = smem + cur * BUF;
    const unsigned char* do_img = q_img + IMG;
    const float* lse_l = reinterpret_cast<const float*>(q_img + 2 * IMG);
    const float* del_l = lse_l + BQ;
    // ILP2: both 32-row halves unrolled so the scheduler can overlap one half's LDS reads and
    // softmax with the other's MFMAs (one wave per SIMD has no other wave to hide latency)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (!ILP2 && half == 1) __builtin_amdgcn_sched_barrier(0);
      const int qh = qt + half * 32;
      if (CAUSAL && wk0 > qh + 31) continue;      // every key of this wave is after every query
      f32x16 sacc = zero16(), dpacc = zero16();
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const int row = half * 32 + lr;
        const u32x4 qa = *reinterpret_cast<const u32x4*>(q_img + dual_off(row, 2 * kk + h));
        const u32x4 ga = *reinterpret_cast<const u32x4*>(do_img + dual_off(row, 2 * kk + h));
        sacc = MF<T>::mma(as_frag<frag>(qa), kf[kk], sacc);
        dpacc = MF<T>::mma(as_frag<frag>(ga), vf[kk], dpacc);
      }
      const bool need_mask = (qh + 32 > S) || (wk0 + 32 > Sk) || (CAUSAL && wk0 + 31 > qh);
      // the mask test is wave-uniform: the unmasked version (all but the diagonal / ragged
      // tiles) carries no per-element compares and selects
      auto probs = [&](auto masked_c) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ql = half * 32 + acc_row(r, h);
          float x = sacc[r] * scale_log2 - lse_l[ql];
          if constexpr (decltype(masked_c)::value) {
            // select on the exponent (2^-inf = 0): a select after the exp became an exec
            // branch per element
            const int qq = qt + ql;
            // bitwise, not short-circuit: || became branches around the lse read
            const bool out = (qq >= S) | (key >= Sk) | (CAUSAL & (key > qq));
            x = out ? -INFINITY : x;
          }
          const float p = fexp2(x);
          sacc[r] = p;
          dpacc[r] = p * (dpacc[r] - del_l[ql]);
        }
      };
      if (!kSplitMaskDkdv || need_mask) probs(std::true_type{});
      else probs(std::false_type{});
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 pw, dw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pw[j] = MF<T>::pack(sacc[8 * s2 + 2 * j], sacc[8 * s2 + 2 * j + 1]);
          dw[j] = MF<T>::pack(dpacc[8 * s2 + 2 * j], dpacc[8 * s2 + 2 * j + 1]);
        }
        const int r0 = half * 32 + 16 * s2 + 4 * h;
#pragma unroll
        for (int db = 0; db < ND; ++db) {
          const u32x4 av = tr_frag(do_img, r0, db, g, tq, tp);
          const u32x4 bv = tr_frag(q_img, r0, db, g, tq, tp);
          dvt[db] = MF<T>::mma(as_frag<frag>(av), as_frag<frag>(pw), dvt[db]);
          dkt[db] = MF<T>::mma(as_frag<frag>(bv), as_frag<frag>(dw), dkt[db]);
        }
      }
    }
    if (t + 1 < ntile) store_tile(cur ^ 1);
    __syncthreads();
  }
  if (key < Sk) {
    T* dkr = dK + ((long)b * Sk + key) * fs.dkv_tok + (long)head * fs.dkv_head;   // per query head (GQA summed by caller)
    T* dvr = dV + ((long)b * Sk + key) * fs.dkv_tok + (long)head * fs.dkv_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 wk, wv;
        wk[0] = MF<T>::pack(dkt[db][4 * gg + 0] * scale, dkt[db][4 * gg + 1] * scale);
        wk[1] = MF<T>::pack(dkt[db][4 * gg + 2] * scale, dkt[db][4 * gg + 3] * scale);
        wv[0] = MF<T>::pack(dvt[db][4 * gg + 0], dvt[db][4 * gg + 1]);
        wv[1] = MF<T>::pack(dvt[db][4 * gg + 2], dvt[db][4 * gg + 3]);
        *reinterpret_cast<u32x2*>(dkr + d) = wk;
        *reinterpret_cast<u32x2*>(dvr + d) = wv;
      }
  }
}


// D (VGPR) += A (VGPR) * B (AGPR) on the 32x32x16 MFMA, D tied in place
template <typename T>
__device__ __forceinline__ void mma_vva(f32x16& d, const u32x4& a, const typename MF<T>::frag& b) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const v4u va = __builtin_bit_cast(v4u, a), vb = __builtin_bit_cast(v4u, b);
  if constexpr (std::is_same<T, bf16_t>::value)
    asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(d) : "v"(va), "a"(vb));
  else
    asm volatile("v_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+v"(d) : "v"(va), "a"(vb));
}

// ============================================================================================
// Backward v3 dK/dV (D = 128, default): fa_bwd_dkdv_v2's geometry (4 waves, 32 keys per wave on
// the lane, K/V fragments and dK^T/dV^T in registers, 64-query tiles as two 32-row halves) with
//  * the row constants as the initial accumulators (CDNA guide App. B "Attention backward"): the
//    S chain starts from -lse/scale and the dP chain from -delta (4 + 4 ds_read_b128 per half
//    instead of 32 scalar reads), so p = exp2(c S') and dS = p dP' need no subtractions;
//  * a software pipeline over halves: step j issues half j's S/dP MFMAs (16) in the same basic
//    block as half j-1's probabilities (VALU) and its dV/dK MFMAs (16), so one wave per SIMD
//    always has independent MFMAs to cover the exp / pack work and the LDS latencies;
//  * a 3-deep Q/dO ring (99 KB): the half pending from the previous tile still reads its buffer
//    while the next tile is written, so one barrier per tile stays enough.
// ============================================================================================
template <typename T, bool CAUSAL>
__global__ __launch_bounds__(NTKV) __attribute__((amdgpu_waves_per_eu(1, 1))) void fa_bwd_dkdv_v3(const T* __restrict__ Q, const T* __restrict__ K,
                                                      const T* __restrict__ V, const T* __restrict__ dO,
                                                      const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                      T* __restrict__ dK, T* __restrict__ dV, int S, int Sk, int H,
                                                      int Hk, float scale, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int NK = 8, ND = 4, BQ = 64;
  constexpr int IMG = BQ * 256;                         // 16 KiB per operand image
  constexpr int BUF = 2 * IMG + 2 * BQ * 4;             // Q, dO, -lse/scale, -delta
  __shared__ __attribute__((aligned(16))) unsigned char smem[3 * BUF];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5, lr = lane & 31;
  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / ((Sk + NTKV / 2 - 1) / (NTKV / 2)), (Sk + NTKV / 2 - 1) / (NTKV / 2), fs.order_g, bh, rank);
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int k0 = rank * (NTKV / 2);
  const int wk0 = k0 + wid * 32;
  const int key = wk0 + lr;
  const long kstride = fs.kv_tok;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const float* lse_b = LSE + ((long)b * H + head) * S;
  const float* del_b = DELTA + ((long)b * H + head) * S;
  const float c2 = scale * kLog2e, nis = -1.f / scale;

  const int keyc = min(key, Sk - 1);
  frag kf[NK], vf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    kf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Kb + (long)keyc * kstride + 16 * kk + 8 * h));
    vf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Vb + (long)keyc * kstride + 16 * kk + 8 * h));
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): see fa_bwd_dkdv_v2
  f32x16 dvt[ND], dkt[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { dvt[i] = zero16(); dkt[i] = zero16(); }

  // Q / dO tiles by LDS-DMA (no staging registers): wave w issues the 1-KiB pieces w*8 .. w*8+7
  // (piece = 4 rows of one operand); lane l writes physical chunk l & 15 of row l >> 4, so it
  // fetches the logical chunk (l & 15) ^ swizzle(row) of dual_off's image
  float srow = 0.f;
  auto load_tile = [&](int qt, int buf) {
    const unsigned lds = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)(smem + buf * BUF);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int gidx = wid * 8 + u, which = gidx >> 4;
      const int row = (gidx & 15) * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      const long rs = which ? fs.o_tok : fs.q_tok;
      const T* base = (which ? dOb : Qb) + (long)qt * rs;
      const unsigned voff = (unsigned)(((long)(min(qt + row, S - 1) - qt) * rs + ch * 8) * 2);
      fa_glds16(voff, base, __builtin_amdgcn_readfirstlane(lds + which * IMG + (gidx & 15) * 1024));
    }
    if (tid < 2 * BQ) srow = (tid < BQ ? lse_b : del_b)[min(qt + (tid & (BQ - 1)), S - 1)];
  };
  auto store_rc = [&](int buf) {   // row constants (the DMA'd images need no store)
    if (tid < 2 * BQ) reinterpret_cast<float*>(smem + buf * BUF + 2 * IMG)[tid] = tid < BQ ? srow * nis : -srow;
  };

  // step of half j (parity P): A = its S / dP chains (row constants as the initial accumulators;
  // masked scores start at -inf, so no per-element select is left after the MFMAs), C = the
  // dV / dK MFMAs of the pending half j-1 (packed P / dS in pw[P^1], dw[P^1], its image pimg),
  // then B = half j's probabilities packed into pw[P], dw[P]. C's 16 MFMAs cover B's VALU (B
  // waits only for A's results), and only the packed half (16 registers) crosses steps. One code
  // path per half (the mask is a branch around the initial values only): step variants behind
  // branches made the register allocator spill the K / V fragments.
  u32x4 pw[2][2], dw[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) { pw[i][j] = u32x4{0, 0, 0, 0}; dw[i][j] = u32x4{0, 0, 0, 0}; }
  // lane parts of the LDS read addresses; the parity / 16-row block / buffer parts are immediates
  // or one scalar base (dual_off's swizzle reduces to these for rows 32P + lr and the transposed
  // rows 32Q + 16 s2 + 4h + tq (+8))
  int aoff[NK], troff[ND][2];
  {
    const int fr = ((lr & 3) << 2) | ((lr >> 2) & 3);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) aoff[kk] = lr * 256 + 16 * ((2 * kk + h) ^ fr);
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi)
        troff[db][hi] = (4 * h + tq) * 256 + hi * 2048 +
                        16 * (4 * (db ^ tq) + ((2 * (g & 1) + (tp >> 1)) ^ ((h + 2 * hi) & 3))) + 8 * (tp & 1);
  }
  const int rcoff = 4 * h * 4;
  auto lds_b128 = [&](const unsigned char* base, int off) { return *reinterpret_cast<const u32x4*>(base + off); };
  auto trf = [&](const unsigned char* base, int db) {
    const u32x2 lo = ds_read_tr16(base + troff[db][0]);
    const u32x2 hi = ds_read_tr16(base + troff[db][1]);
    return u32x4{lo[0], lo[1], hi[0], hi[1]};
  };
  auto step = [&](auto par_c, auto a_c, const unsigned char* img, int qh, bool msk, const unsigned char* pimg) {
    constexpr int P = decltype(par_c)::value, Q = P ^ 1;
    constexpr bool DA = decltype(a_c)::value;
    f32x16 sa, da;
    // C's transposed operand reads (issued under A's MFMAs)
    u32x4 cav[2][ND], cbv[2][ND];
    auto read_c = [&]() {
      const unsigned char* pdo = pimg + IMG;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int db = 0; db < ND; ++db) {
          cav[s2][db] = trf(pdo + Q * 8192 + s2 * 4096, db);
          cbv[s2][db] = trf(pimg + Q * 8192 + s2 * 4096, db);
        }
    };
    if constexpr (DA) {
      const unsigned char* rc = img + 2 * IMG + rcoff + P * 128;
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const float4 l4 = *reinterpret_cast<const float4*>(rc + 32 * jj);
        const float4 d4 = *reinterpret_cast<const float4*>(rc + BQ * 4 + 32 * jj);
        sa[4 * jj + 0] = l4.x; sa[4 * jj + 1] = l4.y; sa[4 * jj + 2] = l4.z; sa[4 * jj + 3] = l4.w;
        da[4 * jj + 0] = d4.x; da[4 * jj + 1] = d4.y; da[4 * jj + 2] = d4.z; da[4 * jj + 3] = d4.w;
      }
      if (msk) {
        // query qh + 4h + rowb(r): masked when past S, when the key is past Sk, or (causal) when
        // the key is after the query
        const int lim = key >= Sk ? 32 : (CAUSAL ? key - qh - 4 * h : -1);
        const int lim2 = S - qh - 4 * h;
        const float mval = c2 > 0.f ? -INFINITY : INFINITY;   // exp2(c2 * mval) = 0 for either sign
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rb = (r & 3) + 8 * (r >> 2);
          sa[r] = ((rb < lim) | (rb >= lim2)) ? mval : sa[r];
        }
      }
      const unsigned char* do_img = img + IMG;
      if constexpr (kDkdvAsmSP) {
        // all 16 operand reads, then C's 32 transposed reads, then the S / dP chains as asm MFMAs
        // accumulating in VGPRs (the probability VALU reads them with no accvgpr copies; K / V
        // fragments come from AGPRs). Inline asm is opaque to the scheduler's grouping, so the
        // order is fixed in the source: reads first, one LDS latency per step.
        u32x4 qa[NK], ga[NK];
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          qa[kk] = lds_b128(img + P * 8192, aoff[kk]);
          ga[kk] = lds_b128(do_img + P * 8192, aoff[kk]);
        }
        read_c();
        __builtin_amdgcn_sched_barrier(0);
        asm volatile("s_nop 1" ::: "memory");   // a VALU write of the initial values (mask select)
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          mma_vva<T>(sa, qa[kk], kf[kk]);
          mma_vva<T>(da, ga[kk], vf[kk]);
        }
        // an MFMA's VGPR result read by VALU needs 18 wait states after its issue (16-pass
        // 32x32x16); the compiler does not insert them behind inline asm
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      } else {
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const u32x4 qa = lds_b128(img + P * 8192, aoff[kk]);
          const u32x4 ga = lds_b128(do_img + P * 8192, aoff[kk]);
          sa = MF<T>::mma(as_frag<frag>(qa), kf[kk], sa);
          da = MF<T>::mma(as_frag<frag>(ga), vf[kk], da);
        }
      }
    }
    if constexpr (!(DA && kDkdvAsmSP)) read_c();
    if constexpr (DA && kDkdvGroups && !kDkdvAsmSP) {
      // region 1 (CDNA guide T19): all 16 A operand reads first (one LDS latency per step, not
      // one per MFMA pair), then A's 16 MFMAs each with two of C's 32 transposed reads
      __builtin_amdgcn_sched_group_barrier(0x100, kDkdvAhead, 0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, (48 - kDkdvAhead + 15) / 16, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // region 2: C's MFMAs with B's VALU (B waits only for A's last MFMAs)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int db = 0; db < ND; ++db) {
        dvt[db] = MF<T>::mma(as_frag<frag>(cav[s2][db]), as_frag<frag>(pw[Q][s2]), dvt[db]);
        dkt[db] = MF<T>::mma(as_frag<frag>(cbv[s2][db]), as_frag<frag>(dw[Q][s2]), dkt[db]);
      }
    if constexpr (DA) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(sa[r] * c2);
        sa[r] = p;
        da[r] = p * da[r];
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pw[P][s2][j] = MF<T>::pack(sa[8 * s2 + 2 * j], sa[8 * s2 + 2 * j + 1]);
          dw[P][s2][j] = MF<T>::pack(da[8 * s2 + 2 * j], da[8 * s2 + 2 * j + 1]);
        }
      if constexpr (kDkdvGroups) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        }
      }
    }
  };
  using yes = std::true_type;
  using no = std::false_type;
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  auto needm = [&](int qh) { return (qh + 32 > S) || (wk0 + 32 > Sk) || (CAUSAL && wk0 + 31 > qh); };

  const int qstart = CAUSAL ? (k0 / BQ) * BQ : 0;
  const int ntile = qstart < S ? (S - qstart + BQ - 1) / BQ : 0;
  if (ntile > 0) {
    load_tile(qstart, 0);
    store_rc(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // halves whose keys all follow all their queries are skipped (causal, at the start only); the
  // first step's C then multiplies the zero-initialised pw / dw (adds nothing)
  bool pend = false;
  const unsigned char* pimg = smem;
  int buf = 0;
  for (int t = 0; t < ntile; ++t) {
    const int qt = qstart + t * BQ;
    const int nbuf = buf == 2 ? 0 : buf + 1;
    if (t + 1 < ntile) load_tile(qt + BQ, nbuf);
    const unsigned char* img = smem + buf * BUF;
    if (!(CAUSAL && wk0 > qt + 31)) {
      step(P0{}, yes{}, img, qt, needm(qt), pimg);
      pend = true;
      pimg = img;
    }
    if (!(CAUSAL && wk0 > qt + 63)) {
      step(P1{}, yes{}, img, qt + 32, needm(qt + 32), pimg);
      pend = true;
      pimg = img;
    }
    buf = nbuf;
    if (t + 1 < ntile) store_rc(buf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA'd tile has landed (asm: untracked)
    __syncthreads();
  }
  if (pend) step(P0{}, no{}, smem, 0, false, pimg);   // C of the last half (parity 1)
  if (key < Sk) {
    T* dkr = dK + ((long)b * Sk + key) * fs.dkv_tok + (long)head * fs.dkv_head;
    T* dvr = dV + ((long)b * Sk + key) * fs.dkv_tok + (long)head * fs.dkv_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 wk, wv;
        wk[0] = MF<T>::pack(dkt[db][4 * gg + 0] * scale, dkt[db][4 * gg + 1] * scale);
        wk[1] = MF<T>::pack(dkt[db][4 * gg + 2] * scale, dkt[db][4 * gg + 3] * scale);
        wv[0] = MF<T>::pack(dvt[db][4 * gg + 0], dvt[db][4 * gg + 1]);
        wv[1] = MF<T>::pack(dvt[db][4 * gg + 2], dvt[db][4 * gg + 3]);
        *reinterpret_cast<u32x2*>(dkr + d) = wk;
        *reinterpret_cast<u32x2*>(dvr + d) = wv;
      }
  }
}

// dQ v3 (default): fa_bwd_dq_v2's geometry with K / V tiles by LDS-DMA (no staging registers, no
// ds_write), the mask folded into the S^T chain's initial accumulator (-inf where masked, so the
// probability loop is one code path with no selects), and each 32-key block's 16 row reads issued
// ahead of its MFMAs (one LDS latency per block).
template <typename T, bool CAUSAL>
// Od (optional): the forward output — delta = rowsum(dO * O) is then formed here from the dO
// fragments already in registers and stored to DELTA for the dK/dV kernel launched after this one
// (no separate preprocess pass re-reading dO).
__global__ __launch_bounds__(NT2) void fa_bwd_dq_v3(const T* __restrict__ Q, const T* __restrict__ K,
                                                    const T* __restrict__ V, const T* __restrict__ dO,
                                                    const float* __restrict__ LSE, float* __restrict__ DELTA,
                                                    T* __restrict__ dQ, int S, int Sk, int H, int Hk, float scale, FaStrides fs,
                                                    const T* __restrict__ Od = nullptr) {
  typedef typename MF<T>::frag frag;
  constexpr int NK = 8, ND = 4;
  constexpr int IMG = BN * 256;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            lr = lane & 31;
  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nqb = (S + BM2 - 1) / BM2;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / nqb, nqb, fs.order_g, bh, rank);
  const int qb = CAUSAL ? (nqb - 1 - rank) : rank;
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM2;
  const int wq0 = q0 + wid * 32;
  const int q = wq0 + lr;
  const long kstride = fs.kv_tok;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const float scale_log2 = scale * kLog2e;
  const float lse2 = (q < S) ? LSE[((long)b * H + head) * S + q] * kLog2e : 0.f;

  frag qf[NK], gf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
    if (q < S) {
      a = *reinterpret_cast<const u32x4*>(Qb + (long)q * fs.q_tok + 16 * kk + 8 * h);
      c = *reinterpret_cast<const u32x4*>(dOb + (long)q * fs.o_tok + 16 * kk + 8 * h);
    }
    qf[kk] = as_frag<frag>(a);
    gf[kk] = as_frag<frag>(c);
  }
  float dlt;
  if (Od) {   // O shares dO's strides (both dense [B, S, H, D] outputs)
    const T* Ob = Od + (long)b * S * fs.o_tok + (long)head * fs.o_head;
    float sdl = 0.f;
    if (q < S) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const frag of = as_frag<frag>(*reinterpret_cast<const u32x4*>(Ob + (long)q * fs.o_tok + 16 * kk + 8 * h));
#pragma unroll
        for (int i = 0; i < 8; ++i) sdl += (float)gf[kk][i] * (float)of[i];
      }
    }
    dlt = sdl + __shfl_xor(sdl, 32, 64);
    if (h == 0 && q < S) DELTA[((long)b * H + head) * S + q] = dlt;
  } else {
    dlt = (q < S) ? DELTA[((long)b * H + head) * S + q] : 0.f;
  }
  f32x16 dq[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dq[i] = zero16();

  // K / V tile (64 keys) by LDS-DMA: 32 1-KiB pieces (4 rows of one operand), 4 per wave
  auto load_tile = [&](int k0, int buf) {
    const unsigned lds = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)(smem + buf * 2 * IMG);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int gidx = wid * 4 + u, which = gidx >> 4;
      const int row = (gidx & 15) * 4 + (lane >> 4);
      const int ch = (lane & 15) ^ (((row & 3) << 2) | ((row >> 2) & 3));
      const T* base = (which ? Vb : Kb) + (long)k0 * kstride;
      const unsigned voff = (unsigned)(((long)(min(k0 + row, Sk - 1) - k0) * kstride + ch * 8) * 2);
      fa_glds16(voff, base, __builtin_amdgcn_readfirstlane(lds + which * IMG + (gidx & 15) * 1024));
    }
  };

  // lane parts of the LDS addresses (see fa_bwd_dkdv_v3): key rows kb*32 + lr, transposed rows
  // kb*32 + 16 s2 + 4h + tq (+8)
  int aoff[NK], troff[ND][2];
  {
    const int fr = ((lr & 3) << 2) | ((lr >> 2) & 3);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) aoff[kk] = lr * 256 + 16 * ((2 * kk + h) ^ fr);
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int hi = 0; hi < 2; ++hi)
        troff[db][hi] = (4 * h + tq) * 256 + hi * 2048 +
                        16 * (4 * (db ^ tq) + ((2 * (g & 1) + (tp >> 1)) ^ ((h + 2 * hi) & 3))) + 8 * (tp & 1);
  }

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM2);
  const int ntile = (kend + BN - 1) / BN;
  if (ntile > 0) {
    load_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  const float mval = scale_log2 > 0.f ? -INFINITY : INFINITY;   // exp2(mval * c) = 0 for either sign
  if (fs.prio != 0 && wid < 4) __builtin_amdgcn_s_setprio(1);   // see fa_fwd_v3_kernel
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * BN;
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(k0 + BN, cur ^ 1);
    const unsigned char* k_img = smem + cur * 2 * IMG;
    const unsigned char* v_img = k_img + IMG;
    if (!(CAUSAL && k0 > wq0 + 31)) {
      const bool need_mask = (k0 + BN > Sk) || (CAUSAL && k0 + BN - 1 > wq0);
#pragma unroll 1
      for (int kb = 0; kb < 2; ++kb) {
        if (CAUSAL && k0 + kb * 32 > wq0 + 31) break;   // every key of the block after every query
        f32x16 st = zero16(), dpt = zero16();
        if (need_mask) {
          // key k0 + 32kb + 4h + rowb(r): masked past Sk or (causal) after the lane's query
          const int base = k0 + kb * 32 + 4 * h;
          const int lim1 = CAUSAL ? q - base : 1 << 20, lim2 = Sk - base;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rb = (r & 3) + 8 * (r >> 2);
            st[r] = ((rb > lim1) | (rb >= lim2)) ? mval : 0.f;
          }
        }
        const unsigned char* kbi = k_img + kb * 8192;
        const unsigned char* vbi = v_img + kb * 8192;
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const u32x4 ka = *reinterpret_cast<const u32x4*>(kbi + aoff[kk]);
          const u32x4 va = *reinterpret_cast<const u32x4*>(vbi + aoff[kk]);
          st = MF<T>::mma(as_frag<frag>(ka), qf[kk], st);
          dpt = MF<T>::mma(as_frag<frag>(va), gf[kk], dpt);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(st[r], scale_log2, -lse2));
          dpt[r] = p * (dpt[r] - dlt);
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int s8 = s2 * 8;
          u32x4 pw;
          pw[0] = MF<T>::pack(dpt[s8 + 0], dpt[s8 + 1]);
          pw[1] = MF<T>::pack(dpt[s8 + 2], dpt[s8 + 3]);
          pw[2] = MF<T>::pack(dpt[s8 + 4], dpt[s8 + 5]);
          pw[3] = MF<T>::pack(dpt[s8 + 6], dpt[s8 + 7]);
          const frag pf = as_frag<frag>(pw);
#pragma unroll
          for (int db = 0; db < ND; ++db) {
            const unsigned char* tb = kbi + s2 * 4096;
            const u32x2 lo = ds_read_tr16(tb + troff[db][0]);
            const u32x2 hi = ds_read_tr16(tb + troff[db][1]);
            dq[db] = MF<T>::mma(as_frag<frag>(u32x4{lo[0], lo[1], hi[0], hi[1]}), pf, dq[db]);
          }
        }
        if constexpr (kDqGroups) {
          // the 16 row reads ahead of the S^T / dP^T MFMAs, the 16 transposed reads under them
          __builtin_amdgcn_sched_group_barrier(0x100, kDqAhead, 0);
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, (32 - kDqAhead + 15) / 16, 0);
          }
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA'd tile has landed (asm: untracked)
    __syncthreads();
  }
  if (q < S) {
    T* qrow = dQ + ((long)b * S + q) * fs.dq_tok + (long)head * fs.dq_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(dq[db][4 * gg + 0] * scale, dq[db][4 * gg + 1] * scale);
        w[1] = MF<T>::pack(dq[db][4 * gg + 2] * scale, dq[db][4 * gg + 3] * scale);
        *reinterpret_cast<u32x2*>(qrow + d) = w;
      }
  }
}

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(NT2) void fa_bwd_dq_v2(const T* __restrict__ Q, const T* __restrict__ K,
                                                    const T* __restrict__ V, const T* __restrict__ dO,
                                                    const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                    T* __restrict__ dQ, int S, int Sk, int H, int Hk, float scale, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int D = 128, NK = 8, ND = 4;
  constexpr int IMG = BN * 256;
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * 2 * IMG];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  const int nqb = (S + BM2 - 1) / BM2;
  int bh, rank;
  fa_block(gridDim.x * gridDim.y / nqb, nqb, fs.order_g, bh, rank);
  const int qb = CAUSAL ? (nqb - 1 - rank) : rank;
  const int head = bh % H, b = bh / H;
  const int hk = head / (H / Hk);
  const int q0 = qb * BM2;
  const int wq0 = q0 + wid * 32;
  const int q = wq0 + lr;
  const long kstride = fs.kv_tok;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * kstride + (long)hk * fs.kv_head;
  const float scale_log2 = scale * kLog2e;
  const float lse2 = (q < S) ? LSE[((long)b * H + head) * S + q] * kLog2e : 0.f;
  const float dlt = (q < S) ? DELTA[((long)b * H + head) * S + q] : 0.f;

  frag qf[NK], gf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
    if (q < S) {
      a = *reinterpret_cast<const u32x4*>(Qb + (long)q * fs.q_tok + 16 * kk + 8 * h);
      c = *reinterpret_cast<const u32x4*>(dOb + (long)q * fs.o_tok + 16 * kk + 8 * h);
    }
    qf[kk] = as_frag<frag>(a);
    gf[kk] = as_frag<frag>(c);
  }
  f32x16 dq[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) dq[i] = zero16();

  u32x4 kreg[2], vreg[2];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + NT2 * i;
      // keys past Sk read row Sk - 1 (finite; masked to P = 0): no exec branch per load
      const int kk = min(k0 + (c >> 4), Sk - 1), ch = c & 15;
      kreg[i] = *reinterpret_cast<const u32x4*>(Kb + (long)kk * kstride + ch * 8);
      vreg[i] = *reinterpret_cast<const u32x4*>(Vb + (long)kk * kstride + ch * 8);
    }
  };
  auto store_tile = [&](int buf) {
    unsigned char* kl = smem + buf * 2 * IMG;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + NT2 * i;
      *reinterpret_cast<u32x4*>(kl + dual_off(c >> 4, c & 15)) = kreg[i];
      *reinterpret_cast<u32x4*>(kl + IMG + dual_off(c >> 4, c & 15)) = vreg[i];
    }
  };

  int kend = Sk;
  if (CAUSAL) kend = min(Sk, q0 + BM2);
  const int ntile = (kend + BN - 1) / BN;
  if (ntile > 0) {
    load_tile(0);
    store_tile(0);
    __syncthreads();
  }
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * BN;
    const int cur = t & 1;
    if (t + 1 < ntile) load_tile(k0 + BN);
    const unsigned char* k_img = smem + cur * 2 * IMG;
    const unsigned char* v_img = k_img + IMG;
    if (!(CAUSAL && k0 > wq0 + 31)) {
      const bool need_mask = (k0 + BN > Sk) || (CAUSAL && k0 + BN - 1 > wq0);
      // one 32-key block at a time keeps only 32 accumulator registers live for S/dP
#pragma unroll 1
      for (int kb = 0; kb < 2; ++kb) {
        f32x16 st = zero16(), dpt = zero16();
#pragma unroll
        for (int kk = 0; kk < NK; ++kk) {
          const u32x4 ka = *reinterpret_cast<const u32x4*>(k_img + dual_off(kb * 32 + lr, 2 * kk + h));
          const u32x4 va = *reinterpret_cast<const u32x4*>(v_img + dual_off(kb * 32 + lr, 2 * kk + h));
          st = MF<T>::mma(as_frag<frag>(ka), qf[kk], st);
          dpt = MF<T>::mma(as_frag<frag>(va), gf[kk], dpt);
        }
        auto probs = [&](auto masked_c) {   // wave-uniform mask test, as in fa_bwd_dkdv_v2
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            float x = st[r] * scale_log2 - lse2;
            if constexpr (decltype(masked_c)::value) {   // select on the exponent, bitwise test
              const int kk = k0 + kb * 32 + acc_row(r, h);
              x = ((kk >= Sk) | (CAUSAL & (kk > q))) ? -INFINITY : x;
            }
            const float p = kDqBareExp ? fexp2(x) : exp2f(x);
            dpt[r] = p * (dpt[r] - dlt);
          }
        };
        if (!kSplitMaskDq || need_mask) probs(std::true_type{});
        else probs(std::false_type{});
        // dQ^T[d][q] += K^T[d][key] dS^T[key][q] for this block's two 16-key steps
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          const int s8 = s2 * 8;
          u32x4 pw;
          pw[0] = MF<T>::pack(dpt[s8 + 0], dpt[s8 + 1]);
          pw[1] = MF<T>::pack(dpt[s8 + 2], dpt[s8 + 3]);
          pw[2] = MF<T>::pack(dpt[s8 + 4], dpt[s8 + 5]);
          pw[3] = MF<T>::pack(dpt[s8 + 6], dpt[s8 + 7]);
          const frag pf = as_frag<frag>(pw);
          const int r0 = kb * 32 + 16 * s2 + 4 * h;
#pragma unroll
          for (int db = 0; db < ND; ++db) {
            const u32x4 a = tr_frag(k_img, r0, db, g, tq, tp);
            dq[db] = MF<T>::mma(as_frag<frag>(a), pf, dq[db]);
          }
        }
      }
    }
    if (t + 1 < ntile) store_tile(cur ^ 1);
    __syncthreads();
  }
  if (q < S) {
    T* qrow = dQ + ((long)b * S + q) * fs.dq_tok + (long)head * fs.dq_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(dq[db][4 * gg + 0] * scale, dq[db][4 * gg + 1] * scale);
        w[1] = MF<T>::pack(dq[db][4 * gg + 2] * scale, dq[db][4 * gg + 3] * scale);
        *reinterpret_cast<u32x2*>(qrow + d) = w;
      }
  }
}

bool dkdv_ilp2() {  // PHA_FA_DKDV_ILP=0 serialises the two 32-row halves (A/B comparisons)
  const char* e = getenv("PHA_FA_DKDV_ILP");
  return !(e && e[0] == '0');
}

bool dkdv_v3() {  // PHA_FA_DKDV=v2 selects the unpipelined dK/dV kernel (A/B comparisons)
  const char* e = getenv("PHA_FA_DKDV");
  return !(e && e[0] == 'v' && e[1] == '2');
}

bool fwd_v3() {  // PHA_FA_FWD=v2 selects the register-staged forward kernel (A/B comparisons)
  const char* e = getenv("PHA_FA_FWD");
  return !(e && e[0] == 'v' && e[1] == '2');
}

bool fwd_v4() {  // PHA_FA_FWD=v4: the 4-wave software-pipelined forward
  const char* e = getenv("PHA_FA_FWD");
  return e && e[0] == 'v' && e[1] == '4';
}

bool dq_v3() {  // PHA_FA_DQ=v2 selects the register-staged dQ kernel (A/B comparisons)
  const char* e = getenv("PHA_FA_DQ");
  return !(e && e[0] == 'v' && e[1] == '2');
}

bool bwd_v2_enabled() {  // PHA_FA_BWD_V1=1 selects the 4-wave kernels (A/B comparisons)
  const char* e = getenv("PHA_FA_BWD_V1");
  return !(e && e[0] == '1');
}

int fa_prio() {  // PHA_FA_PRIO: 8-wave kernels' wave priorities (FaStrides::prio)
  const char* e = getenv("PHA_FA_PRIO");
  return e ? atoi(e) : 0;
}

int fa_order_g() {  // PHA_FA_ORDER_G: blocks of one (b, h) kept together per XCD (0 = plain order)
  const char* e = getenv("PHA_FA_ORDER_G");
  return e ? atoi(e) : 0;   // measured: G = 0 fastest (0.923 ms bwd; G = 4: 1.036 ms)
}

bool fwd_v2_enabled() {  // PHA_FA_FWD_V1=1 selects the 4-wave kernel (A/B comparisons)
  const char* e = getenv("PHA_FA_FWD_V1");
  return !(e && e[0] == '1');
}


template <typename T>
int launch_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Sk, int H, int Hk,
               int D, float scale, int causal, hipStream_t st, const FaStrides* fsp = nullptr) {
  const float sl = scale * kLog2e;
  FaStrides fs = fsp ? *fsp : dense_strides(H, Hk, D);
  fs.order_g = fa_order_g();
  fs.prio = fa_prio();
  const bool v2 = D == 128 && fwd_v2_enabled() && scale > 0.f;   // v2 folds the scale into max / exp
  if (fsp && !v2) return (int)hipErrorInvalidValue;
  if (v2) {
    const dim3 g2(B * H, (S + BM2 - 1) / BM2), b2(NT2);
    if (fwd_v4()) {
      if (causal)
        hipLaunchKernelGGL((fa_fwd_v4_kernel<T, true>), g2, dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, fs);
      else
        hipLaunchKernelGGL((fa_fwd_v4_kernel<T, false>), g2, dim3(256), 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, fs);
    } else if (fwd_v3() && causal)
      hipLaunchKernelGGL((fa_fwd_v3_kernel<T, true>), g2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, fs);
    else if (fwd_v3())
      hipLaunchKernelGGL((fa_fwd_v3_kernel<T, false>), g2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, fs);
    else if (causal)
      hipLaunchKernelGGL((fa_fwd_v2_kernel<T, true>), g2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, fs);
    else
      hipLaunchKernelGGL((fa_fwd_v2_kernel<T, false>), g2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, fs);
    return (int)hipGetLastError();
  }
  const dim3 grid((S + BM - 1) / BM, H, B), block(256);
#define FA_L(DD, CC) hipLaunchKernelGGL((fa_fwd_kernel<T, DD, CC>), grid, block, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl, FaExt{})
  if (D == 128) { if (causal) FA_L(128, true); else FA_L(128, false); }
  else if (D == 64) { if (causal) FA_L(64, true); else FA_L(64, false); }
  else if (D == 256) { if (causal) FA_L(256, true); else FA_L(256, false); }
  else return (int)hipErrorInvalidValue;
#undef FA_L
  return (int)hipGetLastError();
}

template <typename T>
int launch_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse, const float* delta,
               void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, int D, float scale, int causal,
               hipStream_t st, const FaStrides* fsp = nullptr, const void* o = nullptr) {
  FaStrides fs = fsp ? *fsp : dense_strides(H, Hk, D);
  fs.order_g = fa_order_g();
  fs.prio = fa_prio();
  if (fsp && !(D == 128 && bwd_v2_enabled())) return (int)hipErrorInvalidValue;
  if (D == 128 && bwd_v2_enabled()) {
    const dim3 gk2(B * H, (Sk + NTKV / 2 - 1) / (NTKV / 2)), gq2(B * H, (S + BM2 - 1) / BM2), b2(NT2), bk(NTKV);
#define FB2(CC)                                                                                                    \
    if (dkdv_v3())                                                                                                 \
      hipLaunchKernelGGL((fa_bwd_dkdv_v3<T, CC>), gk2, bk, 0, st, (const T*)q, (const T*)k, (const T*)v,          \
                         (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs);                     \
    else if (dkdv_ilp2())                                                                                          \
      hipLaunchKernelGGL((fa_bwd_dkdv_v2<T, CC, true>), gk2, bk, 0, st, (const T*)q, (const T*)k, (const T*)v,    \
                         (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs);                     \
    else                                                                                                           \
    hipLaunchKernelGGL((fa_bwd_dkdv_v2<T, CC, false>), gk2, bk, 0, st, (const T*)q, (const T*)k, (const T*)v,            \
                       (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs);                       \
    if (dq_v3())                                                                                                   \
      hipLaunchKernelGGL((fa_bwd_dq_v3<T, CC>), gq2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v,            \
                         (const T*)dout, lse, const_cast<float*>(delta), (T*)dq, S, Sk, H, Hk, scale, fs);        \
    else                                                                                                           \
      hipLaunchKernelGGL((fa_bwd_dq_v2<T, CC>), gq2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v,            \
                         (const T*)dout, lse, delta, (T*)dq, S, Sk, H, Hk, scale, fs)
    if (o && dq_v3()) {   // delta formed inside dQ (launched first), then read by dK/dV
#define FB3(CC)                                                                                                    \
      hipLaunchKernelGGL((fa_bwd_dq_v3<T, CC>), gq2, b2, 0, st, (const T*)q, (const T*)k, (const T*)v,            \
                         (const T*)dout, lse, const_cast<float*>(delta), (T*)dq, S, Sk, H, Hk, scale, fs,         \
                         (const T*)o);                                                                             \
      if (dkdv_v3())                                                                                               \
        hipLaunchKernelGGL((fa_bwd_dkdv_v3<T, CC>), gk2, bk, 0, st, (const T*)q, (const T*)k, (const T*)v,        \
                           (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs);                   \
      else                                                                                                         \
        hipLaunchKernelGGL((fa_bwd_dkdv_v2<T, CC, true>), gk2, bk, 0, st, (const T*)q, (const T*)k, (const T*)v,  \
                           (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs)
      if (causal) { FB3(true); } else { FB3(false); }
#undef FB3
      return (int)hipGetLastError();
    }
    if (causal) { FB2(true); } else { FB2(false); }
#undef FB2
    return (int)hipGetLastError();
  }
  const dim3 gkv((Sk + 127) / 128, H, B), gq((S + BM - 1) / BM, H, B), block(256);
#define FB_L(DD, CC)                                                                                               \
  hipLaunchKernelGGL((fa_bwd_dkdv_kernel<T, DD, CC>), gkv, block, 0, st, (const T*)q, (const T*)k, (const T*)v,   \
                     (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, FaExt{});                     \
  hipLaunchKernelGGL((fa_bwd_dq_kernel<T, DD, CC>), gq, block, 0, st, (const T*)q, (const T*)k, (const T*)v,       \
                     (const T*)dout, lse, delta, (T*)dq, S, Sk, H, Hk, scale, FaExt{})
  if (D == 128) { if (causal) { FB_L(128, true); } else { FB_L(128, false); } }
  else if (D == 64) { if (causal) { FB_L(64, true); } else { FB_L(64, false); } }
  else if (D == 256) { if (causal) { FB_L(256, true); } else { FB_L(256, false); } }
  else return (int)hipErrorInvalidValue;
#undef FB_L
  return (int)hipGetLastError();
}

// 4-wave kernels with the bias / dropout extensions; head dims 32, 64, 128
template <typename T, int EXT>
int launch_ext(bool bwd, const void* q, const void* k, const void* v, void* o, float* lse, const void* dout,
               const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, int D,
               float scale, int causal, const FaExt& ex, hipStream_t st) {
  const dim3 grid((S + BM - 1) / BM, H, B), gkv((Sk + 127) / 128, H, B), block(256);
#define FX_F(DD, CC) hipLaunchKernelGGL((fa_fwd_kernel<T, DD, CC, EXT>), grid, block, 0, st, (const T*)q, (const T*)k, \
                                        (const T*)v, (T*)o, lse, S, Sk, H, Hk, scale * kLog2e, ex)
#define FX_B(DD, CC)                                                                                               \
  hipLaunchKernelGGL((fa_bwd_dkdv_kernel<T, DD, CC, EXT>), gkv, block, 0, st, (const T*)q, (const T*)k,            \
                     (const T*)v, (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, ex);             \
  hipLaunchKernelGGL((fa_bwd_dq_kernel<T, DD, CC, EXT>), grid, block, 0, st, (const T*)q, (const T*)k,             \
                     (const T*)v, (const T*)dout, lse, delta, (T*)dq, S, Sk, H, Hk, scale, ex)
#define FX(DD)                                                                                                     \
  if (!bwd) { if (causal) FX_F(DD, true); else FX_F(DD, false); }                                                  \
  else { if (causal) { FX_B(DD, true); } else { FX_B(DD, false); } }
  if (D == 128) { FX(128) }
  else if (D == 64) { FX(64) }
  else if (D == 32) { FX(32) }
  else if (D == 256) { FX(256) }
  else return (int)hipErrorInvalidValue;
#undef FX
#undef FX_B
#undef FX_F
  return (int)hipGetLastError();
}

template <typename T>
int dispatch_ext(bool bwd, const void* q, const void* k, const void* v, void* o, float* lse, const void* dout,
                 const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, int D,
                 float scale, int causal, const FaExt& ex, hipStream_t st) {
  const int ext = (ex.bias ? 1 : 0) | (ex.thresh ? 2 : 0);
  switch (ext) {
    case 1: return launch_ext<T, 1>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, ex, st);
    case 2: return launch_ext<T, 2>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, ex, st);
    case 3: return launch_ext<T, 3>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, ex, st);
    default: return launch_ext<T, 0>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, ex, st);
  }
}

}  // namespace

// Attention with an additive fp32 bias (natural-log units, key stride 1; element strides sb / sh /
// sq of batch / head / query, 0 = broadcast: a key-padding mask [B,1,1,Sk] has sh = sq = 0) and/or
// dropout of the probabilities (rate in [0, 1): 16-bit threshold; seed selects the stream, the
// backward regenerates the same mask from it). Head dims 32 / 64 / 128 / 256.
PHA_API int pha_flash_attn_fwd_ext(int dt, const void* q, const void* k, const void* v, void* o, float* lse, int B,
                                   int S, int Sk, int H, int Hk, int D, float scale, int causal, const float* bias,
                                   long sb, long sh, long sq, float dropout, unsigned seed, hipStream_t stream,
                                   const unsigned* seedp) {
  if (H % Hk || (D != 32 && D != 64 && D != 128 && D != 256) || S <= 0 || Sk <= 0 || dropout < 0.f || dropout >= 1.f)
    return (int)hipErrorInvalidValue;
  FaExt ex{bias, sb, sh, sq, seed, (unsigned)(dropout * 65536.f + 0.5f), dropout > 0.f ? 1.f / (1.f - dropout) : 1.f};
  ex.seedp = seedp;
  if (dropout > 0.f && ex.thresh == 0) ex.thresh = 1;
  if (dt == kBF16) return dispatch_ext<bf16_t>(false, q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, B, S, Sk, H, Hk, D, scale, causal, ex, stream);
  if (dt == kF16) return dispatch_ext<half_t>(false, q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, B, S, Sk, H, Hk, D, scale, causal, ex, stream);
  return (int)hipErrorInvalidValue;
}

// g*_tok / g*_head: element strides of the dQ and dK / dV outputs (0 = dense [B, S, H, D]); with
// Hk == H the three may point into one packed [B, S, H, 3D] gradient
PHA_API int pha_flash_attn_bwd_ext(int dt, const void* q, const void* k, const void* v, const void* dout,
                                   const float* lse, const float* delta, void* dq, void* dk, void* dv, int B, int S,
                                   int Sk, int H, int Hk, int D, float scale, int causal, const float* bias, long sb,
                                   long sh, long sq, float dropout, unsigned seed, hipStream_t stream, long gq_tok,
                                   int gq_head, long gkv_tok, int gkv_head, const unsigned* seedp) {
  if (H % Hk || (D != 32 && D != 64 && D != 128 && D != 256) || S <= 0 || Sk <= 0 || dropout < 0.f || dropout >= 1.f)
    return (int)hipErrorInvalidValue;
  if ((gkv_tok || gkv_head) && Hk != H) return (int)hipErrorInvalidValue;
  FaExt ex{bias, sb, sh, sq, seed, (unsigned)(dropout * 65536.f + 0.5f), dropout > 0.f ? 1.f / (1.f - dropout) : 1.f};
  ex.gq_tok = gq_tok;
  ex.gq_head = gq_head;
  ex.gkv_tok = gkv_tok;
  ex.gkv_head = gkv_head;
  ex.seedp = seedp;
  if (dropout > 0.f && ex.thresh == 0) ex.thresh = 1;
  if (dt == kBF16) return dispatch_ext<bf16_t>(true, q, k, v, nullptr, const_cast<float*>(lse), dout, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, ex, stream);
  if (dt == kF16) return dispatch_ext<half_t>(true, q, k, v, nullptr, const_cast<float*>(lse), dout, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, ex, stream);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_flash_attn_fwd(int dt, const void* q, const void* k, const void* v, void* o, float* lse, int B, int S,
                               int Sk, int H, int Hk, int D, float scale, int causal, hipStream_t stream) {
  if (H % Hk || (D != 64 && D != 128 && D != 256) || S <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  if (dt == kBF16) return launch_fwd<bf16_t>(q, k, v, o, lse, B, S, Sk, H, Hk, D, scale, causal, stream);
  if (dt == kF16) return launch_fwd<half_t>(q, k, v, o, lse, B, S, Sk, H, Hk, D, scale, causal, stream);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_flash_attn_bwd_preprocess(int dt, const void* o, const void* dout, float* delta, int B, int S, int H,
                                          int D, hipStream_t stream) {
  const long rows = (long)B * S * H;
  const int rpb = 4 * (64 / (D / 8));   // rows per 256-thread block
  const dim3 grid((rows + rpb - 1) / rpb), block(256);
  if (dt == kBF16) {
    if (D == 128) hipLaunchKernelGGL((fa_bwd_pre_kernel<bf16_t, 128>), grid, block, 0, stream, (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H);
    else if (D == 32) hipLaunchKernelGGL((fa_bwd_pre_kernel<bf16_t, 32>), grid, block, 0, stream, (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H);
    else if (D == 256) hipLaunchKernelGGL((fa_bwd_pre_kernel<bf16_t, 256>), grid, block, 0, stream, (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H);
    else hipLaunchKernelGGL((fa_bwd_pre_kernel<bf16_t, 64>), grid, block, 0, stream, (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H);
  } else if (dt == kF16) {
    if (D == 128) hipLaunchKernelGGL((fa_bwd_pre_kernel<half_t, 128>), grid, block, 0, stream, (const half_t*)o, (const half_t*)dout, delta, B, S, H);
    else if (D == 32) hipLaunchKernelGGL((fa_bwd_pre_kernel<half_t, 32>), grid, block, 0, stream, (const half_t*)o, (const half_t*)dout, delta, B, S, H);
    else if (D == 256) hipLaunchKernelGGL((fa_bwd_pre_kernel<half_t, 256>), grid, block, 0, stream, (const half_t*)o, (const half_t*)dout, delta, B, S, H);
    else hipLaunchKernelGGL((fa_bwd_pre_kernel<half_t, 64>), grid, block, 0, stream, (const half_t*)o, (const half_t*)dout, delta, B, S, H);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// dq: [B, S, H, D] (same dtype as q); dk/dv: [B, Sk, H, D] (per query head; the caller sums
// head groups for GQA).
PHA_API int pha_flash_attn_bwd(int dt, const void* q, const void* k, const void* v, const void* dout, const float* lse,
                               const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk,
                               int D, float scale, int causal, hipStream_t stream) {
  // S, Sk >= 1: the kernels clamp out-of-range rows to S - 1 / Sk - 1
  if (H % Hk || (D != 64 && D != 128 && D != 256) || B <= 0 || S <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  if (dt == kBF16) return launch_bwd<bf16_t>(q, k, v, dout, lse, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, stream);
  if (dt == kF16) return launch_bwd<half_t>(q, k, v, dout, lse, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, stream);
  return (int)hipErrorInvalidValue;
}

// pha_flash_attn_bwd_packed with o: the row constants delta = rowsum(dO * O) are formed inside the
// dQ kernel (launched before dK/dV) into `delta` (scratch [B, H, S] fp32) instead of by the
// separate preprocess pass; falls back to preprocess + the two kernels when the v3 kernels are off
PHA_API int pha_flash_attn_bwd_packed_od(int dt, const void* qkv, const void* o, const void* dout, const float* lse,
                                         float* delta, void* dqkv, int B, int S, int H, int D, float scale, int causal,
                                         hipStream_t stream) {
  if (D != 128 || S <= 0) return (int)hipErrorInvalidValue;
  FaStrides f;
  f.order_g = 0;
  f.q_tok = f.kv_tok = f.dq_tok = f.dkv_tok = 3L * H * D;
  f.q_head = f.kv_head = f.dq_head = f.dkv_head = 3 * D;
  f.o_tok = (long)H * D;
  f.o_head = D;
  const bool inq = bwd_v2_enabled() && dq_v3() && !getenv("PHA_FA_DELTA_PASS");
  if (!inq) {
    const int rc = pha_flash_attn_bwd_preprocess(dt, o, dout, delta, B, S, H, D, stream);
    if (rc) return rc;
  }
  const size_t es = 2;
  const char* in = static_cast<const char*>(qkv);
  char* out = static_cast<char*>(dqkv);
  if (dt == kBF16)
    return launch_bwd<bf16_t>(in, in + D * es, in + 2 * D * es, dout, lse, delta, out, out + D * es, out + 2 * D * es, B,
                              S, S, H, H, D, scale, causal, stream, &f, inq ? o : nullptr);
  if (dt == kF16)
    return launch_bwd<half_t>(in, in + D * es, in + 2 * D * es, dout, lse, delta, out, out + D * es, out + 2 * D * es, B,
                              S, S, H, H, D, scale, causal, stream, &f, inq ? o : nullptr);
  return (int)hipErrorInvalidValue;
}

// Packed-QKV variants: q/k/v (and dq/dk/dv) are views into one [B, S, H, 3D] buffer with
// token stride tok = 3*H*D and head stride 3*D; o / dO are dense [B, S, H, D]. D must be 128.
PHA_API int pha_flash_attn_fwd_packed(int dt, const void* qkv, void* o, float* lse, int B, int S, int H, int D,
                                      float scale, int causal, hipStream_t stream) {
  if (D != 128 || S <= 0) return (int)hipErrorInvalidValue;
  FaStrides f;
  f.order_g = 0;
  f.q_tok = f.kv_tok = f.dq_tok = f.dkv_tok = 3L * H * D;
  f.q_head = f.kv_head = f.dq_head = f.dkv_head = 3 * D;
  f.o_tok = (long)H * D;
  f.o_head = D;
  const size_t es = 2;
  const char* base = static_cast<const char*>(qkv);
  if (dt == kBF16)
    return launch_fwd<bf16_t>(base, base + D * es, base + 2 * D * es, o, lse, B, S, S, H, H, D, scale, causal, stream, &f);
  if (dt == kF16)
    return launch_fwd<half_t>(base, base + D * es, base + 2 * D * es, o, lse, B, S, S, H, H, D, scale, causal, stream, &f);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_flash_attn_bwd_packed(int dt, const void* qkv, const void* dout, const float* lse, const float* delta,
                                      void* dqkv, int B, int S, int H, int D, float scale, int causal,
                                      hipStream_t stream) {
  if (D != 128 || S <= 0) return (int)hipErrorInvalidValue;
  FaStrides f;
  f.order_g = 0;
  f.q_tok = f.kv_tok = f.dq_tok = f.dkv_tok = 3L * H * D;
  f.q_head = f.kv_head = f.dq_head = f.dkv_head = 3 * D;
  f.o_tok = (long)H * D;
  f.o_head = D;
  const size_t es = 2;
  const char* in = static_cast<const char*>(qkv);
  char* out = static_cast<char*>(dqkv);
  if (dt == kBF16)
    return launch_bwd<bf16_t>(in, in + D * es, in + 2 * D * es, dout, lse, delta, out, out + D * es, out + 2 * D * es, B,
                              S, S, H, H, D, scale, causal, stream, &f);
  if (dt == kF16)
    return launch_bwd<half_t>(in, in + D * es, in + 2 * D * es, dout, lse, delta, out, out + D * es, out + 2 * D * es, B,
                              S, S, H, H, D, scale, causal, stream, &f);
  return (int)hipErrorInvalidValue;
}
