// Flash attention for head dim 64 (BERT-base / -large, ViT, GPT-2-sized models) on gfx950, with the
// in-kernel dropout of the probabilities and packed-QKV strides. Reference behaviour:
// paddle/fluid/operators/fused/fmha_ref.h:87-172 (softmax(Q K^T / sqrt(d)) with dropout, then P V)
// and its backward in fused_attention_op.cu; the dropout mask is the counter hash of fa_common.h
// (seed, b*H + h, query, key) with a cheaper per-key draw (fa64_draw); the forward stores the keep bits
// for the backward.
//
// Why separate kernels. The generic 4-wave kernels (flash_attn.hip fa_*_kernel<T, 64, ..>) stage
// K / V through registers with a software transpose of V (u16 shuffles per element), take two
// barriers per tile and work on 32-query tiles in the dK/dV kernel: 262 TF/s forward, ~200 TF/s
// backward at the BERT shape (profiles/fa_bert_time.log). Here, as in the D = 128 v3 kernels:
//  * 8 waves x 32 rows per workgroup, tiles by LDS-DMA (global_load_lds_dwordx4, 1-KiB pieces of 8
//    rows), one barrier per tile, the next tile in flight during the current one;
//  * ONE 128-B-row image layout for every operand, read both by rows (ds_read_b128, the MFMA A
//    operand of Q K^T / K Q^T / dO V^T) and transposed (ds_read_b64_tr_b16: V^T for P V, dO^T / Q^T
//    for dV / dK, K^T for dQ). 16-B chunk c of row r sits at chunk c ^ f(r),
//    f(r) = ((r >> 1) & 1) << 2 | ((r >> 2) & 3): the 32 rows of a b128 fragment read (lane groups
//    {0-3,12-15,20-27} / {4-11,16-19,28-31}) land on 16 distinct 16-B slots per bank row, and the
//    4 rows x 64 B of a transposed read fill all 64 banks;
//  * swapped products with the accumulators as the next MFMA's B operand (P^T / dS^T / P / dS never
//    touch LDS); masks as -inf initial accumulators; row constants (-lse / scale, -delta) as the
//    initial accumulators of the dK/dV kernel's S / dP chains (CDNA guide App. B).
#include "fa_common.h"
#include <cstdlib>

namespace {

constexpr int IMG64 = 64 * 128;   // one 64-row x 64-element operand image (8 KiB)

__device__ __forceinline__ int f64(int row) { return (((row >> 1) & 1) << 2) | ((row >> 2) & 3); }

__device__ __forceinline__ void glds64(unsigned voff, const void* sbase, unsigned m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}

// 1-KiB piece p (rows 8p .. 8p+7) of the 64-row tile starting at row r0 of an operand with row
// stride rs (elements): lane L writes physical chunk L & 7 of row 8p + (L >> 3), so it fetches the
// logical chunk (L & 7) ^ f(row). Rows past rmax read row rmax (finite; masked by the caller).
template <typename T>
__device__ __forceinline__ void dma64(const T* base, long rs, int r0, int rmax, int p, int lane, unsigned lds) {
  const int row = 8 * p + (lane >> 3);
  const int lch = (lane & 7) ^ f64(row);
  const unsigned voff = (unsigned)(((long)(min(r0 + row, rmax) - r0) * rs + lch * 8) * 2);
  glds64(voff, base + (long)r0 * rs, __builtin_amdgcn_readfirstlane(lds + p * 1024));
}

// the keep draw of these kernels: one 32-bit hash per key pair (16 bits per key against the
// threshold) of (row seed + key / 2 * odd 24-bit constant) — one full-rate 24-bit and one 32-bit
// multiply per draw instead of fa_keep's two 32-bit ones (the forward is the only place it runs when
// the backward reads the stored keep bits; the re-hashing backward uses the same function)
__device__ __forceinline__ unsigned fa64_draw(unsigned row, int key) {
  unsigned x = row + __umul24((unsigned)(key >> 1), 0x9e3779u);
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  return x;
}
__device__ __forceinline__ bool fa64_keep(unsigned row, int key, unsigned thresh) {
  const unsigned r = fa64_draw(row, key);
  return ((key & 1) ? (r >> 16) : (r & 0xffffu)) >= thresh;
}

// additive score bias (natural-log units, key stride 1) of the lane's 16 keys of a 32-key block
// (query on the lane: keys base + 8m + 4h + {0..3} are one float4), divided by the softmax scale so it
// can start the unscaled S^T accumulator; keys past Sk read the last aligned quad (masked anyway)
__device__ __forceinline__ void bias16(const float* brow, int base, int Sk, float inv_scale, f32x16& acc) {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int k = min(base + 8 * m, Sk - 4);
    const float4 v = *reinterpret_cast<const float4*>(brow + k);
    acc[4 * m + 0] = v.x * inv_scale;
    acc[4 * m + 1] = v.y * inv_scale;
    acc[4 * m + 2] = v.z * inv_scale;
    acc[4 * m + 3] = v.w * inv_scale;
  }
}

__device__ __forceinline__ unsigned lds_addr(const unsigned char* p) {
  return (unsigned)(size_t)(__attribute__((address_space(3))) const unsigned char*)p;
}

// per-lane offsets of the transposed reads (rows 16 ks + 4h + tq (+8), 32-column block db): the
// A operand of an O^T / dV^T / dK^T / dQ^T product; + ks * 2048 (+ 4096 per 32-row half)
__device__ __forceinline__ void tr_offsets(int lane, int (&troff)[2][2]) {
  const int h = lane >> 5, g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
#pragma unroll
  for (int db = 0; db < 2; ++db)
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int f = (((tq >> 1) & 1) << 2) | ((h + 2 * hi) & 3);
      troff[db][hi] = (4 * h + tq + 8 * hi) * 128 + 16 * ((4 * db + 2 * (g & 1) + (tp >> 1)) ^ f) + 8 * (tp & 1);
    }
}

__device__ __forceinline__ u32x4 trA(const unsigned char* img, const int (&troff)[2][2], int db) {
  const u32x2 lo = ds_read_tr16(img + troff[db][0]);
  const u32x2 hi = ds_read_tr16(img + troff[db][1]);
  return u32x4{lo[0], lo[1], hi[0], hi[1]};
}

// ============================================================================================
// forward: workgroup = 8 waves = 256 queries of one (batch, head), query on the MFMA lane;
// per 64-key tile S^T = K Q^T (2 x 4 MFMAs), online softmax (deferred rescale), dropout on P for
// the P V product only (the row sum is undropped), O^T += V^T P^T (4 x 2 MFMAs)
// ============================================================================================
template <typename T, bool CAUSAL, bool DROP, bool BIAS = false>
__global__ __launch_bounds__(512) void fa64_fwd(const T* __restrict__ Q, const T* __restrict__ K,
                                                const T* __restrict__ V, T* __restrict__ O, float* __restrict__ LSE,
                                                int S, int Sk, int H, int Hk, float scale_log2, FaStrides fs, FaExt ex) {
  typedef typename MF<T>::frag frag;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * 2 * IMG64];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, lr = lane & 31;
  const int nqb = (S + 255) >> 8;
  const int bh = blockIdx.y, rank = blockIdx.x;
  const int qb = CAUSAL ? nqb - 1 - rank : rank;
  const int head = bh % H, b = bh / H, hk = head / (H / Hk);
  const int q0 = qb * 256, wq0 = q0 + wid * 32, q = wq0 + lr;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* Kb = K + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;

  frag qf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    u32x4 v = {0, 0, 0, 0};
    if (q < S) v = *reinterpret_cast<const u32x4*>(Qb + (long)q * fs.q_tok + 16 * kk + 8 * h);
    qf[kk] = as_frag<frag>(v);
  }
  unsigned drow = 0;
  if constexpr (DROP) drow = fa_row(fa_stream(fa_seed(ex), b * H + head), q);
  const float inv_scale = kLog2e / scale_log2;
  const float* brow = BIAS ? ex.bias + (long)b * ex.sb + (long)head * ex.sh + (long)min(q, S - 1) * ex.sq : nullptr;
  f32x16 o[2];
  o[0] = zero16();
  o[1] = zero16();
  float m_run = -INFINITY, l_run = 0.f;
  const int kend = CAUSAL ? min(Sk, q0 + 256) : Sk;
  const int ntile = (kend + 63) >> 6;

  const unsigned lds0 = lds_addr(smem);
  auto load_tile = [&](int k0, int buf) {   // 16 pieces (K 0-7, V 8-15), two per wave
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int gidx = wid * 2 + u, which = gidx >> 3;
      dma64(which ? Vb : Kb, fs.kv_tok, k0, Sk - 1, gidx & 7, lane, lds0 + buf * 2 * IMG64 + which * IMG64);
    }
  };
  int koff[4], troff[2][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) koff[kk] = lr * 128 + 16 * ((2 * kk + h) ^ f64(lr));
  tr_offsets(lane, troff);

  if (ntile > 0) {
    load_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * 64, cur = t & 1;
    if (t + 1 < ntile) load_tile(k0 + 64, cur ^ 1);
    const unsigned char* kl = smem + cur * 2 * IMG64;
    const unsigned char* vl = kl + IMG64;
    if (!(CAUSAL && k0 > wq0 + 31)) {
      f32x16 s[2];
      if constexpr (BIAS) {   // the bias / scale as the S^T chain's initial value
        bias16(brow, k0 + 4 * h, Sk, inv_scale, s[0]);
        bias16(brow, k0 + 32 + 4 * h, Sk, inv_scale, s[1]);
      } else {
        s[0] = zero16();
        s[1] = zero16();
      }
      if ((k0 + 64 > Sk) || (CAUSAL && k0 + 63 > wq0)) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int base = k0 + kb * 32 + 4 * h;
          const int lim1 = CAUSAL ? q - base : 1 << 20, lim2 = Sk - base;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rb = (r & 3) + 8 * (r >> 2);
            s[kb][r] = ((rb > lim1) | (rb >= lim2)) ? -INFINITY : s[kb][r];
          }
        }
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const u32x4 a = *reinterpret_cast<const u32x4*>(kl + kb * 4096 + koff[kk]);
          s[kb] = MF<T>::mma(as_frag<frag>(a), qf[kk], s[kb]);
        }
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
        for (int i = 0; i < 2; ++i)
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
      if constexpr (DROP) {
        // fa64_keep of the lane's 32 keys, one hash per (even, odd) key pair: registers r, r + 1 hold
        // keys 2m, 2m + 1, whose draws are the low / high halves of fa64_draw(row, 2m); the odd key's
        // test x >> 16 >= thresh is the full-word x >= thresh << 16. The keep scale 1 / (1 - rate) is
        // applied once to the output instead of per element. Keep bits are shifted in (bit r: register
        // r), then spread to key positions acc_row(r, h) = (r & 3) + 8 (r >> 2) + 4 h.
        unsigned wb[2];
        const unsigned t16 = ex.thresh << 16;
        const unsigned rk = drow + (unsigned)((k0 + 4 * h) >> 1) * 0x9e3779u;
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          unsigned bits = 0;
#pragma unroll
          for (int pr = 7; pr >= 0; --pr) {
            const int r = 2 * pr;
            unsigned x = rk + (unsigned)(kb * 16 + (pr & 1) + 4 * (pr >> 1)) * 0x9e3779u;
            x ^= x >> 16;
            x *= 0x7feb352du;
            x ^= x >> 15;
            const bool klo = (x & 0xffffu) >= ex.thresh, khi = x >= t16;
            bits = 4 * bits + 2 * (unsigned)khi + (unsigned)klo;
            s[kb][r] = klo ? s[kb][r] : 0.f;
            s[kb][r + 1] = khi ? s[kb][r + 1] : 0.f;
          }
          wb[kb] = ((bits & 0xfu) | (bits & 0xf0u) << 4 | (bits & 0xf00u) << 8 | (bits & 0xf000u) << 12) << (4 * h);
        }
        if (ex.dmask) {   // the two 32-key words of this tile: lane half h stores word h of its 32
          // queries — [word][query] layout, so each half-wave writes 128 contiguous bytes
          const unsigned w0 = wb[0] | (unsigned)__shfl_xor((int)wb[0], 32, 64);
          const unsigned w1 = wb[1] | (unsigned)__shfl_xor((int)wb[1], 32, 64);
          if (q < S) ex.dmask[((long)bh * ex.dmask_w + 2 * t + h) * ((S + 63) & ~63) + q] = h ? w1 : w0;
        }
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
#pragma unroll
        for (int db = 0; db < 2; ++db)
          o[db] = MF<T>::mma(as_frag<frag>(trA(vl + ks * 2048, troff, db)), as_frag<frag>(pw), o[db]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA'd tile has landed (asm: untracked)
    __syncthreads();
  }
  if (q < S) {
    const float inv = l_run > 0.f ? (DROP ? ex.keep_scale : 1.f) / l_run : 0.f;
    T* orow = O + ((long)b * S + q) * fs.o_tok + (long)head * fs.o_head;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(o[db][4 * gg + 0] * inv, o[db][4 * gg + 1] * inv);
        w[1] = MF<T>::pack(o[db][4 * gg + 2] * inv, o[db][4 * gg + 3] * inv);
        *reinterpret_cast<u32x2*>(orow + d) = w;
      }
    if (h == 0) LSE[(long)bh * S + q] = (l_run > 0.f) ? (m_run + log2f(l_run)) * kLn2 : INFINITY;
  }
}

// ============================================================================================
// dQ: the forward's geometry (query on the lane, 256 queries per workgroup); per 64-key tile
//   S^T = K Q^T, dP^T = V dO^T (row reads of the K / V images; Q / dO fragments in registers),
//   P^T = exp2(c S^T - lse), dS^T = P^T (Z dP^T / (1 - rate) - delta), dQ^T += K^T dS^T (transposed
//   reads of the K image, dS^T packed as the B operand)
// ============================================================================================
template <typename T, bool CAUSAL, int DR, bool BIAS = false>
__global__ __launch_bounds__(512) void fa64_dq(const T* __restrict__ Q, const T* __restrict__ K,
                                               const T* __restrict__ V, const T* __restrict__ dO,
                                               const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                               T* __restrict__ dQ, int S, int Sk, int H, int Hk, float scale,
                                               FaStrides fs, FaExt ex) {
  typedef typename MF<T>::frag frag;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * 2 * IMG64];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, lr = lane & 31;
  const int nqb = (S + 255) >> 8;
  const int bh = blockIdx.y, rank = blockIdx.x;
  const int qb = CAUSAL ? nqb - 1 - rank : rank;
  const int head = bh % H, b = bh / H, hk = head / (H / Hk);
  const int q0 = qb * 256, wq0 = q0 + wid * 32, q = wq0 + lr;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const int qc = min(q, S - 1);
  frag qf[4], gf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    qf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Qb + (long)qc * fs.q_tok + 16 * kk + 8 * h));
    gf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(dOb + (long)qc * fs.o_tok + 16 * kk + 8 * h));
  }
  const float c2 = scale * kLog2e;
  const float nl = -LSE[(long)bh * S + qc] * kLog2e, del = DELTA[(long)bh * S + qc];
  const unsigned ksb = __float_as_uint(ex.keep_scale);
  unsigned drow = 0;
  if constexpr (DR == 1) drow = fa_row(fa_stream(fa_seed(ex), b * H + head), q);
  const long msp = (S + 63) & ~63;   // the keep words' row pitch ([B * H][words][msp])
  const unsigned* mrow = DR == 2 ? ex.dmask + (long)bh * ex.dmask_w * msp + qc : nullptr;
  const float* brow = BIAS ? ex.bias + (long)b * ex.sb + (long)head * ex.sh + (long)qc * ex.sq : nullptr;
  f32x16 dqt[2];
  dqt[0] = zero16();
  dqt[1] = zero16();
  const int kend = CAUSAL ? min(Sk, q0 + 256) : Sk;
  const int ntile = (kend + 63) >> 6;
  const unsigned lds0 = lds_addr(smem);
  auto load_tile = [&](int k0, int buf) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int gidx = wid * 2 + u, which = gidx >> 3;
      dma64(which ? Vb : Kb, fs.kv_tok, k0, Sk - 1, gidx & 7, lane, lds0 + buf * 2 * IMG64 + which * IMG64);
    }
  };
  int koff[4], troff[2][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) koff[kk] = lr * 128 + 16 * ((2 * kk + h) ^ f64(lr));
  tr_offsets(lane, troff);

  if (ntile > 0) {
    load_tile(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int t = 0; t < ntile; ++t) {
    const int k0 = t * 64, cur = t & 1;
    if (t + 1 < ntile) load_tile(k0 + 64, cur ^ 1);
    const unsigned char* kl = smem + cur * 2 * IMG64;
    const unsigned char* vl = kl + IMG64;
    if (!(CAUSAL && k0 > wq0 + 31)) {
      u32x2 mw = {0u, 0u};
      if constexpr (DR == 2) {
        mw[0] = mrow[(2 * t) * msp];
        mw[1] = mrow[(2 * t + 1) * msp];
      }
      f32x16 s[2], dp[2];
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        dp[kb] = zero16();
        if constexpr (BIAS) {
          bias16(brow, k0 + kb * 32 + 4 * h, Sk, 1.f / scale, s[kb]);
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) s[kb][r] = 0.f;
        }
      }
      if ((k0 + 64 > Sk) || (CAUSAL && k0 + 63 > wq0)) {
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
          const int base = k0 + kb * 32 + 4 * h;
          const int lim1 = CAUSAL ? q - base : 1 << 20, lim2 = Sk - base;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int rb = (r & 3) + 8 * (r >> 2);
            s[kb][r] = ((rb > lim1) | (rb >= lim2)) ? -INFINITY : s[kb][r];
          }
        }
      }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          const u32x4 ka = *reinterpret_cast<const u32x4*>(kl + kb * 4096 + koff[kk]);
          const u32x4 va = *reinterpret_cast<const u32x4*>(vl + kb * 4096 + koff[kk]);
          s[kb] = MF<T>::mma(as_frag<frag>(ka), qf[kk], s[kb]);
          dp[kb] = MF<T>::mma(as_frag<frag>(va), gf[kk], dp[kb]);
        }
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fexp2(fmaf(s[kb][r], c2, nl));
          const float g = dp[kb][r];
          if constexpr (DR != 0) {   // keep multiplier as in the dK/dV kernel
            unsigned msk;   // all ones = keep (DR 2: one signed bitfield extract)
            if constexpr (DR == 2) msk = (unsigned)__builtin_amdgcn_sbfe((int)mw[kb], (unsigned)acc_row(r, h), 1u);
            else msk = fa64_keep(drow, k0 + kb * 32 + acc_row(r, h), ex.thresh) ? ~0u : 0u;
            s[kb][r] = p * fmaf(g, __uint_as_float(msk & ksb), -del);
          } else {
            s[kb][r] = p * (g - del);
          }
        }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const f32x16& sv = s[ks >> 1];
        const int s8 = (ks & 1) * 8;
        u32x4 w;
        w[0] = MF<T>::pack(sv[s8 + 0], sv[s8 + 1]);
        w[1] = MF<T>::pack(sv[s8 + 2], sv[s8 + 3]);
        w[2] = MF<T>::pack(sv[s8 + 4], sv[s8 + 5]);
        w[3] = MF<T>::pack(sv[s8 + 6], sv[s8 + 7]);
#pragma unroll
        for (int db = 0; db < 2; ++db)
          dqt[db] = MF<T>::mma(as_frag<frag>(trA(kl + ks * 2048, troff, db)), as_frag<frag>(w), dqt[db]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (q < S) {
    const long gt = ex.gq_tok ? ex.gq_tok : (long)H * 64;
    const long gh = ex.gq_head ? ex.gq_head : 64;
    T* row = dQ + ((long)b * S + q) * gt + (long)head * gh;
#pragma unroll
    for (int db = 0; db < 2; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 w;
        w[0] = MF<T>::pack(dqt[db][4 * gg + 0] * scale, dqt[db][4 * gg + 1] * scale);
        w[1] = MF<T>::pack(dqt[db][4 * gg + 2] * scale, dqt[db][4 * gg + 3] * scale);
        *reinterpret_cast<u32x2*>(row + d) = w;
      }
  }
}

// ============================================================================================
// dK / dV: workgroup = 8 waves = 256 keys, key on the MFMA lane, K / V fragments and dK^T / dV^T
// in registers; per 64-query tile (Q, dO images by LDS-DMA; -lse/scale, -delta and the dropout
// row seeds staged in LDS with it), two 32-query halves:
//   S = Q K^T (from -lse/scale), dP = dO V^T (from -delta, or 0 with dropout), p = exp2(c S),
//   dV^T += dO^T (Z p / (1 - rate)), dK^T += Q^T (p (Z dP / (1 - rate) - delta))
// ============================================================================================
constexpr int RC64 = 3 * 64 * 4 + 8 * 64 * 4;   // -lse/scale, -delta, row seeds, keep bits [8 words][64 rows]

template <typename T, bool CAUSAL, int DR, bool BIAS = false, int NW = 8>
__global__ __launch_bounds__(NW * 64) void fa64_dkdv(const T* __restrict__ Q, const T* __restrict__ K,
                                                 const T* __restrict__ V, const T* __restrict__ dO,
                                                 const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                 T* __restrict__ dK, T* __restrict__ dV, int S, int Sk, int H, int Hk,
                                                 float scale, FaStrides fs, FaExt ex) {
  typedef typename MF<T>::frag frag;
  constexpr int BUF = 2 * IMG64 + RC64;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * BUF];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, lr = lane & 31;
  const int bh = blockIdx.y;
  const int head = bh % H, b = bh / H, hk = head / (H / Hk);
  const int k0 = blockIdx.x * (NW * 32), wk0 = k0 + wid * 32, key = wk0 + lr;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const float* lse_b = LSE + (long)bh * S;
  const float* del_b = DELTA + (long)bh * S;
  const float c2 = scale * kLog2e, nis = -1.f / scale;
  constexpr bool DROP = DR != 0;
  const unsigned ksb = __float_as_uint(ex.keep_scale);
  unsigned dstream = 0;
  if constexpr (DR == 1) dstream = fa_stream(fa_seed(ex), b * H + head);

  const int keyc = min(key, Sk - 1);
  // additive bias column of this lane's key (key-padding masks: one value for every query)
  const float inv_sc = 1.f / scale;
  const float* bcol = BIAS ? ex.bias + (long)b * ex.sb + (long)head * ex.sh + keyc : nullptr;
  const float bkey = (BIAS && ex.sq == 0) ? bcol[0] * inv_sc : 0.f;
  frag kf[4], vf[4];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    kf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Kb + (long)keyc * fs.kv_tok + 16 * kk + 8 * h));
    vf[kk] = as_frag<frag>(*reinterpret_cast<const u32x4*>(Vb + (long)keyc * fs.kv_tok + 16 * kk + 8 * h));
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0) through the builtin (see flash_attn.hip dK/dV v2)
  f32x16 dvt[2], dkt[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) { dvt[i] = zero16(); dkt[i] = zero16(); }

  const unsigned lds0 = lds_addr(smem);
  float rcv = 0.f;
  unsigned rseed = 0;
  uint4 mreg = {0u, 0u, 0u, 0u};
  // keep words: NW words x 64 rows per tile, one b128 (4 consecutive rows of one word) per thread
  constexpr int MT0 = NW == 8 ? 256 : 128;
  const long msp = (S + 63) & ~63;
  const unsigned* mbase = DR == 2 ? ex.dmask + ((long)bh * ex.dmask_w + (k0 >> 5)) * msp : nullptr;
  auto load_tile = [&](int qt, int buf) {   // 16 pieces (Q 0-7, dO 8-15) + the row constants
#pragma unroll
    for (int u = 0; u < 16 / NW; ++u) {
      const int gidx = wid * (16 / NW) + u, which = gidx >> 3;
      if (which) dma64(dOb, fs.o_tok, qt, S - 1, gidx & 7, lane, lds0 + buf * BUF + IMG64);
      else dma64(Qb, fs.q_tok, qt, S - 1, gidx & 7, lane, lds0 + buf * BUF);
    }
    if (tid < 128) rcv = (tid < 64 ? lse_b : del_b)[min(qt + (tid & 63), S - 1)];
    if constexpr (DR == 1) {
      if (tid >= 128 && tid < 192) rseed = fa_row(dstream, qt + (tid & 63));
    } else if constexpr (DR == 2) {   // rows past S (pitch padding) are masked out by the -inf row limit
      if (tid >= MT0 && tid < MT0 + 16 * NW) {
        const int i = tid - MT0;
        mreg = *reinterpret_cast<const uint4*>(mbase + (i >> 4) * msp + qt + 4 * (i & 15));
      }
    }
  };
  auto store_rc = [&](int buf) {
    float* rc = reinterpret_cast<float*>(smem + buf * BUF + 2 * IMG64);
    if (tid < 128) rc[tid] = tid < 64 ? rcv * nis : -rcv;
    if constexpr (DR == 1) {
      if (tid >= 128 && tid < 192) reinterpret_cast<unsigned*>(rc)[tid] = rseed;
    } else if constexpr (DR == 2) {   // [word][row] in LDS, as in global memory: a lane's 4 rows are one b128
      if (tid >= MT0 && tid < MT0 + 16 * NW) {
        const int i = tid - MT0;
        *reinterpret_cast<uint4*>(reinterpret_cast<unsigned*>(rc) + 192 + 64 * (i >> 4) + 4 * (i & 15)) = mreg;
      }
    }
  };
  int aoff[4], troff[2][2];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) aoff[kk] = lr * 128 + 16 * ((2 * kk + h) ^ f64(lr));
  tr_offsets(lane, troff);

  const int qstart = CAUSAL ? (k0 / 64) * 64 : 0;
  const int ntile = qstart < S ? (S - qstart + 63) / 64 : 0;
  if (ntile > 0) {
    load_tile(qstart, 0);
    store_rc(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  int buf = 0;
  for (int t = 0; t < ntile; ++t) {
    const int qt = qstart + t * 64;
    if (t + 1 < ntile) load_tile(qt + 64, buf ^ 1);
    const unsigned char* img = smem + buf * BUF;
    const unsigned char* doimg = img + IMG64;
    const float* rc = reinterpret_cast<const float*>(img + 2 * IMG64);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int qh = qt + 32 * j;
      if (CAUSAL && wk0 > qh + 31) continue;   // every key of the wave after every query of the half
      f32x16 sa, da;
      float dl[16];
      unsigned sd[16];
#pragma unroll
      for (int m = 0; m < 4; ++m) {   // rows 32j + 8m + 4h + {0..3}: registers 4m .. 4m+3
        const float4 l4 = *reinterpret_cast<const float4*>(rc + 32 * j + 8 * m + 4 * h);
        const float4 d4 = *reinterpret_cast<const float4*>(rc + 64 + 32 * j + 8 * m + 4 * h);
        sa[4 * m + 0] = l4.x; sa[4 * m + 1] = l4.y; sa[4 * m + 2] = l4.z; sa[4 * m + 3] = l4.w;
        if constexpr (DROP) {
          dl[4 * m + 0] = d4.x; dl[4 * m + 1] = d4.y; dl[4 * m + 2] = d4.z; dl[4 * m + 3] = d4.w;   // -delta
          // DR 1: the rows' hash seeds; DR 2: the rows' keep words of this wave's 32 keys
          const uint4 s4 = *reinterpret_cast<const uint4*>(rc + (DR == 1 ? 128 : 192 + wid * 64) + 32 * j + 8 * m + 4 * h);
          sd[4 * m + 0] = s4.x; sd[4 * m + 1] = s4.y; sd[4 * m + 2] = s4.z; sd[4 * m + 3] = s4.w;
          da[4 * m + 0] = da[4 * m + 1] = da[4 * m + 2] = da[4 * m + 3] = 0.f;
        } else {
          da[4 * m + 0] = d4.x; da[4 * m + 1] = d4.y; da[4 * m + 2] = d4.z; da[4 * m + 3] = d4.w;
        }
      }
      if constexpr (BIAS) {   // + bias / scale of (query row, this lane's key)
        if (ex.sq == 0) {
#pragma unroll
          for (int r = 0; r < 16; ++r) sa[r] += bkey;
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) sa[r] += bcol[(long)min(qh + acc_row(r, h), S - 1) * ex.sq] * inv_sc;
        }
      }
      if ((qh + 32 > S) || (wk0 + 32 > Sk) || (CAUSAL && wk0 + 31 > qh)) {
        const int lim = key >= Sk ? 32 : (CAUSAL ? key - qh - 4 * h : -1);
        const int lim2 = S - qh - 4 * h;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int rb = (r & 3) + 8 * (r >> 2);
          sa[r] = ((rb < lim) | (rb >= lim2)) ? -INFINITY : sa[r];
        }
      }
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        const u32x4 qa = *reinterpret_cast<const u32x4*>(img + j * 4096 + aoff[kk]);
        const u32x4 ga = *reinterpret_cast<const u32x4*>(doimg + j * 4096 + aoff[kk]);
        sa = MF<T>::mma(as_frag<frag>(qa), kf[kk], sa);
        da = MF<T>::mma(as_frag<frag>(ga), vf[kk], da);
      }
      // dropout draws: lanes 2i, 2i+1 hold keys 2m, 2m+1, and fa64_keep takes both keys' 16-bit
      // halves from ONE 32-bit hash of (row seed ^ key / 2): each lane of the pair hashes 8 of the
      // 16 rows and the pair swaps results (DPP quad_perm 1,0,3,2) — half the multiply-heavy hashes
      unsigned rnd[16];
      if constexpr (DR == 1) {
        const bool odd = lane & 1;
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const unsigned mine = fa64_draw(odd ? sd[i + 8] : sd[i], key);
          const unsigned other = (unsigned)__builtin_amdgcn_mov_dpp((int)mine, 0xB1, 0xF, 0xF, false);
          rnd[i] = odd ? other : mine;
          rnd[i + 8] = odd ? mine : other;
        }
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = fexp2(sa[r] * c2);
        if constexpr (DROP) {
          // the keep decision as a multiplier m = keep ? 1 / (1 - rate) : 0, built from the bit with an
          // AND on the scale's bits (no compare / select per element; both DR paths identical arithmetic)
          unsigned msk;   // all ones = keep (DR 2: one signed bitfield extract of the stored bit)
          if constexpr (DR == 2) msk = (unsigned)__builtin_amdgcn_sbfe((int)sd[r], (unsigned)lr, 1u);
          else msk = ((lane & 1) ? (rnd[r] >> 16) : (rnd[r] & 0xffffu)) >= ex.thresh ? ~0u : 0u;   // = fa64_keep
          const float m = __uint_as_float(msk & ksb);
          sa[r] = p * m;
          da[r] = p * fmaf(da[r], m, dl[r]);
        } else {
          sa[r] = p;
          da[r] = p * da[r];
        }
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 pw, dw;
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          pw[jj] = MF<T>::pack(sa[8 * s2 + 2 * jj], sa[8 * s2 + 2 * jj + 1]);
          dw[jj] = MF<T>::pack(da[8 * s2 + 2 * jj], da[8 * s2 + 2 * jj + 1]);
        }
#pragma unroll
        for (int db = 0; db < 2; ++db) {
          dvt[db] = MF<T>::mma(as_frag<frag>(trA(doimg + j * 4096 + s2 * 2048, troff, db)), as_frag<frag>(pw), dvt[db]);
          dkt[db] = MF<T>::mma(as_frag<frag>(trA(img + j * 4096 + s2 * 2048, troff, db)), as_frag<frag>(dw), dkt[db]);
        }
      }
    }
    buf ^= 1;
    if (t + 1 < ntile) store_rc(buf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (key < Sk) {
    const long gt = ex.gkv_tok ? ex.gkv_tok : (long)H * 64;
    const long gh = ex.gkv_head ? ex.gkv_head : 64;
    T* dkr = dK + ((long)b * Sk + key) * gt + (long)head * gh;
    T* dvr = dV + ((long)b * Sk + key) * gt + (long)head * gh;
#pragma unroll
    for (int db = 0; db < 2; ++db)
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

template <typename T, bool C, int DR, bool BI>
void launch64b(bool bwd, const void* q, const void* k, const void* v, void* o, float* lse, const void* dout,
               const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, float scale,
               const FaStrides& fs, const FaExt& ex, hipStream_t st) {
  const dim3 gq((S + 255) / 256, B * H), gk((Sk + 255) / 256, B * H), blk(512);
  if (!bwd) {
    hipLaunchKernelGGL((fa64_fwd<T, C, DR != 0, BI>), gq, blk, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse,
                       S, Sk, H, Hk, scale * kLog2e, fs, ex);
    return;
  }
  // dK/dV workgroup size (PHA_FA64_DKDV_WAVES = 4: 128 keys per workgroup, two workgroups per CU
  // with independent barriers; 8: 256 keys, one per CU)
  const int nwk = getenv("PHA_FA64_DKDV_WAVES") && atoi(getenv("PHA_FA64_DKDV_WAVES")) == 4 ? 4 : 8;
  if (nwk == 4)
    hipLaunchKernelGGL((fa64_dkdv<T, C, DR, BI, 4>), dim3((Sk + 127) / 128, B * H), dim3(256), 0, st, (const T*)q,
                       (const T*)k, (const T*)v, (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs, ex);
  else
    hipLaunchKernelGGL((fa64_dkdv<T, C, DR, BI>), gk, blk, 0, st, (const T*)q, (const T*)k, (const T*)v,
                       (const T*)dout, lse, delta, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs, ex);
  hipLaunchKernelGGL((fa64_dq<T, C, DR, BI>), gq, blk, 0, st, (const T*)q, (const T*)k, (const T*)v, (const T*)dout,
                     lse, delta, (T*)dq, S, Sk, H, Hk, scale, fs, ex);
}

template <typename T, bool C, int DR>
void launch64(bool bwd, const void* q, const void* k, const void* v, void* o, float* lse, const void* dout,
              const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, float scale,
              const FaStrides& fs, const FaExt& ex, hipStream_t st) {
  if (ex.bias) launch64b<T, C, DR, true>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, scale, fs, ex, st);
  else launch64b<T, C, DR, false>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, scale, fs, ex, st);
}

template <typename T>
int dispatch64(bool bwd, const void* q, const void* k, const void* v, void* o, float* lse, const void* dout,
               const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, float scale,
               int causal, const FaStrides& fs, const FaExt& ex, hipStream_t st) {
  const int dr = ex.thresh == 0 ? 0 : (bwd && ex.dmask ? 2 : 1);
#define L64(C, D) launch64<T, C, D>(bwd, q, k, v, o, lse, dout, delta, dq, dk, dv, B, S, Sk, H, Hk, scale, fs, ex, st)
  if (causal) {
    if (dr == 2) L64(true, 2); else if (dr == 1) L64(true, 1); else L64(true, 0);
  } else {
    if (dr == 2) L64(false, 2); else if (dr == 1) L64(false, 1); else L64(false, 0);
  }
#undef L64
  return (int)hipGetLastError();
}

bool check64(const void* q, const void* k, const void* v, int S, int Sk, int H, int Hk, long q_tok, int q_head,
             long kv_tok, int kv_head, long o_tok, int o_head, float dropout) {
  if (S <= 0 || Sk <= 0 || H <= 0 || Hk <= 0 || H % Hk || dropout < 0.f || dropout >= 1.f) return false;
  if (((size_t)q | (size_t)k | (size_t)v) & 15) return false;
  if ((q_tok | kv_tok | o_tok) % 8 || (q_head | kv_head | o_head) % 8) return false;
  // the DMA's 32-bit offsets: 64 rows of the widest row stride
  return 64.0 * (double)(q_tok > kv_tok ? (q_tok > o_tok ? q_tok : o_tok) : (kv_tok > o_tok ? kv_tok : o_tok)) * 2 <
         4294967295.0;
}

// the bias rows are read as float4 quads of keys: 16-B aligned, key count and row strides in quads
bool bias_ok(const float* bias, int Sk, long sb, long sh, long sq) {
  if (!bias) return true;
  return ((size_t)bias & 15) == 0 && Sk % 4 == 0 && sb % 4 == 0 && sh % 4 == 0 && sq % 4 == 0 && sb >= 0 && sh >= 0 &&
         sq >= 0;
}

FaStrides strides64(long q_tok, int q_head, long kv_tok, int kv_head, long o_tok, int o_head) {
  FaStrides f;
  f.order_g = 0;
  f.q_tok = q_tok;
  f.kv_tok = kv_tok;
  f.o_tok = o_tok;
  f.dq_tok = f.dkv_tok = 0;
  f.q_head = q_head;
  f.kv_head = kv_head;
  f.o_head = o_head;
  f.dq_head = f.dkv_head = 0;
  return f;
}

}  // namespace

// keep-mask words per query row (keys rounded up to the dK/dV workgroup's 256): the forward's
// dmask is [B * H][words][S rounded up to 64] uint32 (word-major, so the forward's stores and the
// backward's loads run along the queries)
PHA_API int pha_fa64_mask_words(int Sk) { return 8 * ((Sk + 255) / 256); }
PHA_API long pha_fa64_mask_size(int B, int H, int S, int Sk) {
  return (long)B * H * pha_fa64_mask_words(Sk) * ((S + 63) & ~63);
}

// Head dim 64 forward: q [B, S, H, 64] / k, v [B, Sk, Hk, 64] with element strides (token, head)
// q_tok / q_head, kv_tok / kv_head (a packed [B, S, H, 3 * 64] projection is read in place), o with
// o_tok / o_head, lse [B, H, S] fp32; dropout in [0, 1) with the generic kernels' mask stream.
PHA_API int pha_fa64_fwd(int dt, const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Sk,
                         int H, int Hk, float scale, int causal, long q_tok, int q_head, long kv_tok, int kv_head,
                         long o_tok, int o_head, float dropout, unsigned seed, const unsigned* seedp,
                         hipStream_t stream, unsigned* dmask, const float* bias, long sb, long sh, long sq) {
  if (B <= 0 || !check64(q, k, v, S, Sk, H, Hk, q_tok, q_head, kv_tok, kv_head, o_tok, o_head, dropout) ||
      ((size_t)o & 7) || ((size_t)dmask & 15) || !bias_ok(bias, Sk, sb, sh, sq))
    return (int)hipErrorInvalidValue;
  FaExt ex{bias, sb, sh, sq, seed, (unsigned)(dropout * 65536.f + 0.5f), dropout > 0.f ? 1.f / (1.f - dropout) : 1.f};
  ex.seedp = seedp;
  ex.dmask = dropout > 0.f ? dmask : nullptr;
  ex.dmask_w = pha_fa64_mask_words(Sk);
  if (dropout > 0.f && ex.thresh == 0) ex.thresh = 1;
  const FaStrides fs = strides64(q_tok, q_head, kv_tok, kv_head, o_tok, o_head);
  if (dt == kBF16)
    return dispatch64<bf16_t>(false, q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, B, S, Sk, H, Hk,
                              scale, causal, fs, ex, stream);
  if (dt == kF16)
    return dispatch64<half_t>(false, q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, B, S, Sk, H, Hk,
                              scale, causal, fs, ex, stream);
  return (int)hipErrorInvalidValue;
}

// Head dim 64 backward (delta = rowsum(dO * O) from pha_flash_attn_bwd_preprocess): dout with the
// o strides, dq with gq_tok / gq_head, dk / dv with gkv_tok / gkv_head (0: dense [B, S, H, 64];
// dk / dv per query head — the caller sums GQA groups)
PHA_API int pha_fa64_bwd(int dt, const void* q, const void* k, const void* v, const void* dout, const float* lse,
                         const float* delta, void* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk,
                         float scale, int causal, long q_tok, int q_head, long kv_tok, int kv_head, long o_tok,
                         int o_head, long gq_tok, int gq_head, long gkv_tok, int gkv_head, float dropout,
                         unsigned seed, const unsigned* seedp, hipStream_t stream, const unsigned* dmask,
                         const float* bias, long sb, long sh, long sq) {
  if (B <= 0 || !check64(q, k, v, S, Sk, H, Hk, q_tok, q_head, kv_tok, kv_head, o_tok, o_head, dropout) ||
      ((size_t)dout & 15) || ((size_t)dq & 7) || ((size_t)dk & 7) || ((size_t)dv & 7) || (gq_tok | gkv_tok) % 4 ||
      (gq_head | gkv_head) % 4 || !bias_ok(bias, Sk, sb, sh, sq))
    return (int)hipErrorInvalidValue;
  FaExt ex{bias, sb, sh, sq, seed, (unsigned)(dropout * 65536.f + 0.5f), dropout > 0.f ? 1.f / (1.f - dropout) : 1.f};
  ex.seedp = seedp;
  ex.gq_tok = gq_tok;
  ex.gq_head = gq_head;
  ex.gkv_tok = gkv_tok;
  ex.gkv_head = gkv_head;
  ex.dmask = dropout > 0.f ? const_cast<unsigned*>(dmask) : nullptr;
  ex.dmask_w = pha_fa64_mask_words(Sk);
  if ((size_t)dmask & 15) return (int)hipErrorInvalidValue;
  if (dropout > 0.f && ex.thresh == 0) ex.thresh = 1;
  const FaStrides fs = strides64(q_tok, q_head, kv_tok, kv_head, o_tok, o_head);
  if (dt == kBF16)
    return dispatch64<bf16_t>(true, q, k, v, nullptr, const_cast<float*>(lse), dout, delta, dq, dk, dv, B, S, Sk, H,
                              Hk, scale, causal, fs, ex, stream);
  if (dt == kF16)
    return dispatch64<half_t>(true, q, k, v, nullptr, const_cast<float*>(lse), dout, delta, dq, dk, dv, B, S, Sk, H,
                              Hk, scale, causal, fs, ex, stream);
  return (int)hipErrorInvalidValue;
}
