// Single-kernel flash-attention backward for gfx950 (see the comment above fa_bwd_fused).
//
// Built with -mllvm -amdgpu-mfma-vgpr-form=1 (ops/build.py reads the pha-build-flags line below):
// the S / dP / dQ products then keep their accumulators in VGPRs while the dK^T / dV^T
// accumulators (256 registers) are pinned to the AGPR file by the inline-asm MFMAs of mfma_agpr().
// pha-build-flags: -mllvm -amdgpu-mfma-vgpr-form=1
#include "fa_common.h"
#include <cstdlib>
#include <cstring>

namespace {

// ============================================================================================
// Backward v3 (D = 128): ONE kernel for dK, dV and dQ (CDNA guide App. B "Attention backward").
//  workgroup = 4 waves (one per SIMD) = 256 keys of one (batch, query head); wave w owns keys
//  k0 + 64w .. +63 as two 32-key blocks with the key on the MFMA lane:
//   * K of all 256 keys is staged ONCE in LDS as a dual-use image (row reads for S = Q K^T,
//     transposed reads for dQ = dS K); V B-fragments of the wave's 64 keys live in registers.
//   * the workgroup sweeps 32-row query slices (Q, dO, row constants double-buffered in LDS).
//     S and dP accumulators start from the row constants -lse/scale and -delta, so
//     p = exp2(c S') and dS = p dP' need no per-element subtraction.
//   * dV^T += dO^T P, dK^T += Q^T dS with the accumulators as B operands (no LDS for P / dS),
//     dS^T crosses LDS once; then wave w forms dQ[32 q][32 d] (d block w) over all 256 keys and
//     adds it to an fp32 dQ buffer with float atomics — per wave-instruction two 128-B row
//     segments, the full-rate atomic shape; 4x fewer atomic bytes than 64-key workgroups.
//  dK^T/dV^T of 64 keys = 256 accumulator registers per wave, hence one wave per SIMD.
// Replaces the two-kernel v2 backward (dK/dV kernel + dQ kernel that recomputed S and dP:
// 7 GEMM-units of MFMA work instead of 5).
// ============================================================================================
// acc += A B with the accumulator pinned to AGPRs (AGPR-form MFMA in inline asm; the compiler's
// MFMAs in this file are VGPR-form). hipcc pads no hazards inside asm: `s_nop 1` covers an operand
// written by a VALU instruction (v_cvt_pk of P / dS) or a v_accvgpr_write (the zero init) just
// before; MFMA -> next MFMA on the same accumulator needs no wait.
template <typename T> struct MfmaAsm;
template <> struct MfmaAsm<bf16_t> {
  static __device__ __forceinline__ void run(f32x16& acc, const u32x4& a, const u32x4& b) {
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  }
};
template <> struct MfmaAsm<half_t> {
  static __device__ __forceinline__ void run(f32x16& acc, const u32x4& a, const u32x4& b) {
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  }
};

constexpr int FB_KEYS = 256;   // keys per workgroup
constexpr int FB_BQ = 32;      // query rows per slice

// dS^T image: [key][32 q] bf16, 64-B rows, 16-B chunks XOR-swizzled by (row>>1)&3 so the
// per-key 8-byte stores are 2-way (not 8-way) and the transposed reads stay conflict-free
__device__ __forceinline__ int dst_off(int row, int chunk) { return row * 64 + 16 * (chunk ^ ((row >> 1) & 3)); }

template <typename T, bool CAUSAL>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void fa_bwd_fused(const T* __restrict__ Q, const T* __restrict__ K, const T* __restrict__ V,
                  const T* __restrict__ dO, const float* __restrict__ LSE, const float* __restrict__ DELTA,
                  float* __restrict__ dQacc, T* __restrict__ dK, T* __restrict__ dV, int S, int Sk, int H,
                  int Hk, float scale, FaStrides fs) {
  typedef typename MF<T>::frag frag;
  constexpr int NK = 8, ND = 4;
  constexpr int KIMG = FB_KEYS * 256;              // 64 KiB each for K and V
  constexpr int SIMG = FB_BQ * 256;                // 8 KiB each for the Q and dO slices
  constexpr int DSIMG = FB_KEYS * FB_BQ * 2;       // 16 KiB
  // K | V | Q slice | dO slice | dS^T = exactly the 160 KiB of a CU's LDS
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * KIMG + 2 * SIMG + DSIMG];
  unsigned char* const k_img = smem;
  unsigned char* const v_img = smem + KIMG;
  unsigned char* const q_img = smem + 2 * KIMG;
  unsigned char* const do_img = q_img + SIMG;
  unsigned char* const ds_img = do_img + SIMG;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int g = lane >> 4, gi = lane & 15, tq = gi >> 2, tp = gi & 3;
  // (b, h) fastest in the grid: every pair's heaviest (causal: first) key block is dispatched
  // before any lighter one, so the kernel does not end on a few long workgroups
  const int head = blockIdx.x % H, b = blockIdx.x / H;
  const int hk = head / (H / Hk);
  const int k0 = blockIdx.y * FB_KEYS;
  const int wk0 = k0 + wid * 64;
  const T* Qb = Q + (long)b * S * fs.q_tok + (long)head * fs.q_head;
  const T* dOb = dO + (long)b * S * fs.o_tok + (long)head * fs.o_head;
  const T* Kb = K + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const T* Vb = V + (long)b * Sk * fs.kv_tok + (long)hk * fs.kv_head;
  const float* lse_b = LSE + ((long)b * H + head) * S;
  const float* del_b = DELTA + ((long)b * H + head) * S;
  float* dQb = dQacc + (long)b * S * H * 128 + (long)head * 128;   // dense fp32 [B, S, H, 128]
  const long dq_row = (long)H * 128;
  const float scale_log2 = scale * kLog2e;
  const float inv_scale = 1.f / scale;

  // K and V images of the workgroup's 256 keys (rows past Sk are zero)
#pragma unroll 4
  for (int i = 0; i < 32; ++i) {
    const int c = tid + 256 * i;
    const int which = c >> 12, cc = c & 4095;
    const int row = cc >> 4, ch = cc & 15;
    const int key = k0 + row;
    const T* src = which ? Vb : Kb;
    const u32x4 v = key < Sk ? *reinterpret_cast<const u32x4*>(src + (long)key * fs.kv_tok + ch * 8) : u32x4{0, 0, 0, 0};
    *reinterpret_cast<u32x4*>(smem + which * KIMG + dual_off(row, ch)) = v;
  }
  f32x16 dvt[2][ND], dkt[2][ND];
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int i = 0; i < ND; ++i) { dvt[kb][i] = zero16(); dkt[kb][i] = zero16(); }

  // slice staging in registers: Q and dO (32 rows x 16 chunks each = 1024 chunks, 4 per thread);
  // the row constants -lse/scale (-inf past S, so those rows' p is exactly 0) and -delta stay in
  // registers, lane l holding row l & 31, and reach the accumulator rows by lane shuffles
  u32x4 sreg[4];
  float nxt_lse = 0.f, nxt_del = 0.f;
  auto load_slice = [&](int qs) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int which = c >> 9, cc = c & 511;
      const int qq = qs + (cc >> 4), ch = cc & 15;
      const T* src = which ? dOb : Qb;
      const long rs = which ? fs.o_tok : fs.q_tok;
      sreg[i] = qq < S ? *reinterpret_cast<const u32x4*>(src + (long)qq * rs + ch * 8) : u32x4{0, 0, 0, 0};
    }
    const int qq = qs + lr;
    nxt_lse = qq < S ? -lse_b[qq] * inv_scale : -INFINITY;
    nxt_del = qq < S ? -del_b[qq] : 0.f;
  };
  auto store_slice = [&]() {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + 256 * i;
      const int which = c >> 9, cc = c & 511;
      *reinterpret_cast<u32x4*>(q_img + which * SIMG + dual_off(cc >> 4, cc & 15)) = sreg[i];
    }
  };

  const int qstart = CAUSAL ? k0 : 0;   // k0 is a multiple of 256: slices stay 32-aligned
  const int nslice = qstart < S ? (S - qstart + FB_BQ - 1) / FB_BQ : 0;
  if (nslice > 0) {
    load_slice(qstart);
    store_slice();
  }
  __syncthreads();
  for (int t = 0; t < nslice; ++t) {
    const int q0 = qstart + t * FB_BQ;
    const float cur_lse = nxt_lse, cur_del = nxt_del;
    if (t + 1 < nslice) load_slice(q0 + FB_BQ);
    const bool need_mask = (wk0 + 64 > Sk) || (CAUSAL && wk0 + 63 > q0);
    // Both 32-key blocks are always computed (a block entirely past the causal diagonal or Sk
    // has p = 0 through the mask): a branch per block makes hipcc copy the loop-carried dK/dV
    // accumulators and spill. One block's S / dP is live at a time.
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      // S = Q K^T - lse/scale, dP = dO V^T - delta   (C[q][key], key on the lane); accumulator
      // row of register r: q = acc_row(r, h) = (r&3) + 8(r>>2) + 4h
      f32x16 sacc, dpacc;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        sacc[r] = __shfl(cur_lse, acc_row(r, h), 64);
        dpacc[r] = __shfl(cur_del, acc_row(r, h), 64);
      }
      const int krow = wid * 64 + 32 * kb + lr;
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const u32x4 qa = *reinterpret_cast<const u32x4*>(q_img + dual_off(lr, 2 * kk + h));
        const u32x4 ga = *reinterpret_cast<const u32x4*>(do_img + dual_off(lr, 2 * kk + h));
        const u32x4 ka = *reinterpret_cast<const u32x4*>(k_img + dual_off(krow, 2 * kk + h));
        const u32x4 va = *reinterpret_cast<const u32x4*>(v_img + dual_off(krow, 2 * kk + h));
        sacc = MF<T>::mma(as_frag<frag>(qa), as_frag<frag>(ka), sacc);
        dpacc = MF<T>::mma(as_frag<frag>(ga), as_frag<frag>(va), dpacc);
      }
      const int key = k0 + krow;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = fexp2(sacc[r] * scale_log2);
        if (need_mask && (key >= Sk || (CAUSAL && key > q0 + acc_row(r, h)))) p = 0.f;
        sacc[r] = p;
        dpacc[r] *= p;   // dS (softmax scale applied at the outputs)
      }
      // dV^T += dO^T P, dK^T += Q^T dS (accumulators as B operands); dS^T -> LDS for dQ
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        u32x4 pw, dw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pw[j] = MF<T>::pack(sacc[8 * s2 + 2 * j], sacc[8 * s2 + 2 * j + 1]);
          dw[j] = MF<T>::pack(dpacc[8 * s2 + 2 * j], dpacc[8 * s2 + 2 * j + 1]);
        }
        const int r0 = 16 * s2 + 4 * h;
#pragma unroll
        for (int db = 0; db < ND; ++db) {
          const u32x4 av = tr_frag(do_img, r0, db, g, tq, tp);
          const u32x4 bv = tr_frag(q_img, r0, db, g, tq, tp);
          MfmaAsm<T>::run(dvt[kb][db], av, pw);
          MfmaAsm<T>::run(dkt[kb][db], bv, dw);
        }
        // registers 8s2 .. 8s2+7 = rows q 16s2 + 8(j>>2) + 4h + (j&3): two 4-row runs, 8 B each
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          const int qc = 16 * s2 + 8 * half + 4 * h;   // first q of the run
          *reinterpret_cast<u32x2*>(ds_img + dst_off(krow, qc >> 3) + 2 * (qc & 7)) =
              u32x2{dw[2 * half], dw[2 * half + 1]};
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __syncthreads();   // dS^T of all 256 keys is in LDS; every wave is done with this Q / dO slice
    if (t + 1 < nslice) store_slice();

    // dQ[q][32 wid + n] += sum_key dS[q][key] K[key][d]: A = dS (tr reads of dS^T), B = K (tr reads)
    int nks = FB_KEYS / 16;
    if (CAUSAL) nks = min(nks, (q0 + FB_BQ - k0) / 16);
    nks = min(nks, (Sk - k0 + 15) / 16);
    f32x16 dq = zero16();
    const int ach = 2 * (g & 1) + (tp >> 1);
#pragma unroll 4
    for (int s = 0; s < nks; ++s) {
      const int r0 = 16 * s + 4 * h;
      const u32x2 alo = ds_read_tr16(ds_img + dst_off(r0 + tq, ach) + 8 * (tp & 1));
      const u32x2 ahi = ds_read_tr16(ds_img + dst_off(r0 + 8 + tq, ach) + 8 * (tp & 1));
      const u32x4 a = {alo[0], alo[1], ahi[0], ahi[1]};
      const u32x4 bk = tr_frag(k_img, r0, wid, g, tq, tp);
      dq = MF<T>::mma(as_frag<frag>(a), as_frag<frag>(bk), dq);
    }
    // C[m = q][n = d]: lanes 0-31 / 32-63 each add one 128-B row segment per register
    float* col = dQb + 32 * wid + lr;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int qq = q0 + acc_row(r, h);
      if (qq < S) atomicAdd(col + (long)qq * dq_row, dq[r] * scale);
    }
    __syncthreads();   // next slice staged; dS^T image free
  }

  // the last asm MFMA's result must be complete before the compiler reads the AGPRs (an 8-pass
  // MFMA's D -> other reader: 12 wait states); the empty asm statements order every read after it
  asm volatile("s_nop 15");
#pragma unroll
  for (int kb = 0; kb < 2; ++kb)
#pragma unroll
    for (int db = 0; db < ND; ++db) {
      asm volatile("" : "+a"(dvt[kb][db]));
      asm volatile("" : "+a"(dkt[kb][db]));
    }
#pragma unroll
  for (int kb = 0; kb < 2; ++kb) {
    const int key = wk0 + 32 * kb + lr;
    if (key >= Sk) continue;
    T* dkr = dK + ((long)b * Sk + key) * fs.dkv_tok + (long)head * fs.dkv_head;   // per query head (GQA summed by caller)
    T* dvr = dV + ((long)b * Sk + key) * fs.dkv_tok + (long)head * fs.dkv_head;
#pragma unroll
    for (int db = 0; db < ND; ++db)
#pragma unroll
      for (int gg = 0; gg < 4; ++gg) {
        const int d = db * 32 + 8 * gg + 4 * h;
        u32x2 wk, wv;
        wk[0] = MF<T>::pack(dkt[kb][db][4 * gg + 0] * scale, dkt[kb][db][4 * gg + 1] * scale);
        wk[1] = MF<T>::pack(dkt[kb][db][4 * gg + 2] * scale, dkt[kb][db][4 * gg + 3] * scale);
        wv[0] = MF<T>::pack(dvt[kb][db][4 * gg + 0], dvt[kb][db][4 * gg + 1]);
        wv[1] = MF<T>::pack(dvt[kb][db][4 * gg + 2], dvt[kb][db][4 * gg + 3]);
        *reinterpret_cast<u32x2*>(dkr + d) = wk;
        *reinterpret_cast<u32x2*>(dvr + d) = wv;
      }
  }
}

// fp32 dQ accumulator [B, S, H, 128] -> T at the caller's strides (packed QKV gradient or dense)
template <typename T>
__global__ __launch_bounds__(256) void fa_dq_convert_kernel(const float* __restrict__ acc, T* __restrict__ dQ, long rows,
                                                            int H, long dq_tok, int dq_head) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;   // one 8-element chunk per thread
  if (i >= rows * 16) return;
  const long row = i >> 4;
  const int c = (int)(i & 15);
  float v[8];
  Vec8<float>::ld(acc + row * 128 + c * 8, v);
  u32x4 w;
#pragma unroll
  for (int j = 0; j < 4; ++j) w[j] = MF<T>::pack(v[2 * j], v[2 * j + 1]);
  *reinterpret_cast<u32x4*>(dQ + (row / H) * dq_tok + (row % H) * (long)dq_head + c * 8) = w;
}


// single-kernel backward (D = 128): zero the fp32 dQ workspace [B, S, H, 128], run the fused
// kernel, convert dQ to T at the caller's strides
template <typename T>
int launch_bwd_fused(const void* q, const void* k, const void* v, const void* dout, const float* lse,
                     const float* delta, void* dq, void* dk, void* dv, float* dq_acc, int B, int S, int Sk, int H,
                     int Hk, float scale, int causal, hipStream_t st, const FaStrides& fs) {
  hipError_t e = hipMemsetAsync(dq_acc, 0, (size_t)B * S * H * 128 * sizeof(float), st);
  if (e != hipSuccess) return (int)e;
  const dim3 grid(B * H, (Sk + FB_KEYS - 1) / FB_KEYS), block(256);
  if (causal)
    hipLaunchKernelGGL((fa_bwd_fused<T, true>), grid, block, 0, st, (const T*)q, (const T*)k, (const T*)v,
                       (const T*)dout, lse, delta, dq_acc, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs);
  else
    hipLaunchKernelGGL((fa_bwd_fused<T, false>), grid, block, 0, st, (const T*)q, (const T*)k, (const T*)v,
                       (const T*)dout, lse, delta, dq_acc, (T*)dk, (T*)dv, S, Sk, H, Hk, scale, fs);
  const long rows = (long)B * S * H;
  hipLaunchKernelGGL((fa_dq_convert_kernel<T>), dim3((unsigned)((rows * 16 + 255) / 256)), dim3(256), 0, st,
                     dq_acc, (T*)dq, rows, H, fs.dq_tok, fs.dq_head);
  return (int)hipGetLastError();
}

}  // namespace

// Single-kernel backward (D = 128) with an fp32 dQ workspace of B*S*H*128 floats.
PHA_API int pha_flash_attn_bwd_fused(int dt, const void* q, const void* k, const void* v, const void* dout,
                                     const float* lse, const float* delta, void* dq, void* dk, void* dv,
                                     float* dq_acc, int B, int S, int Sk, int H, int Hk, int D, float scale,
                                     int causal, hipStream_t stream) {
  if (H % Hk || D != 128 || S <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  const FaStrides f = dense_strides(H, Hk, D);
  if (dt == kBF16)
    return launch_bwd_fused<bf16_t>(q, k, v, dout, lse, delta, dq, dk, dv, dq_acc, B, S, Sk, H, Hk, scale, causal, stream, f);
  if (dt == kF16)
    return launch_bwd_fused<half_t>(q, k, v, dout, lse, delta, dq, dk, dv, dq_acc, B, S, Sk, H, Hk, scale, causal, stream, f);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_flash_attn_bwd_packed_fused(int dt, const void* qkv, const void* dout, const float* lse,
                                            const float* delta, void* dqkv, float* dq_acc, int B, int S, int H, int D,
                                            float scale, int causal, hipStream_t stream) {
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
    return launch_bwd_fused<bf16_t>(in, in + D * es, in + 2 * D * es, dout, lse, delta, out, out + D * es,
                                    out + 2 * D * es, dq_acc, B, S, S, H, H, scale, causal, stream, f);
  if (dt == kF16)
    return launch_bwd_fused<half_t>(in, in + D * es, in + 2 * D * es, dout, lse, delta, out, out + D * es,
                                    out + 2 * D * es, dq_acc, B, S, S, H, H, scale, causal, stream, f);
  return (int)hipErrorInvalidValue;
}

