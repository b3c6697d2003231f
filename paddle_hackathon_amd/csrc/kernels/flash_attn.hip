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
// Backward (FA2-style, key-block parallel): workgroup = 4 waves = 128 keys; each wave keeps
// its 32 keys' K and V fragments in registers and accumulates dK^T / dV^T over all query
// tiles; dS goes through LDS once so each wave computes one 32-wide d block of the
// workgroup's dQ contribution (all 128 keys), added with one fp32 atomic per element.
#include "common.h"

using namespace pha;

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

template <typename T> struct MF;
template <> struct MF<bf16_t> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
    return (uint32_t)f32_to_bf16(lo) | ((uint32_t)f32_to_bf16(hi) << 16);
  }
};
template <> struct MF<half_t> {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  }
  static __device__ __forceinline__ uint32_t pack(float lo, float hi) {
    _Float16 l = (_Float16)lo, h = (_Float16)hi;
    return (uint32_t)__builtin_bit_cast(uint16_t, l) | ((uint32_t)__builtin_bit_cast(uint16_t, h) << 16);
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

constexpr int BM = 128;   // query rows per workgroup (4 waves x 32)
constexpr int BN = 64;    // keys per tile
constexpr int VT_PAD = 4; // keys of padding per V^T row (row = 136 B)

// K tile: BN rows x D, 16-B chunks swizzled by (row & (CH-1)), CH = D/8 chunks per row
template <int D>
__device__ __forceinline__ int k_lds_off(int row, int chunk) {
  constexpr int CH = D / 8;
  return row * (D * 2) + ((chunk ^ (row & (CH - 1))) * 16);
}

template <typename T, int D, bool CAUSAL>
__global__ __launch_bounds__(256) void fa_fwd_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                     const T* __restrict__ V, T* __restrict__ O,
                                                     float* __restrict__ LSE, int S, int Sk, int H, int Hk,
                                                     float scale_log2) {
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

  for (int k0 = 0; k0 < kend; k0 += BN) {
    __syncthreads();  // previous tile fully consumed
    // ---- stage K (swizzled rows) and V^T into LDS --------------------------------
#pragma unroll
    for (int i = 0; i < (BN * CH) / 256; ++i) {
      const int c = tid + 256 * i;
      const int row = c / CH, ch = c % CH;
      const int key = k0 + row;
      u32x4 kv = {0, 0, 0, 0}, vv = {0, 0, 0, 0};
      if (key < Sk) {
        kv = *reinterpret_cast<const u32x4*>(Kb + (long)key * kstride + ch * 8);
        vv = *reinterpret_cast<const u32x4*>(Vb + (long)key * kstride + ch * 8);
      }
      *reinterpret_cast<u32x4*>(k_lds + k_lds_off<D>(row, ch)) = kv;
      const uint16_t* ve = reinterpret_cast<const uint16_t*>(&vv);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        *reinterpret_cast<uint16_t*>(vt_lds + (ch * 8 + e) * VT_STRIDE + row * 2) = ve[e];
    }
    __syncthreads();
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
    // ---- masking + online softmax (query on the lane) ---------------------------------
    float tmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = k0 + kb * 32 + acc_row(r, h);
        float v = s[kb][r] * scale_log2;
        const bool masked = (key >= Sk) || (CAUSAL && key > q);
        v = masked ? -INFINITY : v;
        s[kb][r] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float m_new = fmaxf(m_run, tmax);
    const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
    const float alpha = exp2f(m_run - m_use);
    float psum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float p = exp2f(s[kb][r] - m_use);
        s[kb][r] = p;
        psum += p;
      }
    psum += __shfl_xor(psum, 32, 64);
    l_run = l_run * alpha + psum;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < ND; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[i][r] *= alpha;

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

// delta[b,h,q] = sum_d dO * O  (fp32)
template <typename T, int D>
__global__ __launch_bounds__(256) void fa_bwd_pre_kernel(const T* __restrict__ O, const T* __restrict__ dO,
                                                         float* __restrict__ delta, int B, int S, int H) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);  // row over (b, q, head)
  const int lane = threadIdx.x & 63;
  if (row >= (long)B * S * H) return;
  const long off = row * D;
  float s = 0.f;
  for (int c = lane * 8; c < D; c += 512) {
    float a[8], g[8];
    Vec8<T>::ld(O + off + c, a);
    Vec8<T>::ld(dO + off + c, g);
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] * g[i];
  }
  s = wave_sum(s);
  if (lane == 0) {
    const int head = row % H;
    const long bq = row / H;
    const int q = bq % S;
    const int b = bq / S;
    delta[((long)b * H + head) * S + q] = s;
  }
}

// Backward. Workgroup = 4 waves = 128 keys (wave w: keys k0 + 32w .. +31, key on the lane).
// Per query tile of 32 rows (all 4 waves share it through LDS):
//   S  = Q K^T       C[q][key]  (A = Q rows from LDS, B = K^T from registers)
//   P  = exp2(S*c - lse*log2e)
//   dP = dO V^T      C[q][key]  (A = dO rows from LDS, B = V^T from registers)
//   dS = P (dP - delta)
//   dV^T += dO^T P   (A = dO^T from LDS (transposed image), B = P  accumulator-as-operand)
//   dK^T += Q^T dS   (A = Q^T  from LDS (transposed image), B = dS accumulator-as-operand)
//   dQ  += dS K      (dS through LDS [q][key], B = K^T... K[key][d] from LDS transposed)
template <typename T, int D, bool CAUSAL>
__global__ __launch_bounds__(256) void fa_bwd_kernel(const T* __restrict__ Q, const T* __restrict__ K,
                                                     const T* __restrict__ V, const T* __restrict__ dO,
                                                     const float* __restrict__ LSE, const float* __restrict__ DELTA,
                                                     float* __restrict__ dQ, T* __restrict__ dK, T* __restrict__ dV,
                                                     int S, int Sk, int H, int Hk, float scale) {
  typedef typename MF<T>::frag frag;
  constexpr int NK = D / 16;
  constexpr int ND = D / 32;
  constexpr int BQ = 32;                      // query rows per iteration
  constexpr int ROWB = D * 2 + 16;            // padded row bytes for Q/dO row images [q][d]
  constexpr int TB = (BQ + 8) * 2;            // padded row bytes for transposed images [d][q]
  constexpr int KTB = (128 + 8) * 2;          // K^T image rows [d][key] for the workgroup's 128 keys
  constexpr int DSB = (128 + 8) * 2;          // dS image rows [q][key]
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BQ * ROWB + 2 * D * TB + D * KTB + BQ * DSB];
  unsigned char* q_lds = smem;                       // [32][D] rows
  unsigned char* do_lds = q_lds + BQ * ROWB;         // [32][D] rows
  unsigned char* qt_lds = do_lds + BQ * ROWB;        // [D][32]
  unsigned char* dot_lds = qt_lds + D * TB;          // [D][32]
  unsigned char* kt_lds = dot_lds + D * TB;          // [D][128]
  unsigned char* ds_lds = kt_lds + D * KTB;          // [32][128]

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, h = lane >> 5, lr = lane & 31;
  const int head = blockIdx.y, b = blockIdx.z;
  const int group = H / Hk;
  const int hk = head / group;
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

  // K^T / V^T fragments for this wave's keys (B operands: B[k=d][col=key] = K[key][d])
  frag kf[NK], vf[NK];
#pragma unroll
  for (int kk = 0; kk < NK; ++kk) {
    u32x4 a = {0, 0, 0, 0}, c = {0, 0, 0, 0};
    if (key < Sk) {
      a = *reinterpret_cast<const u32x4*>(Kb + (long)key * kstride + 16 * kk + 8 * h);
      c = *reinterpret_cast<const u32x4*>(Vb + (long)key * kstride + 16 * kk + 8 * h);
    }
    kf[kk] = as_frag<frag>(a);
    vf[kk] = as_frag<frag>(c);
  }
  // K^T image of the workgroup's 128 keys for the dQ product (B[k=key][col=d] = K[key][d])
  for (int c = tid; c < 128 * (D / 8); c += 256) {
    const int row = c / (D / 8), ch = c % (D / 8);
    const int kk = k0 + row;
    u32x4 v = {0, 0, 0, 0};
    if (kk < Sk) v = *reinterpret_cast<const u32x4*>(Kb + (long)kk * kstride + ch * 8);
    const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<uint16_t*>(kt_lds + (ch * 8 + i) * KTB + row * 2) = e[i];
  }

  f32x16 dvt[ND], dkt[ND];
#pragma unroll
  for (int i = 0; i < ND; ++i) { dvt[i] = zero16(); dkt[i] = zero16(); }

  int qstart = 0;
  if (CAUSAL) qstart = (k0 / BQ) * BQ;
  for (int qt = qstart; qt < S; qt += BQ) {
    __syncthreads();
    // stage Q, dO rows and their transposed images
    for (int c = tid; c < BQ * (D / 8); c += 256) {
      const int row = c / (D / 8), ch = c % (D / 8);
      const int qq = qt + row;
      u32x4 a = {0, 0, 0, 0}, g = {0, 0, 0, 0};
      if (qq < S) {
        a = *reinterpret_cast<const u32x4*>(Qb + (long)qq * qstride + ch * 8);
        g = *reinterpret_cast<const u32x4*>(dOb + (long)qq * qstride + ch * 8);
      }
      *reinterpret_cast<u32x4*>(q_lds + row * ROWB + ch * 16) = a;
      *reinterpret_cast<u32x4*>(do_lds + row * ROWB + ch * 16) = g;
      const uint16_t* ea = reinterpret_cast<const uint16_t*>(&a);
      const uint16_t* eg = reinterpret_cast<const uint16_t*>(&g);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        *reinterpret_cast<uint16_t*>(qt_lds + (ch * 8 + i) * TB + row * 2) = ea[i];
        *reinterpret_cast<uint16_t*>(dot_lds + (ch * 8 + i) * TB + row * 2) = eg[i];
      }
    }
    __syncthreads();

    const bool active = !(CAUSAL && (k0 + wid * 32) > (qt + BQ - 1));
    f32x16 sacc = zero16(), dpacc = zero16();
    if (active) {
#pragma unroll
      for (int kk = 0; kk < NK; ++kk) {
        const u32x4 qa = *reinterpret_cast<const u32x4*>(q_lds + lr * ROWB + (2 * kk + h) * 16);
        const u32x4 ga = *reinterpret_cast<const u32x4*>(do_lds + lr * ROWB + (2 * kk + h) * 16);
        sacc = MF<T>::mma(as_frag<frag>(qa), kf[kk], sacc);
        dpacc = MF<T>::mma(as_frag<frag>(ga), vf[kk], dpacc);
      }
      // P and dS; rows = queries qt + acc_row(r,h), column = key (lane)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qq = qt + acc_row(r, h);
        float p = 0.f, ds = 0.f;
        if (qq < S && key < Sk && !(CAUSAL && key > qq)) {
          p = exp2f(sacc[r] * scale_log2 - lse_b[qq] * kLog2e);
          ds = p * (dpacc[r] - del_b[qq]);
        }
        sacc[r] = p;
        dpacc[r] = ds;
      }
      // dS image for dQ: ds_lds[q][key_local]
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        T* dst = reinterpret_cast<T*>(ds_lds + acc_row(r, h) * DSB + (wid * 32 + lr) * 2);
        Cvt<T>::st(dst, 0, dpacc[r]);
      }
      // dV^T += dO^T P ; dK^T += Q^T dS  (sum over q = accumulator row index)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        u32x4 pw, dw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          pw[j] = MF<T>::pack(sacc[8 * s + 2 * j], sacc[8 * s + 2 * j + 1]);
          dw[j] = MF<T>::pack(dpacc[8 * s + 2 * j], dpacc[8 * s + 2 * j + 1]);
        }
        const int qbase = 16 * s + 4 * h;
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
    } else {
      // inactive wave still publishes zeros for its dS columns
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        T* dst = reinterpret_cast<T*>(ds_lds + acc_row(r, h) * DSB + (wid * 32 + lr) * 2);
        Cvt<T>::st(dst, 0, 0.f);
      }
    }
    __syncthreads();
    // dQ[32 q][D] += dS[32][128 keys] . K[128][D]: wave w computes d-block(s) w (and w+4 if D>128)
    for (int db = wid; db < ND; db += 4) {
      f32x16 acc = zero16();
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {  // 128 keys = 8 k-steps of 16
        const u32x4 a = *reinterpret_cast<const u32x4*>(ds_lds + lr * DSB + (16 * ks + 8 * h) * 2);
        const unsigned char* kr = kt_lds + (db * 32 + lr) * KTB + (16 * ks + 8 * h) * 2;
        const u32x4 bb = *reinterpret_cast<const u32x4*>(kr);
        acc = MF<T>::mma(as_frag<frag>(a), as_frag<frag>(bb), acc);
      }
      // acc: C[q][d] rows = q, col = d (lane)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qq = qt + acc_row(r, h);
        if (qq < S) atomicAdd(dQ + (((long)b * S + qq) * H + head) * D + db * 32 + lr, acc[r] * scale);
      }
    }
  }
  // ---- store dK, dV (rows = d, col = key on the lane) ----------------------------------
  if (key < Sk) {
    T* dkr = dK + ((long)b * Sk + key) * ((long)H * D) + (long)head * D;   // dK/dV are [B, Sk, H, D]
    T* dvr = dV + ((long)b * Sk + key) * ((long)H * D) + (long)head * D;
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

template <typename T>
int launch_fwd(const void* q, const void* k, const void* v, void* o, float* lse, int B, int S, int Sk, int H, int Hk,
               int D, float scale, int causal, hipStream_t st) {
  const dim3 grid((S + BM - 1) / BM, H, B), block(256);
  const float sl = scale * kLog2e;
#define FA_L(DD, CC) hipLaunchKernelGGL((fa_fwd_kernel<T, DD, CC>), grid, block, 0, st, (const T*)q, (const T*)k, (const T*)v, (T*)o, lse, S, Sk, H, Hk, sl)
  if (D == 128) { if (causal) FA_L(128, true); else FA_L(128, false); }
  else if (D == 64) { if (causal) FA_L(64, true); else FA_L(64, false); }
  else return (int)hipErrorInvalidValue;
#undef FA_L
  return (int)hipGetLastError();
}

template <typename T>
int launch_bwd(const void* q, const void* k, const void* v, const void* dout, const float* lse, const float* delta,
               float* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk, int D, float scale, int causal,
               hipStream_t st) {
  const dim3 grid((Sk + 127) / 128, H, B), block(256);
#define FB_L(DD, CC) hipLaunchKernelGGL((fa_bwd_kernel<T, DD, CC>), grid, block, 0, st, (const T*)q, (const T*)k, (const T*)v, (const T*)dout, lse, delta, dq, (T*)dk, (T*)dv, S, Sk, H, Hk, scale)
  if (D == 128) { if (causal) FB_L(128, true); else FB_L(128, false); }
  else if (D == 64) { if (causal) FB_L(64, true); else FB_L(64, false); }
  else return (int)hipErrorInvalidValue;
#undef FB_L
  return (int)hipGetLastError();
}

}  // namespace

PHA_API int pha_flash_attn_fwd(int dt, const void* q, const void* k, const void* v, void* o, float* lse, int B, int S,
                               int Sk, int H, int Hk, int D, float scale, int causal, hipStream_t stream) {
  if (H % Hk || (D != 64 && D != 128) || S <= 0 || Sk <= 0) return (int)hipErrorInvalidValue;
  if (dt == kBF16) return launch_fwd<bf16_t>(q, k, v, o, lse, B, S, Sk, H, Hk, D, scale, causal, stream);
  if (dt == kF16) return launch_fwd<half_t>(q, k, v, o, lse, B, S, Sk, H, Hk, D, scale, causal, stream);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_flash_attn_bwd_preprocess(int dt, const void* o, const void* dout, float* delta, int B, int S, int H,
                                          int D, hipStream_t stream) {
  const long rows = (long)B * S * H;
  const dim3 grid((rows + 3) / 4), block(256);
  if (dt == kBF16) {
    if (D == 128) hipLaunchKernelGGL((fa_bwd_pre_kernel<bf16_t, 128>), grid, block, 0, stream, (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H);
    else hipLaunchKernelGGL((fa_bwd_pre_kernel<bf16_t, 64>), grid, block, 0, stream, (const bf16_t*)o, (const bf16_t*)dout, delta, B, S, H);
  } else if (dt == kF16) {
    if (D == 128) hipLaunchKernelGGL((fa_bwd_pre_kernel<half_t, 128>), grid, block, 0, stream, (const half_t*)o, (const half_t*)dout, delta, B, S, H);
    else hipLaunchKernelGGL((fa_bwd_pre_kernel<half_t, 64>), grid, block, 0, stream, (const half_t*)o, (const half_t*)dout, delta, B, S, H);
  } else {
    return (int)hipErrorInvalidValue;
  }
  return (int)hipGetLastError();
}

// dq: fp32 [B, S, H, D] zero-initialised by the caller; dk/dv: [B, Sk, H, D] (per query head;
// the caller sums head groups for GQA).
PHA_API int pha_flash_attn_bwd(int dt, const void* q, const void* k, const void* v, const void* dout, const float* lse,
                               const float* delta, float* dq, void* dk, void* dv, int B, int S, int Sk, int H, int Hk,
                               int D, float scale, int causal, hipStream_t stream) {
  if (H % Hk || (D != 64 && D != 128)) return (int)hipErrorInvalidValue;
  if (dt == kBF16) return launch_bwd<bf16_t>(q, k, v, dout, lse, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, stream);
  if (dt == kF16) return launch_bwd<half_t>(q, k, v, dout, lse, delta, dq, dk, dv, B, S, Sk, H, Hk, D, scale, causal, stream);
  return (int)hipErrorInvalidValue;
}
