// Large-tile MFMA GEMM / implicit-GEMM convolution for gfx950 (reference behaviour:
// phi/kernels/gpu/matmul_kernel.cu and conv_kernel.cu — cuBLAS / cuDNN there).
//
//   C[M, N] (row-major, ldc) = sum_k A[m, k] * Bt[n, k]  (+ bias[n]) (relu | gelu)
//
//   A: K-contiguous rows (lda) — or, A_CONV, the NHWC implicit im2col of x: row m = output pixel,
//      k = (kh, kw, cin) with cin fastest (Cin % 8 == 0, so a 16-B chunk never straddles taps)
//   Bt: K-contiguous rows of B^T (ldb) — a [Cout][KH][KW][Cin] filter for convolution
//
// Structure (CDNA guide §5 "glds vs register staging", "Pipelining across barriers"):
//  * 256 x BN x 64 block tile (BN = 64 | 128 | 256), 512 threads = 8 waves laid out
//    (8 / (BN/64)) x (BN/64), each wave a (256 / WM) x 64 sub-tile of 16x16 accumulators
//    (v_mfma_f32_16x16x32_bf16: the shape the chip clocks highest on random data).
//  * A and Bt tiles go global -> LDS with global_load_lds_dwordx4 (no VGPR staging, no ds_write):
//    the LDS image is lane-linear per wave-instruction, so the XOR swizzle (16-B chunk ^= row & 7,
//    conflict-free ds_read_b128 fragment reads) is applied to each lane's SOURCE address and the
//    same involution on the read. The conv gather is just a per-lane source address (a zero page
//    stands in for padding taps and out-of-range rows).
//  * Two LDS stages; tile k+1 is issued before tile k is multiplied and retired by a COUNTED
//    s_waitcnt vmcnt (never 0 in the loop) ahead of a raw s_barrier — __syncthreads() would drain
//    the prefetch too.
#include "common.h"
#include <cstdlib>
#include <type_traits>

namespace pha {
namespace g256 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int NT = 512;

enum Act : int { ACT_NONE = 0, ACT_RELU = 1, ACT_GELU = 2 };

struct ConvGeo {
  int N, H, W, C;   // input NHWC
  int OH, OW;
  int KH, KW;
  int sh, sw, ph, pw, dh, dw;
};

struct Args {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  long M, N, K;
  long lda, ldb, ldc;
  int act;
  const void* zero;   // >= 16 B of zeros
  ConvGeo g;
};

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
  else return row * 64 + ((chunk ^ ((row >> 2) & 3)) << 4);
}

__device__ __forceinline__ void glds16(const void* src, unsigned char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
}

// per-lane row state of the A gather for one of the wave's A instructions
struct ARow {
  const char* base;   // row base (plain) or image pixel base (conv: n, oh*sh-ph, ow*sw-pw folded)
  int ih0, iw0;       // conv: top-left input coordinate of the row's receptive field
  bool ok;
};

template <typename T, int BM, int BN, int BK, bool CONV>
__global__ __launch_bounds__(NT) void gemm256_kernel(Args p) {
  constexpr int NSTAGE = BK == 64 ? 2 : 4;   // BK 64: one tile in flight; BK 32: three
  constexpr int WN = BN / 64, WM = 8 / WN;          // wave grid
  constexpr int WTM = BM / WM;                       // wave tile rows (16 .. 128)
  static_assert(WTM % 16 == 0, "wave tile rows");
  constexpr int RB = WTM / 16, CB = 4;               // 16x16 blocks per wave
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int A_WI = A_BYTES / 1024;                        // A wave-instructions per stage
  constexpr int A_INS = (A_WI + 7) / 8;                       // per thread
  constexpr int B_WI = B_BYTES / 1024;                        // B wave-instructions per stage (4 | 8 | 16)
  constexpr int B_INS = (B_WI + 7) / 8;                       // per thread (waves beyond B_WI repeat one)
  constexpr int INS = A_INS + B_INS;
  constexpr int CROW = BN * 2 + 16;                   // padded LDS row (bytes) of the staged C tile
  constexpr int SMEM = NSTAGE * STAGE > BM * CROW ? NSTAGE * STAGE : BM * CROW;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);   // provably wave-uniform (glds M0 base)
  const int wm = wid / WN, wn = wid % WN;
  const long M = p.M, N = p.N, K = p.K;

  // XCD-aware tile order (CDNA guide T1): the 8 XCDs take contiguous runs of tiles, walked in
  // GROUP_M-row panels so consecutive tiles of an XCD share their A or B panel in its L2
  const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
  const int ntiles = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int q = ntiles / 8, r = ntiles % 8, xcd = bid % 8;
  const int tile = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + bid / 8;
  constexpr int GROUP_M = 8;
  const int group = tile / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (tile % (GROUP_M * tiles_n)) % gsize;
  const int tn = (tile % (GROUP_M * tiles_n)) / gsize;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;

  const T* A = static_cast<const T*>(p.a);
  const T* Bt = static_cast<const T*>(p.b);
  const char* zero = static_cast<const char*>(p.zero);

  // ---- per-lane source rows of this thread's glds instructions ------------------------------
  // wave-instruction i fills image bytes [i * 1024, +1024) = RPI rows of 2*BK bytes; lane l takes
  // row i*RPI + l/CPR and LDS chunk l%CPR; its SOURCE chunk is the swizzle of that (involution)
  constexpr int CPR = BK / 8, RPI = 64 / CPR;      // 16-B chunks per row, rows per wave-instruction
  const int lrow = lane / CPR, lch = lane % CPR;
  ARow ar[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = ((j * 8 + wid) % A_WI) * RPI + lrow;
    const long m = m0 + row;
    ar[j].ok = m < M;
    if constexpr (CONV) {
      const ConvGeo& g = p.g;
      const long mm = ar[j].ok ? m : 0;
      const int hw = g.OH * g.OW;
      const int n = (int)(mm / hw);
      const int rem = (int)(mm - (long)n * hw);
      const int oh = rem / g.OW, ow = rem - (rem / g.OW) * g.OW;
      ar[j].ih0 = oh * g.sh - g.ph;
      ar[j].iw0 = ow * g.sw - g.pw;
      ar[j].base = reinterpret_cast<const char*>(A + (long)n * g.H * g.W * g.C);
    } else {
      ar[j].base = reinterpret_cast<const char*>(A + (ar[j].ok ? m : 0) * p.lda);
      ar[j].ih0 = ar[j].iw0 = 0;
    }
  }
  const char* brow[B_INS];
  bool bok[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = ((j * 8 + wid) % B_WI) * RPI + lrow;
    const long n = n0 + row;
    bok[j] = n < N;
    brow[j] = reinterpret_cast<const char*>(Bt + (bok[j] ? n : 0) * p.ldb);
  }
  // source chunk: row % RPI == lrow for every instruction, so the swizzle is per lane constant
  const int sch = BK == 64 ? (lch ^ (lrow & 7)) : (lch ^ ((lrow >> 2) & 3));

  auto issue = [&](int stage, long k0) {
    unsigned char* sa = smem + stage * STAGE;
    unsigned char* sb = sa + A_BYTES;
    const long k = k0 + sch * 8;
    const bool kok = k < K;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const char* src = zero;
      if (ar[j].ok && kok) {
        if constexpr (CONV) {
          const ConvGeo& g = p.g;
          const int tap = (int)(k / g.C), cin = (int)(k - (long)tap * g.C);
          const int kh = tap / g.KW, kw = tap - kh * g.KW;
          const int ih = ar[j].ih0 + kh * g.dh, iw = ar[j].iw0 + kw * g.dw;
          if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
            src = ar[j].base + (((long)ih * g.W + iw) * g.C + cin) * sizeof(T);
        } else {
          src = ar[j].base + k * sizeof(T);
        }
      }
      glds16(src, sa + ((j * 8 + wid) % A_WI) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const char* src = (bok[j] && kok) ? brow[j] + k * sizeof(T) : zero;
      glds16(src, sb + ((j * 8 + wid) % B_WI) * 1024);   // duplicate waves rewrite identical bytes
    }
  };

  f32x4 acc[RB][CB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((K + BK - 1) / BK);
  // prologue: tiles 0..NSTAGE-2 in flight
#pragma unroll
  for (int t = 0; t < NSTAGE - 1; ++t)
    if (t < nk) issue(t, (long)t * BK);
  const int fr = lane & 15, fk = lane >> 4;   // fragment row / k-chunk of this lane
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NSTAGE;
    // retire tile kt (this thread's loads), leaving the later prefetched tiles in flight
    const int later = min(NSTAGE - 2, nk - 1 - kt);
    if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * INS) : "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(INS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // one barrier publishes every wave's share of tile kt and certifies that the stage read in
    // iteration kt-1 is free for tile kt + NSTAGE - 1
    __builtin_amdgcn_s_barrier();
    if (kt + NSTAGE - 1 < nk) issue((kt + NSTAGE - 1) % NSTAGE, (long)(kt + NSTAGE - 1) * BK);
    const unsigned char* sa = smem + cur * STAGE;
    const unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int kh = 0; kh < BK / 32; ++kh) {
      uint4 bf[CB];
#pragma unroll
      for (int j = 0; j < CB; ++j) bf[j] = *reinterpret_cast<const uint4*>(sb + img_off<BK>(wn * 64 + j * 16 + fr, kh * 4 + fk));
#pragma unroll
      for (int i = 0; i < RB; ++i) {
        const uint4 af = *reinterpret_cast<const uint4*>(sa + img_off<BK>(wm * WTM + i * 16 + fr, kh * 4 + fk));
#pragma unroll
        for (int j = 0; j < CB; ++j) acc[i][j] = Mf<T>::mma(af, bf[j], acc[i][j]);
      }
    }
  }
  __builtin_amdgcn_s_barrier();   // all fragment reads done: the LDS is reused for the C tile

  // ---- epilogue: bias / activation, C tile staged through LDS so every lane stores 16 B --------
  // acc[i][j] register e = C[row 4*(lane>>4) + e][col lane&15] of 16x16 block (i, j)
  unsigned char* ct = smem;
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const int nl = wn * 64 + j * 16 + fr;
    const float bv = (p.bias && n0 + nl < N) ? p.bias[n0 + nl] : 0.f;
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[i][j][e] + bv;
        if (p.act == ACT_RELU) v = fmaxf(v, 0.f);
        else if (p.act == ACT_GELU) v = gelu_tanh(v);
        const int ml = wm * WTM + i * 16 + 4 * fk + e;
        *reinterpret_cast<uint16_t*>(ct + ml * CROW + nl * 2) = Mf<T>::cvt(v);
      }
  }
  __syncthreads();
  T* C = static_cast<T*>(p.c);
  constexpr int CH = BN / 8;                          // 16-B chunks per C row
  const bool full_n = n0 + BN <= N && (p.ldc % 8) == 0;
  for (int idx = tid; idx < BM * CH; idx += NT) {
    const int ml = idx / CH, c8 = idx % CH;
    const long m = m0 + ml, n = n0 + c8 * 8;
    if (m >= M) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + ml * CROW + c8 * 16);
    if (full_n) {
      *reinterpret_cast<uint4*>(C + m * p.ldc + n) = v;
    } else {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
      for (int t = 0; t < 8 && n + t < N; ++t) reinterpret_cast<uint16_t*>(C)[m * p.ldc + n + t] = e[t];
    }
  }
}

// BK = 64 (one tile in flight, half the barriers) suits compute-bound GEMMs; BK = 32 (three tiles
// in flight) the short-K, bandwidth-heavy convolutions. PHA_G256_BK overrides.
// tile: index into cands (-1 = heuristic), bk: 32 | 64 (0 = heuristic); the host autotuner
// (ops/conv_gemm.py) times the candidates once per shape and passes its choice
template <typename T, bool CONV>
int launch(const Args& a, hipStream_t st, int tile = -1, int bk = 0) {
  if (bk != 32 && bk != 64) bk = (CONV || a.K <= 1024) ? 32 : 64;
  // tile shape: the fewest "CU rounds x tile work / tile efficiency" (a 784-tile grid on 256 CUs
  // wastes a quarter of the chip in its last round; small tiles pay in operand re-reads)
  static const int cands[6][2] = {{256, 256}, {256, 128}, {128, 256}, {256, 64}, {128, 128}, {128, 64}};
  static const float eff[6] = {1.0f, 0.9f, 0.88f, 0.72f, 0.75f, 0.55f};
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  int best = 0;
  double best_t = 1e300;
  for (int c = 0; c < 6; ++c) {
    const int bm = cands[c][0], bn = cands[c][1];
    if (bn > 64 && a.N <= bn / 2) continue;   // half-empty column tiles
    const long tiles = ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
    const int per_cu = bm == 128 ? 2 : 1;      // 128-row tiles fit two workgroups per CU
    const double rounds = (double)((tiles + (long)cus * per_cu - 1) / ((long)cus * per_cu));
    const double t = rounds * bm * bn / (eff[c] * per_cu);
    if (t < best_t * 0.97) { best_t = t; best = c; }
  }
  if (tile >= 0 && tile < 6) best = tile;
  const int bm = cands[best][0], bn = cands[best][1];
  auto go = [&](auto bm_c, auto bn_c) {
    constexpr int BMc = decltype(bm_c)::value, BNc = decltype(bn_c)::value;
    const long tiles = ((a.M + BMc - 1) / BMc) * ((a.N + BNc - 1) / BNc);
    if (bk == 32) hipLaunchKernelGGL((gemm256_kernel<T, BMc, BNc, 32, CONV>), dim3((unsigned)tiles), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((gemm256_kernel<T, BMc, BNc, 64, CONV>), dim3((unsigned)tiles), dim3(NT), 0, st, a);
  };
#define G256_CASE(M_, N_) if (bm == M_ && bn == N_) { go(std::integral_constant<int, M_>(), std::integral_constant<int, N_>()); return (int)hipGetLastError(); }
  G256_CASE(256, 256) G256_CASE(256, 128) G256_CASE(256, 64) G256_CASE(128, 256) G256_CASE(128, 128) G256_CASE(128, 64)
#undef G256_CASE
  return (int)hipErrorInvalidValue;
}

}  // namespace g256
}  // namespace pha

using namespace pha;

// C[M,N] = A[M,K] . Bt[N,K]^T (+bias)(act); A, Bt K-contiguous, K % 8 == 0, 16-B aligned rows.
PHA_API int pha_gemm256_nt(int dt, const void* a, const void* bt, void* c, const float* bias, long M, long N, long K,
                           long lda, long ldb, long ldc, int act, const void* zero16, int tile, int bk,
                           hipStream_t stream) {
  if (K % 8 || lda % 8 || ldb % 8 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  g256::Args p{a, bt, c, bias, M, N, K, lda, ldb, ldc, act, zero16, {}};
  if (dt == kBF16) return g256::launch<bf16_t, false>(p, stream, tile, bk);
  if (dt == kF16) return g256::launch<half_t, false>(p, stream, tile, bk);
  return (int)hipErrorInvalidValue;
}

// NHWC conv forward: y[N*OH*OW, Cout] = im2col(x) . w^T, w as [Cout][KH][KW][Cin], Cin % 8 == 0.
PHA_API int pha_conv256_fwd(int dt, const void* x, const void* w, void* y, const float* bias, int N, int H, int W,
                            int C, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw, int act,
                            const void* zero16, int tile, int bk, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  g256::ConvGeo g{N, H, W, C, (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, (W + 2 * pw - dw * (KW - 1) - 1) / sw + 1,
                  KH, KW, sh, sw, ph, pw, dh, dw};
  const long M = (long)N * g.OH * g.OW, K = (long)KH * KW * C;
  g256::Args p{x, w, y, bias, M, (long)Cout, K, 0, K, (long)Cout, act, zero16, g};
  if (dt == kBF16) return g256::launch<bf16_t, true>(p, stream, tile, bk);
  if (dt == kF16) return g256::launch<half_t, true>(p, stream, tile, bk);
  return (int)hipErrorInvalidValue;
}
