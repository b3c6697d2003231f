// 256 x 256 x 64 MFMA GEMM with the 8-phase ping-pong schedule (CDNA guide §5 "The 256² 8-phase
// template", T3+T4 counted vmcnt, T5 setprio) for gfx950; reference behaviour: the cuBLAS GEMMs
// behind phi/kernels/gpu/matmul_kernel.cu (matmul / linear forward and both gradients).
//
//   C[M, N] = sum_k A(m, k) B(k, n) (+ bias[n]) (relu | gelu), bf16 / fp16 in, fp32 accumulate
//
// Either operand may be K-contiguous (A[m][k] / Bt[n][k]: row reads, ds_read_b128) or K-outer
// (A[k][m] / B[k][n]: the LDS image keeps the HBM layout and fragments are read transposed with
// ds_read_b64_tr_b16), so one kernel serves x @ W (NN), dY @ W^T (NT) and X^T @ dY (TN).
//
// Schedule. 8 waves = 2 (M) x 4 (N); wave (wr, wc) owns the 128 x 64 C block at rows wr*128,
// cols wc*64, split into 4 quadrants of 64 x 32 (16 MFMAs of 16x16x32 per K-tile each). A K-tile
// is staged as four 16 KB half-tiles — A0 / A1 (the qm = 0 / 1 quadrant rows of both wave rows),
// B0 / B1 (the qn = 0 / 1 quadrant columns of all wave columns) — into one of two 64 KB buffers.
// Each of the 4 phases of a K-tile reads one quadrant's fragments (A0+B0, B1, A1, -; B0 and B1 stay
// in registers), issues ONE half-tile (2 global_load_lds per thread), waits vmcnt(8) (the 4 most
// recent half-tiles stay in flight, never 0 in the loop), barriers, runs its 16 MFMAs at raised
// priority and barriers again. Wave row 1 runs one barrier behind wave row 0, so one group's
// MFMAs overlap the other's LDS reads and load issue on every SIMD.
//
// Hazards (all waves barrier together; group 1 lags by one barrier):
//  * RAW: a half-tile is read one phase after the phase whose vmcnt(8) retired it.
//  * WAR: a half-tile slot is re-filled >= 2 phases after its last read (A0 / B0 read in phase 0,
//    re-issued in phases 2 / 3 for the K-tile two ahead; B1 / A1 for the next K-tile in phases 0 / 1
//    of the other buffer, last read 3 phases earlier).
//  Issue order: prologue A0 B0 B1 A1 (tile 0), A0 B0 (tile 1); phase j of tile t issues
//  B1(t+1), A1(t+1), A0(t+2), B0(t+2) — each half-tile is retired by the vmcnt(8) of the phase
//  before its first read.
#include "mfma_tile.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace pha {
namespace g8p {

using namespace g256;

struct Args {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  int M, N, K;
  int lda, ldb, ldc;
  int act;
  const void* zero;   // >= 16 B of zeros
  float* ws;          // splits > 1: fp32 partials [splits][M][N] (bias / act applied by the reduction)
  int splits, kchunk; // split-K: split s covers k in [s * kchunk, (s + 1) * kchunk), kchunk % 64 == 0
};

constexpr unsigned kNone = 0xffffffffu;

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// V: schedule ablations (0 = the schedule above; bit 0: no wave-row stagger, bit 1: no setprio,
// bit 2: fragment reads retired before the barrier). Measured at 8192^3 / 16384x6144x2048 bf16:
// dropping the stagger costs 10-12 %, dropping setprio 10-12 %, bit 2 is neutral.
template <typename T, bool AKO, bool BKO, int V = 0>
__global__ __launch_bounds__(512) void gemm8p_kernel(Args p) {
  constexpr int HALF = 16384, BUF = 4 * HALF;
  constexpr int CROW = 256 * 2 + 16;
  constexpr int SMEM = 256 * CROW > 2 * BUF ? 256 * CROW : 2 * BUF;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  const int M = p.M, N = p.N, K = p.K;

  // XCD-bijective tile order, GROUP_M-row panels (as gemm256)
  const int tiles_m = (M + 255) / 256, tiles_n = (N + 255) / 256;
  const int ntiles = tiles_m * tiles_n, total = ntiles * p.splits;
  const int bid = blockIdx.x;
  const int q8 = total / 8, r8 = total % 8, xcd = bid % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int split = lin / ntiles, tile = lin % ntiles;   // an XCD walks consecutive tiles of one split
  const int kbeg = split * p.kchunk, kend = min(K, kbeg + p.kchunk);
  constexpr int GROUP_M = 8;
  const int group = tile / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (tile % (GROUP_M * tiles_n)) % gsize;
  const int tn = (tile % (GROUP_M * tiles_n)) / gsize;
  const int m0 = tm * 256, n0 = tn * 256;

  const T* A = static_cast<const T*>(p.a);
  const T* B = static_cast<const T*>(p.b);
  const char* zero = static_cast<const char*>(p.zero);

  // ---- per-lane glds sources: half-tile h (0 A0, 1 A1, 2 B0, 3 B1), instruction u -----------
  // K-contiguous image: [128 idx][64 k] (128-B rows, chunk ^= idx & 7); instruction w = 2*wid+u
  // fills idx rows 8w .. 8w+7, lane -> idx 8w + lane/8, LDS chunk lane%8 <- source chunk
  // (lane%8) ^ (lane/8). K-outer image: [64 k][128 idx] (256-B rows, tn_mask swizzle), lane ->
  // k-row 4w + lane/16, LDS chunk lane%16 <- source idx chunk (lane%16) ^ tn_mask(k-row).
  unsigned soff[4][2];   // element offset of the lane's source at k0 = 0 (kNone: outside M / N)
  int skoff[4][2];       // k of the lane's source chunk / row relative to k0
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bool isA = h < 2;
      const bool ko = isA ? AKO : BKO;
      const int qd = h & 1, w = wid * 2 + u;
      int idx, koff;
      if (!ko) {
        idx = w * 8 + (lane >> 3);
        koff = ((lane & 7) ^ (lane >> 3)) * 8;
      } else {
        const int kr = w * 4 + (lane >> 4);
        idx = ((lane & 15) ^ tn_mask(kr, 256)) * 8;
        koff = kr;
      }
      const int g = isA ? m0 + (idx >> 6) * 128 + qd * 64 + (idx & 63) : n0 + (idx >> 5) * 64 + qd * 32 + (idx & 31);
      const int dim = isA ? M : N, ld = isA ? p.lda : p.ldb;
      soff[h][u] = g < dim ? (ko ? (unsigned)g + (unsigned)koff * (unsigned)ld : (unsigned)g * (unsigned)ld + (unsigned)koff)
                           : kNone;
      skoff[h][u] = koff;
    }
  const int nk = (kend - kbeg + 63) / 64;

  auto issue = [&](int h, int t, int buf) {
    const bool isA = h < 2;
    const bool ko = isA ? AKO : BKO;
    const T* base = isA ? A : B;
    const int ld = isA ? p.lda : p.ldb;
    const int k0 = kbeg + t * 64;
    unsigned char* dst = smem + buf * BUF + h * HALF + wid * 2048;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const char* src = zero;
      if (t < nk && soff[h][u] != kNone && k0 + skoff[h][u] < kend)
        src = reinterpret_cast<const char*>(base + soff[h][u] + (ko ? (long)k0 * ld : (long)k0));
      glds16(src, dst + u * 1024);
    }
  };

  const int fr = lane & 15, fk = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  // fragments of one quadrant: A (4 row blocks x 2 k-halves), B (2 column blocks x 2 k-halves)
  auto readA = [&](const unsigned char* img, uint4 (&af)[4][2]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        if constexpr (!AKO) {
          const int row = wr * 64 + i * 16 + fr;
          af[i][kh] = *reinterpret_cast<const uint4*>(img + row * 128 + (((kh * 4 + fk) ^ (row & 7)) << 4));
        } else {
          af[i][kh] = tn_frag<256>(img, kh * 32 + 8 * fk, wr * 64 + i * 16, tq, tp);
        }
      }
  };
  auto readB = [&](const unsigned char* img, uint4 (&bf)[2][2]) {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        if constexpr (!BKO) {
          const int row = wc * 32 + j * 16 + fr;
          bf[j][kh] = *reinterpret_cast<const uint4*>(img + row * 128 + (((kh * 4 + fk) ^ (row & 7)) << 4));
        } else {
          bf[j][kh] = tn_frag<256>(img, kh * 32 + 8 * fk, wc * 32 + j * 16, tq, tp);
        }
      }
  };

  f32x4 acc[2][2][4][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[a][b][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mfma = [&](f32x4 (&c)[4][2], const uint4 (&af)[4][2], const uint4 (&bf)[2][2]) {
    if constexpr (!(V & 4)) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(V & 2)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kh = 0; kh < 2; ++kh)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) c[i][j] = Mf<T>::mma(af[i][kh], bf[j][kh], c[i][j]);
    if constexpr (!(V & 2)) __builtin_amdgcn_s_setprio(0);
  };
  auto wait_bar = [&]() {
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    if constexpr (V & 4) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
  };

  // prologue: A0 B0 B1 A1 of tile 0, A0 B0 of tile 1; retire tile 0's A0 and B0
  issue(0, 0, 0);
  issue(2, 0, 0);
  issue(3, 0, 0);
  issue(1, 0, 0);
  issue(0, 1, 1);
  issue(2, 1, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  bar();
  if (!(V & 1) && wr == 1) bar();   // the ping-pong stagger

  uint4 af[4][2], b0[2][2], b1[2][2];
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1;
    const unsigned char* img = smem + buf * BUF;
    // phase 0: quadrant (0, 0)
    readA(img + 0 * HALF, af);
    readB(img + 2 * HALF, b0);
    issue(3, t + 1, buf ^ 1);
    wait_bar();
    mfma(acc[0][0], af, b0);
    bar();
    // phase 1: quadrant (0, 1)
    readB(img + 3 * HALF, b1);
    issue(1, t + 1, buf ^ 1);
    wait_bar();
    mfma(acc[0][1], af, b1);
    bar();
    // phase 2: quadrant (1, 1)
    readA(img + 1 * HALF, af);
    issue(0, t + 2, buf);
    wait_bar();
    mfma(acc[1][1], af, b1);
    bar();
    // phase 3: quadrant (1, 0)
    issue(2, t + 2, buf);
    wait_bar();
    mfma(acc[1][0], af, b0);
    bar();
  }
  if (!(V & 1) && wr == 0) bar();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();

  // acc[qm][qn][i][j] register e = C[wr*128 + qm*64 + i*16 + 4*fk + e][wc*64 + qn*32 + j*16 + fr]
  if (p.splits > 1) {   // split-K: fp32 partials straight from the accumulators (16 lanes = 64 B of a row)
    float* ws = p.ws + (long)split * M * N;
#pragma unroll
    for (int qn = 0; qn < 2; ++qn)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wc * 64 + qn * 32 + j * 16 + fr;
        if (n >= N) continue;
#pragma unroll
        for (int qm = 0; qm < 2; ++qm)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int m = m0 + wr * 128 + qm * 64 + i * 16 + 4 * fk + e;
              if (m < M) ws[(long)m * N + n] = acc[qm][qn][i][j][e];
            }
      }
    return;
  }

  // ---- epilogue: bias / activation, C tile staged through LDS so every lane stores 16 B ------
  unsigned char* ct = smem;
#pragma unroll
  for (int qn = 0; qn < 2; ++qn)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int nl = wc * 64 + qn * 32 + j * 16 + fr;
      const float bv = (p.bias && n0 + nl < N) ? p.bias[n0 + nl] : 0.f;
#pragma unroll
      for (int qm = 0; qm < 2; ++qm)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float v = acc[qm][qn][i][j][e] + bv;
            if (p.act == ACT_RELU) v = fmaxf(v, 0.f);
            else if (p.act == ACT_GELU) v = gelu_tanh(v);
            const int ml = wr * 128 + qm * 64 + i * 16 + 4 * fk + e;
            *reinterpret_cast<uint16_t*>(ct + ml * CROW + nl * 2) = Mf<T>::cvt(v);
          }
    }
  __syncthreads();
  T* C = static_cast<T*>(p.c);
  const bool full_n = n0 + 256 <= N && (p.ldc % 8) == 0;
  for (int idx = tid; idx < 256 * 32; idx += 512) {
    const int ml = idx >> 5, c8 = idx & 31;
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

// C = sum of the split partials (+ bias)(act), 4 columns per thread
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, T* __restrict__ C,
                                                            const float* __restrict__ bias, int M, int N, int ldc,
                                                            int S, int act) {
  const long MN = (long)M * N;
  for (long i4 = ((long)blockIdx.x * 256 + threadIdx.x) * 4; i4 < MN; i4 += (long)gridDim.x * 256 * 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(ws + i4);
    for (int s = 1; s < S; ++s) v += *reinterpret_cast<const f32x4*>(ws + s * MN + i4);
    const long m = i4 / N;
    const int n = (int)(i4 - m * N);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float x = v[e] + (bias ? bias[n + e] : 0.f);
      if (act == ACT_RELU) x = fmaxf(x, 0.f);
      else if (act == ACT_GELU) x = gelu_tanh(x);
      Cvt<T>::st(C, m * ldc + n + e, x);
    }
  }
}

template <typename T>
int launch(const Args& a, int ako, int bko, hipStream_t st) {
  const unsigned grid = (unsigned)(((a.M + 255) / 256) * ((a.N + 255) / 256) * a.splits);
  if (!ako && !bko) hipLaunchKernelGGL((gemm8p_kernel<T, false, false>), dim3(grid), dim3(512), 0, st, a);
  else if (!ako && bko) hipLaunchKernelGGL((gemm8p_kernel<T, false, true>), dim3(grid), dim3(512), 0, st, a);
  else if (ako && !bko) hipLaunchKernelGGL((gemm8p_kernel<T, true, false>), dim3(grid), dim3(512), 0, st, a);
  else hipLaunchKernelGGL((gemm8p_kernel<T, true, true>), dim3(grid), dim3(512), 0, st, a);
  if (a.splits > 1) {
    const long MN = (long)a.M * a.N;
    const unsigned rg = (unsigned)std::min((MN / 4 + 255) / 256, 8192L);
    hipLaunchKernelGGL((splitk_reduce_kernel<T>), dim3(rg), dim3(256), 0, st, a.ws, static_cast<T*>(a.c), a.bias, a.M,
                       a.N, a.ldc, a.splits, a.act);
  }
  return (int)hipGetLastError();
}

}  // namespace g8p
}  // namespace pha

using namespace pha;

// C[M,N] = A . B (+bias)(act). a_kouter: A stored [K][lda] (else [M][lda]); b_kouter: B stored
// [K][ldb] (else B^T stored [N][ldb]). M, N, K, lda, ldb % 8 == 0; every operand < 2^32 elements.
// splits > 1: split-K over fp32 partials in ws (>= splits * M * N floats, ldc == N), for products
// with few output tiles and a long K (a weight gradient of a square projection).
PHA_API int pha_gemm8p(int dt, const void* a, const void* b, void* c, const float* bias, long M, long N, long K,
                       long lda, long ldb, long ldc, int a_kouter, int b_kouter, int act, const void* zero16,
                       int splits, float* ws, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % 8 || N % 8 || K % 8 || lda % 8 || ldb % 8) return (int)hipErrorInvalidValue;
  const double asz = (double)(a_kouter ? K : M) * lda, bsz = (double)(b_kouter ? K : N) * ldb;
  if (asz >= 4294967295.0 || bsz >= 4294967295.0 || M > (1L << 30) || N > (1L << 30) || K > (1L << 30))
    return (int)hipErrorInvalidValue;
  if (splits < 1) splits = 1;
  const long kchunk = ((K + 64L * splits - 1) / (64L * splits)) * 64;
  splits = (int)((K + kchunk - 1) / kchunk);
  if (splits > 1 && (!ws || N % 4 || ldc != N)) return (int)hipErrorInvalidValue;
  g8p::Args p{a, b, c, bias, (int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)ldc, act, zero16, ws, splits, (int)kchunk};
  if (dt == kBF16) return g8p::launch<bf16_t>(p, a_kouter, b_kouter, stream);
  if (dt == kF16) return g8p::launch<half_t>(p, a_kouter, b_kouter, stream);
  return (int)hipErrorInvalidValue;
}
