// 8-wave (two waves per SIMD) 256 x 256 x 64 bf16/fp16 MFMA GEMM for gfx950, NT layout:
//
//   C[M, N] = A[M, K] . B^T[N, K]^T (+ bias[n]),  fp32 accumulate, bf16/fp16 out
//
// Reference behaviour: the cuBLAS NT products behind phi/kernels/impl/matmul_kernel_impl.h:88
// (linear forward on the transposed weight, dX = dY W) and the bias epilogue of
// fused_gemm_epilogue_op.cu:29.
//
// Why a second NT kernel. gemm4p (one wave per SIMD, 128 x 128 per wave) issues 16 LDS-DMAs, 32
// fragment reads and 128 MFMAs per wave and K-tile; every DMA issue (~60-185 cycles) and every
// wait stalls the only wave of its SIMD, so its long-K NT products stay 8-13 % behind hipBLASLt
// (profiles/gemm4p_early_ab_r3.log, PMC in gemm4p_early_pmc_r3/). Here two waves share each SIMD:
// waves w and w + 4 own the upper / lower 128 rows of the same 64 output columns, and whenever one
// of them stalls on a DMA issue, an LDS read or a wait, its partner's MFMAs keep the SIMD's matrix
// pipe busy (MI355X_MICROARCH.md, "Two waves per SIMD"). Per wave and K-tile: 8 DMAs (1 KiB), 24
// ds_read_b128, 64 v_mfma_f32_16x16x32; 128 AGPR accumulators + two 12-fragment register sets.
//
// K-loop, two LDS stages (tile kt in buffer kt & 1), two phases per K-tile:
//   phase A: MFMAs of k-half 0 (fragment set F0) | reads of k-half 1 of buffer kt&1 -> F1 in MFMA
//            groups 0-5; lgkmcnt(0) + barrier before group 6 (every wave holds all of tile kt:
//            the buffer is free); DMAs of tile kt+2 into it start (groups 6, 7)
//   A/B:     vmcnt(2) + barrier — tile kt+1 (issued one iteration earlier) has landed
//   phase B: MFMAs of k-half 1 (F1) | reads of k-half 0 of tile kt+1 -> F0 and the remaining 6
//            DMAs of tile kt+2 in groups 0-5
// so every DMA has >= 1.5 phases (~1.5k SIMD cycles) of latency cover. The LDS image and the DMA
// source swizzle are gemm4p's (128-B rows, 16-B chunk ^= row & 7, conflict-free ds_read_b128).
// Epilogue: each lane converts and pairs its accumulators with v_permlane16_swap into 16-B rows
// and writes them with bounds-checked buffer stores (rows past M and columns past N dropped).
#include "mfma_tile.h"
#include <type_traits>

namespace pha {
namespace g8w {

template <typename T> struct Ty { using type = T; };

using namespace g256;

enum : int {
  EPI_BIAS = 1,
  EPI_PRIO = 2,      // waves 4-7 run at s_setprio 1 (the second-dispatched half, guide item 4)
  EPI_NOSTORE = 4096, // measurement only: stores dropped by the bounds check
  // bits 8-10: the phase-A release group RELG (2, 3 or 6; 0 = 3)
};

struct Args {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  int M, N, K;
  int lda, ldb, ldc;
  int epi;
  int group_m;
};

constexpr int OPB = 256 * 64 * 2;   // one operand image (32 KB)
constexpr int STAGE = 2 * OPB;      // A image, B image
constexpr int SMEM = 2 * STAGE;     // two stages (128 KB)

__device__ __forceinline__ unsigned lds_u32(const unsigned char* p) {
  return (unsigned)(size_t)(__attribute__((address_space(3))) const unsigned char*)p;
}

// LDS-DMA 16 B per lane: global (sbase + voff) -> LDS m0 + lane * 16. Inline asm: hipcc's waitcnt
// pass would drain every DMA it can see with vmcnt(0) before the next ds_read (mfma_tile.h).
__device__ __forceinline__ void glds_sv(unsigned voff, const void* sbase, unsigned m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <typename T>
__device__ __forceinline__ unsigned pk(float lo, float hi) {
  if constexpr (std::is_same<T, bf16_t>::value) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, bf2{(__bf16)lo, (__bf16)hi});
  } else {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, h2{(_Float16)lo, (_Float16)hi});
  }
}

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

template <typename T, bool BIAS, int RELG>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2))) void gemm8w_nt_kernel(Args p) {
  static_assert(RELG >= 2 && RELG <= 6 && 12 % RELG == 0, "phase A reads 12 fragments over RELG groups");
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;   // rows wr*128 .. +127, columns wc*64 .. +63
  const int M = p.M, N = p.N;
  const int nk = p.K >> 6;

  // ---- tile: XCD-contiguous chunks of the linear order (bijective for any grid), GROUP_M panels
  int tm, tn;
  {
    const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
    const int bid = blockIdx.x, G = gridDim.x;
    const int q8 = G >> 3, r8 = G & 7, xcd = bid & 7;
    const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    const int gm = p.group_m;
    const int group = lin / (gm * tiles_n);
    const int first_m = group * gm;
    const int gsize = min(tiles_m - first_m, gm);
    const int in = lin - group * gm * tiles_n;
    tm = __builtin_amdgcn_readfirstlane(first_m + in % gsize);
    tn = __builtin_amdgcn_readfirstlane(in / gsize);
  }
  const int m0 = tm << 8, n0 = tn << 8;
  if ((p.epi & EPI_PRIO) && wr) __builtin_amdgcn_s_setprio(1);

  // ---- DMA: wave w fills 1-KiB pieces w*4 .. w*4+3 (8 rows x 128 B) of each operand image ------
  unsigned aoff[4], boff[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int row = (wid * 4 + u) * 8 + (lane >> 3);
    const unsigned sw = (unsigned)(((lane & 7) ^ (row & 7)) * 8);
    aoff[u] = ((unsigned)(min(m0 + row, M - 1) - m0) * (unsigned)p.lda + sw) * 2u;
    boff[u] = ((unsigned)(min(n0 + row, N - 1) - n0) * (unsigned)p.ldb + sw) * 2u;
  }
  const char* abase = static_cast<const char*>(p.a) + (size_t)m0 * p.lda * 2;
  const char* bbase = static_cast<const char*>(p.b) + (size_t)n0 * p.ldb * 2;
  const unsigned lds0 = lds_u32(smem);
  auto dma = [&](int kt, int buf, int d) {   // d = 0..7: piece d >> 1 of operand d & 1
    const int u = d >> 1;
    const unsigned dst = lds0 + buf * STAGE + (d & 1) * OPB + (wid * 4 + u) * 1024;
    if (d & 1) glds_sv(boff[u], bbase + (size_t)kt * 128, dst);
    else glds_sv(aoff[u], abase + (size_t)kt * 128, dst);
  };

  // ---- fragments: lane (fr, fk) holds k 8fk .. 8fk+7 of row fr of a 16-row block -------------
  const int fr = lane & 15, fk = lane >> 4;
  auto rdA = [&](int buf, int kh, int i) -> uint4 {
    const int row = wr * 128 + i * 16 + fr;
    return *reinterpret_cast<const uint4*>(smem + buf * STAGE + row * 128 + (((kh * 4 + fk) ^ (fr & 7)) << 4));
  };
  auto rdB = [&](int buf, int kh, int j) -> uint4 {
    const int row = wc * 64 + j * 16 + fr;
    return *reinterpret_cast<const uint4*>(smem + buf * STAGE + OPB + row * 128 + (((kh * 4 + fk) ^ (fr & 7)) << 4));
  };

  f32x4 acc[8][4];
  uint4 fa0[8], fb0[4], fa1[8], fb1[4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one phase: 8 MFMA groups (A fragment i x the 4 B fragments) on (ca, cb);
  // phase A (REL): the 12 fragment reads of (rbuf, rkh) into (na, nb) in groups 0 .. RELG-1 (B
  //   first), lgkmcnt(0) + barrier before group RELG (every wave holds all of its buffer's tile:
  //   the buffer is free), DMAs 0 .. 7-RELG of tile dkt in groups RELG .. 7;
  // phase B: the 12 reads two per group in groups 0-5, DMAs 8-RELG .. 7 in groups 0 .. RELG-1
  auto phase = [&](auto rd_c, auto rel_c, auto dma_c, uint4 (&ca)[8], uint4 (&cb)[4], uint4 (&na)[8],
                   uint4 (&nb)[4], int rbuf, int rkh, int dkt, int dbuf) {
    constexpr bool RD = decltype(rd_c)::value;
    constexpr bool REL = decltype(rel_c)::value;
    constexpr bool DM = decltype(dma_c)::value;
    constexpr int RPG = REL ? 12 / RELG : 2;   // reads per group
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      if constexpr (RD) {
        if (g * RPG < 12) {
#pragma unroll
          for (int r = RPG * g; r < RPG * g + RPG; ++r) {
            if (r < 4) nb[r] = rdB(rbuf, rkh, r);
            else na[r - 4] = rdA(rbuf, rkh, r - 4);
          }
        }
      }
      if constexpr (REL) {
        if (g == RELG) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          bar();
        }
        if (DM && g >= RELG) dma(dkt, dbuf, g - RELG);
      } else if constexpr (DM) {
        if (g < RELG) dma(dkt, dbuf, 8 - RELG + g);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[g][j] = Mf<T>::mma(cb[j], ca[g], acc[g][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using yes = std::true_type;
  using no = std::false_type;

  // ---- prologue: tiles 0 and 1 in flight, tile 0's k-half-0 fragments --------------------------
#pragma unroll
  for (int d = 0; d < 8; ++d) dma(0, 0, d);
  if (nk > 1) {
#pragma unroll
    for (int d = 0; d < 8; ++d) dma(1, 1, d);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
#pragma unroll
  for (int j = 0; j < 4; ++j) fb0[j] = rdB(0, 0, j);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = rdA(0, 0, i);

  int kt = 0;
  for (; kt + 2 < nk; ++kt) {   // steady state: tile kt+2 staged into this iteration's buffer
    const int buf = kt & 1;
    phase(yes{}, yes{}, yes{}, fa0, fb0, fa1, fb1, buf, 1, kt + 2, buf);
    asm volatile("s_waitcnt vmcnt(%0)" :: "n"(8 - RELG) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    bar();
    phase(yes{}, no{}, yes{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, kt + 2, buf);
  }
  if (kt + 1 < nk) {   // tile nk-2: nothing more to stage
    const int buf = kt & 1;
    phase(yes{}, yes{}, no{}, fa0, fb0, fa1, fb1, buf, 1, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bar();
    phase(yes{}, no{}, no{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, 0, 0);
    ++kt;
  }
  {   // last tile
    const int buf = kt & 1;
    phase(yes{}, no{}, no{}, fa0, fb0, fa1, fb1, buf, 1, 0, 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    phase(no{}, no{}, no{}, fa1, fb1, fa0, fb0, 0, 0, 0, 0);
  }

  // ---- epilogue ----------------------------------------------------------------------------------
  // acc[i][j][e] = C[m0 + wr*128 + i*16 + fr][n0 + wc*64 + j*16 + 4fk + e]. After the pair swap a
  // lane holds 8 consecutive columns from (pair base)*16 + (fk & 1)*16 + (fk >> 1)*8.
  const int ldc2 = p.ldc * 2;
  const int e_rows = (p.epi & EPI_NOSTORE) ? 0 : M - m0 - wr * 128;
  const int e_cols = N - n0;
  const int lcol = wc * 64 + (fk & 1) * 16 + (fk >> 1) * 8;
  const unsigned lane_voff = (unsigned)(fr * ldc2 + lcol * 2);
  const char* e_base = static_cast<const char*>(p.c) + ((size_t)(m0 + wr * 128) * ldc2 + (size_t)n0 * 2);
  __builtin_amdgcn_sched_barrier(0);
  f32x4 bv[4];
  if constexpr (BIAS) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = n0 + wc * 64 + j * 16 + 4 * fk;
      bv[j] = *reinterpret_cast<const f32x4*>(p.bias + (col < N ? col : 0));
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int cb = 0; cb < 4; cb += 2) {
      f32x4 x0 = acc[i][cb], x1 = acc[i][cb + 1];
      if constexpr (BIAS) {
        x0 += bv[cb];
        x1 += bv[cb + 1];
      }
      const unsigned q00 = pk<T>(x0[0], x0[1]), q01 = pk<T>(x0[2], x0[3]);
      const unsigned q10 = pk<T>(x1[0], x1[1]), q11 = pk<T>(x1[2], x1[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(q00, q10, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(q01, q11, false, false);
      const u32x4v q = u32x4v{s0[0], s1[0], s0[1], s1[1]};
      const int nbytes = __builtin_amdgcn_readfirstlane(max(min(e_rows - i * 16, 16), 0) * ldc2);
      const size_t bp = (size_t)(e_base + (size_t)i * 16 * ldc2);
      const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp);
      const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((size_t)bhi << 32) | blo), (short)0,
                                                        nbytes, 0x00020000);
      const unsigned voff = (lcol + cb * 16 < e_cols) ? lane_voff : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b128(q, rs, voff + cb * 32, 0, 2);
    }
  }
}

}  // namespace g8w
}  // namespace pha

using namespace pha;

// C[M, N] = A[M, K] . Bt[N, K]^T (+ bias[n]) on the 8-wave kernel. Requires K % 64 == 0;
// M, N, lda, ldb, ldc % 8 == 0; 16-B aligned pointers; 256 * lda * 2 and 256 * ldb * 2 < 2^32;
// 256 rows x ldc x 2 B < 2^31.
PHA_API int pha_gemm8w(int dt, const void* a, const void* b, void* c, long M, long N, long K, long lda, long ldb,
                       long ldc, int epi, const float* bias, int group_m, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8)
    return (int)hipErrorInvalidValue;
  if (lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (M > (1L << 30) || N > (1L << 30) || K > (1L << 30)) return (int)hipErrorInvalidValue;
  if (256.0 * lda * 2 >= 4294967295.0 || 256.0 * ldb * 2 >= 4294967295.0) return (int)hipErrorInvalidValue;
  if (256.0 * ldc * 2 >= 2147483647.0) return (int)hipErrorInvalidValue;
  if (((size_t)a | (size_t)b | (size_t)c) & 15) return (int)hipErrorInvalidValue;
  if ((epi & g8w::EPI_BIAS) && (!bias || ((size_t)bias & 15))) return (int)hipErrorInvalidValue;
  const long tiles = ((M + 255) / 256) * ((N + 255) / 256);
  if (tiles > (1L << 30)) return (int)hipErrorInvalidValue;
  if (group_m <= 0) group_m = 4;
  g8w::Args p{a, b, c, bias, (int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)ldc, epi, group_m};
  const bool bs = epi & g8w::EPI_BIAS;
  const dim3 grid((unsigned)tiles), block(512);
  const int relg = (epi >> 8) & 7;   // release group (schedule variant; 0 = the default 3)
  auto go = [&](auto t_c, auto r_c) {
    using TT = typename decltype(t_c)::type;
    constexpr int R = decltype(r_c)::value;
    if (bs) hipLaunchKernelGGL((g8w::gemm8w_nt_kernel<TT, true, R>), grid, block, 0, stream, p);
    else hipLaunchKernelGGL((g8w::gemm8w_nt_kernel<TT, false, R>), grid, block, 0, stream, p);
  };
  auto by_r = [&](auto t_c) {
    if (relg == 2) go(t_c, std::integral_constant<int, 2>{});
    else if (relg == 6) go(t_c, std::integral_constant<int, 6>{});
    else go(t_c, std::integral_constant<int, 3>{});
  };
  if (dt == kBF16) by_r(g8w::Ty<bf16_t>{});
  else if (dt == kF16) by_r(g8w::Ty<half_t>{});
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
