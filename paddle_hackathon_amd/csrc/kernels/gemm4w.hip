// 256 x 256 x 64 bf16/fp16 MFMA GEMM, ONE wave per SIMD (4 waves, 512 VGPR+AGPR per lane) with
// fused epilogues, for gfx950. Reference behaviour: the cuBLAS/cuBLASLt GEMMs behind
// phi/kernels/impl/matmul_kernel_impl.h:88 (matmul / linear forward and both gradients) and the
// fused_gemm_epilogue op (paddle/fluid/operators/fused/fused_gemm_epilogue_op.cu:29,298: bias +
// gelu/relu forward, dgelu + bias-grad backward).
//
//   C[M, N] = epilogue( sum_k A(m, k) B(k, n) ),  fp32 accumulate
//
// Why one wave per SIMD. Each wave owns a 128 x 128 C block (8 x 8 tiles of 16x16x32 MFMA, 256
// accumulator registers) so a K-tile is 128 MFMAs (~2k cycles) per wave against 32 fragment reads:
// half the LDS read traffic of the 8-wave / 128x64-per-wave layout and ONE workgroup barrier per
// K-tile instead of eight. Latency is hidden inside the wave: fragments are double-buffered by
// k-half (F0 = k 0..31, F1 = k 32..63 of a K-tile), so every phase issues the reads of the NEXT
// k-half between the MFMAs of the current one, and the MFMAs after the barrier run on registers
// that were loaded before it.
//
//   prologue: glds tile 0 -> buf 0, tile 1 -> buf 1; wait tile 0; barrier; read F0(0)
//   K-tile t (buf b = t & 1):
//     phase A: read F1(t) from buf b             | 64 MFMA on F0
//     boundary: vmcnt(0) (tile t+1 landed), lgkmcnt(0) (buf b reads done), barrier
//     phase B: glds tile t+2 -> buf b, read F0(t+1) from buf b^1 | 64 MFMA on F1
//
// Operands: K-contiguous (A[m][k] / B^T[n][k]) tiles are LDS images [256][64] (128-B rows, 16-B
// chunk ^= row & 7, read with ds_read_b128); K-outer (A[k][m] / B[k][n]) tiles are two
// [64 k][128 idx] images (256-B rows, tn_mask swizzle, read transposed with ds_read_b64_tr_b16).
// The LDS-DMA (global_load_lds_dwordx4) uses the SGPR-base + 32-bit VGPR-offset form: the per-lane
// offsets are fixed for the whole K loop and only the wave-uniform base advances.
//
// Epilogue: the fp32 accumulators are staged through LDS in two 128-row halves; each thread then
// owns 8 consecutive columns of a row: bias, GELU (optionally also storing the pre-activation for
// the backward), ReLU, dGELU against a stored pre-activation, fp32 column partial sums (bias
// gradients), and 16-B global stores.
#include "mfma_tile.h"
#include <type_traits>

namespace pha {
namespace g4w {

using namespace g256;

enum : int {
  EPI_BIAS = 1,     // + bias[n] (fp32)
  EPI_GELU = 2,     // C = gelu_tanh(v); with EPI_AUXOUT the pre-activation v goes to aux
  EPI_RELU = 4,
  EPI_DGELU = 8,    // C = v * gelu_tanh'(aux[m][n])
  EPI_COLSUM = 16,  // colsum[tile_m][n] = sum of the tile's rows of the final fp32 C
  EPI_AUXOUT = 32,
  EPI_TRANS = 64,   // store C^T: the kernel computes the transposed product (see pha_gemm4w)
  EPI_SKIP = 128,      // measurement only: no epilogue (tools/g4w_fixed.py)
  EPI_NOSTORE = 512,   // measurement only: epilogue without its global stores
  EPI_NOSTAGE = 1024,  // measurement only: epilogue without the LDS staging writes
  EPI_NTSTORE = 2048,  // output stores with the non-temporal (streaming) hint
  EPI_STAGGER = 4096,  // first-round workgroups start in G = (epi >> 24) & 15 phase groups, group g
                       // after g * ((epi >> 16) & 255) s_sleep(127) — the tiles' output bursts then
                       // fall on different CUs at different times instead of all at once
};

// Epilogue builds (a kernel template parameter): the dGELU build loads the stored pre-activation,
// the AUX build also stores the pre-activation; keeping them out of the plain build keeps its
// epilogue free of register spills (every scratch reload is an exposed memory latency per tile)
enum : int { EK_PLAIN = 0, EK_DGELU = 1, EK_AUX = 2, EK_GEN = 3 };   // PLAIN: convert + store only

struct Args {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  void* aux;
  float* colsum;
  int M, N, K;
  int lda, ldb, ldc, ldaux;
  int epi;
};

constexpr int OPB = 256 * 64 * 2;   // one operand image (32 KB)
constexpr int STAGE = 2 * OPB;      // A image, B image
constexpr int CROWF = 256 * 4 + 16; // fp32 epilogue staging row (bytes)
constexpr int SMEM = (128 * CROWF > 2 * STAGE) ? 128 * CROWF : 2 * STAGE;

__device__ __forceinline__ unsigned lds_u32(const unsigned char* p) {
  return (unsigned)(size_t)(__attribute__((address_space(3))) const unsigned char*)p;
}

// LDS-DMA 16 B per lane: global (sbase + voff) -> LDS m0 + lane * 16
__device__ __forceinline__ void glds_sv(unsigned voff, const void* sbase, unsigned m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ float fast_tanh(float u) {
  const float e = __expf(2.f * u);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}
__device__ __forceinline__ float gelu_t(float x) {
  const float u = 0.7978845608028654f * (x + 0.044715f * x * x * x);
  return 0.5f * x * (1.f + fast_tanh(u));
}
__device__ __forceinline__ float gelu_t_grad(float x) {
  const float k = 0.7978845608028654f, x2 = x * x;
  const float t = fast_tanh(k * (x + 0.044715f * x2 * x));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x2);
}

template <typename T>
__device__ __forceinline__ float ld_elem(uint4 v, int e) {
  const uint16_t u = reinterpret_cast<const uint16_t*>(&v)[e];
  if constexpr (std::is_same<T, bf16_t>::value) return __uint_as_float((unsigned)u << 16);
  else return (float)__builtin_bit_cast(_Float16, u);
}

// SCHED bit 0: compiler-scheduled (else fragment reads / LDS-DMA issues pinned between groups of
// 4 MFMAs by sched_barrier); bit 1: reads spread one per MFMA group (else front-loaded); bit 2:
// early staging (tile t+2 issued mid phase A behind a second barrier)
template <typename T, bool AKO, bool BKO, int SCHED, bool OT = false, int EK = EK_PLAIN>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4w_kernel(Args p) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int M = p.M, N = p.N, K = p.K;

  // XCD-bijective block order, GROUP_M-row panels
  const int tiles_m = (M + 255) >> 8, tiles_n = (N + 255) >> 8;
  const int total = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int q8 = total >> 3, r8 = total & 7, xcd = bid & 7;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // GROUP_M-row panels (4: measured best or tied at every GPT NT / NN / TN shape against 2..32,
  // profiles/gemm4w_group_m_r2.log); measurement override: (epi >> 28) & 7 = log2(GROUP_M)
  const int GROUP_M = ((p.epi >> 28) & 7) ? (1 << ((p.epi >> 28) & 7)) : 4;
  const int group = lin / (GROUP_M * tiles_n);
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (lin % (GROUP_M * tiles_n)) % gsize;
  const int tn = (lin % (GROUP_M * tiles_n)) / gsize;
  const int m0 = tm << 8, n0 = tn << 8;

  // ---- LDS-DMA sources: 8 instructions per operand per wave, g = wid * 8 + u fills LDS bytes
  // [g * 1024, g * 1024 + 1024) of the operand image
  unsigned aoff[8], boff[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int g = wid * 8 + u;
#pragma unroll
    for (int op = 0; op < 2; ++op) {
      const bool ko = op == 0 ? AKO : BKO;
      const int dim = op == 0 ? M : N, base = op == 0 ? m0 : n0, ld = op == 0 ? p.lda : p.ldb;
      unsigned off;
      if (!ko) {
        const int row = g * 8 + (lane >> 3);
        const int grow = min(base + row, dim - 1) - base;
        off = ((unsigned)grow * (unsigned)ld + (unsigned)(((lane & 7) ^ (row & 7)) * 8)) * 2u;
      } else {
        const int half = g >> 4, krow = (g & 15) * 4 + (lane >> 4);
        const int src = (lane & 15) ^ tn_mask(krow, 256);
        const int idx = min(half * 128 + src * 8, dim - base - 8);
        off = ((unsigned)krow * (unsigned)ld + (unsigned)idx) * 2u;
      }
      if (op == 0) aoff[u] = off; else boff[u] = off;
    }
  }
  const char* abase = static_cast<const char*>(p.a) +
                      (AKO ? (size_t)m0 * 2 : (size_t)m0 * p.lda * 2);
  const char* bbase = static_cast<const char*>(p.b) +
                      (BKO ? (size_t)n0 * 2 : (size_t)n0 * p.ldb * 2);
  const size_t astep = AKO ? (size_t)64 * p.lda * 2 : 128, bstep = BKO ? (size_t)64 * p.ldb * 2 : 128;
  const unsigned lds0 = lds_u32(smem);
  const int nk = K >> 6;

  auto glds_one = [&](int t, int u, int op) {
    const unsigned dst = lds0 + (t & 1) * STAGE + op * OPB + (wid * 8 + u) * 1024;
    if (op == 0) glds_sv(aoff[u], abase + (size_t)t * astep, dst);
    else glds_sv(boff[u], bbase + (size_t)t * bstep, dst);
  };
  auto stage_all = [&](int t) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      glds_one(t, u, 0);
      glds_one(t, u, 1);
    }
  };

  const int fr = lane & 15, fk = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  auto readA = [&](int buf, int kh, int i) -> uint4 {
    const unsigned char* img = smem + buf * STAGE;
    if constexpr (!AKO) {
      const int row = wr * 128 + i * 16 + fr;
      return *reinterpret_cast<const uint4*>(img + row * 128 + (((kh * 4 + fk) ^ (fr & 7)) << 4));
    } else {
      return tn_frag<256>(img + wr * 16384, kh * 32 + 8 * fk, i * 16, tq, tp);
    }
  };
  auto readB = [&](int buf, int kh, int j) -> uint4 {
    const unsigned char* img = smem + buf * STAGE + OPB;
    if constexpr (!BKO) {
      const int row = wc * 128 + j * 16 + fr;
      return *reinterpret_cast<const uint4*>(img + row * 128 + (((kh * 4 + fk) ^ (fr & 7)) << 4));
    } else {
      return tn_frag<256>(img + wc * 16384, kh * 32 + 8 * fk, j * 16, tq, tp);
    }
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 fa0[8], fb0[8], fa1[8], fb1[8];

  // MFMA groups [g0, g1) of a phase (16 groups of 4 MFMAs = 64 MFMAs on (ca, cb)). With RD the 16
  // fragment reads of (rbuf, rkh) into (na, nb); with ST, GPG LDS-DMA issues of tile st per group
  // (numbered from gl0).
  auto phase = [&](auto rd_c, auto st_c, auto gpg_c, auto g0_c, auto g1_c, uint4 (&ca)[8], uint4 (&cb)[8],
                   uint4 (&na)[8], uint4 (&nb)[8], int rbuf, int rkh, int st, int gl0) {
    constexpr bool RD = decltype(rd_c)::value, ST = decltype(st_c)::value;
    constexpr int GPG = decltype(gpg_c)::value, G0 = decltype(g0_c)::value, G1 = decltype(g1_c)::value;
#pragma unroll
    for (int s = G0; s < G1; ++s) {
      if constexpr (RD && (SCHED & 2)) {   // one read per MFMA group, alternating A / B
        if (s & 1) nb[s >> 1] = readB(rbuf, rkh, s >> 1);
        else na[s >> 1] = readA(rbuf, rkh, s >> 1);
      } else if constexpr (RD) {
        // all 16 reads in the first half of the phase, in the order the next phase consumes them
        // (A0, B0..B7, A1..A7), so they have retired before its first MFMAs
        if (s < 8) {
#pragma unroll
          for (int r = 2 * s; r < 2 * s + 2; ++r) {
            if (r == 0) na[0] = readA(rbuf, rkh, 0);
            else if (r <= 8) nb[r - 1] = readB(rbuf, rkh, r - 1);
            else na[r - 8] = readA(rbuf, rkh, r - 8);
          }
        }
      }
      if constexpr (ST) {
#pragma unroll
        for (int q = 0; q < GPG; ++q) {
          const int gi = gl0 + (s - G0) * GPG + q;   // 0..15: (u = gi >> 1, operand gi & 1)
          glds_one(st, gi >> 1, gi & 1);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int idx = s * 4 + q, i = idx >> 3, j = idx & 7;
        // operand order picks the accumulator layout: (A, B) leaves a lane 4 consecutive C ROWS of
        // one column, (B, A) 4 consecutive C COLUMNS of one row; the epilogue wants the latter
        // along the output's rows (C^T rows with OT), so it can stage with 16-B LDS writes
        if constexpr (OT) acc[i][j] = Mf<T>::mma(ca[i], cb[j], acc[i][j]);
        else acc[i][j] = Mf<T>::mma(cb[j], ca[i], acc[i][j]);
      }
      if constexpr (!(SCHED & 1)) __builtin_amdgcn_sched_barrier(0);
    }
  };
  using yes = std::true_type;
  using no = std::false_type;
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I8 = std::integral_constant<int, 8>;
  using I16 = std::integral_constant<int, 16>;
  auto sync = [&](auto vm_c) {   // counted vmcnt + lgkmcnt(0) + barrier
    constexpr int VM = decltype(vm_c)::value;
    if constexpr (VM == 0) asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bar();
  };
  auto lgkm0 = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  if ((p.epi & EPI_STAGGER) && bid < 256) {
    const int groups = max((p.epi >> 24) & 15, 1);
    const int n = ((bid >> 3) % groups) * ((p.epi >> 16) & 255);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(127);
  }

  // prologue
  stage_all(0);
  if (nk > 1) {
    stage_all(1);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  bar();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa0[i] = readA(0, 0, i);
    fb0[i] = readB(0, 0, i);
  }

  int t = 0;
  static_assert(!((SCHED & 4) && (SCHED & 2)), "early staging needs the front-loaded reads");
  if constexpr (SCHED & 4) {
    // early staging: buffer b is free once every wave has its F1 fragments (mid phase A), so tile
    // t+2 is issued there and has ~1.5 K-tiles to land; the boundary waits only for tile t+1
    // (vmcnt(16): tile t+2's 16 DMAs stay in flight)
    for (; t + 2 < nk; ++t) {
      const int buf = t & 1;
      phase(yes{}, no{}, I0{}, I0{}, I8{}, fa0, fb0, fa1, fb1, buf, 1, 0, 0);
      sync(I0{});   // F1 reads of buf retired everywhere (vmcnt(0): nothing newer than tile t+1 yet)
      phase(no{}, yes{}, I2{}, I8{}, I16{}, fa0, fb0, fa1, fb1, buf, 1, t + 2, 0);
      sync(I16{});  // tile t+1 landed
      phase(yes{}, no{}, I0{}, I0{}, I16{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, 0, 0);
    }
  } else {
    for (; t + 2 < nk; ++t) {   // steady state: reads of the next k-half every phase, tile t+2 staged
      const int buf = t & 1;
      phase(yes{}, no{}, I0{}, I0{}, I16{}, fa0, fb0, fa1, fb1, buf, 1, 0, 0);
      sync(I0{});
      phase(yes{}, yes{}, I1{}, I0{}, I16{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, t + 2, 0);
    }
  }
  if (t + 1 < nk) {   // second-to-last tile: nothing left to stage
    const int buf = t & 1;
    phase(yes{}, no{}, I0{}, I0{}, I16{}, fa0, fb0, fa1, fb1, buf, 1, 0, 0);
    sync(I0{});
    phase(yes{}, no{}, I0{}, I0{}, I16{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, 0, 0);
    ++t;
  }
  {   // last tile
    const int buf = t & 1;
    phase(yes{}, no{}, I0{}, I0{}, I16{}, fa0, fb0, fa1, fb1, buf, 1, 0, 0);
    lgkm0();
    phase(no{}, no{}, I0{}, I0{}, I16{}, fa1, fb1, fa0, fb0, 0, 0, 0, 0);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  bar();

  // ---- epilogue ---------------------------------------------------------------------------------
  // OT: the tile is C^T (kernel rows = output columns). Output rows [r0, r0 + 256) of the Mo x No
  // result, columns [c0, c0 + 256); the accumulators are staged through LDS in two 128-row halves
  // of the OUTPUT (kernel row halves wr, or with OT kernel column halves wc, written as 16-B
  // vectors since a fragment's 4 accumulator rows are 4 consecutive output columns)
  const int epi = p.epi;
  if (epi & EPI_SKIP) return;
  const int Mo = OT ? N : M, No = OT ? M : N, r0 = OT ? n0 : m0, c0 = OT ? m0 : n0, rt = OT ? tn : tm;
  T* C = static_cast<T*>(p.c);
  T* AUX = static_cast<T*>(p.aux);
  float* stg = reinterpret_cast<float*>(smem);
  const int c8 = tid & 31, rl = tid >> 5;   // this thread: columns c0 + c8*8 .. +7, rows rl + 8 r
  const int n = c0 + c8 * 8;
  const bool ncol = n < No;
  constexpr bool GEN = EK != EK_PLAIN;   // bias / activation / column sums (runtime flags)
  float bv[8], cs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    bv[e] = (GEN && (epi & EPI_BIAS) && ncol) ? p.bias[n + e] : 0.f;
    cs[e] = 0.f;
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (epi & EPI_NOSTAGE) {
    } else if constexpr (OT) {   // acc[i][j][e] = C^T[wc*128 + j*16 + fr][wr*128 + i*16 + 4fk + e]
      if (wc == h) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            *reinterpret_cast<f32x4*>(smem + (j * 16 + fr) * CROWF + (wr * 128 + i * 16 + 4 * fk) * 4) = acc[i][j];
      }
    } else {   // acc[i][j][e] = C[wr*128 + i*16 + fr][wc*128 + j*16 + 4fk + e] (operands swapped)
      if (wr == h) {
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            *reinterpret_cast<f32x4*>(smem + (i * 16 + fr) * CROWF + (wc * 128 + j * 16 + 4 * fk) * 4) = acc[i][j];
      }
    }
    __syncthreads();
    // rows in batches of RB: all RB results are computed into distinct registers before their
    // stores issue. A register that still holds an in-flight store's data can only be rewritten
    // after vmcnt(0), i.e. after that store COMPLETED, and a load among the rows (the dGELU aux
    // read) waits vmcnt(0) too: row-by-row code paid a full memory round trip per row. The dGELU
    // build loads a batch's aux rows before computing it; the others load nothing.
    constexpr bool DG = EK == EK_DGELU, AX = EK == EK_AUX;
    constexpr int RB = (DG || AX) ? 4 : 8;   // the aux builds hold twice the registers per row
    // the batch loop stays rolled: unrolled, the compiler hoists every row's addresses and bounds
    // tests (C and aux) ahead of the epilogue and spills them
#pragma unroll 1
    for (int rb = 0; rb < 16; rb += RB) {
      uint4 ov[RB], pv[AX ? RB : 1], auxv[DG ? RB : 1];
      if constexpr (DG) {
#pragma unroll
        for (int r8 = 0; r8 < RB; ++r8) {
          const long m = r0 + h * 128 + rl + 8 * (rb + r8);
          auxv[r8] = (m < Mo && ncol) ? *reinterpret_cast<const uint4*>(AUX + m * p.ldaux + n) : uint4{0, 0, 0, 0};
        }
      }
#pragma unroll
      for (int r8 = 0; r8 < RB; ++r8) {
        const int ml = rl + 8 * (rb + r8);
        const f32x4 lo = *reinterpret_cast<const f32x4*>(smem + ml * CROWF + c8 * 32);
        const f32x4 hi = *reinterpret_cast<const f32x4*>(smem + ml * CROWF + c8 * 32 + 16);
        const bool ok = r0 + h * 128 + ml < Mo && ncol;
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        uint16_t pre[8], out[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float x = v[e];
          if constexpr (GEN) {
            x += bv[e];
            if constexpr (AX) pre[e] = Mf<T>::cvt(x);
            if (epi & EPI_GELU) x = gelu_t(x);
            else if (epi & EPI_RELU) x = fmaxf(x, 0.f);
            if constexpr (DG) x *= gelu_t_grad(ld_elem<T>(auxv[r8], e));
            if (ok) cs[e] += x;
          }
          out[e] = Mf<T>::cvt(x);
        }
        ov[r8] = *reinterpret_cast<const uint4*>(out);
        if constexpr (AX) pv[r8] = *reinterpret_cast<const uint4*>(pre);
        // one row's GELU math at a time: interleaving the rows' transcendental chains is what
        // made the aux builds spill
        if constexpr (DG || AX) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int r8 = 0; r8 < RB; ++r8) {
        const long m = r0 + h * 128 + rl + 8 * (rb + r8);
        if (m >= Mo || !ncol || (epi & EPI_NOSTORE)) continue;
        if (epi & EPI_NTSTORE) {
          typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
          __builtin_nontemporal_store(__builtin_bit_cast(u32x4_t, ov[r8]), reinterpret_cast<u32x4_t*>(C + m * p.ldc + n));
        }
        else *reinterpret_cast<uint4*>(C + m * p.ldc + n) = ov[r8];
        if constexpr (AX) *reinterpret_cast<uint4*>(AUX + m * p.ldaux + n) = pv[r8];
      }
    }
    __syncthreads();
  }
  if (GEN && (epi & EPI_COLSUM)) {
    // reduce the 8 row-lanes (rl) of every column group through LDS, one fp32 row per tile
#pragma unroll
    for (int e = 0; e < 8; ++e) stg[rl * 264 + c8 * 8 + e] = cs[e];
    __syncthreads();
    const int col = tid;   // 256 columns of the tile
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 8; ++r) s += stg[r * 264 + col];
    if (c0 + col < No) p.colsum[(long)rt * No + c0 + col] = s;
  }
}

template <typename T, int SCHED, int EK>
int launch_ek(const Args& a, int ako, int bko, hipStream_t st) {
  const unsigned grid = (unsigned)(((a.M + 255) / 256) * ((a.N + 255) / 256));
  if (a.epi & EPI_TRANS) {   // only the layout whose main loop keeps every accumulator in AGPRs
    if (!(ako && !bko)) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm4w_kernel<T, true, false, SCHED, true, EK>), dim3(grid), dim3(256), 0, st, a);
    return (int)hipGetLastError();
  }
  if constexpr (EK == EK_PLAIN || EK == EK_GEN) {
    if (!ako && !bko) hipLaunchKernelGGL((gemm4w_kernel<T, false, false, SCHED, false, EK>), dim3(grid), dim3(256), 0, st, a);
    else if (!ako && bko) hipLaunchKernelGGL((gemm4w_kernel<T, false, true, SCHED, false, EK>), dim3(grid), dim3(256), 0, st, a);
    else if (ako && !bko) hipLaunchKernelGGL((gemm4w_kernel<T, true, false, SCHED, false, EK>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gemm4w_kernel<T, true, true, SCHED, false, EK>), dim3(grid), dim3(256), 0, st, a);
  } else {   // the dGELU / pre-activation builds: NT (fc2 dgrad) and the transposed store (fc1 fwd)
    if (ako || bko) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL((gemm4w_kernel<T, false, false, SCHED, false, EK>), dim3(grid), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

template <typename T, int SCHED>
int launch(const Args& a, int ako, int bko, hipStream_t st) {
  const bool dg = a.epi & EPI_DGELU, ax = a.epi & EPI_AUXOUT;
  if (dg && ax) return (int)hipErrorInvalidValue;
  if (dg) return launch_ek<T, SCHED, EK_DGELU>(a, ako, bko, st);
  if (ax) return launch_ek<T, SCHED, EK_AUX>(a, ako, bko, st);
  if (a.epi & (EPI_BIAS | EPI_GELU | EPI_RELU | EPI_COLSUM)) return launch_ek<T, SCHED, EK_GEN>(a, ako, bko, st);
  return launch_ek<T, SCHED, EK_PLAIN>(a, ako, bko, st);
}

// colsum partials [rows][N] fp32 -> out[N] (T), one thread per column
template <typename T>
__global__ __launch_bounds__(256) void colsum_finish_kernel(const float* __restrict__ part, T* __restrict__ out,
                                                            int rows, int N) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int r = 0; r < rows; ++r) s += part[(long)r * N + n];
  Cvt<T>::st(out, n, s);
}

}  // namespace g4w
}  // namespace pha

using namespace pha;

// C[M,N] = epi(A . B). a_kouter: A stored [K][lda] (else [M][lda]); b_kouter: B stored [K][ldb]
// (else B^T stored [N][ldb]). Requires K % 64 == 0; M, N, lda, ldb, ldc, ldaux % 8 == 0; K-outer
// operand dims >= 8; every byte offset inside one 256-row / 64-k operand panel < 2^32.
// epi: see g4w::EPI_*; bias fp32 [N]; aux [M][ldaux] (pre-activation in or out);
// colsum fp32 [ceil(M/256)][N] partials (finish with pha_colsum_finish).
// EPI_DGELU / EPI_AUXOUT (mutually exclusive): NT layout or EPI_TRANS only.
// EPI_TRANS (a_kouter = 1, b_kouter = 0 only): C (and aux) hold the TRANSPOSED product, [N][ldc];
// bias is indexed by C's column (the kernel's m), colsum is [ceil(N/256)][M]. The NN product
// x[M][K] . W[K][N] runs as this with A = W (K-outer) and B^T = x: the direct NN instantiation
// leaves accumulators cycling through VGPRs (serialised MFMAs), this one keeps them in AGPRs.
PHA_API int pha_gemm4w(int dt, const void* a, const void* b, void* c, long M, long N, long K, long lda, long ldb,
                       long ldc, int a_kouter, int b_kouter, int epi, const float* bias, void* aux, long ldaux,
                       float* colsum, int sched, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8)
    return (int)hipErrorInvalidValue;
  if ((a_kouter && M < 8) || (b_kouter && N < 8)) return (int)hipErrorInvalidValue;
  if (M > (1L << 30) || N > (1L << 30) || K > (1L << 30) || lda > (1L << 30) || ldb > (1L << 30))
    return (int)hipErrorInvalidValue;
  // per-lane 32-bit byte offsets inside one panel
  if ((a_kouter ? 64.0 * lda : 256.0 * lda) * 2 >= 4294967295.0 || (b_kouter ? 64.0 * ldb : 256.0 * ldb) * 2 >= 4294967295.0)
    return (int)hipErrorInvalidValue;
  if ((epi & (g4w::EPI_BIAS)) && !bias) return (int)hipErrorInvalidValue;
  if ((epi & (g4w::EPI_DGELU | g4w::EPI_AUXOUT)) && (!aux || ldaux % 8)) return (int)hipErrorInvalidValue;
  if ((epi & g4w::EPI_COLSUM) && !colsum) return (int)hipErrorInvalidValue;
  g4w::Args p{a, b, c, bias, aux, colsum, (int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)ldc, (int)ldaux, epi};
  if (dt == kBF16) {
    switch (sched) {
      case 2: return g4w::launch<bf16_t, 2>(p, a_kouter, b_kouter, stream);
      default: return g4w::launch<bf16_t, 0>(p, a_kouter, b_kouter, stream);
    }
  }
  if (dt == kF16) return g4w::launch<half_t, 0>(p, a_kouter, b_kouter, stream);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_colsum_finish(int dt, const float* part, void* out, int rows, int N, hipStream_t stream) {
  if (rows <= 0 || N <= 0) return (int)hipErrorInvalidValue;
  const unsigned grid = (unsigned)((N + 255) / 256);
  if (dt == kBF16) hipLaunchKernelGGL((g4w::colsum_finish_kernel<bf16_t>), dim3(grid), dim3(256), 0, stream, part,
                                      static_cast<bf16_t*>(out), rows, N);
  else if (dt == kF16) hipLaunchKernelGGL((g4w::colsum_finish_kernel<half_t>), dim3(grid), dim3(256), 0, stream, part,
                                          static_cast<half_t*>(out), rows, N);
  else if (dt == kF32) hipLaunchKernelGGL((g4w::colsum_finish_kernel<float>), dim3(grid), dim3(256), 0, stream, part,
                                          static_cast<float*>(out), rows, N);
  else return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}
