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
#include "mfma_tile.h"
#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace pha {
namespace g256 {


constexpr int NT = 512;


struct ConvGeo {
  int N, H, W, C;   // input NHWC
  int OH, OW;
  int KH, KW;
  int sh, sw, ph, pw, dh, dw;
  // output row remap (osh > 0): output pixel (n, oh, ow) is stored at row
  // (n * OHF + oh0 + oh * osh) * OWF + ow0 + ow * osw — one phase of a strided conv's dgrad
  int OHF, OWF, oh0, ow0, osh, osw;
  int ozero;   // also store zeros at the osh x osw - 1 other pixels of the output's stride cell
  // grouped convolution (blockIdx.y = group): the image's pixel stride in channels (0: C) and the
  // per-group element offsets of the image channels (ga), the filter / A rows (gb) and the output
  // columns (gc); C, the GEMM N and K are the ONE group's
  int cs = 0;
  long ga = 0, gb = 0, gc = 0;
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
  float* stats;       // optional [tiles_m][2][N]: per-tile column sum / sum of squares of the stored C
  // optional fused batch-norm backward reduction over the stored C (= dL/dy of a BN whose input
  // was bn_x, same layout as C): per-tile column sums of dy' and dy' * (bn_x - mean), with
  // dy' = dy masked by bn_x * scale + shift > 0 when bn_aff ([scale | shift]) is given
  const void* bn_x;
  const float* bn_mean;
  const float* bn_aff;
  float* bn_part;     // [bn_row0 + tiles_m][2][N]
  int bn_row0;
  // optional C += addend (same layout and ldc as C, after the bias / activation): a conv dgrad
  // that also receives the residual branch's gradient stores the sum, no separate add pass
  const void* addend = nullptr;
  // C is fp32 (ldc in floats): the accumulators are stored directly (bias / activation / output
  // remap applied; no stats, bn_part or addend) — the fp32 products split into three bf16 terms
  int out_f32 = 0;
};



// one 16-bit element (bf16 / fp16 bits) as float
template <typename T>
__device__ __forceinline__ float u16f(uint16_t u) {
  if constexpr (std::is_same<T, bf16_t>::value) return __uint_as_float((unsigned)u << 16);
  else return (float)__builtin_bit_cast(_Float16, u);
}

// workgroup barrier over LDS only: waits for this wave's LDS operations, not for its global stores
// (__syncthreads' release fence drains vmcnt — in the epilogues below that parked every wave on its
// C-tile stores before the statistics reduction could start)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// per-lane row state of the A gather for one of the wave's A instructions
struct ARow {
  const char* base;   // row base (plain) or image pixel base (conv: n, oh*sh-ph, ow*sw-pw folded)
  int ih0, iw0;       // conv: top-left input coordinate of the row's receptive field
  bool ok;
};

template <typename T, int BM, int BN, int BK, bool CONV, bool F32OUT = false>
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
  long goff_c = 0;   // grouped conv: this group's output column offset
  int CS = 0;        // conv: image pixel stride in channels
  if constexpr (CONV) {
    const int grp = blockIdx.y;
    A += grp * p.g.ga;
    Bt += grp * p.g.gb;
    goff_c = grp * p.g.gc;
    CS = p.g.cs ? p.g.cs : p.g.C;
  }

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
      ar[j].base = reinterpret_cast<const char*>(A + (long)n * g.H * g.W * CS);
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
  const int sch = BK == 64 ? (lch ^ (lrow & 7)) : (lch ^ ((0x78 >> (((lrow >> 2) & 3) << 1)) & 3));   // img_off<BK>

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
            src = ar[j].base + (((long)ih * g.W + iw) * CS + cin) * sizeof(T);
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

  // ---- fp32 output: straight from the accumulators (16 lanes store 64 contiguous bytes of a row)
  if constexpr (F32OUT) {
    float* Cf = static_cast<float*>(p.c) + goff_c;
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const long n = n0 + wn * 64 + j * 16 + fr;
      if (n >= N) continue;
      const float bv = p.bias ? p.bias[n] : 0.f;
#pragma unroll
      for (int i = 0; i < RB; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          long m = m0 + wm * WTM + i * 16 + 4 * fk + e;
          if (m >= M) continue;
          float v = acc[i][j][e] + bv;
          if (p.act == ACT_RELU) v = fmaxf(v, 0.f);
          else if (p.act == ACT_GELU) v = gelu_tanh(v);
          if constexpr (CONV) {
            const ConvGeo& g = p.g;
            if (g.osh > 0) {
              const int hw = g.OH * g.OW;
              const int b = (int)(m / hw), rem = (int)(m - (long)b * hw);
              const int oh = rem / g.OW, ow = rem - oh * g.OW;
              const int fh = g.oh0 + oh * g.osh, fw = g.ow0 + ow * g.osw;
              m = ((long)b * g.OHF + fh) * g.OWF + fw;
              if (g.ozero)
                for (int a = 0; a < g.osh; ++a)
                  for (int c = 0; c < g.osw; ++c)
                    if ((a | c) && fh + a < g.OHF && fw + c < g.OWF) Cf[(m + (long)a * g.OWF + c) * p.ldc + n] = 0.f;
            }
          }
          Cf[m * p.ldc + n] = v;
        }
    }
    return;
  }

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
  T* C = static_cast<T*>(p.c) + goff_c;
  constexpr int CH = BN / 8;                          // 16-B chunks per C row
  const bool full_n = n0 + BN <= N && (p.ldc % 8) == 0;
  for (int idx = tid; idx < BM * CH; idx += NT) {
    const int ml = idx / CH, c8 = idx % CH;
    long m = m0 + ml;
    const long n = n0 + c8 * 8;
    if (m >= M) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + ml * CROW + c8 * 16);
    if constexpr (CONV) {
      const ConvGeo& g = p.g;
      if (g.osh > 0) {
        const int hw = g.OH * g.OW;
        const int b = (int)(m / hw), rem = (int)(m - (long)b * hw);
        const int oh = rem / g.OW, ow = rem - oh * g.OW;
        const int fh = g.oh0 + oh * g.osh, fw = g.ow0 + ow * g.osw;
        m = ((long)b * g.OHF + fh) * g.OWF + fw;
        if (g.ozero && full_n) {   // taps reach only phase (0, 0): the rest of the cell is zero
          for (int a = 0; a < g.osh; ++a)
            for (int c = 0; c < g.osw; ++c)
              if ((a | c) && fh + a < g.OHF && fw + c < g.OWF)
                *reinterpret_cast<uint4*>(C + (m + (long)a * g.OWF + c) * p.ldc + n) = uint4{0, 0, 0, 0};
        }
      }
    }
    if (full_n) {
      uint4 o = v;
      if (p.addend) {
        const uint4 r = *reinterpret_cast<const uint4*>(static_cast<const T*>(p.addend) + m * p.ldc + n);
        const uint16_t* ev = reinterpret_cast<const uint16_t*>(&v);
        const uint16_t* er = reinterpret_cast<const uint16_t*>(&r);
        uint16_t* eo = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
        for (int t = 0; t < 8; ++t) eo[t] = Mf<T>::cvt(u16f<T>(ev[t]) + u16f<T>(er[t]));
      }
      *reinterpret_cast<uint4*>(C + m * p.ldc + n) = o;
    } else {
      const uint16_t* e = reinterpret_cast<const uint16_t*>(&v);
      const uint16_t* ad = static_cast<const uint16_t*>(p.addend);
      for (int t = 0; t < 8 && n + t < N; ++t)
        reinterpret_cast<uint16_t*>(C)[m * p.ldc + n + t] =
            ad ? Mf<T>::cvt(u16f<T>(e[t]) + u16f<T>(ad[m * p.ldc + n + t])) : e[t];
    }
  }
  if (p.bn_part) {
    // batch-norm backward sums over this tile (this product is the BN's output gradient dy; the
    // BN then skips its own reduction pass): thread = 8-column chunk x row group, 16-B loads of
    // bn_x and of the staged C rows, so a tile costs a few vector loads per thread, not a
    // dependent scalar loop
    constexpr int CW = BN / 8, G2 = NT / CW;
    const int c8 = tid % CW, rg2 = tid / CW;
    const int rows = (int)min((long)BM, M - m0);
    const long n = n0 + c8 * 8;
    float a1[8], a2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a1[k] = a2[k] = 0.f;
    if (n < N) {
      const T* bx = static_cast<const T*>(p.bn_x);
      float mu[8], sc[8], sh[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mu[k] = p.bn_mean[n + k];
        sc[k] = p.bn_aff ? p.bn_aff[n + k] : 0.f;
        sh[k] = p.bn_aff ? p.bn_aff[N + n + k] : 0.f;
      }
      for (int r = rg2; r < rows; r += G2) {
        long m = m0 + r;
        if constexpr (CONV) {
          const ConvGeo& g = p.g;
          if (g.osh > 0) {
            const int hw = g.OH * g.OW;
            const int b = (int)(m / hw), rem = (int)(m - (long)b * hw);
            const int oh = rem / g.OW, ow = rem - oh * g.OW;
            m = ((long)b * g.OHF + g.oh0 + oh * g.osh) * g.OWF + g.ow0 + ow * g.osw;
          }
        }
        float xv[8], d[8];
        Vec8<T>::ld(bx + m * p.ldc + n, xv);
        Vec8<T>::ld(reinterpret_cast<const T*>(ct + r * CROW + c8 * 16), d);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dd = (p.bn_aff && !(fmaf(xv[k], sc[k], sh[k]) > 0.f)) ? 0.f : d[k];
          a1[k] += dd;
          a2[k] = fmaf(dd, xv[k] - mu[k], a2[k]);
        }
      }
    }
    lds_barrier();                                      // C tile read out of the LDS: reuse it (32 KiB)
    float* red = reinterpret_cast<float*>(smem);        // [G2][2][BN]
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[(rg2 * 2) * BN + c8 * 8 + k] = a1[k];
      red[(rg2 * 2 + 1) * BN + c8 * 8 + k] = a2[k];
    }
    lds_barrier();
    if (tid < BN && n0 + tid < N) {
      float s1 = 0.f, s2 = 0.f;
      for (int g2 = 0; g2 < G2; ++g2) {
        s1 += red[(g2 * 2) * BN + tid];
        s2 += red[(g2 * 2 + 1) * BN + tid];
      }
      float* out = p.bn_part + (long)(p.bn_row0 + tm) * 2 * N;
      out[n0 + tid] = s1;
      out[N + n0 + tid] = s2;
    }
  } else if (p.stats) {
    // batch-norm statistics of this tile (the BN that follows a convolution then skips its own
    // read of the output): column sums over the tile's rows of the values as stored (rounded to T).
    // Thread = 8-column chunk x row group with 16-B LDS reads (a 2-byte read per column per row
    // made this loop as long as a K = 64 tile's whole main loop: the 1x1 expansion convolutions
    // ran at 2.1-2.6 TB/s against 3.9 for the same shapes' dgrad, profiles/resnet_wgrad_s2d_r5/)
    constexpr int CW = BN / 8, G2 = NT / CW;
    const int c8 = tid % CW, rg2 = tid / CW;
    const int rows = (int)min((long)BM, M - m0);
    float a1[8], a2[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a1[k] = a2[k] = 0.f;
#pragma unroll 2
    for (int r = rg2; r < rows; r += G2) {
      float d[8];
      Vec8<T>::ld(reinterpret_cast<const T*>(ct + r * CROW + c8 * 16), d);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a1[k] += d[k];
        a2[k] = fmaf(d[k], d[k], a2[k]);
      }
    }
    lds_barrier();                                      // C tile read out of the LDS: reuse it
    float* red = reinterpret_cast<float*>(smem);        // [G2][2][BN] (16 KiB)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[(rg2 * 2) * BN + c8 * 8 + k] = a1[k];
      red[(rg2 * 2 + 1) * BN + c8 * 8 + k] = a2[k];
    }
    lds_barrier();
    if (tid < BN && n0 + tid < N) {
      float s1 = 0.f, s2 = 0.f;
      for (int g2 = 0; g2 < G2; ++g2) {
        s1 += red[(g2 * 2) * BN + tid];
        s2 += red[(g2 * 2 + 1) * BN + tid];
      }
      p.stats[(long)tm * 2 * N + n0 + tid] = s1;
      p.stats[(long)tm * 2 * N + N + n0 + tid] = s2;
    }
  }
}

// BK = 64 (one tile in flight, half the barriers) suits compute-bound GEMMs; BK = 32 (three tiles
// in flight) the short-K, bandwidth-heavy convolutions. PHA_G256_BK overrides.
// tile: index into cands (-1 = heuristic), bk: 32 | 64 (0 = heuristic); the host autotuner
// (ops/conv_gemm.py) times the candidates once per shape and passes its choice
template <typename T, bool CONV>
int launch(const Args& a, hipStream_t st, int tile = -1, int bk = 0, int* stats_rows = nullptr, int groups_ = 1) {
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
  if (stats_rows) *stats_rows = (int)((a.M + bm - 1) / bm);   // row tiles with stats / bn_part rows
  const unsigned groups = (unsigned)std::max(1, groups_);
  if (a.out_f32) {
    // fp32 products (three-term bf16 split, bf16 operands only): the split triples K, so the
    // products are long-K — the large tiles with BK = 64 when the heuristic picks them, else
    // 128 x 128 x 32
    if constexpr (std::is_same<T, bf16_t>::value) {
      auto gof = [&](auto bm_c, auto bn_c, auto bk_c) {
        constexpr int BMc = decltype(bm_c)::value, BNc = decltype(bn_c)::value, BKc = decltype(bk_c)::value;
        const long tiles = ((a.M + BMc - 1) / BMc) * ((a.N + BNc - 1) / BNc);
        hipLaunchKernelGGL((gemm256_kernel<T, BMc, BNc, BKc, CONV, true>), dim3((unsigned)tiles, groups), dim3(NT),
                           0, st, a);
      };
      using I256 = std::integral_constant<int, 256>;
      using I128 = std::integral_constant<int, 128>;
      using I64 = std::integral_constant<int, 64>;
      using I32 = std::integral_constant<int, 32>;
      // (the 256 x 256 conv variant spills: its gather state and the fp32 epilogue exceed the budget)
      bool done = false;
      if constexpr (!CONV) {
        if (a.K >= 512 && bm == 256 && bn == 256) {
          gof(I256{}, I256{}, I64{});
          done = true;
        }
      }
      if (done) {
      } else if (a.K >= 512 && bm == 256 && bn >= 128) gof(I256{}, I128{}, I64{});
      else if (a.K >= 512 && bn == 256) gof(I128{}, I256{}, I64{});
      else if (a.K >= 512 && bm >= 128 && bn >= 128) gof(I128{}, I128{}, I64{});
      else gof(I128{}, I128{}, I32{});
      return (int)hipGetLastError();
    } else {
      return (int)hipErrorInvalidValue;
    }
  }
  auto go = [&](auto bm_c, auto bn_c) {
    constexpr int BMc = decltype(bm_c)::value, BNc = decltype(bn_c)::value;
    const long tiles = ((a.M + BMc - 1) / BMc) * ((a.N + BNc - 1) / BNc);
    if (bk == 32) hipLaunchKernelGGL((gemm256_kernel<T, BMc, BNc, 32, CONV>), dim3((unsigned)tiles, groups), dim3(NT), 0, st, a);
    else hipLaunchKernelGGL((gemm256_kernel<T, BMc, BNc, 64, CONV>), dim3((unsigned)tiles, groups), dim3(NT), 0, st, a);
  };
#define G256_CASE(M_, N_) if (bm == M_ && bn == N_) { go(std::integral_constant<int, M_>(), std::integral_constant<int, N_>()); return (int)hipGetLastError(); }
  G256_CASE(256, 256) G256_CASE(256, 128) G256_CASE(256, 64) G256_CASE(128, 256) G256_CASE(128, 128) G256_CASE(128, 64)
#undef G256_CASE
  return (int)hipErrorInvalidValue;
}


// ================================================================================================
// TN: C[M, N] = sum_k A[k, m] * B[k, n] — both operands K-OUTER (M / N contiguous): the weight
// gradient of a linear layer (dW = X^T dY over tokens) and of a convolution (dW = dY^T im2col(X)
// over output pixels, B_CONV gathers the im2col rows). K is long and M x N small, so the K range
// is split over blockIdx (split s writes fp32 partials ws[s][M][N]; tn_finalize sums the splits,
// converts and, for convolutions, permutes [Cout][tap][Cin] to the [Cout][Cin][KH][KW] filter).
//
// The LDS images are [BK k-rows][BM | BN] exactly as the operands lie in HBM (glds, lane-linear),
// and the MFMA fragments are read TRANSPOSED with ds_read_b64_tr_b16 (CDNA guide T10): per 16-lane
// group a 4 k-row x 16 column block arrives column-major, i.e. as 4 consecutive k of one m / n —
// two reads give the 8-k operand of v_mfma_f32_16x16x32. Chunk swizzle: the 8 k-rows a 32-lane
// half reads (rows r0+{0..3} and r0+8+{0..3}) land on 8 distinct 32-B bank groups.
// ================================================================================================

struct TnArgs {
  const void* a;   // [K][lda] (M contiguous)
  const void* b;   // [K][ldb] (N contiguous) — or the NHWC input x (B_CONV)
  float* ws;       // [S][M][N] fp32 partials
  long M, N, K;
  long lda, ldb;
  long kchunk;     // rows of K per split (multiple of BK)
  int splits;
  const void* zero;
  ConvGeo g;       // B_CONV: K = N*OH*OW output pixels, N = KH*KW*C
};

template <typename T, int BM, int BN, bool BCONV>
__global__ __launch_bounds__(NT) void gemm256_tn_kernel(TnArgs p) {
  constexpr int BK = 32, NSTAGE = 4;
  constexpr int WN = BN / 64, WM = 8 / WN, WTM = BM / WM;
  static_assert(WTM % 16 == 0, "wave tile rows");
  constexpr int RB = WTM / 16, CB = 4;
  constexpr int RA = BM * 2, RBB = BN * 2;                  // image row bytes
  constexpr int A_BYTES = BK * RA, B_BYTES = BK * RBB, STAGE = A_BYTES + B_BYTES;
  constexpr int A_WI = A_BYTES / 1024, B_WI = B_BYTES / 1024;
  constexpr int A_INS = (A_WI + 7) / 8, B_INS = (B_WI + 7) / 8, INS = A_INS + B_INS;
  constexpr int ACPR = RA / 16, ARPI = 1024 / RA;           // chunks per row / rows per wave-instr
  constexpr int BCPR = RBB / 16, BRPI = 1024 / RBB;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NSTAGE * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const long M = p.M, N = p.N;

  // XCD-bijective order over (split, tile): an XCD walks consecutive tiles of one K split, so
  // they share the split's A / B rows in its L2
  const int tiles_m = (int)((M + BM - 1) / BM), tiles_n = (int)((N + BN - 1) / BN);
  const int ntiles = tiles_m * tiles_n, total = ntiles * p.splits;
  const int bid = blockIdx.x;
  const int q8 = total / 8, r8 = total % 8, xcd = bid % 8;
  const int lin = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int split = lin / ntiles, tile = lin % ntiles;
  const int tm = tile % tiles_m, tn = tile / tiles_m;
  const long m0 = (long)tm * BM, n0 = (long)tn * BN;
  const long kbeg = (long)split * p.kchunk;
  const long kend = min(p.K, kbeg + p.kchunk);

  const T* A = static_cast<const T*>(p.a);
  const T* B = static_cast<const T*>(p.b);
  const char* zero = static_cast<const char*>(p.zero);
  int CS = 0;   // B_CONV: image pixel stride in channels
  float* wsg = p.ws;
  if constexpr (BCONV) {   // grouped conv weight gradient: blockIdx.y = group
    const int grp = blockIdx.y;
    A += grp * p.g.gc;                       // the group's dY columns
    B += grp * p.g.ga;                       // the group's input channels
    wsg += (long)grp * p.splits * M * N;     // the group's partial slabs
    CS = p.g.cs ? p.g.cs : p.g.C;
  }

  // per-lane source columns (constant over the K loop) and image rows of each glds instruction
  int arow[A_INS];
  const char* acol[A_INS];
#pragma unroll
  for (int j = 0; j < A_INS; ++j) {
    const int row = ((j * 8 + wid) % A_WI) * ARPI + lane / ACPR;
    const int sch = (lane % ACPR) ^ tn_mask(row, RA);
    const long m = m0 + sch * 8;
    arow[j] = row;
    acol[j] = m < M ? reinterpret_cast<const char*>(A + m) : nullptr;
  }
  int brow[B_INS];
  const char* bcol[B_INS];
  int bkh[B_INS], bkw[B_INS];   // conv: tap offsets kh*dh - ph, kw*dw - pw of the lane's column
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = ((j * 8 + wid) % B_WI) * BRPI + lane / BCPR;
    const int sch = (lane % BCPR) ^ tn_mask(row, RBB);
    const long n = n0 + sch * 8;
    brow[j] = row;
    bkh[j] = bkw[j] = 0;
    if constexpr (BCONV) {
      const ConvGeo& g = p.g;
      const int tap = (int)(n / g.C), cin = (int)(n - (long)tap * g.C);
      const int kh = tap / g.KW, kw = tap - kh * g.KW;
      bkh[j] = kh * g.dh - g.ph;
      bkw[j] = kw * g.dw - g.pw;
      bcol[j] = n < N ? reinterpret_cast<const char*>(B + cin) : nullptr;
    } else {
      bcol[j] = n < N ? reinterpret_cast<const char*>(B + n) : nullptr;
    }
  }

  auto issue = [&](int stage, long k0) {
    unsigned char* sa = smem + stage * STAGE;
    unsigned char* sb = sa + A_BYTES;
#pragma unroll
    for (int j = 0; j < A_INS; ++j) {
      const long k = k0 + arow[j];
      const char* src = (acol[j] && k < kend) ? acol[j] + k * p.lda * (long)sizeof(T) : zero;
      glds16(src, sa + ((j * 8 + wid) % A_WI) * 1024);
    }
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const long k = k0 + brow[j];
      const char* src = zero;
      if (bcol[j] && k < kend) {
        if constexpr (BCONV) {
          const ConvGeo& g = p.g;
          const int hw = g.OH * g.OW, ki = (int)k;   // pixel count < 2^31: 32-bit division
          const int b = ki / hw, rem = ki - b * hw;
          const int oh = rem / g.OW, ow = rem - oh * g.OW;
          const int ih = oh * g.sh + bkh[j], iw = ow * g.sw + bkw[j];
          if ((unsigned)ih < (unsigned)g.H && (unsigned)iw < (unsigned)g.W)
            src = bcol[j] + (((long)b * g.H + ih) * g.W + iw) * CS * (long)sizeof(T);
        } else {
          src = bcol[j] + k * p.ldb * (long)sizeof(T);
        }
      }
      glds16(src, sb + ((j * 8 + wid) % B_WI) * 1024);
    }
  };

  f32x4 acc[RB][CB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;
#pragma unroll
  for (int t = 0; t < NSTAGE - 1; ++t)
    if (t < nk) issue(t, kbeg + (long)t * BK);
  const int fk = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NSTAGE;
    const int later = min(NSTAGE - 2, nk - 1 - kt);
    if (later >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * INS) : "memory");
    else if (later == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(INS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kt + NSTAGE - 1 < nk) issue((kt + NSTAGE - 1) % NSTAGE, kbeg + (long)(kt + NSTAGE - 1) * BK);
    const unsigned char* sa = smem + cur * STAGE;
    const unsigned char* sb = sa + A_BYTES;
    const int r0 = 8 * fk;
    uint4 bf[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) bf[j] = tn_frag<RBB>(sb, r0, wn * 64 + j * 16, q, pp);
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const uint4 af = tn_frag<RA>(sa, r0, wm * WTM + i * 16, q, pp);
#pragma unroll
      for (int j = 0; j < CB; ++j) acc[i][j] = Mf<T>::mma(af, bf[j], acc[i][j]);
    }
  }

  // fp32 partials straight from the accumulators: register e of block (i, j) is
  // C[4 * (lane >> 4) + e][lane & 15]; 16 lanes store 64 contiguous bytes of a row
  float* ws = wsg + (long)split * M * N;
  const int fr = lane & 15;
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const long n = n0 + wn * 64 + j * 16 + fr;
    if (n >= N) continue;
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const long m = m0 + wm * WTM + i * 16 + 4 * fk + e;
        if (m < M) ws[m * N + n] = acc[i][j][e];
      }
  }
}

// first level of the split-K sum: ws2[g][i] = sum of splits [16g, 16g + 16) of ws, 4 floats per thread
// (grid.y = split groups: the sum reads S x M x N floats across the whole chip, not 16 CUs)
__global__ __launch_bounds__(256) void tn_reduce16_kernel(const float* __restrict__ ws, float* __restrict__ ws2, long MN,
                                                         int S) {
  const long i4 = (blockIdx.x * 256L + threadIdx.x) * 4;
  if (i4 >= MN) return;
  const int s0 = blockIdx.y * 16, s1 = min(S, s0 + 16);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int s = s0; s < s1; ++s) acc += *reinterpret_cast<const f32x4*>(ws + s * MN + i4);
  *reinterpret_cast<f32x4*>(ws2 + blockIdx.y * MN + i4) = acc;
}

// out = sum_s ws[s] (+ out if accumulate), converted to T (or fp32 when OUTF32); conv_c > 0
// permutes column n = tap * conv_c + cin of row m to out[m][cin][tap] (taps = N / conv_c)
template <typename T, bool OUTF32>
__global__ __launch_bounds__(256) void tn_finalize_kernel(const float* __restrict__ ws, void* out, long M, long N,
                                                           int S, int conv_c, int accumulate) {
  const long total = M * N;
  // grouped conv weight gradients: blockIdx.y = group, slabs [group][S][M][N] -> out rows of the group
  ws += (long)blockIdx.y * S * total;
  out = static_cast<char*>(out) + (long)blockIdx.y * total * (OUTF32 ? sizeof(float) : sizeof(T));
  for (long idx = blockIdx.x * 256L + threadIdx.x; idx < total; idx += (long)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < S; ++s) v += ws[s * total + idx];
    long o = idx;
    if (conv_c > 0) {
      const long m = idx / N, n = idx - m * N;
      const int taps = (int)(N / conv_c);
      const int tap = (int)(n / conv_c), cin = (int)(n - (long)tap * conv_c);
      o = m * N + (long)cin * taps + tap;
    }
    if constexpr (OUTF32) {
      float* y = static_cast<float*>(out);
      y[o] = accumulate ? y[o] + v : v;
    } else {
      T* y = static_cast<T*>(out);
      if (accumulate) v += Cvt<T>::ld(y, o);
      Cvt<T>::st(y, o, v);
    }
  }
}

// tile: 0 (256x256) 1 (256x128) 2 (128x256) 3 (128x128) 4 (64x256) 5 (256x64) 6 (128x64) 7 (64x128)
template <typename T, bool BCONV>
int launch_tn(TnArgs a, void* out, int out_f32, int conv_c, int accumulate, int tile, int splits, hipStream_t st,
              int groups_ = 1) {
  const unsigned groups = (unsigned)std::max(1, groups_);
  static const int cands[8][2] = {{256, 256}, {256, 128}, {128, 256}, {128, 128},
                                  {64, 256}, {256, 64}, {128, 64}, {64, 128}};
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  if (tile < 0 || tile > 7) {   // the fewest MFMA-padded tiles, then the largest tile
    tile = 0;
    double best = 1e300;
    for (int c = 0; c < 8; ++c) {
      const int bm = cands[c][0], bn = cands[c][1];
      const double pad = (double)((a.M + bm - 1) / bm * bm) * ((a.N + bn - 1) / bn * bn);
      const double cost = pad * (1.0 + 0.15 * (bm < 256) + 0.15 * (bn < 256));
      if (cost < best * 0.999) { best = cost; tile = c; }
    }
  }
  const int bm = cands[tile][0], bn = cands[tile][1];
  const long tiles = ((a.M + bm - 1) / bm) * ((a.N + bn - 1) / bn);
  const long kblocks = (a.K + 31) / 32;
  if (splits <= 0) splits = (int)std::max(1L, std::min(kblocks / 8, (2L * cus + tiles - 1) / tiles));
  splits = (int)std::max(1L, std::min((long)splits, kblocks));
  a.kchunk = ((kblocks + splits - 1) / splits) * 32;
  a.splits = (int)((a.K + a.kchunk - 1) / a.kchunk);
  const unsigned grid = (unsigned)(tiles * a.splits);
#define TN_CASE(M_, N_) \
  if (bm == M_ && bn == N_) hipLaunchKernelGGL((gemm256_tn_kernel<T, M_, N_, BCONV>), dim3(grid, groups), dim3(NT), 0, st, a);
  TN_CASE(256, 256) TN_CASE(256, 128) TN_CASE(128, 256) TN_CASE(128, 128)
  TN_CASE(64, 256) TN_CASE(256, 64) TN_CASE(128, 64) TN_CASE(64, 128)
#undef TN_CASE
  const long total = a.M * a.N;
  const float* part = a.ws;
  int S = a.splits;
  if (S > 32 && groups > 1) return (int)hipErrorInvalidValue;   // (grouped: the caller caps the splits)
  if (S > 32) {   // ws holds (S + ceil(S / 16)) x M x N floats
    float* ws2 = a.ws + (long)S * total;
    const int G = (S + 15) / 16;
    hipLaunchKernelGGL(tn_reduce16_kernel, dim3((unsigned)((total / 4 + 255) / 256), G), dim3(256), 0, st, a.ws, ws2,
                       total, S);
    part = ws2;
    S = G;
  }
  const unsigned fg = (unsigned)std::min((total + 255) / 256, 8192L);
  if (out_f32) hipLaunchKernelGGL((tn_finalize_kernel<T, true>), dim3(fg, groups), dim3(256), 0, st, part, out, a.M, a.N,
                                  S, conv_c, accumulate);
  else hipLaunchKernelGGL((tn_finalize_kernel<T, false>), dim3(fg, groups), dim3(256), 0, st, part, out, a.M, a.N,
                          S, conv_c, accumulate);
  return (int)hipGetLastError();
}


}  // namespace g256
}  // namespace pha

using namespace pha;

// C[M,N] = A[M,K] . Bt[N,K]^T (+bias)(act); A, Bt K-contiguous, K % 8 == 0, 16-B aligned rows.
PHA_API int pha_gemm256_nt(int dt, const void* a, const void* bt, void* c, const float* bias, long M, long N, long K,
                           long lda, long ldb, long ldc, int act, const void* zero16, int tile, int bk,
                           hipStream_t stream) {
  if (K % 8 || lda % 8 || ldb % 8 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  g256::Args p{a, bt, c, bias, M, N, K, lda, ldb, ldc, act, zero16, {}, nullptr, nullptr, nullptr, nullptr, nullptr, 0};
  if (dt == kBF16) return g256::launch<bf16_t, false>(p, stream, tile, bk);
  if (dt == kF16) return g256::launch<half_t, false>(p, stream, tile, bk);
  return (int)hipErrorInvalidValue;
}

// NHWC conv forward: y[N*OH*OW, Cout] = im2col(x) . w^T, w as [Cout][KH][KW][Cin], Cin % 8 == 0.
// oremap (host int[9], may be null): strided output rows and explicit output size, see ConvGeo.
// stats (may be null, >= ceil(M/128)*2*Cout floats): per-row-tile channel sum / sum of squares of y
// for a following batch norm; *stats_rows receives the number of row tiles written.
// bn_part (may be null): y is the output gradient of a batch norm with input bn_x / batch mean
// bn_mean (/ ReLU affine bn_aff): rows [bn_row0, bn_row0 + *stats_rows) of bn_part receive the
// per-tile sums of the BN backward (the BN then skips its own reduction pass).
PHA_API int pha_conv256_fwd(int dt, const void* x, const void* w, void* y, const float* bias, int N, int H, int W,
                            int C, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw, int act,
                            const void* zero16, int tile, int bk, const int* oremap, float* stats, int* stats_rows,
                            const void* bn_x, const float* bn_mean, const float* bn_aff, float* bn_part, int bn_row0,
                            const void* addend, hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  if (addend && (stats || bn_part || (oremap && oremap[8]))) return (int)hipErrorInvalidValue;
  g256::ConvGeo g{N, H, W, C, (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, (W + 2 * pw - dw * (KW - 1) - 1) / sw + 1,
                  KH, KW, sh, sw, ph, pw, dh, dw, 0, 0, 0, 0, 0, 0, 0};
  if (oremap) {   // {OHF, OWF, oh0, ow0, osh, osw, OH, OW, ozero}: phase output size given explicitly
    g.OHF = oremap[0]; g.OWF = oremap[1]; g.oh0 = oremap[2]; g.ow0 = oremap[3]; g.osh = oremap[4]; g.osw = oremap[5];
    g.OH = oremap[6]; g.OW = oremap[7]; g.ozero = oremap[8];
  }
  const long M = (long)N * g.OH * g.OW, K = (long)KH * KW * C;
  if (stats && (oremap || bn_part)) return (int)hipErrorInvalidValue;
  if (bn_part && (!bn_x || !bn_mean || Cout % 8)) return (int)hipErrorInvalidValue;
  g256::Args p{x, w, y, bias, M, (long)Cout, K, 0, K, (long)Cout, act, zero16, g, stats,
               bn_x, bn_mean, bn_aff, bn_part, bn_row0, addend};
  if (dt == kBF16) return g256::launch<bf16_t, true>(p, stream, tile, bk, stats_rows);
  if (dt == kF16) return g256::launch<half_t, true>(p, stream, tile, bk, stats_rows);
  return (int)hipErrorInvalidValue;
}

// grouped NHWC convolution on the implicit-GEMM kernel: x [N, H, W, groups*cig], w [groups*cog][KH][KW][cig],
// y [N*OH*OW][ldy] (group g writes columns g*cog.. of y + its own offset); cig % 8 == 0. One launch,
// blockIdx.y = group. out_f32: fp32 y (bias / act / remap as pha_conv256_fwd_f32out). oremap as
// pha_conv256_fwd (dgrad phases).
PHA_API int pha_conv256_fwd_grouped(int dt, const void* x, const void* w, void* y, const float* bias, int N, int H,
                                    int W, int cig, int cog, int groups, int KH, int KW, int sh, int sw, int ph,
                                    int pw, int dh, int dw, int act, long ldy, int out_f32, const void* zero16,
                                    int tile, int bk, const int* oremap, hipStream_t stream) {
  if (cig % 8 || groups < 1) return (int)hipErrorInvalidValue;
  g256::ConvGeo g{N, H, W, cig, (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, (W + 2 * pw - dw * (KW - 1) - 1) / sw + 1,
                  KH, KW, sh, sw, ph, pw, dh, dw, 0, 0, 0, 0, 0, 0, 0};
  if (oremap) {
    g.OHF = oremap[0]; g.OWF = oremap[1]; g.oh0 = oremap[2]; g.ow0 = oremap[3]; g.osh = oremap[4]; g.osw = oremap[5];
    g.OH = oremap[6]; g.OW = oremap[7]; g.ozero = oremap[8];
  }
  const long K = (long)KH * KW * cig;
  g.cs = cig * groups;
  g.ga = cig;
  g.gb = (long)cog * K;
  g.gc = cog;
  const long M = (long)N * g.OH * g.OW;
  g256::Args p{x, w, y, bias, M, (long)cog, K, 0, K, ldy, act, zero16, g, nullptr,
               nullptr, nullptr, nullptr, nullptr, 0, nullptr, out_f32 ? 1 : 0};
  if (dt == kBF16) return g256::launch<bf16_t, true>(p, stream, tile, bk, nullptr, groups);
  if (dt == kF16) return g256::launch<half_t, true>(p, stream, tile, bk, nullptr, groups);
  return (int)hipErrorInvalidValue;
}

// grouped conv weight gradient: dw [groups*cog][cig][KH][KW] from dy [N*OH*OW][groups*cog] and x
// [N, H, W, groups*cig]; ws >= groups * splits * cog * KH*KW*cig floats, splits <= 32
PHA_API int pha_conv256_wgrad_grouped(int dt, const void* dy, const void* x, void* dw, float* ws, int N, int H, int W,
                                      int cig, int cog, int groups, int KH, int KW, int sh, int sw, int ph, int pw,
                                      int dh, int dw_, int out_f32, const void* zero16, int tile, int splits,
                                      hipStream_t stream) {
  if (cig % 8 || cog % 8 || groups < 1 || splits > 32) return (int)hipErrorInvalidValue;
  g256::ConvGeo g{N, H, W, cig, (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, (W + 2 * pw - dw_ * (KW - 1) - 1) / sw + 1,
                  KH, KW, sh, sw, ph, pw, dh, dw_, 0, 0, 0, 0, 0, 0, 0};
  g.cs = cig * groups;
  g.ga = cig;
  g.gc = cog;
  const long K = (long)N * g.OH * g.OW;
  g256::TnArgs p{dy, x, ws, (long)cog, (long)KH * KW * cig, K, (long)cog * groups, (long)cig, 0, 1, zero16, g};
  if (dt == kBF16) return g256::launch_tn<bf16_t, true>(p, dw, out_f32, cig, 0, tile, splits, stream, groups);
  if (dt == kF16) return g256::launch_tn<half_t, true>(p, dw, out_f32, cig, 0, tile, splits, stream, groups);
  return (int)hipErrorInvalidValue;
}

// pha_conv256_fwd with an fp32 y (ldc = Cout floats): bias / act / output remap only (the fp32
// convolution as one bf16 implicit GEMM over the [hi, hi, lo] x [hi, lo, hi] channel split)
PHA_API int pha_conv256_fwd_f32out(int dt, const void* x, const void* w, float* y, const float* bias, int N, int H,
                                   int W, int C, int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh,
                                   int dw, int act, const void* zero16, int tile, int bk, const int* oremap,
                                   hipStream_t stream) {
  if (C % 8) return (int)hipErrorInvalidValue;
  g256::ConvGeo g{N, H, W, C, (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, (W + 2 * pw - dw * (KW - 1) - 1) / sw + 1,
                  KH, KW, sh, sw, ph, pw, dh, dw, 0, 0, 0, 0, 0, 0, 0};
  if (oremap) {
    g.OHF = oremap[0]; g.OWF = oremap[1]; g.oh0 = oremap[2]; g.ow0 = oremap[3]; g.osh = oremap[4]; g.osw = oremap[5];
    g.OH = oremap[6]; g.OW = oremap[7]; g.ozero = oremap[8];
  }
  const long M = (long)N * g.OH * g.OW, K = (long)KH * KW * C;
  g256::Args p{x, w, y, bias, M, (long)Cout, K, 0, K, (long)Cout, act, zero16, g, nullptr,
               nullptr, nullptr, nullptr, nullptr, 0, nullptr, 1};
  if (dt == kBF16) return g256::launch<bf16_t, true>(p, stream, tile, bk);
  if (dt == kF16) return g256::launch<half_t, true>(p, stream, tile, bk);
  return (int)hipErrorInvalidValue;
}

// C[M,N] = sum_k A[k][m] B[k][n] (K-outer operands, M/N contiguous, lda/ldb % 8 == 0), split-K over
// `splits` fp32 partials in ws (>= (splits + (splits > 32 ? ceil(splits/16) : 0))*M*N floats), summed into out (T, or fp32 when out_f32; += when accumulate).
PHA_API int pha_gemm256_tn(int dt, const void* a, const void* b, void* out, float* ws, long M, long N, long K, long lda,
                           long ldb, int out_f32, int accumulate, const void* zero16, int tile, int splits,
                           hipStream_t stream) {
  if (M % 8 || N % 8 || lda % 8 || ldb % 8 || M <= 0 || N <= 0 || K <= 0) return (int)hipErrorInvalidValue;
  g256::TnArgs p{a, b, ws, M, N, K, lda, ldb, 0, 1, zero16, {}};
  if (dt == kBF16) return g256::launch_tn<bf16_t, false>(p, out, out_f32, 0, accumulate, tile, splits, stream);
  if (dt == kF16) return g256::launch_tn<half_t, false>(p, out, out_f32, 0, accumulate, tile, splits, stream);
  return (int)hipErrorInvalidValue;
}

// NHWC conv weight gradient: dw[Cout][Cin][KH][KW] = sum over output pixels of dy[p][cout] *
// im2col(x)[p][(kh, kw, cin)]; dy [N*OH*OW][Cout], Cin % 8 == 0, Cout % 8 == 0.
PHA_API int pha_conv256_wgrad(int dt, const void* dy, const void* x, void* dw, float* ws, int N, int H, int W, int C,
                              int Cout, int KH, int KW, int sh, int sw, int ph, int pw, int dh, int dw_,
                              int out_f32, const void* zero16, int tile, int splits, hipStream_t stream) {
  if (C % 8 || Cout % 8) return (int)hipErrorInvalidValue;
  g256::ConvGeo g{N, H, W, C, (H + 2 * ph - dh * (KH - 1) - 1) / sh + 1, (W + 2 * pw - dw_ * (KW - 1) - 1) / sw + 1,
                  KH, KW, sh, sw, ph, pw, dh, dw_, 0, 0, 0, 0, 0, 0, 0};
  const long K = (long)N * g.OH * g.OW;
  g256::TnArgs p{dy, x, ws, (long)Cout, (long)KH * KW * C, K, (long)Cout, (long)C, 0, 1, zero16, g};
  if (dt == kBF16) return g256::launch_tn<bf16_t, true>(p, dw, out_f32, C, 0, tile, splits, stream);
  if (dt == kF16) return g256::launch_tn<half_t, true>(p, dw, out_f32, C, 0, tile, splits, stream);
  return (int)hipErrorInvalidValue;
}
