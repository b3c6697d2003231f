// Persistent 256 x 256 x 64 bf16/fp16 MFMA GEMM for gfx950, one wave per SIMD, whose epilogue runs
// UNDER the next tile's MFMAs. Reference behaviour: the cuBLAS GEMMs behind
// phi/kernels/impl/matmul_kernel_impl.h:88 (matmul / linear forward and both gradients) and the
// bias epilogue of fused_gemm_epilogue_op.cu:29.
//
//   C[M, N] = sum_k A(m, k) B(k, n) (+ bias[n]),  fp32 accumulate, bf16/fp16 out
//
// Why. gemm4w.hip's main loop runs at ~1.6 PF/s, but every tile then stages its 256 x 256 fp32
// result through LDS and issues a 128 KB store burst while the MFMA pipe idles: ~10 us per tile,
// 15-25 % of a GPT-sized GEMM (profiles/README.md, round 2 session 3/4). Here each workgroup walks a
// sequence of tiles as ONE continuous stream of K-tiles (the LDS-DMA prefetch of the next tile's
// first K-tiles is issued during the current tile's last two, exactly like any other prefetch), and
// the finished accumulators are written out from registers while the next tile's first k-half
// multiplies: before MFMA (i, j) first overwrites acc[i][j] (with a zero C operand), the old value is
// converted to bf16, paired with its neighbour tile through v_permlane16_swap into 16-byte rows, and
// stored with a bounds-checked buffer store. No LDS staging, no barrier, no idle MFMA pipe.
//
// Stores and LDS-DMA share the wave's vmcnt counter (in issue order). The stores of the epilogue
// phase are the youngest operations when that phase ends, so its wait is vmcnt(#stores): the
// prefetch it needs has landed, the stores stay in flight.
//
// Layouts (template AKO / BKO / OT):
//   NT  A[m][k],  B^T[n][k]                 forward on the cached W^T, dX = dY W
//   TN  A[k][m],  B[k][n]                   weight gradients X^T dY
//   NN  as (W^T X^T)^T: A = W [k][m'] (K-outer), B^T = X [n'][k], transposed store (OT)
#include "mfma_tile.h"
#include <type_traits>

namespace pha {
namespace g4p {

using namespace g256;

#ifndef PHA_G4P_RELG_NT
#define PHA_G4P_RELG_NT 8
#endif
#ifndef PHA_G4P_CS_SPLITLOOP
#define PHA_G4P_CS_SPLITLOOP 1
#endif
#ifndef PHA_G4P_RELG_TN
#define PHA_G4P_RELG_TN 8
#endif

enum : int {
  EPI_BIAS = 1,       // + bias[output column] (fp32)
  EPI_GELU = 2,       // NT only: C = gelu_tanh(acc + bias), and aux = acc (the pre-activation before
                      // the bias, what the HIP dGELU + bias-grad pass reads back)
  EPI_NOSTORE = 512,  // measurement only: stores dropped by the buffer bounds check (tools/bench_g4p.py)
  EPI_SKIP = 128,     // measurement only: no epilogue at all (fresh tiles just start at C = 0)
  EPI_STAGGER = 4096, // measurement only: workgroup w starts after (w & 7) * ((epi >> 16) & 255) s_sleep(16)
  EPI_ROUNDS = 8192,  // measurement only: round-robin tile order (lin = r * G + pos) instead of XCD chunks
  EPI_TEMPORAL = 16384,  // stores with the default cache policy (else non-temporal)
  EPI_RSTAGE = 32768,    // NT: register-staged operands (global_load -> VGPR -> ds_write) instead of LDS-DMA
  EPI_EARLY = 65536,     // early-release schedule (see the EARLY main loop)
  EPI_LATE_SHIFT = 17,   // NT + EARLY, bits 17-20: schedule variant LV (lv_lwg / lv_ldma / PIN)
  EPI_L2ONLY = 1 << 21,  // measurement only: every DMA re-reads the item's first K-tile (L2-resident
                         // operands: isolates the main loop from HBM / MALL latency; wrong results)
  EPI_RING = 1 << 22,    // NT: the 4-slot ring of 32-deep stages (gemm4r_kernel), K % 64 == 0, K >= 128
  EPI_ADEEP = 1 << 23,   // NT without bias / GELU: 3 A + 2 B LDS slots (gemm4a_kernel), K >= 256
  EPI_WSTAG = 1 << 24,   // NT + EARLY: wave w issues its LDS-DMA after MFMA w of the group (LV + 16)
  EPI_KSTAG_SHIFT = 25,  // bits 25-26: K-start stagger (1: per XCD, 2: per tile, 3: per slot in the XCD)
  EPI_COLSUM = 1 << 27,  // TN + EARLY: column sums of B (a linear layer's bias gradient: the sum of dY over
                         // the tokens) from the B fragments the MFMAs already hold, into aux (see CS)
  EPI_SPREAD_SHIFT = 28, // NT + EARLY + PIN, bits 28-29: DMA placement (see sp_na / sp_gb)
};

// SPREAD (LV bits 5-6): where the 16 DMAs of the next-next K-tile go. The plain EARLY schedule
// issues one per MFMA group over A groups 8-15 + B groups 0-7: 16 consecutive groups in which the
// CU's four waves push 4 KiB per 64 MFMA cycles into the texture path (its 64 B / clk), and none in
// the other 16. SPREAD puts sp_na of them over A groups RELG-15 and the rest over B groups
// 0..sp_gb-1, so the same bytes go out at up to half the rate (less issue back-pressure on the
// MFMA stream), at the price of less latency cover for the last ones (>= 16 groups instead of 24).
constexpr int sp_mode(int lv) { return (lv >> 5) & 3; }
constexpr int sp_na(int lv, int relg) { return sp_mode(lv) == 3 ? 6 : sp_mode(lv) ? 8 : 16 - relg; }
constexpr int sp_gb(int lv, int relg) { return sp_mode(lv) == 2 ? 12 : sp_mode(lv) ? 16 : relg; }

// late-wait variants (LV): {LWG = phase-B group of the buffer wait (0: at the A/B boundary),
// LDMA = DMAs of the next-next K-tile issued in phase A (groups RELG-15), the rest in phase B}
// LV & 8 (PIN): an empty "memory" asm closes every MFMA group, so no IR pass sinks a group's LDS
// fragment reads out of it (hipcc sank phase B's last reads past the loop latch: an uncovered
// read burst + lgkmcnt stall at every K-tile boundary, profiles/README.md round 5).
constexpr int lv_lwg(int lv) { return (lv & 7) == 1 ? 8 : (lv & 7) == 4 ? 12 : 0; }
constexpr int lv_ldma(int lv) { return 8; }
// LV & 7 in {2, 3, 5}: phase B reads in consumption order (LORD); phase A's 16 reads over the first
// lv_rg groups (8: two per group up to the release at group 8; 6 / 4: two / four groups of MFMAs
// between the last read and the release barrier's lgkmcnt(0))
constexpr bool lv_lord(int lv) { return (lv & 7) == 2 || (lv & 7) == 3 || (lv & 7) == 5; }
constexpr int lv_rg(int lv, int relg) { return (lv & 7) == 3 ? 6 : (lv & 7) == 5 ? 4 : relg; }
// LV & 7 == 6 (BURST): phase B's 16 reads two per group over groups 0-7 in consumption order, so the
// next phase A's first groups never wait on reads issued in phase B's last groups (the counted
// lgkmcnt waits at the top of every phase in the LV 0 / 8 ISA, profiles/README.md round 5)
constexpr bool lv_burst(int lv) { return (lv & 7) == 6; }
// LV & 7 == 7 (STAMP, diagnostic build, tools/g4p_stamp.py): the LV 0 / 8 schedule with s_memtime
// stamps around its two waits per K-tile (release: lgkmcnt(0) + barrier; A/B boundary: counted
// vmcnt + barrier); each wave writes {total, A/B-wait, release-wait, K-tiles} cycles to p.ws
constexpr bool lv_stamp(int lv) { return (lv & 7) == 7; }
// LV & 16 (WSTAG): the four waves' LDS-DMAs of one MFMA group go out 16 cycles apart (wave w after
// the group's MFMA w) instead of together at the group start: the CU's texture-address path takes
// one 1-KiB piece at a time, so four simultaneous issues stall three waves' MFMA streams
constexpr bool lv_wstag(int lv) { return (lv & 16) != 0; }

struct Args {
  const void* a;
  const void* b;
  void* c;
  const float* bias;
  int M, N, K;
  int lda, ldb, ldc;
  int epi;
  int group_m;
  float* ws;    // split-K: fp32 partial slabs [splits][M][N] (C unused)
  int splits;
  void* aux;    // EPI_GELU: pre-activation output, same shape and row stride as C
  int batch;    // batched products: item b reads A + b * sa, B + b * sb and writes C + b * sc
  long long sa, sb, sc;   // (element strides; the tiles of all batches share one persistent grid)
};

constexpr int OPB = 256 * 64 * 2;   // one operand image (32 KB)
constexpr int STAGE = 2 * OPB;      // A image, B image
constexpr int BIAS_OFF = 2 * STAGE; // 4 bias slots of 256 fp32 after the two stages
constexpr int SMEM = 2 * STAGE + 4 * 1024;

__device__ __forceinline__ unsigned lds_u32(const unsigned char* p) {
  return (unsigned)(size_t)(__attribute__((address_space(3))) const unsigned char*)p;
}

// LDS-DMA 16 B per lane: global (sbase + voff) -> LDS m0 + lane * 16
__device__ __forceinline__ void glds_sv(unsigned voff, const void* sbase, unsigned m0) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :: "v"(voff), "s"(sbase), "s"(m0) : "memory", "m0");
}
// LDS-DMA 4 B per lane (the bias slot)
__device__ __forceinline__ void glds4(const void* src, unsigned m0) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off"
               :: "v"(src), "s"(m0) : "memory", "m0");
}

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

// tanh-GELU as x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3) — the same function as
// 0.5 x (1 + tanh u), in 5 VALU + 2 transcendental instructions (exp2 with log2(e) folded into the
// polynomial, one reciprocal) instead of ~10 + 2: the epilogue runs beside the next tile's MFMAs at
// one wave per SIMD, so its VALU count is its cost
__device__ __forceinline__ float gelu_t(float x) {
  constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f;
  constexpr float c1 = c0 * 0.044715f;
  const float arg = x * __builtin_fmaf(x * x, c1, c0);
  return x * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(arg) + 1.f);
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

// d = a . b (C = 0) written over d's registers (see the fresh-tile phase). The leading s_nop 1 is
// the VALU-write -> MFMA-operand wait the compiler cannot insert inside an asm statement.
template <typename T>
__device__ __forceinline__ void mma0(f32x4& d, const uint4& a, const uint4& b) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  const v4u va = __builtin_bit_cast(v4u, a), vb = __builtin_bit_cast(v4u, b);
  if constexpr (std::is_same<T, bf16_t>::value)
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "+a"(d) : "v"(va), "v"(vb));
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, 0" : "+a"(d) : "v"(va), "v"(vb));
}

// c + x . sel for two 16-bit values (v_dot2, fp32 accumulate): sel = ONES2 sums x's pair, 0 adds 0
template <typename T>
constexpr unsigned ONES2 = std::is_same<T, bf16_t>::value ? 0x3f803f80u : 0x3c003c00u;
template <typename T>
__device__ __forceinline__ float dot2sel(unsigned x, unsigned sel, float c) {
  if constexpr (std::is_same<T, bf16_t>::value) {
    typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf2, x), __builtin_bit_cast(bf2, sel), c, false);
  } else {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, x), __builtin_bit_cast(h2, sel), c, false);
  }
}

// tile schedule of one workgroup. With G % 8 == 0 (G / 8 workgroups per XCD under round-robin
// placement) every XCD owns a contiguous chunk of the linear tile order and its workgroups walk it
// together: lin = chunk_start + r * (G / 8) + slot, so the 8 XCDs work on far-apart panels (their
// HBM / MALL reads spread over the channels) while the 32 CUs of an XCD share panels in its L2.
// Otherwise lin = r * G + pos. lin -> (tm, tn) in GROUP_M-row panels.
struct Sched {
  int tiles_m, tiles_n, total, G, pos, gm, splits, per_batch;
  int c0, c1, step;   // this workgroup's chunk [c0, c1) and stride
  __device__ __forceinline__ bool valid(int r) const { return c0 + r * step < c1; }
  // work item of round r: tile (tm, tn) and K slice (the slices of a tile are adjacent items)
  __device__ __forceinline__ void tile(int r, int& tm, int& tn, int& slice, int& bi) const {
    const int item = c0 + r * step;
    int lin = item / splits;
    slice = __builtin_amdgcn_readfirstlane(item - lin * splits);
    bi = __builtin_amdgcn_readfirstlane(lin / per_batch);   // batch index (tiles of one batch adjacent)
    lin -= bi * per_batch;
    const int group = lin / (gm * tiles_n);
    const int first_m = group * gm;
    const int gsize = min(tiles_m - first_m, gm);
    const int in = lin - group * gm * tiles_n;
    // wave-uniform by construction; readfirstlane tells the compiler (the integer divisions run
    // on the VALU), so the DMA bases and store descriptors stay scalar — no waterfall loops
    tm = __builtin_amdgcn_readfirstlane(first_m + in % gsize);
    tn = __builtin_amdgcn_readfirstlane(in / gsize);
  }
};

// SPLIT: the K range of every tile is cut into p.splits slices (separate work items, for problems
// with fewer tiles than CUs); each item writes its fp32 partial tile to its slab of p.ws and
// pha_gemm4p's reduce kernel sums the slabs in slice order (deterministic) into C (+ bias).
template <typename T, bool AKO, bool BKO, bool OT, bool BIAS, bool SKIPEPI = false, bool SPLIT = false,
          bool GELU = false, bool RS = false, bool EARLY = false, int LV = 0, bool CS = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4p_kernel(Args p) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int M = p.M, N = p.N, K = p.K;
  const int nsplit = SPLIT ? p.splits : 1;
  const int nk = (K >> 6) / nsplit;   // K-tiles per work item

  Sched sc;
  sc.tiles_m = (M + 255) >> 8;
  sc.tiles_n = (N + 255) >> 8;
  sc.splits = nsplit;
  sc.per_batch = sc.tiles_m * sc.tiles_n;
  sc.total = sc.per_batch * nsplit * p.batch;
  sc.G = gridDim.x;
  sc.gm = p.group_m;
  {
    const int bid = blockIdx.x, G = gridDim.x;
    const int q8 = G >> 3, r8 = G & 7, xcd = bid & 7;
    sc.pos = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (r8 == 0 && !(p.epi & EPI_ROUNDS)) {
      const int qt = sc.total >> 3, rt = sc.total & 7;
      sc.c0 = (xcd < rt ? xcd * (qt + 1) : rt * (qt + 1) + (xcd - rt) * qt) + (bid >> 3);
      sc.c1 = sc.c0 - (bid >> 3) + qt + (xcd < rt ? 1 : 0);
      sc.step = q8;
    } else {
      sc.c0 = sc.pos;
      sc.c1 = sc.total;
      sc.step = G;
    }
  }
  if (!sc.valid(0)) return;
  if (p.epi & EPI_STAGGER) {
    const int n = (blockIdx.x & 7) * ((p.epi >> 16) & 255);
    for (int i = 0; i < n; ++i) __builtin_amdgcn_s_sleep(16);
  }

  // ---- staging cursor: (round rs, k-tile ks); per-lane DMA offsets of the cursor's tile --------
  unsigned aoff[8], boff[8];
  const char* abase;
  const char* bbase;
  int rs = 0, ks = 0;
  const size_t astep = AKO ? (size_t)64 * p.lda * 2 : 128, bstep = BKO ? (size_t)64 * p.ldb * 2 : 128;
  const unsigned lds0 = lds_u32(smem);

  // K-start stagger: the cursor walks a tile's K-tiles from kofs, wrapping (every work item still
  // sums all of its K-tiles; only the order rotates). With power-of-two row pitches every workgroup
  // reading the same K columns at once lands on a fraction of the memory channels
  const int ksm = (p.epi >> EPI_KSTAG_SHIFT) & 3;
  int kofs = 0;
  auto set_tile = [&](int r) {   // DMA offsets + bases of round r's tile
    int tm, tn, slice, bi;
    sc.tile(r, tm, tn, slice, bi);
    if (ksm == 1) kofs = ((blockIdx.x & 7) * nk) >> 3;
    else if (ksm == 2) kofs = __builtin_amdgcn_readfirstlane(((tm * 5 + tn * 3) & 15) * nk >> 4);
    else if (ksm == 3) kofs = (((blockIdx.x >> 3) & 7) * nk) >> 3;
    const size_t k0 = (size_t)slice * nk * 64;   // first K of the item
    const int m0 = tm << 8, n0 = tn << 8;
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
    abase = static_cast<const char*>(p.a) + (size_t)bi * p.sa * 2 +
            (AKO ? (size_t)m0 * 2 + k0 * p.lda * 2 : (size_t)m0 * p.lda * 2 + k0 * 2);
    bbase = static_cast<const char*>(p.b) + (size_t)bi * p.sb * 2 +
            (BKO ? (size_t)n0 * 2 + k0 * p.ldb * 2 : (size_t)n0 * p.ldb * 2 + k0 * 2);
    if constexpr (BIAS && !SPLIT) {   // the tile's 256 output-column biases -> slot r & 3 (wave w: 64 of them)
      const int c0 = OT ? m0 : n0, No = OT ? M : N;
      const int col = min(c0 + wid * 64 + lane, No - 1);
      glds4(p.bias + col, lds0 + BIAS_OFF + (r & 3) * 1024 + wid * 256);
    }
  };
  // the cursor's K-tile goes into LDS buffer st_buf as 16 DMAs per wave, one per MFMA group of a
  // phase (a burst of them ahead of the MFMAs stalls the pipe: each costs ~60 issue cycles)
  const char* st_a = nullptr;
  const char* st_b = nullptr;
  bool st_on = false;
  int st_buf = 0;
  // Past the last tile the cursor stays on the last K-tile: those DMAs land in a buffer nothing
  // reads any more (no branch in the MFMA stream); the kernel drains them before it exits.
  const bool l2only = (p.epi & EPI_L2ONLY) != 0;
  auto stage_begin = [&](int buf) {
    st_on = sc.valid(rs);
    int kk = l2only ? 0 : (st_on ? ks : nk - 1) + kofs;
    if (kk >= nk) kk -= nk;
    st_a = abase + (size_t)kk * astep;
    st_b = bbase + (size_t)kk * bstep;
    st_buf = buf;
  };
  auto stage_one = [&](int gi) {   // DMA gi (0..15): u = gi >> 1, operand gi & 1
    const int u = gi >> 1;
    const unsigned dst = lds0 + st_buf * STAGE + (wid * 8 + u) * 1024 + (gi & 1) * OPB;
    if (gi & 1) glds_sv(boff[u], st_b, dst);
    else glds_sv(aoff[u], st_a, dst);
  };
  // RS (register staging, NT): the cursor's K-tile is loaded into 16 x 16 B of VGPRs per lane
  // (global_load_dwordx4) one K-tile ahead and written to its LDS slots (ds_write_b128, the same
  // swizzled image the DMA produces) during the next K-tile's phase B. Each load then has a whole
  // K-tile of latency cover and no wait drains the prefetch at the phase boundary.
  typedef unsigned u32x4s __attribute__((ext_vector_type(4)));
  u32x4s sreg[RS ? 16 : 1];
  auto stage_load = [&](int gi) {
    const int u = gi >> 1;
    if (gi & 1) asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(sreg[RS ? gi : 0]) : "v"(boff[u]), "s"(st_b) : "memory");
    else asm volatile("global_load_dwordx4 %0, %1, %2" : "=v"(sreg[RS ? gi : 0]) : "v"(aoff[u]), "s"(st_a) : "memory");
  };
  auto stage_write = [&](int gi) {
    const int u = gi >> 1;
    const unsigned dst = lds0 + st_buf * STAGE + (wid * 8 + u) * 1024 + (gi & 1) * OPB + lane * 16;
    asm volatile("ds_write_b128 %0, %1" :: "v"(dst), "v"(sreg[RS ? gi : 0]) : "memory");
  };
  auto stage_end = [&]() {   // advance the cursor; a new tile's offsets + bias DMA
    if (!st_on) return;
    if (++ks == nk) {
      ks = 0;
      ++rs;
      if (sc.valid(rs)) set_tile(rs);
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

  // ---- epilogue geometry (output coordinates; OT swaps the kernel's rows and columns) ----------
  // Non-OT: acc[i][j][e] = C[wr*128 + i*16 + fr][wc*128 + j*16 + 4fk + e]; tiles j, j+1 pair.
  // OT:     acc[i][j][e] = C_out[wc*128 + j*16 + fr][wr*128 + i*16 + 4fk + e]; tiles i, i+1 pair.
  // After the pair swap a lane holds 8 consecutive output columns starting at
  // (pair base)*16 + (fk & 1) * 16 + (fk >> 1) * 8 of output row (row base) + fr.
  const int Mo = OT ? N : M, No = OT ? M : N;
  const int ldc2 = SPLIT ? No * 4 : p.ldc * 2;   // output row bytes (split-K: the fp32 slab)
  const int wrow = (OT ? wc : wr) * 128;                                  // wave's first output row
  const int lcol = (OT ? wr : wc) * 128 + (fk & 1) * 16 + (fk >> 1) * 8;   // + pair base * 16
  const unsigned lane_voff = (unsigned)(fr * ldc2 + lcol * 2);
  // split-K (non-OT only): a lane's 4 fp32 of tile j sit at columns wc*128 + j*16 + 4fk
  const int lcol4 = wc * 128 + 4 * fk;
  const unsigned lane_voff4 = (unsigned)(fr * ldc2 + lcol4 * 4);
  // the tile being written out: output origin (bytes), valid rows / columns from the wave's origin,
  // bias slot
  const char* e_base = static_cast<const char*>(p.c);
  const char* e_aux = static_cast<const char*>(p.aux);
  int e_rows = 0, e_cols = 0, e_slot = 0;
  auto set_epi = [&](int r) {
    int tm, tn, slice, bi;
    sc.tile(r, tm, tn, slice, bi);
    const int r0 = OT ? tn << 8 : tm << 8, c0 = OT ? tm << 8 : tn << 8;
    e_slot = r & 3;
    if constexpr (SPLIT)
      e_base = reinterpret_cast<const char*>(p.ws) + (size_t)slice * Mo * No * 4 +
               ((size_t)(r0 + wrow) * ldc2 + (size_t)c0 * 4);
    else
      e_base = static_cast<const char*>(p.c) + (size_t)bi * p.sc * 2 + ((size_t)(r0 + wrow) * ldc2 + (size_t)c0 * 2);
    if constexpr (GELU) e_aux = static_cast<const char*>(p.aux) + ((size_t)(r0 + wrow) * ldc2 + (size_t)c0 * 2);
    // (EPI_NOSTORE, measurement only: zero rows, every store is issued and dropped)
    e_rows = (p.epi & EPI_NOSTORE) ? 0 : Mo - r0 - wrow;
    e_cols = No - c0;
  };
  // pair (t0, t0 + 1) of the wave's output-row block rb: one 16-B store of the lane's 8 columns.
  // Bounds: the buffer's base is the block's first row and its size the rows left, so rows past
  // the output are dropped by the buffer range check; a lane whose 8 columns (multiples of 8,
  // No % 8 == 0) start past the last column gets an offset past any size. Only the lane's
  // column offset is a VGPR; row block and pair go to the scalar base / the immediate offset.
  auto store_pair = [&](const f32x4& x0, const f32x4& x1, int rb, int cb) {
    // AGPR -> VGPR reads as asm: as plain C++ uses, the register allocator answered the
    // epilogue's reads by splitting every accumulator's live range into VGPR copies at the tile
    // boundary (60-150 spilled VGPRs); opaque, it keeps them in place (0 spills). The last MFMA
    // writing any of these registers is >= 60 MFMAs back (no hazard wait states needed).
    float v0[4], v1[4];
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v0[0]), "=v"(v0[1]), "=v"(v0[2]), "=v"(v0[3]) : "a"(x0[0]), "a"(x0[1]), "a"(x0[2]), "a"(x0[3]));
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v1[0]), "=v"(v1[1]), "=v"(v1[2]), "=v"(v1[3]) : "a"(x1[0]), "a"(x1[1]), "a"(x1[2]), "a"(x1[3]));
    const int nbytes = __builtin_amdgcn_readfirstlane(max(min(e_rows - rb * 16, 16), 0) * ldc2);
    const unsigned voff = (lcol + cb * 16 < e_cols) ? lane_voff : 0x80000000u;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    // 8 values -> the lane's 16-B row segment: pack, then lanes of odd 16-lane rows trade their
    // tile-t0 half for the even rows' tile-(t0+1) half
    auto pack_swap = [&](const float (&a)[4], const float (&b)[4]) {
      unsigned q00 = pk<T>(a[0], a[1]), q01 = pk<T>(a[2], a[3]);
      unsigned q10 = pk<T>(b[0], b[1]), q11 = pk<T>(b[2], b[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(q00, q10, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(q01, q11, false, false);
      return u32x4{s0[0], s1[0], s0[1], s1[1]};
    };
    // descriptor inputs readfirstlane'd: provably uniform, so the descriptor lives in SGPRs
    // (no per-store waterfall loop, cdna_hip_programming.md T20)
    auto rsrc = [&](const char* base) {
      const size_t bp = (size_t)(base + (size_t)rb * 16 * ldc2);
      const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp);
      const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
      return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((size_t)bhi << 32) | blo), (short)0, nbytes,
                                               0x00020000);
    };
    if constexpr (GELU)   // the pre-activation (before the bias) for the backward pass
      __builtin_amdgcn_raw_buffer_store_b128(pack_swap(v0, v1), rsrc(e_aux), voff + cb * 32, 0, 2);
    if constexpr (BIAS) {   // bias of the lane's pre-swap columns cb*16 + 4fk .. +3 and (cb+1)*16 + ...
      const unsigned char* bs = smem + BIAS_OFF + e_slot * 1024 + (OT ? wr : wc) * 512 + 16 * fk;
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(bs + cb * 64);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(bs + cb * 64 + 64);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] += b0[e];
        v1[e] += b1[e];
      }
    }
    if constexpr (GELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] = gelu_t(v0[e]);
        v1[e] = gelu_t(v1[e]);
      }
    }
    const auto rs = rsrc(e_base);
    const u32x4 q = pack_swap(v0, v1);
    // non-temporal by default (the output is not re-read by this kernel; 3 % faster measured,
    // profiles/gemm4p_store_ab_r3.log)
    if (p.epi & EPI_TEMPORAL) __builtin_amdgcn_raw_buffer_store_b128(q, rs, voff + cb * 32, 0, 0);
    else __builtin_amdgcn_raw_buffer_store_b128(q, rs, voff + cb * 32, 0, 2);
  };

  // split-K: acc tile (rb, cb) of the wave as fp32, one 16-B store per lane
  auto store_f32 = [&](const f32x4& x, int rb, int cb) {
    float v[4];
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]) : "a"(x[0]), "a"(x[1]), "a"(x[2]), "a"(x[3]));
    const size_t bp = (size_t)(e_base + (size_t)rb * 16 * ldc2);
    const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp);
    const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
    const int nbytes = __builtin_amdgcn_readfirstlane(max(min(e_rows - rb * 16, 16), 0) * ldc2);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((size_t)bhi << 32) | blo), (short)0, nbytes, 0x00020000);
    const unsigned voff = (lcol4 + cb * 16 < e_cols) ? lane_voff4 : 0x80000000u;
    typedef float f4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, f4{v[0], v[1], v[2], v[3]}), rs, voff + cb * 64, 0, 2);
  };

  f32x4 acc[8][8];
  uint4 fa0[8], fb0[8], fa1[8], fb1[8];
  // CS: per-lane column sums of the B fragments (fragment j: column wc*128 + 16j + fr, k-quarter fk)
  float csum[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  constexpr int SCHED = AKO ? 0 : 2;   // read placement, as gemm4w's per-layout winners
  // EARLY: MFMA group at which phase A's fragment-read burst ends and the buffer is released
  constexpr int RELG = AKO ? PHA_G4P_RELG_TN : PHA_G4P_RELG_NT;
  static_assert(16 % RELG == 0 && RELG < 16, "the read burst covers the 16 fragment reads in whole groups");
  constexpr int LWG = lv_lwg(LV), LDMA = lv_ldma(LV), LDMB = 16 - LDMA;
  constexpr bool PIN = (LV & 8) != 0;
  constexpr bool LORD = lv_lord(LV);
  constexpr bool BURST = lv_burst(LV);
  constexpr bool STAMP = lv_stamp(LV);
  constexpr bool WSTAG = lv_wstag(LV);
  unsigned long long sp_t = 0, sp_ab = 0, sp_rel = 0, sp_n = 0;
  constexpr int LRG = lv_rg(LV, RELG);
  constexpr int SPM = sp_mode(LV), SNA = sp_na(LV, RELG), SGB = sp_gb(LV, RELG);
  static_assert(SPM == 0 || (LWG == 0 && !WSTAG), "SPREAD: the early schedule without late waits / wave stagger");
  static_assert(LWG == 0 || (LDMB <= LWG && RELG == 8), "late variants: every phase-B DMA before the wait");

  // One k-half phase: MFMA groups of 4 on (ca, cb); with RD the 16 fragment reads of (rbuf, rkh)
  // into (na, nb). MODE 0: accumulate; 1: fresh tile (C = 0); 2: fresh tile with the previous
  // tile's accumulators written out right before the MFMA that overwrites them.
  auto phase = [&](auto rd_c, auto mode_c, auto st_c, uint4 (&ca)[8], uint4 (&cb)[8], uint4 (&na)[8],
                   uint4 (&nb)[8], int rbuf, int rkh) {
    constexpr bool RD = decltype(rd_c)::value;
    constexpr int MODE = decltype(mode_c)::value;
    constexpr int STV = decltype(st_c)::value;   // 0: no staging; else staging (RS: vmcnt STV - 1)
    constexpr bool ST = STV != 0;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if constexpr (RD && (SCHED & 2)) {
        if (s & 1) nb[s >> 1] = readB(rbuf, rkh, s >> 1);
        else na[s >> 1] = readA(rbuf, rkh, s >> 1);
      } else if constexpr (RD) {
        if (s < 8) {
#pragma unroll
          for (int r = 2 * s; r < 2 * s + 2; ++r) {
            if (r == 0) na[0] = readA(rbuf, rkh, 0);
            else if (r <= 8) nb[r - 1] = readB(rbuf, rkh, r - 1);
            else na[r - 8] = readA(rbuf, rkh, r - 8);
          }
        }
      }
      if constexpr (ST && RS) {
        // the previous set's load s has landed (STV - 1 younger ops: its 15 later loads + this
        // set's s earlier ones [+ the epilogue's stores]), then it is written and reloaded
        asm volatile("s_waitcnt vmcnt(%0)" :: "n"(STV - 1) : "memory");
        stage_write(s);
        stage_load(s);
      } else if constexpr (ST) {
        stage_one(s);
      }
      const int i = s >> 1, jb = (s & 1) * 4;
      if constexpr (MODE == 2 && SPLIT) {
#pragma unroll
        for (int q = 0; q < 4; ++q) store_f32(acc[i][jb + q], i, jb + q);
      } else if constexpr (MODE == 2) {
        if constexpr (!OT) {   // pairs (j, j+1) of row block i
          store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
          store_pair(acc[i][jb + 2], acc[i][jb + 3], i, jb + 2);
        } else if ((i & 1) == 0) {   // pairs (i, i+1) of output-row block j
#pragma unroll
          for (int q = 0; q < 4; ++q) store_pair(acc[i][jb + q], acc[i + 1][jb + q], jb + q, i);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = jb + q;
        if constexpr (MODE == 0) {
          if constexpr (OT) acc[i][j] = Mf<T>::mma(ca[i], cb[j], acc[i][j]);
          else acc[i][j] = Mf<T>::mma(cb[j], ca[i], acc[i][j]);
        } else {
          // fresh tile, C = 0, result IN PLACE of the old accumulator: as a builtin with a zero C
          // the register allocator gives the new value other AGPRs and copies every old
          // accumulator still waiting for its store into VGPRs (spills); tied "+a" it cannot.
          // The next reader is the following k-half's MFMA taking it whole as C (no wait states).
          if constexpr (OT) mma0<T>(acc[i][j], ca[i], cb[j]);
          else mma0<T>(acc[i][j], cb[j], ca[i]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PIN) asm volatile("" ::: "memory");
    }
  };
  using yes = std::true_type;
  using no = std::false_type;
  using M0 = std::integral_constant<int, 0>;
  using M1 = std::integral_constant<int, 1>;
  using M2 = std::integral_constant<int, 2>;
  // stores one epilogue phase issues per lane: 32 pairs
  constexpr int NST = 32;

  // EARLY schedule (the buffer-release pattern of hipBLASLt's gfx950 NT kernel, profiles/README.md
  // round 3): phase A reads its 16 next-k-half fragments in a burst (groups 0-3), then
  // lgkmcnt(0) + barrier releases the K-tile's LDS buffer at group 4, so the next-next K-tile's 16
  // DMAs go out in A's groups 4-15 and B's groups 0-3 — one K-tile ahead of where the plain
  // schedule can issue them; the A/B boundary waits with a counted vmcnt for the previous set only.
  // Each DMA gets >= 112 MFMAs of latency cover instead of >= 64.
  auto phaseE = [&](auto mode_c, auto rel_c, auto vbw_c, uint4 (&ca)[8], uint4 (&cb)[8], uint4 (&na)[8],
                    uint4 (&nb)[8], int rbuf, int rkh, int stbuf, auto cs_c, unsigned onesel) {
    constexpr int MODE = decltype(mode_c)::value;
    constexpr bool REL = decltype(rel_c)::value;   // phase A: read burst, release barrier, DMAs 0-11
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      int dq = -1;   // WSTAG: this group's DMA, issued after MFMA wid
      (void)dq;
      if constexpr (REL) {
        if (s < LRG) {   // the 16 reads over groups 0..LRG-1 (LRG < RELG: LDS-latency cover before the release)
#pragma unroll
          for (int r = s * 16 / LRG; r < (s + 1) * 16 / LRG; ++r) {
            if (r & 1) nb[r >> 1] = readB(rbuf, rkh, r >> 1);
            else na[r >> 1] = readA(rbuf, rkh, r >> 1);
          }
        }
        if (s == RELG) {
          if constexpr (STAMP) sp_t = __builtin_amdgcn_s_memtime();
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          bar();
          if constexpr (STAMP) {
            sp_rel += __builtin_amdgcn_s_memtime() - sp_t;
            __builtin_amdgcn_sched_barrier(0);
          }
          stage_begin(stbuf);
        }
        if constexpr (LWG > 0) {
          // LDMA DMAs over groups RELG-15 (one or two per group), the other LDMB in phase B
          if (s >= RELG) {
#pragma unroll
            for (int d = (s - RELG) * LDMA / (16 - RELG); d < (s - RELG + 1) * LDMA / (16 - RELG); ++d) stage_one(d);
          }
        } else if constexpr (SPM != 0) {
          if (s >= RELG) {
#pragma unroll
            for (int d = (s - RELG) * SNA / (16 - RELG); d < (s - RELG + 1) * SNA / (16 - RELG); ++d) stage_one(d);
          }
        } else if (s >= RELG) {
          if constexpr (WSTAG) dq = s - RELG;
          else stage_one(s - RELG);
        }
      } else if constexpr (LWG > 0) {
        // LATE (LV != 0): the next K-tile's LDS buffer is waited for at group LWG of phase B instead
        // of at the A/B boundary, and its 16 fragment reads (A0, B0-7, A1-7: the order the next
        // phase A's groups consume them) follow in groups LWG-15. hipBLASLt's gfx950 NT kernel waits
        // about two thirds into its iteration the same way (profiles/README.md round 5): each DMA
        // gets 4 * LWG more MFMAs of latency cover.
        if (s < LDMB) stage_one(LDMA + s);
        if (s == LWG) {
          asm volatile("s_waitcnt vmcnt(%0)" :: "n"(decltype(vbw_c)::value) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          bar();
        }
        if (s >= LWG) {
#pragma unroll
          for (int r = (s - LWG) * 16 / (16 - LWG); r < (s - LWG + 1) * 16 / (16 - LWG); ++r) {
            if (r == 0) na[0] = readA(rbuf, rkh, 0);
            else if (r <= 8) nb[r - 1] = readB(rbuf, rkh, r - 1);
            else na[r - 8] = readA(rbuf, rkh, r - 8);
          }
        }
      } else {
        if constexpr (BURST) {
          if (s < 8) {
#pragma unroll
            for (int r = 2 * s; r < 2 * s + 2; ++r) {
              if (r == 0) na[0] = readA(rbuf, rkh, 0);
              else if (r <= 8) nb[r - 1] = readB(rbuf, rkh, r - 1);
              else na[r - 8] = readA(rbuf, rkh, r - 8);
            }
          }
        } else if constexpr ((SCHED & 2) && !LORD) {
          if (s & 1) nb[s >> 1] = readB(rbuf, rkh, s >> 1);
          else na[s >> 1] = readA(rbuf, rkh, s >> 1);
        } else if constexpr (LORD) {
          // one read per group in the order the next phase A consumes them (A0, B0-7, A1-7): its
          // group 1 needs B4-7, read by group 8 here (the alternating order reads B7 last)
          if (s == 0) na[0] = readA(rbuf, rkh, 0);
          else if (s <= 8) nb[s - 1] = readB(rbuf, rkh, s - 1);
          else na[s - 8] = readA(rbuf, rkh, s - 8);
        } else if (s < 8) {
#pragma unroll
          for (int r = 2 * s; r < 2 * s + 2; ++r) {
            if (r == 0) na[0] = readA(rbuf, rkh, 0);
            else if (r <= 8) nb[r - 1] = readB(rbuf, rkh, r - 1);
            else na[r - 8] = readA(rbuf, rkh, r - 8);
          }
        }
        if constexpr (SPM != 0) {
          if (s < SGB) {
#pragma unroll
            for (int d = SNA + s * (16 - SNA) / SGB; d < SNA + (s + 1) * (16 - SNA) / SGB; ++d) stage_one(d);
          }
        } else if (s < RELG) {
          if constexpr (WSTAG) dq = 16 - RELG + s;
          else stage_one(16 - RELG + s);
        }
      }
      const int i = s >> 1, jb = (s & 1) * 4;
      if constexpr (MODE == 2 && SPLIT) {
#pragma unroll
        for (int q = 0; q < 4; ++q) store_f32(acc[i][jb + q], i, jb + q);
      } else if constexpr (MODE == 2) {
        if constexpr (!OT) {
          store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
          store_pair(acc[i][jb + 2], acc[i][jb + 3], i, jb + 2);
        } else if ((i & 1) == 0) {
#pragma unroll
          for (int q = 0; q < 4; ++q) store_pair(acc[i][jb + q], acc[i + 1][jb + q], jb + q, i);
        }
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = jb + q;
        if constexpr (WSTAG) {
          if (dq >= 0 && wid == q) stage_one(dq);
        }
        if constexpr (MODE == 0) {
          if constexpr (OT) acc[i][j] = Mf<T>::mma(ca[i], cb[j], acc[i][j]);
          else acc[i][j] = Mf<T>::mma(cb[j], ca[i], acc[i][j]);
        } else {
          if constexpr (OT) mma0<T>(acc[i][j], ca[i], cb[j]);
          else mma0<T>(acc[i][j], cb[j], ca[i]);
        }
      }
      // CS phases (branch-free: a taken branch per group cost 12 % of the TN kernel): group s < 8
      // adds the 8 k-values of B fragment s (column wc*128 + 16s + fr) dotted with onesel — 1.0 x 2
      // on the wave row that sums this k-half of this K-tile, 0 on the other
      if constexpr (decltype(cs_c)::value) {
        if (s < 8) {   // (s is a constant after unrolling: no branch)
          csum[s & 7] = dot2sel<T>(cb[s & 7].x, onesel, csum[s & 7]);
          csum[s & 7] = dot2sel<T>(cb[s & 7].y, onesel, csum[s & 7]);
          csum[s & 7] = dot2sel<T>(cb[s & 7].z, onesel, csum[s & 7]);
          csum[s & 7] = dot2sel<T>(cb[s & 7].w, onesel, csum[s & 7]);
        }
      } else {
        (void)onesel;
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (PIN) asm volatile("" ::: "memory");
    }
  };

  // ---- prologue ----------------------------------------------------------------------------------
  set_tile(0);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    stage_begin(b);
#pragma unroll
    for (int gi = 0; gi < 16; ++gi) stage_one(gi);
    stage_end();
  }
  if constexpr (RS) {   // the register stage starts one K-tile ahead of the two LDS buffers
    stage_begin(0);
#pragma unroll
    for (int gi = 0; gi < 16; ++gi) stage_load(gi);
    stage_end();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa0[i] = readA(0, 0, i);
    fb0[i] = readB(0, 0, i);
  }

  // the first epilogue phase has no previous tile: zero rows, its stores are dropped
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int s = 0;   // global K-tile step; buffer s & 1
  if constexpr (EARLY && !SKIPEPI && !RS) {
    using yes = std::true_type;
    using no = std::false_type;
    using M0 = std::integral_constant<int, 0>;
    using M2 = std::integral_constant<int, 2>;
    // VMEM ops younger than the previous K-tile's DMAs at the A/B boundary: phase A's 12 DMAs, plus
    // an epilogue phase's stores (capped at the counter's 63)
    constexpr int NSTE = (SPLIT || GELU) ? 64 : 32;
    constexpr int VB2 = SNA + NSTE > 63 ? 63 : SNA + NSTE;
    // LATE: the wait sits in phase B after all 16 DMAs of the next-next K-tile (+ the stores)
    constexpr int VL2 = 16 + NSTE > 63 ? 63 : 16 + NSTE;
    using VW1 = std::integral_constant<int, LWG ? 16 : 0>;
    using VW2 = std::integral_constant<int, LWG ? VL2 : 0>;
    const unsigned long long sp_0 = STAMP ? __builtin_amdgcn_s_memtime() : 0;
    for (int r = 0; sc.valid(r); ++r) {
      // CS: the item's K-tiles [klo, khi) are summed by this tile row (each of the tiles_m tile rows
      // takes its own 1/tiles_m of the K range, so the extra VALU work is spread over the grid);
      // wave row wr takes k-half wr of each of them
      int klo = 0, khi = 0;
      if constexpr (CS) {
        int tm, tn, slice, bi;
        sc.tile(r, tm, tn, slice, bi);
        klo = __builtin_amdgcn_readfirstlane(tm * nk / sc.tiles_m);
        khi = __builtin_amdgcn_readfirstlane((tm + 1) * nk / sc.tiles_m);
      }
      // CS: K-tile k's k-half h is summed by wave row h when klo <= k < khi (sel below)
      using CSY = std::integral_constant<bool, CS>;
      auto sel = [&](int k, int h) -> unsigned {
        return (CS && k >= klo && k < khi && wr == h) ? ONES2<T> : 0u;
      };
      {
        const int buf = s & 1;
        phaseE(M2{}, yes{}, VW2{}, fa0, fb0, fa1, fb1, buf, 1, buf, CSY{}, sel(0, 0));
        if constexpr (LWG == 0) {
          if constexpr (STAMP) sp_t = __builtin_amdgcn_s_memtime();
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" :: "n"(VB2) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          bar();
          if constexpr (STAMP) {
            sp_ab += __builtin_amdgcn_s_memtime() - sp_t;
            ++sp_n;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        set_epi(r);
        phaseE(M0{}, no{}, VW2{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, buf, CSY{}, sel(0, 1));
        stage_end();
        ++s;
      }
      auto ktile = [&](auto cs_c, int k) {
        const int buf = s & 1;
        phaseE(M0{}, yes{}, VW1{}, fa0, fb0, fa1, fb1, buf, 1, buf, cs_c, sel(k, 0));
        if constexpr (LWG == 0) {
          if constexpr (STAMP) sp_t = __builtin_amdgcn_s_memtime();
          asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" :: "n"(SNA) : "memory");
          __builtin_amdgcn_sched_barrier(0);
          bar();
          if constexpr (STAMP) {
            sp_ab += __builtin_amdgcn_s_memtime() - sp_t;
            ++sp_n;
            __builtin_amdgcn_sched_barrier(0);
          }
        }
        phaseE(M0{}, no{}, VW1{}, fa1, fb1, fa0, fb0, buf ^ 1, 0, buf, cs_c, sel(k, 1));
        stage_end();
      };
      // the K-tile loop cut at klo / khi: only the phases of [klo, khi) carry the dot2s (all-on
      // dot2 phases cost the TN kernel 9-13 %, profiles/tn_colsum_r6/)
      if constexpr (CS && PHA_G4P_CS_SPLITLOOP) {
        using CSN = std::false_type;
        int k = 1;
        for (; k < klo; ++k, ++s) ktile(CSN{}, k);
        for (; k < khi; ++k, ++s) ktile(CSY{}, k);
        for (; k < nk; ++k, ++s) ktile(CSN{}, k);
      } else {
        for (int k = 1; k < nk; ++k, ++s) ktile(CSY{}, k);
      }
      if constexpr (CS) {
        // the item is done: sum the 4 k-quarters (lanes l, l+16, l+32, l+48) of every fragment. The
        // swaps pair DIFFERENT fragments (a swap of a register with itself is a no-op): after
        // permlane32_swap(f_j, f_j+4) + add, lanes 0-31 hold f_j's half sums and lanes 32-63 f_j+4's;
        // after permlane16_swap(u_j, u_j+1) + add, 16-lane row 0..3 holds the totals of fragments
        // (j, j+1, j+4, j+5). Lane row fk then stores two fragments to row
        // (slice * tiles_m + tm) * 2 + wr of the fp32 partials [2 * splits * tiles_m][N]
        int tm, tn, slice, bi;
        sc.tile(r, tm, tn, slice, bi);
        // (asm swaps: hipcc's permlane*_swap builtins fed into an add came out as vdst + vdst, the
        // second result dropped — the ISA showed v_add_f32 vX, vA, vA after v_permlane32_swap vA, vB)
        float u[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float x0 = csum[j], x1 = csum[j + 4];
          asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x0), "+v"(x1));
          u[j] = x0 + x1;
        }
        float w[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float x0 = u[2 * j], x1 = u[2 * j + 1];
          asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x0), "+v"(x1));
          w[j] = x0 + x1;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) csum[j] = 0.f;
        const int f0 = (fk & 1) + (fk >> 1) * 4;   // w[0]: fragment f0, w[1]: fragment f0 + 2
        float* row = static_cast<float*>(p.aux) + (size_t)((slice * sc.tiles_m + tm) * 2 + wr) * N;
        const int c0 = (tn << 8) + wc * 128 + 16 * f0 + fr;
        if (c0 < N) row[c0] = w[0];
        if (c0 + 32 < N) row[c0 + 32] = w[1];
      }
    }
    if constexpr (STAMP) {   // diagnostic output (vector stores from lane 0 into the workspace)
      const unsigned long long tot = __builtin_amdgcn_s_memtime() - sp_0;
      if (lane == 0) {
        unsigned long long* o = reinterpret_cast<unsigned long long*>(p.ws) + ((size_t)blockIdx.x * 4 + wid) * 4;
        o[0] = tot;
        o[1] = sp_ab;
        o[2] = sp_rel;
        o[3] = sp_n;
      }
    }
  } else {
  using ST1 = std::integral_constant<int, 1>;
  using STB = std::integral_constant<int, RS ? 16 : 1>;         // phase B staging (RS: vmcnt(15))
  using STB2 = std::integral_constant<int, RS ? 16 + 32 : 1>;   // after an epilogue phase's stores
  (void)sizeof(ST1);
  for (int r = 0; sc.valid(r); ++r) {
    {   // K-tile 0 of tile r: the previous tile is written out under its k-half-0 MFMAs
      const int buf = s & 1;
      if constexpr (SKIPEPI) phase(yes{}, M1{}, M0{}, fa0, fb0, fa1, fb1, buf, 1);
      else phase(yes{}, M2{}, M0{}, fa0, fb0, fa1, fb1, buf, 1);
      static_assert(NST == 32, "vmcnt literal");
      // GELU builds store twice per pair (64 > the counter's 63): wait to 63, one store retired
      if constexpr (RS) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else if constexpr (SPLIT || GELU) asm volatile("s_waitcnt vmcnt(63)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(32)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bar();
      set_epi(r);   // the next epilogue phase writes this tile
      stage_begin(buf);
      phase(yes{}, M0{}, STB2{}, fa1, fb1, fa0, fb0, buf ^ 1, 0);
      stage_end();
      ++s;
    }
    for (int k = 1; k < nk; ++k, ++s) {
      const int buf = s & 1;
      // phase A: F1 reads of this K-tile | MFMAs on F0 (k-half 0)
      phase(yes{}, M0{}, M0{}, fa0, fb0, fa1, fb1, buf, 1);
      if constexpr (RS) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bar();
      // phase B: stage the cursor into this buffer, F0 reads of the next K-tile (after the last
      // K-tile they read a stale buffer, unused) | MFMAs on F1
      stage_begin(buf);
      phase(yes{}, M0{}, STB{}, fa1, fb1, fa0, fb0, buf ^ 1, 0);
      stage_end();
    }
  }
  }
  // last tile: stores only (after the cursor's trailing DMAs have landed)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i) {
#pragma unroll
    for (int jb = 0; jb < 8; jb += 2) {
      if constexpr (SPLIT) {
        store_f32(acc[i][jb], i, jb);
        store_f32(acc[i][jb + 1], i, jb + 1);
      } else if constexpr (!OT) store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
      else if ((i & 1) == 0) {
        store_pair(acc[i][jb], acc[i + 1][jb], jb, i);
        store_pair(acc[i][jb + 1], acc[i + 1][jb + 1], jb + 1, i);
      }
    }
  }
}

// C[m][n] = sum_s ws[s][m][n] (+ bias[n]), slices summed in order; 8 columns per thread
template <typename T, bool BIAS>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, T* __restrict__ c,
                                                            const float* __restrict__ bias, int M, int N, int ldc,
                                                            int splits) {
  const long i = ((long)blockIdx.x * 256 + threadIdx.x) * 8;
  if (i >= (long)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (long)m * N);
  float acc[8];
  {
    const float4 a = *reinterpret_cast<const float4*>(ws + i), b = *reinterpret_cast<const float4*>(ws + i + 4);
    acc[0] = a.x; acc[1] = a.y; acc[2] = a.z; acc[3] = a.w; acc[4] = b.x; acc[5] = b.y; acc[6] = b.z; acc[7] = b.w;
  }
  for (int s = 1; s < splits; ++s) {
    const float* w = ws + (size_t)s * M * N + i;
    const float4 a = *reinterpret_cast<const float4*>(w), b = *reinterpret_cast<const float4*>(w + 4);
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w; acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
  }
  if constexpr (BIAS) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += bias[n + e];
  }
  Vec8<T>::st(c + (long)m * ldc + n, acc);
}

// ================================================================================================
// RING: the NT main loop on a 4-slot ring of 32-deep K stages (EPI_RING). gemm4p's two 64-deep LDS
// buffers leave each LDS-DMA 1.5-2.5 MFMA phases of latency cover, and the long-K NT products are
// latency-bound on the HBM / MALL fetches: the same schedule with L2-resident operands
// (EPI_L2ONLY) runs at hipBLASLt's speed (profiles/README.md round 5). Here stage q + 4 is DMA'd
// into slot q % 4 during phase q (one phase = one 32-deep stage = 64 MFMAs per wave) and read
// during phase q + 3: 2.1-3 phases of cover, one barrier per phase. A stage's operand images are
// plain [256][32] bf16 rows (64 B): a fragment read (16 rows x 4 chunks) and a DMA piece (16 rows)
// are both one contiguous KiB, conflict-free without a swizzle.
//
// Per phase, at its start: s_waitcnt vmcnt(N) (the stage read in this phase has landed: N = the
// VMEM ops issued after its DMAs — two phases of DMAs plus the stores of an epilogue phase among
// them) + lgkmcnt(0) (this wave's reads of the slot about to be overwritten are done) + barrier.
// Then 16 MFMA groups: DMA d of the cursor stage before even groups, the next stage's 16 fragment
// reads two per group over groups 0-7, and in a tile's first phase the previous tile's
// accumulators stored right before the MFMAs that overwrite them (gemm4p's overlapped epilogue).
// ================================================================================================
constexpr int R_OPB = 256 * 32 * 2;            // one operand image of a 32-deep stage (16 KiB)
constexpr int R_STAGE = 2 * R_OPB;             // A image, B image
constexpr int R_NS = 4;                        // ring slots
constexpr int R_BIAS_OFF = R_NS * R_STAGE;     // 4 bias slots of 256 fp32 after the ring
constexpr int R_SMEM = R_BIAS_OFF + 4 * 1024;

template <typename T, bool BIAS, bool GELU>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4r_kernel(Args p) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[R_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int M = p.M, N = p.N, K = p.K;
  const int nst = K >> 5;   // stages per tile (even, >= 4: the launcher checks)

  Sched sc;
  sc.tiles_m = (M + 255) >> 8;
  sc.tiles_n = (N + 255) >> 8;
  sc.splits = 1;
  sc.per_batch = sc.tiles_m * sc.tiles_n;
  sc.total = sc.per_batch * p.batch;
  sc.G = gridDim.x;
  sc.gm = p.group_m;
  {
    const int bid = blockIdx.x, G = gridDim.x;
    const int q8 = G >> 3, r8 = G & 7, xcd = bid & 7;
    sc.pos = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (r8 == 0 && !(p.epi & EPI_ROUNDS)) {
      const int qt = sc.total >> 3, rt = sc.total & 7;
      sc.c0 = (xcd < rt ? xcd * (qt + 1) : rt * (qt + 1) + (xcd - rt) * qt) + (bid >> 3);
      sc.c1 = sc.c0 - (bid >> 3) + qt + (xcd < rt ? 1 : 0);
      sc.step = q8;
    } else {
      sc.c0 = sc.pos;
      sc.c1 = sc.total;
      sc.step = G;
    }
  }
  if (!sc.valid(0)) return;

  // ---- DMA cursor: round rs, stage ks; 4 A + 4 B pieces (16 rows x 64 B) per wave and stage ----
  unsigned aoff[4], boff[4];
  const char* abase;
  const char* bbase;
  int rs = 0, ks = 0;
  const unsigned lds0 = lds_u32(smem);
  const bool l2only = (p.epi & EPI_L2ONLY) != 0;
  auto set_tile = [&](int r) {
    int tm, tn, slice, bi;
    sc.tile(r, tm, tn, slice, bi);
    const int m0 = tm << 8, n0 = tn << 8;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = (wid * 4 + u) * 16 + (lane >> 2);
      const int ga = min(m0 + row, M - 1) - m0, gb = min(n0 + row, N - 1) - n0;
      aoff[u] = ((unsigned)ga * (unsigned)p.lda + (unsigned)((lane & 3) * 8)) * 2u;
      boff[u] = ((unsigned)gb * (unsigned)p.ldb + (unsigned)((lane & 3) * 8)) * 2u;
    }
    abase = static_cast<const char*>(p.a) + (size_t)bi * p.sa * 2 + (size_t)m0 * p.lda * 2;
    bbase = static_cast<const char*>(p.b) + (size_t)bi * p.sb * 2 + (size_t)n0 * p.ldb * 2;
    if constexpr (BIAS) {
      const int col = min(n0 + wid * 64 + lane, N - 1);
      glds4(p.bias + col, lds0 + R_BIAS_OFF + (r & 3) * 1024 + wid * 256);
    }
  };
  const char* st_a = nullptr;
  const char* st_b = nullptr;
  bool st_on = false;
  int st_slot = 0;
  auto stage_begin = [&](int slot) {   // past the last tile the cursor repeats its last stage (unread slots)
    st_on = sc.valid(rs);
    const int kk = l2only ? 0 : (st_on ? ks : nst - 1);
    st_a = abase + (size_t)kk * 64;
    st_b = bbase + (size_t)kk * 64;
    st_slot = slot;
  };
  auto stage_one = [&](int d) {   // d = 0..7: piece d >> 1 of operand d & 1
    const int u = d >> 1;
    const unsigned dst = lds0 + st_slot * R_STAGE + (d & 1) * R_OPB + (wid * 4 + u) * 1024;
    if (d & 1) glds_sv(boff[u], st_b, dst);
    else glds_sv(aoff[u], st_a, dst);
  };
  auto stage_end = [&]() {
    if (!st_on) return;
    if (++ks == nst) {
      ks = 0;
      ++rs;
      if (sc.valid(rs)) set_tile(rs);
    }
  };

  const int fr = lane & 15, fk = lane >> 4;
  auto readA = [&](int slot, int i) -> uint4 {
    return *reinterpret_cast<const uint4*>(smem + slot * R_STAGE + (wr * 128 + i * 16 + fr) * 64 + fk * 16);
  };
  auto readB = [&](int slot, int j) -> uint4 {
    return *reinterpret_cast<const uint4*>(smem + slot * R_STAGE + R_OPB + (wc * 128 + j * 16 + fr) * 64 + fk * 16);
  };

  // ---- epilogue geometry (gemm4p's non-OT layout) ------------------------------------------------
  const int ldc2 = p.ldc * 2;
  const int wrow = wr * 128;
  const int lcol = wc * 128 + (fk & 1) * 16 + (fk >> 1) * 8;
  const unsigned lane_voff = (unsigned)(fr * ldc2 + lcol * 2);
  const char* e_base = static_cast<const char*>(p.c);
  const char* e_aux = static_cast<const char*>(p.aux);
  int e_rows = 0, e_cols = 0, e_slot = 0;
  auto set_epi = [&](int r) {
    int tm, tn, slice, bi;
    sc.tile(r, tm, tn, slice, bi);
    const int r0 = tm << 8, c0 = tn << 8;
    e_slot = r & 3;
    e_base = static_cast<const char*>(p.c) + (size_t)bi * p.sc * 2 + ((size_t)(r0 + wrow) * ldc2 + (size_t)c0 * 2);
    if constexpr (GELU) e_aux = static_cast<const char*>(p.aux) + ((size_t)(r0 + wrow) * ldc2 + (size_t)c0 * 2);
    e_rows = (p.epi & EPI_NOSTORE) ? 0 : M - r0 - wrow;
    e_cols = N - c0;
  };
  auto store_pair = [&](const f32x4& x0, const f32x4& x1, int rb, int cb) {
    float v0[4], v1[4];
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v0[0]), "=v"(v0[1]), "=v"(v0[2]), "=v"(v0[3]) : "a"(x0[0]), "a"(x0[1]), "a"(x0[2]), "a"(x0[3]));
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v1[0]), "=v"(v1[1]), "=v"(v1[2]), "=v"(v1[3]) : "a"(x1[0]), "a"(x1[1]), "a"(x1[2]), "a"(x1[3]));
    const int nbytes = __builtin_amdgcn_readfirstlane(max(min(e_rows - rb * 16, 16), 0) * ldc2);
    const unsigned voff = (lcol + cb * 16 < e_cols) ? lane_voff : 0x80000000u;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    auto pack_swap = [&](const float (&a)[4], const float (&b)[4]) {
      unsigned q00 = pk<T>(a[0], a[1]), q01 = pk<T>(a[2], a[3]);
      unsigned q10 = pk<T>(b[0], b[1]), q11 = pk<T>(b[2], b[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(q00, q10, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(q01, q11, false, false);
      return u32x4{s0[0], s1[0], s0[1], s1[1]};
    };
    auto rsrc = [&](const char* base) {
      const size_t bp = (size_t)(base + (size_t)rb * 16 * ldc2);
      const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp);
      const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
      return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((size_t)bhi << 32) | blo), (short)0, nbytes,
                                               0x00020000);
    };
    if constexpr (GELU) __builtin_amdgcn_raw_buffer_store_b128(pack_swap(v0, v1), rsrc(e_aux), voff + cb * 32, 0, 2);
    if constexpr (BIAS) {
      const unsigned char* bs = smem + R_BIAS_OFF + e_slot * 1024 + wc * 512 + 16 * fk;
      const f32x4 b0 = *reinterpret_cast<const f32x4*>(bs + cb * 64);
      const f32x4 b1 = *reinterpret_cast<const f32x4*>(bs + cb * 64 + 64);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] += b0[e];
        v1[e] += b1[e];
      }
    }
    if constexpr (GELU) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v0[e] = gelu_t(v0[e]);
        v1[e] = gelu_t(v1[e]);
      }
    }
    const auto rs_ = rsrc(e_base);
    const u32x4 q = pack_swap(v0, v1);
    if (p.epi & EPI_TEMPORAL) __builtin_amdgcn_raw_buffer_store_b128(q, rs_, voff + cb * 32, 0, 0);
    else __builtin_amdgcn_raw_buffer_store_b128(q, rs_, voff + cb * 32, 0, 2);
  };

  f32x4 acc[8][8];
  uint4 fa0[8], fb0[8], fa1[8], fb1[8];
  // VMEM ops allowed outstanding at the start of phase kq of a tile: the two phases of DMAs issued
  // after the needed stage's, plus the stores of an epilogue phase among them (capped at 63:
  // waiting for more than needed is only slower)
  constexpr int NSTO = GELU ? 64 : 32;
  auto phase = [&](auto epi_c, auto nv_c, uint4 (&ca)[8], uint4 (&cb)[8], uint4 (&na)[8], uint4 (&nb)[8], int q) {
    constexpr bool EP = decltype(epi_c)::value;
    constexpr int NV = decltype(nv_c)::value;
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" :: "n"(NV) : "memory");
    __builtin_amdgcn_sched_barrier(0);
    bar();
    stage_begin(q & 3);
    const int rslot = (q + 1) & 3;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if ((s & 1) == 0) stage_one(s >> 1);
      if (s < 8) {
#pragma unroll
        for (int r = 2 * s; r < 2 * s + 2; ++r) {   // consumption order: A0, B0-7, A1-7
          if (r == 0) na[0] = readA(rslot, 0);
          else if (r <= 8) nb[r - 1] = readB(rslot, r - 1);
          else na[r - 8] = readA(rslot, r - 8);
        }
      }
      const int i = s >> 1, jb = (s & 1) * 4;
      if constexpr (EP) {
        store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
        store_pair(acc[i][jb + 2], acc[i][jb + 3], i, jb + 2);
      }
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const int j = jb + qq;
        if constexpr (EP) mma0<T>(acc[i][j], cb[j], ca[i]);
        else acc[i][j] = Mf<T>::mma(cb[j], ca[i], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
    }
    stage_end();
  };
  using yes = std::true_type;
  using no = std::false_type;
  constexpr int NV_E = 16 + 0;                                  // phase 0: the previous tile's last 3
  constexpr int NV_1 = 16 + NSTO > 63 ? 63 : 16 + NSTO;         // phase 1: the epilogue phase is in the window
  constexpr int NV_3 = 16 + 4 * (NSTO / 32);                    // phase 3: its stores after the last DMA
  using V0 = std::integral_constant<int, NV_E>;
  using V1 = std::integral_constant<int, NV_1>;
  using V3 = std::integral_constant<int, NV_3>;

  // ---- prologue: stages 0-3 into slots 0-3, stage 0's fragments -----------------------------------
  set_tile(0);
#pragma unroll
  for (int b = 0; b < R_NS; ++b) {
    stage_begin(b);
#pragma unroll
    for (int d = 0; d < 8; ++d) stage_one(d);
    stage_end();
  }
  asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  bar();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa0[i] = readA(0, i);
    fb0[i] = readB(0, i);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int q = 0;   // global phase = stage index; slot q & 3
  for (int r = 0; sc.valid(r); ++r) {
    phase(yes{}, V0{}, fa0, fb0, fa1, fb1, q);   // kq 0: the previous tile written out
    set_epi(r);
    phase(no{}, V1{}, fa1, fb1, fa0, fb0, q + 1);
    phase(no{}, V1{}, fa0, fb0, fa1, fb1, q + 2);
    phase(no{}, V3{}, fa1, fb1, fa0, fb0, q + 3);
    q += 4;
    for (int k = 4; k < nst; k += 2, q += 2) {
      phase(no{}, V0{}, fa0, fb0, fa1, fb1, q);
      phase(no{}, V0{}, fa1, fb1, fa0, fb0, q + 1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jb = 0; jb < 8; jb += 2) store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
}

// ================================================================================================
// A-DEEP (EPI_ADEEP, NT, no bias / GELU yet): gemm4p's early-release schedule with the LDS split
// 3 : 2 between the operands — three 32 KiB slots for the activation panel A (streamed from HBM)
// and two for the weight panel B^T (re-read across the chip, mostly L2 / MALL hits): 160 KiB.
// K-tile t reads A slot t % 3 and B slot t % 2; B of tile t + 2 is DMA'd in phase A(t) after the
// release barrier, A of tile t + 3 in phase B(t): the A fetches get ~2 K-tiles of latency cover
// (one in gemm4p), B's 1.25. One counted vmcnt + two barriers per K-tile, as gemm4p.
// ================================================================================================
constexpr int AD_SLOT = 256 * 64 * 2;           // 32 KiB operand image of one 64-deep K-tile
constexpr int AD_B0 = 3 * AD_SLOT;              // B slots after the three A slots
constexpr int AD_SMEM = 5 * AD_SLOT;            // 160 KiB

template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm4a_kernel(Args p) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[AD_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  const int M = p.M, N = p.N, K = p.K;
  const int nk = K >> 6;   // >= 4 (launcher)

  Sched sc;
  sc.tiles_m = (M + 255) >> 8;
  sc.tiles_n = (N + 255) >> 8;
  sc.splits = 1;
  sc.per_batch = sc.tiles_m * sc.tiles_n;
  sc.total = sc.per_batch * p.batch;
  sc.G = gridDim.x;
  sc.gm = p.group_m;
  {
    const int bid = blockIdx.x, G = gridDim.x;
    const int q8 = G >> 3, r8 = G & 7, xcd = bid & 7;
    sc.pos = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
    if (r8 == 0 && !(p.epi & EPI_ROUNDS)) {
      const int qt = sc.total >> 3, rt = sc.total & 7;
      sc.c0 = (xcd < rt ? xcd * (qt + 1) : rt * (qt + 1) + (xcd - rt) * qt) + (bid >> 3);
      sc.c1 = sc.c0 - (bid >> 3) + qt + (xcd < rt ? 1 : 0);
      sc.step = q8;
    } else {
      sc.c0 = sc.pos;
      sc.c1 = sc.total;
      sc.step = G;
    }
  }
  if (!sc.valid(0)) return;

  const unsigned lds0 = lds_u32(smem);
  const bool l2only = (p.epi & EPI_L2ONLY) != 0;
  // two DMA cursors (A three K-tiles ahead, B two): per operand a round, a K-tile, the tile's base
  // and the lanes' 8 piece offsets (gemm4p's NT geometry: piece g = 8 rows x 128 B, chunk ^ row & 7)
  struct Cur {
    int rs, ks;
    const char* base;
    unsigned off[8];
    const char* st;
    bool on;
    int slot;
  };
  Cur ca_{0, 0, nullptr, {}, nullptr, false, 0}, cb_{0, 0, nullptr, {}, nullptr, false, 0};
  auto set_tile = [&](Cur& c, bool isA, int r) {
    int tm, tn, slice, bi;
    sc.tile(r, tm, tn, slice, bi);
    const int base = isA ? tm << 8 : tn << 8, dim = isA ? M : N, ld = isA ? p.lda : p.ldb;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int row = (wid * 8 + u) * 8 + (lane >> 3);
      const int grow = min(base + row, dim - 1) - base;
      c.off[u] = ((unsigned)grow * (unsigned)ld + (unsigned)(((lane & 7) ^ (row & 7)) * 8)) * 2u;
    }
    c.base = static_cast<const char*>(isA ? p.a : p.b) + (size_t)bi * (isA ? p.sa : p.sb) * 2 + (size_t)base * ld * 2;
  };
  auto begin = [&](Cur& c, int slot) {
    c.on = sc.valid(c.rs);
    const int kk = l2only ? 0 : (c.on ? c.ks : nk - 1);
    c.st = c.base + (size_t)kk * 128;
    c.slot = slot;
  };
  auto dma = [&](Cur& c, unsigned img0, int u) {
    glds_sv(c.off[u], c.st, img0 + c.slot * AD_SLOT + (wid * 8 + u) * 1024);
  };
  auto end = [&](Cur& c, bool isA) {
    if (!c.on) return;
    if (++c.ks == nk) {
      c.ks = 0;
      ++c.rs;
      if (sc.valid(c.rs)) set_tile(c, isA, c.rs);
    }
  };

  const int fr = lane & 15, fk = lane >> 4;
  auto readA = [&](int slot, int kh, int i) -> uint4 {
    const int row = wr * 128 + i * 16 + fr;
    return *reinterpret_cast<const uint4*>(smem + slot * AD_SLOT + row * 128 + (((kh * 4 + fk) ^ (fr & 7)) << 4));
  };
  auto readB = [&](int slot, int kh, int j) -> uint4 {
    const int row = wc * 128 + j * 16 + fr;
    return *reinterpret_cast<const uint4*>(smem + AD_B0 + slot * AD_SLOT + row * 128 + (((kh * 4 + fk) ^ (fr & 7)) << 4));
  };

  const int ldc2 = p.ldc * 2;
  const int wrow = wr * 128;
  const int lcol = wc * 128 + (fk & 1) * 16 + (fk >> 1) * 8;
  const unsigned lane_voff = (unsigned)(fr * ldc2 + lcol * 2);
  const char* e_base = static_cast<const char*>(p.c);
  int e_rows = 0, e_cols = 0;
  auto set_epi = [&](int r) {
    int tm, tn, slice, bi;
    sc.tile(r, tm, tn, slice, bi);
    const int r0 = tm << 8, c0 = tn << 8;
    e_base = static_cast<const char*>(p.c) + (size_t)bi * p.sc * 2 + ((size_t)(r0 + wrow) * ldc2 + (size_t)c0 * 2);
    e_rows = (p.epi & EPI_NOSTORE) ? 0 : M - r0 - wrow;
    e_cols = N - c0;
  };
  auto store_pair = [&](const f32x4& x0, const f32x4& x1, int rb, int cb) {
    float v0[4], v1[4];
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v0[0]), "=v"(v0[1]), "=v"(v0[2]), "=v"(v0[3]) : "a"(x0[0]), "a"(x0[1]), "a"(x0[2]), "a"(x0[3]));
    asm volatile("v_accvgpr_read_b32 %0, %4\n\tv_accvgpr_read_b32 %1, %5\n\tv_accvgpr_read_b32 %2, %6\n\t"
                 "v_accvgpr_read_b32 %3, %7"
                 : "=v"(v1[0]), "=v"(v1[1]), "=v"(v1[2]), "=v"(v1[3]) : "a"(x1[0]), "a"(x1[1]), "a"(x1[2]), "a"(x1[3]));
    const int nbytes = __builtin_amdgcn_readfirstlane(max(min(e_rows - rb * 16, 16), 0) * ldc2);
    const unsigned voff = (lcol + cb * 16 < e_cols) ? lane_voff : 0x80000000u;
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    unsigned q00 = pk<T>(v0[0], v0[1]), q01 = pk<T>(v0[2], v0[3]);
    unsigned q10 = pk<T>(v1[0], v1[1]), q11 = pk<T>(v1[2], v1[3]);
    const auto s0 = __builtin_amdgcn_permlane16_swap(q00, q10, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(q01, q11, false, false);
    const size_t bp = (size_t)(e_base + (size_t)rb * 16 * ldc2);
    const unsigned blo = __builtin_amdgcn_readfirstlane((unsigned)bp);
    const unsigned bhi = __builtin_amdgcn_readfirstlane((unsigned)(bp >> 32));
    const auto rsc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((size_t)bhi << 32) | blo), (short)0,
                                                       nbytes, 0x00020000);
    const u32x4 qv{s0[0], s1[0], s0[1], s1[1]};
    if (p.epi & EPI_TEMPORAL) __builtin_amdgcn_raw_buffer_store_b128(qv, rsc, voff + cb * 32, 0, 0);
    else __builtin_amdgcn_raw_buffer_store_b128(qv, rsc, voff + cb * 32, 0, 2);
  };

  f32x4 acc[8][8];
  uint4 fa0[8], fb0[8], fa1[8], fb1[8];
  // phase A of K-tile t: MFMAs on k-half 0; k-half 1's 16 reads in a burst over groups 0-7; release
  // barrier at group 8 (A slot t % 3 and B slot t % 2 are fully read); B of tile t + 2 DMA'd over
  // groups 8-15
  auto phaseA = [&](auto ep_c, uint4 (&ca)[8], uint4 (&cb)[8], uint4 (&na)[8], uint4 (&nb)[8], int t) {
    constexpr bool EP = decltype(ep_c)::value;
    const int as = t % 3, bs = t & 1;
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s < 8) {
#pragma unroll
        for (int r = 2 * s; r < 2 * s + 2; ++r) {
          if (r & 1) nb[r >> 1] = readB(bs, 1, r >> 1);
          else na[r >> 1] = readA(as, 1, r >> 1);
        }
      }
      if (s == 8) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        bar();
        begin(cb_, bs);
      }
      if (s >= 8) dma(cb_, lds0 + AD_B0, s - 8);
      const int i = s >> 1, jb = (s & 1) * 4;
      if constexpr (EP) {
        store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
        store_pair(acc[i][jb + 2], acc[i][jb + 3], i, jb + 2);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = jb + q;
        if constexpr (EP) mma0<T>(acc[i][j], cb[j], ca[i]);
        else acc[i][j] = Mf<T>::mma(cb[j], ca[i], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
    }
    end(cb_, false);
  };
  // phase B of K-tile t: MFMAs on k-half 1; k-half 0 of tile t + 1 read one per group (consumption
  // order); A of tile t + 3 DMA'd over groups 0-7 into A slot t % 3
  auto phaseB = [&](uint4 (&ca)[8], uint4 (&cb)[8], uint4 (&na)[8], uint4 (&nb)[8], int t) {
    const int as = t % 3, as1 = (t + 1) % 3, bs1 = (t + 1) & 1;
    begin(ca_, as);
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      if (s == 0) na[0] = readA(as1, 0, 0);
      else if (s <= 8) nb[s - 1] = readB(bs1, 0, s - 1);
      else na[s - 8] = readA(as1, 0, s - 8);
      if (s < 8) dma(ca_, lds0, s);
      const int i = s >> 1, jb = (s & 1) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = jb + q;
        acc[i][j] = Mf<T>::mma(cb[j], ca[i], acc[i][j]);
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
    }
    end(ca_, true);
  };

  // ---- prologue: A tiles 0-2 into A slots 0-2, B tiles 0-1 into B slots 0-1 ----------------------
  set_tile(ca_, true, 0);
  set_tile(cb_, false, 0);
  for (int b = 0; b < 2; ++b) {
    begin(cb_, b);
#pragma unroll
    for (int u = 0; u < 8; ++u) dma(cb_, lds0 + AD_B0, u);
    end(cb_, false);
  }
  for (int a = 0; a < 3; ++a) {
    begin(ca_, a);
#pragma unroll
    for (int u = 0; u < 8; ++u) dma(ca_, lds0, u);
    end(ca_, true);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar();
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa0[i] = readA(0, 0, i);
    fb0[i] = readB(0, 0, i);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // boundary A(t) -> B(t): tile t + 1's B (DMA'd in A(t-1)) and A (in B(t-2)) have landed; younger:
  // A(t+2)'s 8 DMAs (B(t-1)), B(t+2)'s 8 (A(t)) and an epilogue phase's 32 stores
  int t = 0;
  for (int r = 0; sc.valid(r); ++r) {
    phaseA(std::true_type{}, fa0, fb0, fa1, fb1, t);
    asm volatile("s_waitcnt vmcnt(48)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    bar();
    set_epi(r);
    phaseB(fa1, fb1, fa0, fb0, t);
    ++t;
    for (int k = 1; k < nk; ++k, ++t) {
      phaseA(std::false_type{}, fa0, fb0, fa1, fb1, t);
      asm volatile("s_waitcnt vmcnt(16)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      bar();
      phaseB(fa1, fb1, fa0, fb0, t);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int jb = 0; jb < 8; jb += 2) store_pair(acc[i][jb], acc[i][jb + 1], i, jb);
}

template <typename T, bool BIAS, bool E>
int launch_e(const Args& a, int ako, int bko, int trans, int grid, hipStream_t st) {
  if (a.splits > 1) {   // TN only (weight gradients)
    if (!(ako && bko && !trans)) return (int)hipErrorInvalidValue;
    bool cs = false;
    if constexpr (E) {
      if (a.epi & EPI_COLSUM) {
        cs = true;
        hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, false, false, true, false, false, E, 0, true>), dim3(grid), dim3(256), 0, st, a);
      }
    }
    if (!cs) hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, false, false, true, false, false, E>), dim3(grid), dim3(256), 0, st, a);
    const long elems = (long)a.M * a.N;
    hipLaunchKernelGGL((splitk_reduce_kernel<T, BIAS>), dim3((unsigned)((elems / 8 + 255) / 256)), dim3(256), 0, st,
                       a.ws, static_cast<T*>(a.c), a.bias, a.M, a.N, a.ldc, a.splits);
    return (int)hipGetLastError();
  }
  if constexpr (std::is_same<T, bf16_t>::value && !BIAS && !E) {   // measurement build (EPI_SKIP)
    if ((a.epi & EPI_SKIP) && !ako && !bko && !trans) {
      hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, false, true>), dim3(grid), dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
  }
  if constexpr (!BIAS) {
    if ((a.epi & EPI_ADEEP) && !(a.epi & EPI_GELU) && !ako && !bko && !trans && a.K >= 256) {
      hipLaunchKernelGGL((gemm4a_kernel<T>), dim3(grid), dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
  }
  if ((a.epi & EPI_RING) && !ako && !bko && !trans && a.K >= 128 && a.K % 64 == 0) {
    if (a.epi & EPI_GELU)
      hipLaunchKernelGGL((gemm4r_kernel<T, BIAS, true>), dim3(grid), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((gemm4r_kernel<T, BIAS, false>), dim3(grid), dim3(256), 0, st, a);
    return (int)hipGetLastError();
  }
  if (!E && (a.epi & EPI_RSTAGE) && !ako && !bko && !trans) {
    if (a.epi & EPI_GELU)
      hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, true, true>), dim3(grid), dim3(256), 0, st, a);
    else
      hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, true>), dim3(grid), dim3(256), 0, st, a);
  } else if ((a.epi & EPI_GELU) && !ako && !bko && !trans)
    hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, true, false, E>), dim3(grid), dim3(256), 0, st, a);
  else if (a.epi & EPI_GELU)
    return (int)hipErrorInvalidValue;
  else if (!ako && !bko && !trans) {
    const int lv = E && std::is_same<T, bf16_t>::value
                       ? ((a.epi >> EPI_LATE_SHIFT) & 15) | ((a.epi & EPI_WSTAG) ? 16 : 0) | (((a.epi >> EPI_SPREAD_SHIFT) & 3) << 5)
                       : 0;
    if (lv == 40) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 40>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 72) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 72>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 104) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 104>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 47 && a.ws) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 47>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 8)hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 8>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 10) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 10>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 11) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 11>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 13) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 13>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 14) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 14>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 24) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 24>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 31 && a.ws) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 31>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 15 && a.ws) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 15>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 6) hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E, 6>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gemm4p_kernel<T, false, false, false, BIAS, false, false, false, false, E>), dim3(grid), dim3(256), 0, st, a);
  }
  else if (ako && bko && !trans) {
    // TN schedule variants (weight gradients): LV 8 (PIN) / 40 (PIN + SPREAD, the ops/gemm.py default:
    // 1.2-4.3 % on the GPT dW products, tools/tn_lv_ab.py)
    const int lv = E && std::is_same<T, bf16_t>::value && !BIAS
                       ? ((a.epi >> EPI_LATE_SHIFT) & 15) | (((a.epi >> EPI_SPREAD_SHIFT) & 3) << 5) : 0;
    if constexpr (E) {
      if (a.epi & EPI_COLSUM) {
        if (lv == 40) hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, BIAS, false, false, false, false, E, 40, true>), dim3(grid), dim3(256), 0, st, a);
        else if (lv == 8) hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, BIAS, false, false, false, false, E, 8, true>), dim3(grid), dim3(256), 0, st, a);
        else hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, BIAS, false, false, false, false, E, 0, true>), dim3(grid), dim3(256), 0, st, a);
        return (int)hipGetLastError();
      }
    }
    if (lv == 40) hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, BIAS, false, false, false, false, E, 40>), dim3(grid), dim3(256), 0, st, a);
    else if (lv == 8) hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, BIAS, false, false, false, false, E, 8>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((gemm4p_kernel<T, true, true, false, BIAS, false, false, false, false, E>), dim3(grid), dim3(256), 0, st, a);
  }
  else if (ako && !bko && trans)
    hipLaunchKernelGGL((gemm4p_kernel<T, true, false, true, BIAS, false, false, false, false, E>), dim3(grid), dim3(256), 0, st, a);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

template <typename T, bool BIAS>
int launch(const Args& a, int ako, int bko, int trans, int grid, hipStream_t st) {
  if (a.epi & EPI_EARLY) return launch_e<T, BIAS, true>(a, ako, bko, trans, grid, st);
  return launch_e<T, BIAS, false>(a, ako, bko, trans, grid, st);
}

}  // namespace g4p
}  // namespace pha

using namespace pha;

// C = A . B (+ bias[output column]) on the persistent epilogue-overlapped kernel.
// Layouts: (a_kouter, b_kouter, trans) = (0,0,0) NT, (1,1,0) TN, (1,0,1) NN as (W^T X^T)^T with the
// transposed store (C is then [N][ldc]). Requires K % 64 == 0; M, N, lda, ldb, ldc % 8 == 0; 16-B
// aligned base pointers; K-outer operand dims >= 8; per-panel byte offsets < 2^32; 256 output rows
// x ldc x 2 bytes < 2^31. grid: workgroups (<= tiles; the caller passes the CU count).
// batch > 1: C_i = A_i . B_i for i < batch, A_i = a + i * sa (elements; likewise b, c), all tiles of
// all items in one persistent launch (torch.bmm / paddle.bmm with per-batch right operands).
PHA_API int pha_gemm4p_batched(int dt, const void* a, const void* b, void* c, long M, long N, long K, long lda,
                               long ldb, long ldc, int a_kouter, int b_kouter, int trans, int epi, const float* bias,
                               int grid, int group_m, float* ws, int splits, hipStream_t stream, void* aux, int batch,
                               long sa, long sb, long sc) {
  if (M <= 0 || N <= 0 || K <= 0 || K % 64 || M % 8 || N % 8 || lda % 8 || ldb % 8 || ldc % 8)
    return (int)hipErrorInvalidValue;
  if ((a_kouter && M < 8) || (b_kouter && N < 8)) return (int)hipErrorInvalidValue;
  if (M > (1L << 30) || N > (1L << 30) || K > (1L << 30) || lda > (1L << 30) || ldb > (1L << 30))
    return (int)hipErrorInvalidValue;
  if ((a_kouter ? 64.0 * lda : 256.0 * lda) * 2 >= 4294967295.0 || (b_kouter ? 64.0 * ldb : 256.0 * ldb) * 2 >= 4294967295.0)
    return (int)hipErrorInvalidValue;
  if (256.0 * ldc * 2 >= 2147483647.0) return (int)hipErrorInvalidValue;
  if (((size_t)a | (size_t)b | (size_t)c) & 15) return (int)hipErrorInvalidValue;
  if ((epi & g4p::EPI_BIAS) && !bias) return (int)hipErrorInvalidValue;
  if ((epi & g4p::EPI_GELU) && (!aux || ((size_t)aux & 15) || splits > 1)) return (int)hipErrorInvalidValue;
  // COLSUM: TN, early schedule, no K-start stagger (the K sub-ranges of the tile rows must tile the
  // item's K-tiles in cursor order), fp32 partials [2 * splits * ceil(M / 256)][N] in aux
  if ((epi & g4p::EPI_COLSUM) && (!aux || ((size_t)aux & 3) || !a_kouter || !b_kouter || trans || batch != 1 ||
                                  !(epi & g4p::EPI_EARLY) || ((epi >> g4p::EPI_KSTAG_SHIFT) & 3) || (epi & g4p::EPI_GELU)))
    return (int)hipErrorInvalidValue;
  if (splits < 1) splits = 1;
  if (batch < 1 || (batch > 1 && (splits > 1 || (epi & g4p::EPI_GELU) || (sa | sb | sc) % 8 || sa < 0 || sb < 0 || sc < 0)))
    return (int)hipErrorInvalidValue;
  if ((double)batch * ((M + 255) / 256) * ((N + 255) / 256) >= 2147483647.0) return (int)hipErrorInvalidValue;
  if (splits > 1 && (!ws || (K / 64) % splits || !a_kouter || !b_kouter || trans || (size_t)ws & 15))
    return (int)hipErrorInvalidValue;
  const long tiles = ((M + 255) / 256) * ((N + 255) / 256) * splits * batch;
  if (grid <= 0 || grid > tiles) grid = (int)tiles;
  if (group_m <= 0) group_m = 4;
  g4p::Args p{a, b, c, bias, (int)M, (int)N, (int)K, (int)lda, (int)ldb, (int)ldc, epi, group_m, ws, splits, aux,
              batch, sa, sb, sc};
  const bool bs = epi & g4p::EPI_BIAS;
  if (dt == kBF16) return bs ? g4p::launch<bf16_t, true>(p, a_kouter, b_kouter, trans, grid, stream)
                             : g4p::launch<bf16_t, false>(p, a_kouter, b_kouter, trans, grid, stream);
  if (dt == kF16) return bs ? g4p::launch<half_t, true>(p, a_kouter, b_kouter, trans, grid, stream)
                            : g4p::launch<half_t, false>(p, a_kouter, b_kouter, trans, grid, stream);
  return (int)hipErrorInvalidValue;
}

PHA_API int pha_gemm4p(int dt, const void* a, const void* b, void* c, long M, long N, long K, long lda, long ldb,
                       long ldc, int a_kouter, int b_kouter, int trans, int epi, const float* bias, int grid,
                       int group_m, float* ws, int splits, hipStream_t stream, void* aux) {
  return pha_gemm4p_batched(dt, a, b, c, M, N, K, lda, ldb, ldc, a_kouter, b_kouter, trans, epi, bias, grid, group_m,
                            ws, splits, stream, aux, 1, 0, 0, 0);
}
