// bf16/fp16 MFMA GEMM and implicit-GEMM convolution for gfx950 (reference behaviour:
// phi/kernels/gpu/matmul_kernel.cu, conv_kernel.cu / conv_grad_kernel.cu — cuDNN there).
//
//   C[M, N] (row-major, ldc) = sum_k A[m, k] * B[k, n]   (+ bias[n]) (+ relu/gelu)
//
// Operand staging modes (the GEMM is the same; only the tile loaders differ):
//   A_ROW : A[m][k] at a[m*lda + k]            (K contiguous)
//   A_COL : A[m][k] at a[k*lda + m]            (M contiguous — e.g. dY^T in weight grads)
//   A_CONV: A[m][k] = x[pixel(m, tap(k))][cin(k)] NHWC implicit im2col (zero padding)
//   B_ROW : B[k][n] at b[n*ldb + k]            (K contiguous, i.e. "B^T" storage)
//   B_COL : B[k][n] at b[k*ldb + n]            (N contiguous)
//   B_CONV: B[k][n] = x[pixel(k, tap(n))][cin(n)] (weight-grad: k runs over output pixels)
//
// Geometry: 128x128x64 block tile, 256 threads = 4 waves (2x2), 64x64 per wave as 2x2
// mfma_f32_32x32x16_bf16 tiles. LDS holds K-contiguous [row][64] images (128-B rows, 16-B
// chunks XOR-swizzled by row&7 so the 32-row ds_read_b128 fragment reads are 2-way at most),
// double buffered; the next K-tile is fetched into registers while the current one is
// multiplied (register staging, one barrier per K-tile). Column-major operands (A_COL,
// B_COL, B_CONV) are transposed in registers: each thread loads a 4(k)x8(m) block as four
// 16-B vectors and writes eight 8-B rows. Grid: 1-D over output tiles, remapped so each XCD
// gets a contiguous, GROUP_M-ordered slab of tiles (L2 reuse of A/B panels per XCD), plus
// grid.y = split-K slices writing fp32 partials that a second kernel reduces.
#include "common.h"

namespace pha {
namespace gemm {

enum AMode { A_ROW = 0, A_COL = 1, A_CONV = 2 };
enum BMode { B_ROW = 0, B_COL = 1, B_CONV = 2 };
enum Epi { E_NONE = 0, E_RELU = 1, E_GELU = 2 };

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int GROUP_M = 8;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct ConvGeo {
  int N, H, W, C;          // input NHWC
  int OH, OW;              // output grid
  int KH, KW;              // taps
  int sh, sw, ph, pw, dh, dw;
};

struct Params {
  const void* a;
  const void* b;
  void* c;        // output (T) or fp32 partials when split-K
  const float* bias;
  long M, N, K;
  long lda, ldb, ldc;
  int splitk;     // number of K slices (grid.y)
  long k_per_split;
  ConvGeo g;      // for A_CONV / B_CONV
  const void* zero;  // 16-B aligned zero page for padding taps
};

// -------------------------------------------------------------------------- LDS addressing
// image: [128 rows][64 k] bf16, 128-B rows of 8 16-B chunks; chunk ^= row & 7
__device__ __forceinline__ int lds_off(int row, int k) {  // byte offset of element (row, k), k%4==0 ok
  const int chunk = (k >> 3) ^ (row & 7);
  return row * 128 + chunk * 16 + (k & 7) * 2;
}

// -------------------------------------------------------------------------- tile loaders
// Row-mode (K-contiguous) tile: 128 rows x 64 k = 1024 chunks of 16 B, 4 per thread.
struct RowRegs { uint4 v[4]; };
// Col-mode (M/N-contiguous) tile: 64 k x 128 cols = 256 blocks of 4k x 8col, 1 per thread.
struct ColRegs { uint4 v[4]; };

template <typename T>
__device__ __forceinline__ const T* conv_pixel(const ConvGeo& g, const T* x, int n, int oh, int ow, int tap,
                                               const T* zero) {
  const int kh = tap / g.KW, kw = tap - (tap / g.KW) * g.KW;
  const int ih = oh * g.sh - g.ph + kh * g.dh;
  const int iw = ow * g.sw - g.pw + kw * g.dw;
  if ((unsigned)ih >= (unsigned)g.H || (unsigned)iw >= (unsigned)g.W) return zero;
  return x + (((long)n * g.H + ih) * g.W + iw) * g.C;
}

// A_ROW / B_ROW: plain K-contiguous rows
template <typename T>
__device__ __forceinline__ void load_row_plain(RowRegs& r, const T* base, long ld, long row0, long rows, long k0,
                                               long kend) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = threadIdx.x + NT * j;
    const int row = i >> 3, ch = i & 7;
    const long gr = row0 + row, gk = k0 + ch * 8;
    if (gr < rows && gk < kend)
      r.v[j] = *reinterpret_cast<const uint4*>(base + gr * ld + gk);
    else
      r.v[j] = make_uint4(0, 0, 0, 0);
  }
}

// A_CONV: row = output pixel, k chunk = 8 channels of one tap (requires C % 8 == 0)
struct ConvRows { int n[4], oh[4], ow[4]; bool ok[4]; };

__device__ __forceinline__ void conv_rows_init(ConvRows& cr, const ConvGeo& g, long row0, long M) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = threadIdx.x + NT * j;
    const long m = row0 + (i >> 3);
    cr.ok[j] = m < M;
    const long mm = cr.ok[j] ? m : 0;
    const int hw = g.OH * g.OW;
    cr.n[j] = (int)(mm / hw);
    const int rem = (int)(mm - (long)cr.n[j] * hw);
    cr.oh[j] = rem / g.OW;
    cr.ow[j] = rem - cr.oh[j] * g.OW;
  }
}

template <typename T>
__device__ __forceinline__ void load_row_conv(RowRegs& r, const T* x, const ConvGeo& g, const ConvRows& cr, long k0,
                                              long K, const T* zero) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = threadIdx.x + NT * j;
    const int ch = i & 7;
    const long gk = k0 + ch * 8;
    if (cr.ok[j] && gk < K) {
      const int tap = (int)(gk / g.C);
      const int cin = (int)(gk - (long)tap * g.C);
      const T* p = conv_pixel(g, x, cr.n[j], cr.oh[j], cr.ow[j], tap, zero);
      r.v[j] = p == zero ? make_uint4(0, 0, 0, 0) : *reinterpret_cast<const uint4*>(p + cin);
    } else {
      r.v[j] = make_uint4(0, 0, 0, 0);
    }
  }
}

// Column-major plain: element (k, col) at base[k*ld + col]; 4 k rows x 8 cols per thread.
template <typename T>
__device__ __forceinline__ void load_col_plain(ColRegs& r, const T* base, long ld, long col0, long cols, long k0,
                                               long kend) {
  const int cb = threadIdx.x & 15, kb = threadIdx.x >> 4;  // 16 col-blocks x 16 k-blocks
  const long gc = col0 + cb * 8;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long gk = k0 + kb * 4 + q;
    if (gk < kend && gc < cols)
      r.v[q] = *reinterpret_cast<const uint4*>(base + gk * ld + gc);
    else
      r.v[q] = make_uint4(0, 0, 0, 0);
  }
}

// B_CONV: element (k = output pixel m, n = (tap, cin)) = x[pixel(m, tap)][cin]
template <typename T>
__device__ __forceinline__ void load_col_conv(ColRegs& r, const T* x, const ConvGeo& g, long col0, long cols, long k0,
                                              long kend, const T* zero) {
  const int cb = threadIdx.x & 15, kb = threadIdx.x >> 4;
  const long gc = col0 + cb * 8;
  const int tap = (int)(gc / g.C);
  const int cin = (int)(gc - (long)tap * g.C);
  const int hw = g.OH * g.OW;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const long m = k0 + kb * 4 + q;
    if (m < kend && gc < cols) {
      const int n = (int)(m / hw);
      const int rem = (int)(m - (long)n * hw);
      const int oh = rem / g.OW, ow = rem - (rem / g.OW) * g.OW;
      const T* p = conv_pixel(g, x, n, oh, ow, tap, zero);
      r.v[q] = p == zero ? make_uint4(0, 0, 0, 0) : *reinterpret_cast<const uint4*>(p + cin);
    } else {
      r.v[q] = make_uint4(0, 0, 0, 0);
    }
  }
}

__device__ __forceinline__ void store_row(char* lds, const RowRegs& r) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int i = threadIdx.x + NT * j;
    const int row = i >> 3, ch = i & 7;
    *reinterpret_cast<uint4*>(lds + lds_off(row, ch * 8)) = r.v[j];
  }
}

// transpose the 4(k) x 8(col) block into 8 rows of 4 k (8 bytes each)
__device__ __forceinline__ void store_col(char* lds, const ColRegs& r) {
  const int cb = threadIdx.x & 15, kb = threadIdx.x >> 4;
  const uint16_t* e0 = reinterpret_cast<const uint16_t*>(&r.v[0]);
  const uint16_t* e1 = reinterpret_cast<const uint16_t*>(&r.v[1]);
  const uint16_t* e2 = reinterpret_cast<const uint16_t*>(&r.v[2]);
  const uint16_t* e3 = reinterpret_cast<const uint16_t*>(&r.v[3]);
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    uint2 w;
    w.x = (uint32_t)e0[c] | ((uint32_t)e1[c] << 16);
    w.y = (uint32_t)e2[c] | ((uint32_t)e3[c] << 16);
    *reinterpret_cast<uint2*>(lds + lds_off(cb * 8 + c, kb * 4)) = w;
  }
}

template <typename T> struct Mfma;
template <> struct Mfma<bf16_t> {
  static __device__ __forceinline__ f32x16 run(const uint4& a, const uint4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(*reinterpret_cast<const bf16x8*>(&a),
                                                   *reinterpret_cast<const bf16x8*>(&b), c, 0, 0, 0);
  }
};
template <> struct Mfma<half_t> {
  static __device__ __forceinline__ f32x16 run(const uint4& a, const uint4& b, const f32x16& c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(*reinterpret_cast<const f16x8*>(&a),
                                                  *reinterpret_cast<const f16x8*>(&b), c, 0, 0, 0);
  }
};

__device__ __forceinline__ float gelu_f(float x) {
  return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
}

// bijective XCD remap + GROUP_M raster
__device__ __forceinline__ void tile_coords(long tiles_m, long tiles_n, long& tm, long& tn) {
  const long nwg = tiles_m * tiles_n;
  const long orig = blockIdx.x;
  const long nx = 8;
  long wgid = orig;
  if (nwg > nx) {
    const long q = nwg / nx, r = nwg % nx, xcd = orig % nx, idx = orig / nx;
    wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const long group = GROUP_M * tiles_n;
  const long gid = wgid / group;
  const long first_m = gid * GROUP_M;
  const long gsize = (tiles_m - first_m) < GROUP_M ? (tiles_m - first_m) : GROUP_M;
  tm = first_m + (wgid % group) % gsize;
  tn = (wgid % group) / gsize;
}

template <typename T, int AM, int BMd, int EP, bool SPLIT>
__global__ __launch_bounds__(NT, 2) void gemm_kernel(Params p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * BM * BK * 2];  // [buf][A|B] 64 KiB
  long tm, tn;
  const long tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  tile_coords(tiles_m, tiles_n, tm, tn);
  const long row0 = tm * BM, col0 = tn * BN;
  const long kbeg = SPLIT ? blockIdx.y * p.k_per_split : 0;
  const long kend = SPLIT ? (kbeg + p.k_per_split < p.K ? kbeg + p.k_per_split : p.K) : p.K;
  const int ntile = kend > kbeg ? (int)((kend - kbeg + BK - 1) / BK) : 0;

  const T* A = reinterpret_cast<const T*>(p.a);
  const T* B = reinterpret_cast<const T*>(p.b);
  const T* zero = reinterpret_cast<const T*>(p.zero);
  ConvRows cr;
  if (AM == A_CONV) conv_rows_init(cr, p.g, row0, p.M);

  RowRegs ra, rb;
  ColRegs ca, cb;
  auto fetch = [&](long k0) {
    if (AM == A_ROW) load_row_plain(ra, A, p.lda, row0, p.M, k0, kend);
    else if (AM == A_CONV) load_row_conv(ra, A, p.g, cr, k0, kend, zero);
    else load_col_plain(ca, A, p.lda, row0, p.M, k0, kend);
    if (BMd == B_ROW) load_row_plain(rb, B, p.ldb, col0, p.N, k0, kend);
    else if (BMd == B_COL) load_col_plain(cb, B, p.ldb, col0, p.N, k0, kend);
    else load_col_conv(cb, B, p.g, col0, p.N, k0, kend, zero);
  };
  auto stash = [&](int buf) {
    char* la = smem + buf * (2 * BM * BK * 2);
    char* lb = la + BM * BK * 2;
    if (AM == A_COL) store_col(la, ca); else store_row(la, ra);
    if (BMd == B_ROW) store_row(lb, rb); else store_col(lb, cb);
  };

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int fr = lane & 31, fh = lane >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (ntile > 0) {
    fetch(kbeg);
    stash(0);
    __syncthreads();
  }
  for (int t = 0; t < ntile; ++t) {
    const int cur = t & 1;
    if (t + 1 < ntile) fetch(kbeg + (long)(t + 1) * BK);
    const char* la = smem + cur * (2 * BM * BK * 2);
    const char* lb = la + BM * BK * 2;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      uint4 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        af[i] = *reinterpret_cast<const uint4*>(la + lds_off(wm * 64 + i * 32 + fr, s * 16 + fh * 8));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(lb + lds_off(wn * 64 + j * 32 + fr, s * 16 + fh * 8));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = Mfma<T>::run(af[i], bfr[j], acc[i][j]);
    }
    if (t + 1 < ntile) {
      stash(cur ^ 1);
    }
    __syncthreads();
  }

  // epilogue: acc[i][j][r] -> C[row0 + wm*64 + i*32 + (r&3) + 8*(r>>2) + 4*fh][col0 + wn*64 + j*32 + fr]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long col = col0 + wn * 64 + j * 32 + fr;
      if (col >= p.N) continue;
      float bv = 0.f;
      if (!SPLIT && p.bias) bv = p.bias[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const long row = row0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * fh;
        if (row >= p.M) continue;
        float v = acc[i][j][r];
        if (SPLIT) {
          reinterpret_cast<float*>(p.c)[(long)blockIdx.y * p.M * p.N + row * p.N + col] = v;
        } else {
          v += bv;
          if (EP == E_RELU) v = fmaxf(v, 0.f);
          if (EP == E_GELU) v = gelu_f(v);
          Cvt<T>::st(reinterpret_cast<T*>(p.c), row * p.ldc + col, v);
        }
      }
    }
  }
}

// split-K reduction: out[m, n] = sum_s part[s, m, n] (+bias) (+act), written with ldc.
template <typename T, int EP>
__global__ void splitk_reduce_kernel(const float* __restrict__ part, int splits, long M, long N, const float* bias,
                                     T* __restrict__ out, long ldc) {
  const long total = M * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    for (int s = 0; s < splits; ++s) v += part[(long)s * total + i];
    const long m = i / N, n = i - m * N;
    if (bias) v += bias[n];
    if (EP == E_RELU) v = fmaxf(v, 0.f);
    if (EP == E_GELU) v = gelu_f(v);
    Cvt<T>::st(out, m * ldc + n, v);
  }
}

template <typename T, int AM, int BMd, int EP>
int launch_t(const Params& p0, float* ws, hipStream_t s) {
  Params p = p0;
  const long tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  if (p.splitk <= 1) {
    hipLaunchKernelGGL((gemm_kernel<T, AM, BMd, EP, false>), dim3((unsigned)tiles, 1), dim3(NT), 0, s, p);
    return (int)hipGetLastError();
  }
  void* out = p.c;
  p.c = ws;
  hipLaunchKernelGGL((gemm_kernel<T, AM, BMd, E_NONE, true>), dim3((unsigned)tiles, p.splitk), dim3(NT), 0, s, p);
  long blocks = (p.M * p.N + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL((splitk_reduce_kernel<T, EP>), dim3((unsigned)blocks), dim3(256), 0, s, ws, p.splitk, p.M, p.N,
                     p.bias, (T*)out, p.ldc);
  return (int)hipGetLastError();
}

template <typename T>
int dispatch(int am, int bm, int ep, const Params& p, float* ws, hipStream_t s) {
#define PHA_GEMM_EP(AM_, BM_)                                                   \
  switch (ep) {                                                                 \
    case E_NONE: return launch_t<T, AM_, BM_, E_NONE>(p, ws, s);               \
    case E_RELU: return launch_t<T, AM_, BM_, E_RELU>(p, ws, s);               \
    case E_GELU: return launch_t<T, AM_, BM_, E_GELU>(p, ws, s);               \
    default: return (int)hipErrorInvalidValue;                                  \
  }
  if (am == A_ROW && bm == B_ROW) { PHA_GEMM_EP(A_ROW, B_ROW) }
  if (am == A_ROW && bm == B_COL) { PHA_GEMM_EP(A_ROW, B_COL) }
  if (am == A_COL && bm == B_ROW) { PHA_GEMM_EP(A_COL, B_ROW) }
  if (am == A_COL && bm == B_COL) { PHA_GEMM_EP(A_COL, B_COL) }
  if (am == A_CONV && bm == B_ROW) { PHA_GEMM_EP(A_CONV, B_ROW) }
  if (am == A_COL && bm == B_CONV) { PHA_GEMM_EP(A_COL, B_CONV) }
#undef PHA_GEMM_EP
  return (int)hipErrorInvalidValue;
}

}  // namespace gemm
}  // namespace pha

using namespace pha;
using namespace pha::gemm;

// dt: 1 = bf16, 2 = fp16. ws: fp32 workspace of splitk*M*N floats when splitk > 1.
// conv: int[12] = {N,H,W,C, OH,OW, KH,KW, sh,sw, ph,pw} (+ dilation dh,dw in conv[12..13]).
PHA_API int pha_gemm(int dt, int amode, int bmode, int epi, const void* a, long lda, const void* b, long ldb,
                     void* c, long ldc, const float* bias, long M, long N, long K, int splitk, float* ws,
                     const int* conv, const void* zero, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  // K must be a multiple of 8 only when it is a contiguous (16-byte vector) dimension
  if ((amode == A_ROW || amode == A_CONV || bmode == B_ROW) && K % 8 != 0) return (int)hipErrorInvalidValue;
  Params p{};
  p.a = a; p.b = b; p.c = c; p.bias = bias;
  p.M = M; p.N = N; p.K = K; p.lda = lda; p.ldb = ldb; p.ldc = ldc;
  p.splitk = splitk < 1 ? 1 : splitk;
  p.k_per_split = ((K + p.splitk - 1) / p.splitk + BK - 1) / BK * BK;
  p.zero = zero;
  if (conv) {
    p.g = ConvGeo{conv[0], conv[1], conv[2], conv[3], conv[4], conv[5], conv[6], conv[7], conv[8], conv[9], conv[10],
                  conv[11], conv[12], conv[13]};
    if (p.g.C % 8 != 0) return (int)hipErrorInvalidValue;
  }
  if ((amode == A_COL && M % 8 != 0) || ((bmode == B_COL || bmode == B_CONV) && N % 8 != 0))
    return (int)hipErrorInvalidValue;
  if (p.splitk > 1 && !ws) return (int)hipErrorInvalidValue;
  if (dt == kBF16) return dispatch<bf16_t>(amode, bmode, epi, p, ws, s);
  if (dt == kF16) return dispatch<half_t>(amode, bmode, epi, p, ws, s);
  return (int)hipErrorInvalidValue;
}
