// Channels-last (NHWC) batch norm for training, with optional fused residual-add + ReLU
// (reference behaviour: phi/kernels/gpu/batch_norm_kernel.cu, batch_norm_grad_kernel.cu and
// fluid/operators/fused/fused_bn_add_activation_op.cu).
//
// x is viewed as [M, C] (M = N*H*W rows, C contiguous). Each thread owns 8 consecutive
// channels (one 16-byte vector for bf16/fp16) of a row, so a row of C channels is read by
// C/8 adjacent lanes and a wave reads 64*16 B contiguous — fully coalesced for every C.
//
// Forward (3 launches, 2 reads + 1 write of x):
//   bn_stats   : per-block partial sums of (x - shift), (x - shift)^2 with one per-channel
//                shift (row 0), so partials add exactly and the variance avoids the
//                E[x^2]-E[x]^2 cancellation at 3M rows/channel.
//   bn_finalize: 1024-thread sum of the block partials -> mean / inv-std, running-stat update (Paddle momentum
//                semantics), per-channel scale = g*istd and shift = b - mean*scale.
//   bn_apply   : y = relu?(x*scale + shift (+ residual)).
// Backward (3 launches, reads dy/x(/y) twice, writes dx (+ d_residual)):
//   bn_bwd_reduce  : sum(dy') and sum(dy'*(x-mean)), dy' = relu-masked dy (mask from saved y).
//   bn_bwd_finalize: dgamma, dbeta and the affine dx = A*dy' + B*x + C0 coefficients.
//   bn_bwd_apply   : dx (+ d_residual = dy').
#include "common.h"

namespace pha {
namespace {

constexpr int kThreads = 256;
constexpr int kMaxVecTile = 256;  // vectors (of 8 channels) per channel tile -> 2048 channels

struct Geo {
  int cv;        // vectors per row = C/8
  int cvt;       // vectors in this tile
  int rows_it;   // rows handled per block iteration
  int v;         // this thread's vector index within the row (global)
  int r;         // this thread's row offset within an iteration
  bool active;
};

__device__ __forceinline__ Geo geo(int C) {
  Geo g;
  g.cv = C >> 3;
  const int tile0 = blockIdx.y * kMaxVecTile;
  g.cvt = min(kMaxVecTile, g.cv - tile0);
  g.rows_it = kThreads / g.cvt;
  g.r = threadIdx.x / g.cvt;
  g.v = tile0 + threadIdx.x % g.cvt;
  g.active = g.r < g.rows_it;
  return g;
}

// ------------------------------------------------------------------------- forward stats
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_stats_kernel(const T* __restrict__ x, long M, int C,
                                                            float* __restrict__ part) {
  // Sums of (x - shift) and (x - shift)^2 with ONE shift per channel (row 0's value) for every
  // thread and block, so partials combine by plain addition; |mean - shift| ~ std keeps the
  // variance free of the E[x^2] - E[x]^2 cancellation.
  __shared__ float sm[2][kThreads][8];
  const Geo g = geo(C);
  float s1[8], s2[8], x0[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s2[i] = x0[i] = 0.f;
  if (g.active) {
    Vec8<T>::ld(x + g.v * 8, x0);
    const long stride = (long)gridDim.x * g.rows_it;
    for (long row = (long)blockIdx.x * g.rows_it + g.r; row < M; row += stride) {
      float v[8];
      Vec8<T>::ld(x + row * C + g.v * 8, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[i] - x0[i];
        s1[i] += d;
        s2[i] = fmaf(d, d, s2[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sm[0][threadIdx.x][i] = s1[i];
    sm[1][threadIdx.x][i] = s2[i];
  }
  __syncthreads();
  if (g.active && g.r == 0) {
    for (int rr = 1; rr < g.rows_it; ++rr) {
      const int t = rr * g.cvt + threadIdx.x;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s1[i] += sm[0][t][i];
        s2[i] += sm[1][t][i];
      }
    }
    float* p = part + (long)blockIdx.x * 2 * C + g.v * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      p[i] = s1[i];
      p[C + i] = s2[i];
    }
  }
}

// Sum `nblk` partial rows of [2][C] floats: block = 64 channels x 16 slices (1024 threads).
__device__ __forceinline__ void sum_partials(const float* __restrict__ part, int nblk, int C, int c, float& a,
                                             float& b, float (*sm)[2][64]) {
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  a = b = 0.f;
  if (c < C) {
    for (int k = sl; k < nblk; k += 16) {
      a += part[(long)k * 2 * C + c];
      b += part[(long)k * 2 * C + C + c];
    }
  }
  sm[sl][0][cl] = a;
  sm[sl][1][cl] = b;
  __syncthreads();
  a = b = 0.f;
  for (int k = 0; k < 16; ++k) {
    a += sm[k][0][cl];
    b += sm[k][1][cl];
  }
}

// First stage for many partial rows: block (channel block, g) sums rows [g*rows_per, +rows_per)
// of `part` into out[g][2][C] (64 channels x 16 slices, four independent accumulators per thread
// so the loads overlap), so the finalize kernels read <= 64 rows instead of thousands.
__global__ __launch_bounds__(1024) void bn_partial_reduce_kernel(const float* __restrict__ part, int nblk, int C,
                                                                 int rows_per, float* __restrict__ out) {
  __shared__ float sm[16][2][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  const int r0 = blockIdx.y * rows_per, r1 = min(nblk, r0 + rows_per);
  float a[4] = {0.f, 0.f, 0.f, 0.f}, b[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
    int k = r0 + sl, u = 0;
    for (; k < r1; k += 16, u = (u + 1) & 3) {
      a[u] += part[(long)k * 2 * C + c];
      b[u] += part[(long)k * 2 * C + C + c];
    }
  }
  sm[sl][0][cl] = (a[0] + a[1]) + (a[2] + a[3]);
  sm[sl][1][cl] = (b[0] + b[1]) + (b[2] + b[3]);
  __syncthreads();
  if (sl == 0 && c < C) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k < 16; ++k) {
      sa += sm[k][0][cl];
      sb += sm[k][1][cl];
    }
    out[(long)blockIdx.y * 2 * C + c] = sa;
    out[(long)blockIdx.y * 2 * C + C + c] = sb;
  }
}

__global__ __launch_bounds__(1024) void bn_finalize_kernel(const float* __restrict__ part, int nblk, int C, long M,
                                                           const void* __restrict__ x, int dt, float eps,
                                                           float momentum, const float* __restrict__ w,
                                                           const float* __restrict__ b, float* __restrict__ run_mean,
                                                           float* __restrict__ run_var, float* __restrict__ save_mean,
                                                           float* __restrict__ save_istd, float* __restrict__ scale,
                                                           float* __restrict__ shift) {
  __shared__ float sm[16][2][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float s1, s2;
  sum_partials(part, nblk, C, c, s1, s2, sm);
  if (threadIdx.x >= 64 || c >= C) return;
  // x == nullptr: unshifted partial sums (from the producing convolution's epilogue)
  const float x0 = !x ? 0.f : dt == kF32 ? ((const float*)x)[c]
                   : dt == kBF16 ? bf16_to_f32(((const uint16_t*)x)[c]) : (float)((const _Float16*)x)[c];
  const float n = (float)M;
  const float dm = s1 / n;
  const float mean = x0 + dm;
  const float var = fmaxf(s2 / n - dm * dm, 0.f);
  const float istd = rsqrtf(var + eps);
  save_mean[c] = mean;
  save_istd[c] = istd;
  if (run_mean) {
    const float unbiased = n > 1.f ? var * n / (n - 1.f) : var;
    run_mean[c] = run_mean[c] * momentum + mean * (1.f - momentum);
    run_var[c] = run_var[c] * momentum + unbiased * (1.f - momentum);
  }
  const float gw = w ? w[c] : 1.f, gb = b ? b[c] : 0.f;
  scale[c] = gw * istd;
  shift[c] = gb - mean * gw * istd;
}

// ------------------------------------------------------------------------- forward apply
template <typename T, bool kRes, bool kRelu>
__global__ __launch_bounds__(kThreads) void bn_apply_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                            const float* __restrict__ scale,
                                                            const float* __restrict__ shift, T* __restrict__ y,
                                                            long nvec, int cv) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * 8;
    float v[8];
    Vec8<T>::ld(x + i * 8, v);
    const float4 s0 = *reinterpret_cast<const float4*>(scale + c), s1 = *reinterpret_cast<const float4*>(scale + c + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(shift + c), h1 = *reinterpret_cast<const float4*>(shift + c + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
    float r[8];
    if (kRes) Vec8<T>::ld(res + i * 8, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float o = fmaf(v[k], sc[k], sh[k]);
      if (kRes) o += r[k];
      if (kRelu) o = fmaxf(o, 0.f);
      v[k] = o;
    }
    Vec8<T>::st(y + i * 8, v);
  }
}

// ------------------------------------------------------------------------- backward
// ReLU mask: from the saved output y, or — y == nullptr, no residual was added — recomputed from x
// as x*scale + shift > 0 with the forward's affine (aff = [scale | shift]); y > 0 <=> that > 0, and
// the backward then reads two tensors per pass instead of three.
template <typename T>
__device__ __forceinline__ void relu_mask(const T* __restrict__ y, const float* __restrict__ aff, int C, long off, int c,
                                          const float (&xv)[8], float (&d)[8]) {
  if (y) {
    float yv[8];
    Vec8<T>::ld(y + off, yv);
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = yv[i] > 0.f ? d[i] : 0.f;
  } else {
    const float4 s0 = *reinterpret_cast<const float4*>(aff + c), s1 = *reinterpret_cast<const float4*>(aff + c + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(aff + C + c), h1 = *reinterpret_cast<const float4*>(aff + C + c + 4);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = fmaf(xv[i], sc[i], sh[i]) > 0.f ? d[i] : 0.f;
  }
}

template <typename T, bool kRelu>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                 const T* __restrict__ y,
                                                                 const float* __restrict__ mean, long M, int C,
                                                                 float* __restrict__ part,
                                                                 const float* __restrict__ aff) {
  __shared__ float sm[2][kThreads][8];
  const Geo g = geo(C);
  float sdy[8], sdx[8], mu[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sdy[i] = sdx[i] = 0.f;
  if (g.active) {
    const float4 m0 = *reinterpret_cast<const float4*>(mean + g.v * 8);
    const float4 m1 = *reinterpret_cast<const float4*>(mean + g.v * 8 + 4);
    mu[0] = m0.x; mu[1] = m0.y; mu[2] = m0.z; mu[3] = m0.w;
    mu[4] = m1.x; mu[5] = m1.y; mu[6] = m1.z; mu[7] = m1.w;
    const long stride = (long)gridDim.x * g.rows_it;
    for (long row = (long)blockIdx.x * g.rows_it + g.r; row < M; row += stride) {
      const long off = row * C + g.v * 8;
      float d[8], xv[8];
      Vec8<T>::ld(dy + off, d);
      Vec8<T>::ld(x + off, xv);
      if (kRelu) relu_mask<T>(y, aff, C, off, g.v * 8, xv, d);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sdy[i] += d[i];
        sdx[i] = fmaf(d[i], xv[i] - mu[i], sdx[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sm[0][threadIdx.x][i] = sdy[i];
    sm[1][threadIdx.x][i] = sdx[i];
  }
  __syncthreads();
  if (g.active && g.r == 0) {
    for (int rr = 1; rr < g.rows_it; ++rr) {
      const int t = rr * g.cvt + threadIdx.x;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sdy[i] += sm[0][t][i];
        sdx[i] += sm[1][t][i];
      }
    }
    float* p = part + (long)blockIdx.x * 2 * C + g.v * 8;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      p[i] = sdy[i];
      p[C + i] = sdx[i];
    }
  }
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(const float* __restrict__ part, int nblk, int C,
                                                               float inv_m, const float* __restrict__ w,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ istd, float* __restrict__ dw,
                                                               float* __restrict__ db, float* __restrict__ coef) {
  __shared__ float sm[16][2][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float sdy, sdx;
  sum_partials(part, nblk, C, c, sdy, sdx, sm);
  if (threadIdx.x >= 64 || c >= C) return;
  const float is = istd[c], gw = w ? w[c] : 1.f;
  if (dw) dw[c] = sdx * is;
  if (db) db[c] = sdy;
  const float A = gw * is;
  const float B = -gw * is * is * is * sdx * inv_m;
  coef[c] = A;
  coef[C + c] = B;
  coef[2 * C + c] = -A * sdy * inv_m - B * mean[c];
}

template <typename T, bool kRelu, bool kDres>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                                const T* __restrict__ y,
                                                                const float* __restrict__ coef, T* __restrict__ dx,
                                                                T* __restrict__ dres, long nvec, int cv,
                                                                const float* __restrict__ aff) {
  const int C = cv * 8;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nvec; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i % cv) * 8;
    float d[8], xv[8];
    Vec8<T>::ld(dy + i * 8, d);
    Vec8<T>::ld(x + i * 8, xv);
    if (kRelu) relu_mask<T>(y, aff, C, i * 8, c, xv, d);
    if (kDres) Vec8<T>::st(dres + i * 8, d);
    float A[8], B[8], C0[8], o[8];
    *reinterpret_cast<float4*>(A) = *reinterpret_cast<const float4*>(coef + c);
    *reinterpret_cast<float4*>(A + 4) = *reinterpret_cast<const float4*>(coef + c + 4);
    *reinterpret_cast<float4*>(B) = *reinterpret_cast<const float4*>(coef + C + c);
    *reinterpret_cast<float4*>(B + 4) = *reinterpret_cast<const float4*>(coef + C + c + 4);
    *reinterpret_cast<float4*>(C0) = *reinterpret_cast<const float4*>(coef + 2 * C + c);
    *reinterpret_cast<float4*>(C0 + 4) = *reinterpret_cast<const float4*>(coef + 2 * C + c + 4);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(A[k], d[k], fmaf(B[k], xv[k], C0[k]));
    Vec8<T>::st(dx + i * 8, o);
  }
}

int grid_rows(long M, int C, int* tiles) {
  const int cv = C / 8;
  *tiles = (cv + kMaxVecTile - 1) / kMaxVecTile;
  const int cvt = cv < kMaxVecTile ? cv : kMaxVecTile;
  const int rows_it = kThreads / cvt;
  // ~16 row-iterations per thread, between 64 and 1024 blocks
  long want = (M + (long)rows_it * 16 - 1) / ((long)rows_it * 16);
  if (want < 64) want = 64;
  if (want > 1024) want = 1024;
  const long maxb = (M + rows_it - 1) / rows_it;
  if (want > maxb) want = maxb > 0 ? maxb : 1;
  return (int)want;
}

int grid_elem(long nvec) {
  long b = (nvec + kThreads - 1) / kThreads;
  if (b > 8192) b = 8192;
  return (int)(b > 0 ? b : 1);
}

// fold `nblk` partial rows to <= 64 in `scratch` (>= 64 x 2 x C floats) when there are many
const float* fold_rows(const float* part, int& nblk, int C, float* scratch, hipStream_t s) {
  if (nblk <= 64) return part;
  const int G = min(64, (nblk + 31) / 32);
  const int rows_per = (nblk + G - 1) / G;
  hipLaunchKernelGGL(bn_partial_reduce_kernel, dim3((C + 63) / 64, G), dim3(1024), 0, s, part, nblk, C, rows_per,
                     scratch);
  nblk = (nblk + rows_per - 1) / rows_per;
  return scratch;
}

}  // namespace
}  // namespace pha

using namespace pha;

// Number of row blocks the stats / reduce kernels use; the host sizes the partial buffer for
// (this + 64) rows of [2][C] floats (the tail takes the folded first-stage sums).
PHA_API int pha_bn_num_blocks(long M, int C) {
  int tiles;
  return grid_rows(M, C, &tiles);
}

PHA_API int pha_bn_fwd_train(int dt, const void* x, const void* res, void* y, long M, int C, const float* w,
                             const float* b, float* run_mean, float* run_var, float* save_mean, float* save_istd,
                             float* scale, float* shift, float* part, float eps, float momentum, int relu,
                             const float* ext_part, int ext_rows, hipStream_t s) {
  if (C % 8 != 0 || M <= 0) return (int)hipErrorInvalidValue;
  // part: >= (pha_bn_num_blocks + 64) x 2 x C floats; its tail holds the folded rows
  if (ext_part) {   // [ext_rows][2][C] unshifted sums computed by the producer of x
    int rows = ext_rows;
    const float* pp = fold_rows(ext_part, rows, C, part, s);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, pp, rows, C, M, nullptr, dt,
                       eps, momentum, w, b, run_mean, run_var, save_mean, save_istd, scale, shift);
  } else {
    int tiles;
    int nb = grid_rows(M, C, &tiles);
    PHA_DISPATCH_T(dt, T, {
      hipLaunchKernelGGL((bn_stats_kernel<T>), dim3(nb, tiles), dim3(kThreads), 0, s, (const T*)x, M, C, part);
    });
    const float* pp = fold_rows(part, nb, C, part + (long)grid_rows(M, C, &tiles) * 2 * C, s);
    hipLaunchKernelGGL(bn_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, pp, nb, C, M, x, dt, eps, momentum,
                       w, b, run_mean, run_var, save_mean, save_istd, scale, shift);
  }
  const long nvec = M * (C / 8);
  const int ge = grid_elem(nvec);
  PHA_DISPATCH_T(dt, T, {
    const T* xr = (const T*)x;
    const T* rr = (const T*)res;
    T* yr = (T*)y;
    if (res && relu)
      hipLaunchKernelGGL((bn_apply_kernel<T, true, true>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
    else if (res)
      hipLaunchKernelGGL((bn_apply_kernel<T, true, false>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
    else if (relu)
      hipLaunchKernelGGL((bn_apply_kernel<T, false, true>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
    else
      hipLaunchKernelGGL((bn_apply_kernel<T, false, false>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
  });
  return (int)hipGetLastError();
}

// Inference / frozen-stats affine: y = relu?(x*scale + shift (+res)) with given per-channel scale/shift.
PHA_API int pha_bn_apply(int dt, const void* x, const void* res, void* y, long M, int C, const float* scale,
                         const float* shift, int relu, hipStream_t s) {
  if (C % 8 != 0 || M <= 0) return (int)hipErrorInvalidValue;
  const long nvec = M * (C / 8);
  const int ge = grid_elem(nvec);
  PHA_DISPATCH_T(dt, T, {
    const T* xr = (const T*)x;
    const T* rr = (const T*)res;
    T* yr = (T*)y;
    if (res && relu)
      hipLaunchKernelGGL((bn_apply_kernel<T, true, true>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
    else if (res)
      hipLaunchKernelGGL((bn_apply_kernel<T, true, false>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
    else if (relu)
      hipLaunchKernelGGL((bn_apply_kernel<T, false, true>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
    else
      hipLaunchKernelGGL((bn_apply_kernel<T, false, false>), dim3(ge), dim3(kThreads), 0, s, xr, rr, scale, shift, yr, nvec, C / 8);
  });
  return (int)hipGetLastError();
}

PHA_API int pha_bn_bwd(int dt, const void* dy, const void* x, const void* y, long M, int C, const float* w,
                       const float* save_mean, const float* save_istd, void* dx, void* dres, float* dw, float* db,
                       float* part, float* coef, int relu, const float* aff, const float* ext_part, int ext_rows,
                       hipStream_t s) {
  if (C % 8 != 0 || M <= 0) return (int)hipErrorInvalidValue;
  if (relu && !y && !aff) return (int)hipErrorInvalidValue;
  int tiles;
  const int nb = grid_rows(M, C, &tiles);
  if (ext_part) {   // [ext_rows][2][C] sums of dy' and dy' (x - mean) from the producer of dy
    int rows = ext_rows;
    const float* pp = fold_rows(ext_part, rows, C, part, s);
    hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, pp, rows, C, 1.f / (float)M, w,
                       save_mean, save_istd, dw, db, coef);
  } else {
  PHA_DISPATCH_T(dt, T, {
    if (relu)
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, true>), dim3(nb, tiles), dim3(kThreads), 0, s, (const T*)dy,
                         (const T*)x, (const T*)y, save_mean, M, C, part, aff);
    else
      hipLaunchKernelGGL((bn_bwd_reduce_kernel<T, false>), dim3(nb, tiles), dim3(kThreads), 0, s, (const T*)dy,
                         (const T*)x, (const T*)y, save_mean, M, C, part, aff);
  });
  int rows = nb;
  const float* pp = fold_rows(part, rows, C, part + (long)nb * 2 * C, s);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(1024), 0, s, pp, rows, C, 1.f / (float)M, w,
                     save_mean, save_istd, dw, db, coef);
  }
  const long nvec = M * (C / 8);
  const int ge = grid_elem(nvec);
  PHA_DISPATCH_T(dt, T, {
    const T* d = (const T*)dy;
    const T* xr = (const T*)x;
    const T* yr = (const T*)y;
    if (relu && dres)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true, true>), dim3(ge), dim3(kThreads), 0, s, d, xr, yr, coef, (T*)dx, (T*)dres, nvec, C / 8, aff);
    else if (relu)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, true, false>), dim3(ge), dim3(kThreads), 0, s, d, xr, yr, coef, (T*)dx, (T*)dres, nvec, C / 8, aff);
    else if (dres)
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false, true>), dim3(ge), dim3(kThreads), 0, s, d, xr, yr, coef, (T*)dx, (T*)dres, nvec, C / 8, aff);
    else
      hipLaunchKernelGGL((bn_bwd_apply_kernel<T, false, false>), dim3(ge), dim3(kThreads), 0, s, d, xr, yr, coef, (T*)dx, (T*)dres, nvec, C / 8, aff);
  });
  return (int)hipGetLastError();
}
