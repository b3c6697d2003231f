// DistributedFusedLamb's shard update as three kernels over the flat fp32 shard (reference:
// paddle/fluid/operators/optimizers/distributed_fused_lamb_op.cu — one fused op there too):
//
//   lamb_sq      sum of squares of the shard's gradient (deterministic two-level reduction) — the
//                global-norm clip's input, all-reduced over the ranks by the caller;
//   lamb_moment  clip scale from the all-reduced square sum (device scalar: no host sync),
//                m1 / m2 moments, the LAMB direction r = m1^ / (sqrt(m2^) + eps) + wd[p] w written
//                over the gradient buffer, and per-parameter sums of w^2 and r^2 (one wave-level
//                reduction per parameter run inside a wave + one float atomic) — the trust-ratio
//                inputs, all-reduced by the caller (parameters straddle shards);
//   lamb_apply   w -= lr * lr_ratio[p] * trust[p] * r, trust = ||w|| / ||r|| (1 when either is 0).
//
// 48 bytes of HBM traffic per element and step against ~200 for the unfused torch sequence.
#include "common.h"

namespace {

__device__ __forceinline__ float wave_sum_f(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(256) void lamb_sq_partial(const float* __restrict__ g, long n, float* __restrict__ part) {
  float s = 0.f;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) s += g[i] * g[i];
  __shared__ float red[4];
  s = wave_sum_f(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void lamb_sq_final(const float* __restrict__ part, int n, float* __restrict__ out) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += part[i];
  __shared__ float red[4];
  s = wave_sum_f(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

struct MomentArgs {
  float b1, b2, bc1, bc2, eps, gmul, clip;   // bc = 1 - beta^t; gmul: 1 / world when not pre-scaled
  const float* gsq;                           // all-reduced gradient square sum (clip > 0)
};

// per-parameter accumulation of (a, b) for the lanes' parameter ids (non-decreasing over lanes):
// one iteration per distinct id in the wave, one atomic pair per id
__device__ __forceinline__ void seg_add(int pid, float a, float b, float* __restrict__ norms, int npar) {
  const int lane = threadIdx.x & 63;
  unsigned long long left = __ballot(1);
  while (left) {
    const int first = __ffsll((long long)left) - 1;
    const int p = __shfl(pid, first, 64);
    const bool mine = pid == p;
    const float sa = wave_sum_f(mine ? a : 0.f), sb = wave_sum_f(mine ? b : 0.f);
    if (lane == first) {
      atomicAdd(norms + p, sa);
      atomicAdd(norms + npar + p, sb);
    }
    left &= ~__ballot(mine);
  }
}

__global__ __launch_bounds__(256) void lamb_moment_kernel(float* __restrict__ g, float* __restrict__ m1,
                                                          float* __restrict__ m2, const float* __restrict__ w,
                                                          const int* __restrict__ pid, const float* __restrict__ wd,
                                                          float* __restrict__ norms, int npar, long n, MomentArgs a) {
  float scale = a.gmul;
  if (a.clip > 0.f) {
    const float nrm = sqrtf(a.gsq[0]);
    scale *= a.clip / fmaxf(nrm, a.clip);
  }
  for (long base = (long)blockIdx.x * 256; base < n; base += (long)gridDim.x * 256) {
    const long i = base + threadIdx.x;
    float ww = 0.f, rr = 0.f;
    int p = npar - 1;   // the padding slot (its sums are never used)
    if (i < n) {
      p = pid[i];
      const float gv = g[i] * scale;
      const float v1 = a.b1 * m1[i] + (1.f - a.b1) * gv;
      const float v2 = a.b2 * m2[i] + (1.f - a.b2) * gv * gv;
      m1[i] = v1;
      m2[i] = v2;
      const float wv = w[i];
      const float r = (v1 / a.bc1) / (sqrtf(v2 / a.bc2) + a.eps) + wd[p] * wv;
      g[i] = r;
      ww = wv * wv;
      rr = r * r;
    }
    seg_add(p, ww, rr, norms, npar);
  }
}

__global__ __launch_bounds__(256) void lamb_apply_kernel(float* __restrict__ w, const float* __restrict__ r,
                                                         const int* __restrict__ pid, const float* __restrict__ norms,
                                                         const float* __restrict__ lr_ratio, int npar, long n,
                                                         float lr, const float* __restrict__ lr_dev) {
  const float l = lr_dev ? lr_dev[0] : lr;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    const int p = pid[i];
    const float wn = sqrtf(norms[p]), rn = sqrtf(norms[npar + p]);
    const float trust = (wn > 0.f && rn > 0.f) ? wn / rn : 1.f;
    w[i] -= l * lr_ratio[p] * trust * r[i];
  }
}

unsigned grid_for(long n) {
  const long b = (n + 255) / 256;
  return (unsigned)(b < 1 ? 1 : (b > 8192 ? 8192 : b));
}

}  // namespace

// part: >= 8192 floats of scratch
PHA_API int pha_lamb_sq(const float* g, long n, float* part, float* out, hipStream_t st) {
  const unsigned gb = grid_for(n);
  hipLaunchKernelGGL(lamb_sq_partial, dim3(gb), dim3(256), 0, st, g, n, part);
  hipLaunchKernelGGL(lamb_sq_final, dim3(1), dim3(256), 0, st, part, (int)gb, out);
  return (int)hipGetLastError();
}

// norms: [2, npar] fp32, zeroed by the caller; pid values in [0, npar)
PHA_API int pha_lamb_moment(float* g, float* m1, float* m2, const float* w, const int* pid, const float* wd,
                            float* norms, int npar, long n, float b1, float b2, float bc1, float bc2, float eps,
                            float gmul, float clip, const float* gsq, hipStream_t st) {
  if (n <= 0) return 0;
  if (clip > 0.f && !gsq) return (int)hipErrorInvalidValue;
  MomentArgs a{b1, b2, bc1, bc2, eps, gmul, clip, gsq};
  hipLaunchKernelGGL(lamb_moment_kernel, dim3(grid_for(n)), dim3(256), 0, st, g, m1, m2, w, pid, wd, norms, npar, n, a);
  return (int)hipGetLastError();
}

PHA_API int pha_lamb_apply(float* w, const float* r, const int* pid, const float* norms, const float* lr_ratio,
                           int npar, long n, float lr, const float* lr_dev, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(lamb_apply_kernel, dim3(grid_for(n)), dim3(256), 0, st, w, r, pid, norms, lr_ratio, npar, n, lr,
                     lr_dev);
  return (int)hipGetLastError();
}
