// HBM-resident sparse embedding table (the GPU-PS of the reference: paddle/fluid/framework/fleet/
// heter_ps/hashtable_kernel.cu, heter_comm_inl.h, optimizer.cuh.h) for MI355X.
//
// Design: a 288 GB HBM3E GPU holds hundreds of millions of embedding rows itself, so the hot
// sparse table of a CTR / recommender model lives in HBM instead of behind a CPU server:
//  * open-addressing hash map keys[cap] (u64, EMPTY = ~0) -> row[cap] (i32), linear probing with
//    a 64-bit mix; cap a power of two >= 2x the row budget keeps probes short;
//  * rows of [dim] fp32 weights + one AdaGrad g2sum per row in two dense arrays indexed by row;
//  * inserts: one lane per (already de-duplicated) key; the slot is claimed with a 64-bit
//    compare-and-swap and the row number drawn from a device counter with an atomic add
//    (vector-memory global atomics); new rows are initialised from a hash of the key, so the
//    result does not depend on thread order;
//  * pull = gather of the rows (one wave per 64-lane row chunk); push = AdaGrad applied to the
//    touched rows (duplicates summed by the caller), fused in one pass.
// Keys are de-duplicated per call on the caller's side (torch.unique), so no two lanes of one
// call race for the same key and no lane ever waits on another.
#include "common.h"

using namespace pha;

namespace {

constexpr unsigned long long kEmpty = ~0ULL;
constexpr unsigned long long kTomb = ~0ULL - 1;   // a slot claimed by an insert that found no free row

__device__ __forceinline__ unsigned long long mix64(unsigned long long x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  return x ^ (x >> 31);
}

__device__ __forceinline__ float init_val(unsigned long long key, int j, unsigned seed, float range) {
  const unsigned long long h = mix64(key ^ ((unsigned long long)seed << 32) ^ (unsigned long long)(j + 1) * 0x9e3779b97f4a7c15ULL);
  const float u = (float)(h >> 40) * (1.0f / 16777216.0f);   // [0, 1)
  return (2.f * u - 1.f) * range;
}

// keys[n] (unique; never ~0 or ~0 - 1, the empty / tombstone markers) -> rows[n]; create = 0:
// missing keys give -1; create = 1: insert (row counter in *next_row, capped at max_rows: overflow
// gives -2 and leaves a tombstone)
__global__ __launch_bounds__(256) void ps_find_insert_kernel(const unsigned long long* __restrict__ keys,
                                                             int* __restrict__ rows_out, long n,
                                                             unsigned long long* __restrict__ tkeys,
                                                             int* __restrict__ trow, long cap_mask,
                                                             int* __restrict__ next_row, int max_rows, int create,
                                                             float* __restrict__ W, float* __restrict__ g2, int dim,
                                                             unsigned seed, float init_range) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const unsigned long long k = keys[i];
  long s = (long)(mix64(k) & (unsigned long long)cap_mask);
  for (long probe = 0; probe <= cap_mask; ++probe) {
    const unsigned long long cur = tkeys[s];
    if (cur == k) {
      rows_out[i] = trow[s];
      return;
    }
    if (cur == kEmpty) {
      if (!create) {
        rows_out[i] = -1;
        return;
      }
      const unsigned long long prev = atomicCAS(tkeys + s, kEmpty, k);
      if (prev == kEmpty) {
        const int r = atomicAdd(next_row, 1);
        if (r >= max_rows) {
          // give the row number back (next_row settles at max_rows) and leave a tombstone: the
          // slot stays occupied for probing (keys placed past it stay reachable) but matches no
          // key and is not exported
          atomicSub(next_row, 1);
          trow[s] = -2;
          tkeys[s] = kTomb;
          rows_out[i] = -2;
          return;
        }
        float* w = W + (long)r * dim;
        for (int j = 0; j < dim; ++j) w[j] = init_val(k, j, seed, init_range);
        g2[r] = 0.f;
        trow[s] = r;
        rows_out[i] = r;
        return;
      }
      if (prev == k) {   // cannot happen for de-duplicated keys within one call
        rows_out[i] = trow[s];
        return;
      }
    }
    s = (s + 1) & cap_mask;
  }
  rows_out[i] = -3;   // table full
}

// AdaGrad (the CPU server's row rule): ratio = lr * sqrt(ig2 / (ig2 + g2sum)); w -= ratio * g;
// g2sum += mean(g^2); clamp to [lo, hi]. One wave per row, lanes over dim.
__global__ __launch_bounds__(256) void ps_adagrad_kernel(const int* __restrict__ rows, const float* __restrict__ grads,
                                                         long n, float* __restrict__ W, float* __restrict__ g2,
                                                         int dim, float lr, float ig2, float lo, float hi) {
  const long w = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= n) return;
  const int r = rows[w];
  if (r < 0) return;
  float* wr = W + (long)r * dim;
  const float* gr = grads + w * dim;
  const float ratio = lr * sqrtf(ig2 / (ig2 + g2[r]));
  float add = 0.f;
  for (int j = lane; j < dim; j += 64) {
    const float g = gr[j];
    wr[j] = fminf(fmaxf(wr[j] - ratio * g, lo), hi);
    add += g * g;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) add += __shfl_xor(add, o);
  if (lane == 0) g2[r] += add / dim;
}

}  // namespace

PHA_API int pha_ps_gpu_find(const void* keys, int* rows, long n, void* tkeys, int* trow, long cap, int* next_row,
                            int max_rows, int create, float* W, float* g2, int dim, unsigned seed, float init_range,
                            hipStream_t stream) {
  if (n <= 0) return 0;
  if (cap <= 0 || (cap & (cap - 1)) || dim <= 0) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(ps_find_insert_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream,
                     (const unsigned long long*)keys, rows, n, (unsigned long long*)tkeys, trow, cap - 1, next_row,
                     max_rows, create, W, g2, dim, seed, init_range);
  return (int)hipGetLastError();
}

PHA_API int pha_ps_gpu_adagrad(const int* rows, const float* grads, long n, float* W, float* g2, int dim, float lr,
                               float ig2, float lo, float hi, hipStream_t stream) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(ps_adagrad_kernel, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, stream, rows, grads, n,
                     W, g2, dim, lr, ig2, lo, hi);
  return (int)hipGetLastError();
}
