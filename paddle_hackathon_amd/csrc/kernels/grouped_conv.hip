// Direct NHWC convolution for the layouts the implicit-GEMM kernels do not take: grouped and
// depthwise convolutions (MobileNet / ShuffleNet / ResNeXt), dilated + strided convolutions and
// channel counts that are not multiples of 8. Reference behaviour: phi/kernels/gpu/conv_kernel.cu
// (grouped cuDNN path) and the depthwise kernels of phi/kernels/gpu/depthwise_conv.h (forward,
// input gradient, filter gradient).
//
//   y[n, oh, ow, co] = sum_{kh, kw, ci < cig} x[n, oh*sh - ph + kh*dh, ow*sw - pw + kw*dw, g*cig + ci]
//                                            * w[co, ci, kh, kw] (+ b[co]),   g = co / cog
//
// Design. Per-channel arithmetic intensity is a few MACs per byte, so these kernels are HBM /
// L2 bound, not MFMA work: each thread owns 8 consecutive channels of one pixel (16-B vector
// loads and stores for 2-byte types, fp32 accumulation), the weight is re-laid out by the caller
// so the 8 channels a thread needs are one contiguous vector, and the grid has one thread per
// (pixel, 8 channels) so even a 7x7 feature map fills the chip. Channel modes, fixed per launch:
//   SAME  — the 8 output channels share one group (cog % 8 == 0): 8-wide weight vectors against
//           the group's input channels, 8 of them per 16-B load when cig % 8 == 0;
//   DEPTH — depthwise, one input channel per output channel (cig == cog == 1): input, weight and
//           output are all 8-wide vectors;
//   GRP2 / GRP4 — cig == cog == 2 / 4 (ResNeXt 32x4d's first stage): the 8 output channels read
//           exactly the 8 input channels at the same offsets, one vector load per tap;
//   ANY   — anything else (e.g. channel multiplier > 1): per channel.
// The filter gradient reduces over all output pixels: blocks own (tap, block of input channels,
// 8 output channels) x a chunk of pixels and write fp32 partials that a second kernel sums in chunk
// order (deterministic, no atomics).
#include "common.h"

namespace pha {
namespace gconv {

enum Mode : int { SAME = 0, DEPTH = 1, ANY = 2, GRP2 = 3, GRP4 = 4 };

template <int MODE> constexpr int grp_cig() { return MODE == GRP2 ? 2 : 4; }

struct Geo {
  int N, H, W, C, OH, OW, CO, KH, KW, sh, sw, ph, pw, dh, dw, groups, cig, cog;
};

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float (&o)[8]) { Vec8<T>::ld(p, o); }

// y = conv(x, wr) (+ bias); wr [KH][KW][cig][CO]
template <typename T, int MODE, bool BIAS>
__global__ __launch_bounds__(256) void fwd_kernel(const T* __restrict__ x, const T* __restrict__ wr,
                                                  const float* __restrict__ bias, T* __restrict__ y, Geo g) {
  const int cb = g.CO >> 3;
  const long tid = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.N * g.OH * g.OW * cb;
  if (tid >= total) return;
  const int c8 = (int)(tid % cb);
  const long pix = tid / cb;
  const int ow = (int)(pix % g.OW);
  const int oh = (int)((pix / g.OW) % g.OH);
  const int n = (int)(pix / ((long)g.OW * g.OH));
  const int co0 = c8 * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = BIAS ? bias[co0 + j] : 0.f;
  const T* xn = x + (long)n * g.H * g.W * g.C;
  for (int kh = 0; kh < g.KH; ++kh) {
    const int ih = oh * g.sh - g.ph + kh * g.dh;
    if (ih < 0 || ih >= g.H) continue;
    for (int kw = 0; kw < g.KW; ++kw) {
      const int iw = ow * g.sw - g.pw + kw * g.dw;
      if (iw < 0 || iw >= g.W) continue;
      const T* xp = xn + ((long)ih * g.W + iw) * g.C;
      const T* wp = wr + (long)(kh * g.KW + kw) * g.cig * g.CO;
      if constexpr (MODE == DEPTH) {
        float xv[8], wv[8];
        ld8(xp + co0, xv);
        ld8(wp + co0, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv[j], wv[j], acc[j]);
      } else if constexpr (MODE == GRP2 || MODE == GRP4) {
        // cig == cog == CIG: output channels co0 .. co0+7 read input channels co0 .. co0+7
        constexpr int CIG = grp_cig<MODE>();
        float xv[8];
        ld8(xp + co0, xv);
#pragma unroll
        for (int ci = 0; ci < CIG; ++ci) {
          float wv[8];
          ld8(wp + (long)ci * g.CO + co0, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv[(j / CIG) * CIG + ci], wv[j], acc[j]);
        }
      } else if constexpr (MODE == SAME) {
        const T* xg = xp + (co0 / g.cog) * g.cig;
        if ((g.cig & 7) == 0) {   // 8 input channels per 16-B load
          for (int ci = 0; ci < g.cig; ci += 8) {
            float xv[8];
            ld8(xg + ci, xv);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              float wv[8];
              ld8(wp + (long)(ci + q) * g.CO + co0, wv);
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv[q], wv[j], acc[j]);
            }
          }
        } else {
          for (int ci = 0; ci < g.cig; ++ci) {
            const float xv = Cvt<T>::ld(xg, ci);
            float wv[8];
            ld8(wp + (long)ci * g.CO + co0, wv);
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, wv[j], acc[j]);
          }
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int co = co0 + j;
          const T* xg = xp + (co / g.cog) * g.cig;
          float a = 0.f;
          for (int ci = 0; ci < g.cig; ++ci) a = fmaf(Cvt<T>::ld(xg, ci), Cvt<T>::ld(wp, (long)ci * g.CO + co), a);
          acc[j] += a;
        }
      }
    }
  }
  Vec8<T>::st(y + pix * g.CO + co0, acc);
}

// dx = conv^T(dy, w); for SAME / ANY / GRP the weight is wt [KH][KW][CO][cig], for DEPTH wr [KH][KW][1][C]
template <typename T, int MODE>
__global__ __launch_bounds__(256) void dgrad_kernel(const T* __restrict__ dy, const T* __restrict__ wt,
                                                    T* __restrict__ dx, Geo g) {
  const int cb = g.C >> 3;
  const long tid = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)g.N * g.H * g.W * cb;
  if (tid >= total) return;
  const int c8 = (int)(tid % cb);
  const long pix = tid / cb;
  const int iw = (int)(pix % g.W);
  const int ih = (int)((pix / g.W) % g.H);
  const int n = (int)(pix / ((long)g.W * g.H));
  const int ci0 = c8 * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const T* dyn = dy + (long)n * g.OH * g.OW * g.CO;
  for (int kh = 0; kh < g.KH; ++kh) {
    const int th = ih + g.ph - kh * g.dh;
    if (th < 0 || th % g.sh) continue;
    const int oh = th / g.sh;
    if (oh >= g.OH) continue;
    for (int kw = 0; kw < g.KW; ++kw) {
      const int tw = iw + g.pw - kw * g.dw;
      if (tw < 0 || tw % g.sw) continue;
      const int ow = tw / g.sw;
      if (ow >= g.OW) continue;
      const T* dyp = dyn + ((long)oh * g.OW + ow) * g.CO;
      const T* wp = wt + (long)(kh * g.KW + kw) * g.cig * g.CO;
      if constexpr (MODE == DEPTH) {
        float dv[8], wv[8];
        ld8(dyp + ci0, dv);
        ld8(wp + ci0, wv);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = fmaf(dv[j], wv[j], acc[j]);
      } else if constexpr (MODE == GRP2 || MODE == GRP4) {
        // input channels ci0 .. ci0+7 receive from output channels ci0 .. ci0+7; their weights
        // w[co][ci_l], co in that range, are 8 * CIG consecutive elements of wt
        constexpr int CIG = grp_cig<MODE>();
        float dv[8], wv[8 * CIG];
        ld8(dyp + ci0, dv);
#pragma unroll
        for (int q = 0; q < CIG; ++q) {
          float t8[8];
          ld8(wp + (long)ci0 * CIG + q * 8, t8);
#pragma unroll
          for (int e = 0; e < 8; ++e) wv[q * 8 + e] = t8[e];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int jg = (j / CIG) * CIG;
#pragma unroll
          for (int cl = 0; cl < CIG; ++cl) acc[j] = fmaf(dv[jg + cl], wv[(jg + cl) * CIG + (j % CIG)], acc[j]);
        }
      } else if constexpr (MODE == SAME) {   // the 8 input channels share one group (cig % 8 == 0)
        const int grp = ci0 / g.cig, cl0 = ci0 - grp * g.cig;
        const int c_lo = grp * g.cog, c_hi = c_lo + g.cog;
        int co = c_lo;
        if ((g.cog & 7) == 0) {   // 8 output channels per 16-B load
          for (; co < c_hi; co += 8) {
            float dv[8];
            ld8(dyp + co, dv);
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              float wv[8];
              ld8(wp + (long)(co + q) * g.cig + cl0, wv);
#pragma unroll
              for (int j = 0; j < 8; ++j) acc[j] = fmaf(dv[q], wv[j], acc[j]);
            }
          }
        }
        for (; co < c_hi; ++co) {
          const float dv = Cvt<T>::ld(dyp, co);
          float wv[8];
          ld8(wp + (long)co * g.cig + cl0, wv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = fmaf(dv, wv[j], acc[j]);
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int ci = ci0 + j, grp = ci / g.cig, cl = ci - grp * g.cig;
          float a = 0.f;
          for (int co = grp * g.cog; co < (grp + 1) * g.cog; ++co)
            a = fmaf(Cvt<T>::ld(dyp, co), Cvt<T>::ld(wp, (long)co * g.cig + cl), a);
          acc[j] += a;
        }
      }
    }
  }
  Vec8<T>::st(dx + pix * g.C + ci0, acc);
}

// input channels (per group) one filter-gradient block covers: all of them (GRP), 8 (SAME with
// cig % 8 == 0), else 1
template <int MODE> constexpr int wg_civ() { return MODE == GRP2 ? 2 : MODE == GRP4 ? 4 : MODE == SAME ? 8 : 1; }

// partial filter gradients: block (item, chunk); item = ((tap * (cig / CIV) + cblk) * CO/8 + c8);
// part[chunk][tap][ci][CO] (fp32) = sum over the chunk's output pixels of dy[.., co] x[.., g*cig+ci]
template <typename T, int MODE>
__global__ __launch_bounds__(256) void wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                    float* __restrict__ part, Geo g, long chunk_pix) {
  constexpr int CIV = wg_civ<MODE>();
  __shared__ float red[4][CIV * 8];
  const int cb = g.CO >> 3;
  const int nblk = g.cig / CIV;
  const int item = blockIdx.x;
  const int c8 = item % cb;
  const int cblk = (item / cb) % nblk;
  const int tap = item / (cb * nblk);
  const int kh = tap / g.KW, kw = tap - kh * g.KW;
  const int co0 = c8 * 8, ci0 = cblk * CIV;
  const long npix = (long)g.N * g.OH * g.OW;
  const long p0 = (long)blockIdx.y * chunk_pix, p1 = min(npix, p0 + chunk_pix);
  float acc[CIV][8];
#pragma unroll
  for (int c = 0; c < CIV; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[c][j] = 0.f;
  for (long p = p0 + threadIdx.x; p < p1; p += 256) {
    const int ow = (int)(p % g.OW);
    const int oh = (int)((p / g.OW) % g.OH);
    const int n = (int)(p / ((long)g.OW * g.OH));
    const int ih = oh * g.sh - g.ph + kh * g.dh, iw = ow * g.sw - g.pw + kw * g.dw;
    if (ih < 0 || ih >= g.H || iw < 0 || iw >= g.W) continue;
    const T* xp = x + (((long)n * g.H + ih) * g.W + iw) * g.C;
    const T* dyp = dy + p * g.CO;
    float dv[8];
    ld8(dyp + co0, dv);
    if constexpr (MODE == DEPTH) {
      float xv[8];
      ld8(xp + co0, xv);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[0][j] = fmaf(dv[j], xv[j], acc[0][j]);
    } else if constexpr (MODE == GRP2 || MODE == GRP4) {
      float xv[8];
      ld8(xp + co0, xv);
#pragma unroll
      for (int c = 0; c < CIV; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c][j] = fmaf(dv[j], xv[(j / CIV) * CIV + c], acc[c][j]);
    } else if constexpr (MODE == SAME) {   // cig % 8 == 0: 8 input channels of the group
      float xv[8];
      ld8(xp + (co0 / g.cog) * g.cig + ci0, xv);
#pragma unroll
      for (int c = 0; c < 8; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[c][j] = fmaf(dv[j], xv[c], acc[c][j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        acc[0][j] = fmaf(dv[j], Cvt<T>::ld(xp, ((co0 + j) / g.cog) * g.cig + ci0), acc[0][j]);
    }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < CIV; ++c)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = wave_sum(acc[c][j]);
      if (lane == 0) red[wid][c * 8 + j] = v;
    }
  __syncthreads();
  if (threadIdx.x < CIV * 8) {
    const int c = threadIdx.x >> 3, j = threadIdx.x & 7;
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    part[(((long)blockIdx.y * g.KH * g.KW + tap) * g.cig + ci0 + c) * g.CO + co0 + j] = v;
  }
}

// dw[co][ci][kh][kw] = sum over chunks (in order) of part[chunk][tap][ci][co]
template <typename T>
__global__ __launch_bounds__(256) void wgrad_finish_kernel(const float* __restrict__ part, T* __restrict__ dw, Geo g,
                                                           int chunks) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  const long per = (long)g.KH * g.KW * g.cig * g.CO;
  if (i >= per) return;
  // i indexes dw's own layout [CO][cig][KH][KW]
  const int taps = g.KH * g.KW;
  const int tap = (int)(i % taps);
  const int ci = (int)((i / taps) % g.cig);
  const int co = (int)(i / ((long)taps * g.cig));
  const long src = ((long)tap * g.cig + ci) * g.CO + co;
  float s = 0.f;
  for (int c = 0; c < chunks; ++c) s += part[c * per + src];
  Cvt<T>::st(dw, i, s);
}

// channel mode of a launch: input_side selects the input-gradient condition (its 8 channels are
// input channels); the filter gradient uses the output-side mode
inline int mode_of(const Geo& g, bool input_side) {
  if (g.cig == 1 && g.cog == 1) return DEPTH;
  if (g.cig == g.cog && g.cig == 2) return GRP2;
  if (g.cig == g.cog && g.cig == 4) return GRP4;
  if (input_side ? (g.cig % 8 == 0) : (g.cog % 8 == 0)) return SAME;
  return ANY;
}

inline unsigned blocks(long n) { return (unsigned)((n + 255) / 256); }

}  // namespace gconv
}  // namespace pha

using namespace pha;
using gconv::Geo;

static bool geo_ok(const Geo& g) {
  return g.N > 0 && g.H > 0 && g.W > 0 && g.OH > 0 && g.OW > 0 && g.KH > 0 && g.KW > 0 && g.sh > 0 && g.sw > 0 &&
         g.dh > 0 && g.dw > 0 && g.groups > 0 && g.C % g.groups == 0 && g.CO % g.groups == 0 && g.C % 8 == 0 &&
         g.CO % 8 == 0 && g.cig == g.C / g.groups && g.cog == g.CO / g.groups;
}

static Geo make_geo(const int* d) {
  Geo g{d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7], d[8], d[9], d[10], d[11], d[12], d[13], d[14], d[15], 0, 0};
  if (g.groups > 0) {
    g.cig = g.C / g.groups;
    g.cog = g.CO / g.groups;
  }
  return g;
}

#define PHA_GCONV_MODES(mode, M, ...)                                     \
  switch (mode) {                                                         \
    case gconv::DEPTH: { constexpr int M = gconv::DEPTH; __VA_ARGS__; break; } \
    case gconv::GRP2: { constexpr int M = gconv::GRP2; __VA_ARGS__; break; }   \
    case gconv::GRP4: { constexpr int M = gconv::GRP4; __VA_ARGS__; break; }   \
    case gconv::SAME: { constexpr int M = gconv::SAME; __VA_ARGS__; break; }   \
    default: { constexpr int M = gconv::ANY; __VA_ARGS__; break; }             \
  }

// dims: N, H, W, C, OH, OW, CO, KH, KW, sh, sw, ph, pw, dh, dw, groups (C and CO multiples of 8).
// x [N][H][W][C], wr [KH][KW][C/groups][CO], bias fp32 [CO] or null, y [N][OH][OW][CO].
PHA_API int pha_gconv_fwd(int dt, const int* dims, const void* x, const void* wr, const float* bias, void* y,
                          hipStream_t st) {
  const Geo g = make_geo(dims);
  if (!geo_ok(g)) return (int)hipErrorInvalidValue;
  const unsigned nb = gconv::blocks((long)g.N * g.OH * g.OW * (g.CO / 8));
  PHA_DISPATCH_T(dt, T, {
    PHA_GCONV_MODES(gconv::mode_of(g, false), M, {
      if (bias) hipLaunchKernelGGL((gconv::fwd_kernel<T, M, true>), dim3(nb), dim3(256), 0, st, (const T*)x, (const T*)wr, bias, (T*)y, g);
      else hipLaunchKernelGGL((gconv::fwd_kernel<T, M, false>), dim3(nb), dim3(256), 0, st, (const T*)x, (const T*)wr, bias, (T*)y, g);
    });
  });
  return (int)hipGetLastError();
}

// dy [N][OH][OW][CO] -> dx [N][H][W][C]; w2: [KH][KW][CO][C/groups] (or [KH][KW][1][C] when
// depthwise, the forward's layout)
PHA_API int pha_gconv_dgrad(int dt, const int* dims, const void* dy, const void* w2, void* dx, hipStream_t st) {
  const Geo g = make_geo(dims);
  if (!geo_ok(g)) return (int)hipErrorInvalidValue;
  const unsigned nb = gconv::blocks((long)g.N * g.H * g.W * (g.C / 8));
  PHA_DISPATCH_T(dt, T, {
    PHA_GCONV_MODES(gconv::mode_of(g, true), M, {
      hipLaunchKernelGGL((gconv::dgrad_kernel<T, M>), dim3(nb), dim3(256), 0, st, (const T*)dy, (const T*)w2, (T*)dx, g);
    });
  });
  return (int)hipGetLastError();
}

// filter-gradient mode: SAME needs both the 8 output channels in one group and 8 input channels
static int wgrad_mode(const Geo& g) {
  const int m = gconv::mode_of(g, false);
  return (m == gconv::SAME && g.cig % 8) ? (int)gconv::ANY : m;
}

// workspace floats the filter gradient needs for `chunks` pixel chunks
PHA_API long pha_gconv_wgrad_ws(const int* dims, int chunks) {
  const Geo g = make_geo(dims);
  return (long)chunks * g.KH * g.KW * (g.groups > 0 ? g.C / g.groups : 0) * g.CO;
}

// blocks per chunk of the filter gradient (tap x input-channel block x 8 output channels)
PHA_API long pha_gconv_wgrad_items(const int* dims) {
  const Geo g = make_geo(dims);
  if (!geo_ok(g)) return 0;
  int civ = 1;
  switch (wgrad_mode(g)) {
    case gconv::GRP2: civ = 2; break;
    case gconv::GRP4: civ = 4; break;
    case gconv::SAME: civ = 8; break;
    default: civ = 1;
  }
  return (long)g.KH * g.KW * (g.cig / civ) * (g.CO / 8);
}

// x, dy -> dw [CO][C/groups][KH][KW] (dtype dt); ws: pha_gconv_wgrad_ws(dims, chunks) floats
PHA_API int pha_gconv_wgrad(int dt, const int* dims, const void* x, const void* dy, void* dw, float* ws, int chunks,
                            hipStream_t st) {
  const Geo g = make_geo(dims);
  if (!geo_ok(g) || chunks < 1 || !ws) return (int)hipErrorInvalidValue;
  const long npix = (long)g.N * g.OH * g.OW;
  const long chunk_pix = (npix + chunks - 1) / chunks;
  const dim3 grid((unsigned)pha_gconv_wgrad_items(dims), (unsigned)chunks);
  const long per = (long)g.KH * g.KW * g.cig * g.CO;
  PHA_DISPATCH_T(dt, T, {
    PHA_GCONV_MODES(wgrad_mode(g), M, {
      hipLaunchKernelGGL((gconv::wgrad_kernel<T, M>), grid, dim3(256), 0, st, (const T*)x, (const T*)dy, ws, g, chunk_pix);
    });
    hipLaunchKernelGGL((gconv::wgrad_finish_kernel<T>), dim3(gconv::blocks(per)), dim3(256), 0, st, ws, (T*)dw, g, chunks);
  });
  return (int)hipGetLastError();
}
