// Recurrent layers (SimpleRNN tanh / relu, LSTM, GRU) for gfx950: the time loop of one (layer,
// direction). Reference behaviour: the cudnn "rnn" op, paddle/phi/kernels/gpu/rnn_kernel.cu.cc and
// rnn_grad_kernel.cu.cc (paddle/fluid/operators/rnn_op.cc), with the cell equations of
// python/paddle/nn/layer/rnn.py (SimpleRNNCell / LSTMCell / GRUCell):
//
//   LSTM  a = gx + h W_hh^T + b_hh, [i f g o] = [s s tanh s](a), c' = f c + i g, h' = o tanh(c')
//   GRU   r = s(gx_r + h W_hr^T + b_hr), z = s(gx_z + ..), n = tanh(gx_n + r (h W_hn^T + b_hn)),
//         h' = z h + (1 - z) n
//   RNN   h' = act(gx + h W_hh^T + b_hh)
//
// gx = x W_ih^T + b_ih for ALL time steps is one large GEMM done by the caller (ops/rnn.py, on the
// own GEMM kernels). What remains is sequential: per step a [B, H] x [H, G*H] product and the cell.
// One launch per step (the host loop below, graph-capturable), grid = (H / 16 units) x (B / 64
// rows); wave w of a workgroup owns 16 batch rows x 16 hidden units x all G gates, so the cell
// update of a (row, unit) needs no data from other lanes. The hidden-state product runs on
// v_mfma_f32_16x16x4_f32 (exact fp32, k-ordered fma chain): A = h rows, B = W_hh^T columns, one
// accumulator per gate; the operands are staged through LDS in 32-deep k chunks (row pitch 33
// floats: the 16 lanes of a fragment column read 16 distinct banks).
//
// Variable-length batches (SequenceLength): a step t >= len[b] leaves row b's state unchanged and
// writes a zero output, in both directions (a reverse pass over padded steps carries h0 until the
// row's last valid step, which is then the first one it processes).
//
// Backward (reverse over the steps): per step one launch computes, for its units, the recurrent
// gradient dh = dG_h(s+1) W_hh (K = G*H, MFMA again, B operand = W_hh rows) + the direct part
// carried from step s+1 + dy(s), then the cell's gate gradients: dG_x (for x / W_ih / b_ih) and
// dG_h (for h / W_hh / b_hh; equal to dG_x except GRU's candidate gate). The weight gradients are
// large GEMMs over all steps afterwards (ops/rnn.py).
#include "common.h"

#include <cstdlib>

namespace pha {
namespace rnn {

typedef float f32x4 __attribute__((ext_vector_type(4)));

enum : int { M_TANH = 0, M_RELU = 1, M_LSTM = 2, M_GRU = 3 };
template <int MODE> struct Gates { static constexpr int G = MODE == M_LSTM ? 4 : MODE == M_GRU ? 3 : 1; };
// saved per step and (row, unit): LSTM i f g o; GRU r z n hc; RNN none (h' itself)
template <int MODE> struct Saved { static constexpr int S = MODE == M_LSTM ? 4 : MODE == M_GRU ? 4 : 0; };

constexpr int KC = 32;        // k chunk
constexpr int PITCH = KC + 1; // LDS row pitch (floats)
constexpr int UB = 16;        // hidden units per workgroup
constexpr int BB = 64;        // batch rows per workgroup (16 per wave)

__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = expf(-2.f * fabsf(x));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, x);
}

struct FwdArgs {
  const float* gx;     // [T][B][G*H] (time index)
  const float* whh;    // [G*H][H]
  const float* bhh;    // [G*H] or null
  const int* lens;     // [B] or null
  float* y;            // [T][B][H] (time index)
  float* hall;         // [T+1][B][H] (step index; hall[0] = h0)
  float* call;         // [T+1][B][H] (LSTM)
  float* save;         // [T][B][S*H] (step index)
  int T, B, H, s, t;   // current step s, its time t
};

template <int MODE>
__global__ __launch_bounds__(256) void rnn_fwd_step(FwdArgs p) {
  constexpr int G = Gates<MODE>::G, S = Saved<MODE>::S;
  __shared__ float hs[BB * PITCH];
  __shared__ float ws[G * UB * PITCH];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j0 = blockIdx.x * UB, b0 = blockIdx.y * BB;
  const int B = p.B, H = p.H, GH = G * H;
  const float* hprev = p.hall + (size_t)p.s * B * H;
  f32x4 acc[G];
#pragma unroll
  for (int g = 0; g < G; ++g) acc[g] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < H; k0 += KC) {
    // stage h rows b0..b0+63 and the G x 16 weight rows, k0..k0+31 (zero outside)
    for (int e = tid; e < BB * KC; e += 256) {
      const int r = e / KC, k = e - r * KC;
      const int b = b0 + r, kk = k0 + k;
      hs[r * PITCH + k] = (b < B && kk < H) ? hprev[(size_t)b * H + kk] : 0.f;
    }
    for (int e = tid; e < G * UB * KC; e += 256) {
      const int r = e / KC, k = e - r * KC;
      const int g = r / UB, j = j0 + (r - g * UB), kk = k0 + k;
      ws[r * PITCH + k] = (j < H && kk < H) ? p.whh[(size_t)(g * H + j) * H + kk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < KC; kk += 4) {
      const float a = hs[(wid * 16 + (lane & 15)) * PITCH + kk + (lane >> 4)];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float bv = ws[(g * UB + (lane & 15)) * PITCH + kk + (lane >> 4)];
        acc[g] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bv, acc[g], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  // cell update: lane owns rows b0 + 16 wid + 4 (lane >> 4) + r, unit j0 + (lane & 15)
  const int j = j0 + (lane & 15);
  if (j >= H) return;
  const size_t tBG = (size_t)p.t * B;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + wid * 16 + 4 * (lane >> 4) + r;
    if (b >= B) continue;
    const bool valid = !p.lens || p.t < p.lens[b];
    const float hp = hprev[(size_t)b * H + j];
    float hn = hp, cn = 0.f;
    const float* gxr = p.gx + (tBG + b) * GH;
    float* sv = S ? p.save + ((size_t)p.s * B + b) * (S * H) : nullptr;
    float bh[G];
#pragma unroll
    for (int g = 0; g < G; ++g) bh[g] = p.bhh ? p.bhh[g * H + j] : 0.f;
    if constexpr (MODE == M_LSTM) {
      const float cp = p.call[(size_t)p.s * B * H + (size_t)b * H + j];
      cn = cp;
      if (valid) {
        const float ig = sigm(gxr[j] + acc[0][r] + bh[0]);
        const float fg = sigm(gxr[H + j] + acc[1][r] + bh[1]);
        const float gg = tanh_f(gxr[2 * H + j] + acc[2][r] + bh[2]);
        const float og = sigm(gxr[3 * H + j] + acc[3][r] + bh[3]);
        cn = fg * cp + ig * gg;
        hn = og * tanh_f(cn);
        sv[j] = ig; sv[H + j] = fg; sv[2 * H + j] = gg; sv[3 * H + j] = og;
      }
      p.call[(size_t)(p.s + 1) * B * H + (size_t)b * H + j] = cn;
    } else if constexpr (MODE == M_GRU) {
      if (valid) {
        const float rg = sigm(gxr[j] + acc[0][r] + bh[0]);
        const float zg = sigm(gxr[H + j] + acc[1][r] + bh[1]);
        const float hc = acc[2][r] + bh[2];
        const float ng = tanh_f(gxr[2 * H + j] + rg * hc);
        hn = zg * hp + (1.f - zg) * ng;
        sv[j] = rg; sv[H + j] = zg; sv[2 * H + j] = ng; sv[3 * H + j] = hc;
      }
    } else {
      if (valid) {
        const float a = gxr[j] + acc[0][r] + bh[0];
        hn = MODE == M_TANH ? tanh_f(a) : fmaxf(a, 0.f);
      }
    }
    p.hall[(size_t)(p.s + 1) * B * H + (size_t)b * H + j] = hn;
    p.y[(tBG + b) * H + j] = valid ? hn : 0.f;
  }
}

struct BwdArgs {
  const float* dy;       // [T][B][H] (time index) or null
  const float* whh;      // [G*H][H]
  const int* lens;
  const float* hall;     // [T+1][B][H]
  const float* call;     // [T+1][B][H]
  const float* save;     // [T][B][S*H]
  float* dgx;            // [T][B][G*H] (step index)
  float* dgh;            // [T][B][G*H] (step index)
  float* dpass;          // [B][H]: the direct part of dh carried to the step before (in: from s+1)
  float* dc;             // [B][H]: LSTM cell gradient (in: from s+1, out: to s-1)
  float* dh0;            // [B][H] written by the final (s = -1) launch
  int T, B, H, s, t;     // s = -1: dh0 = dG_h(0) W_hh + dpass only
};

template <int MODE>
__global__ __launch_bounds__(256) void rnn_bwd_step(BwdArgs p) {
  constexpr int G = Gates<MODE>::G, S = Saved<MODE>::S;
  __shared__ float as[BB * PITCH];
  __shared__ float ws[KC * (UB + 1)];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int j0 = blockIdx.x * UB, b0 = blockIdx.y * BB;
  const int B = p.B, H = p.H, GH = G * H;
  // recurrent part of dh(s): dG_h(s+1) W_hh (nothing past the last step)
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (p.s + 1 < p.T) {
    const float* gnext = p.dgh + (size_t)(p.s + 1) * B * GH;
    for (int k0 = 0; k0 < GH; k0 += KC) {
      for (int e = tid; e < BB * KC; e += 256) {
        const int r = e / KC, k = e - r * KC;
        const int b = b0 + r, kk = k0 + k;
        as[r * PITCH + k] = (b < B && kk < GH) ? gnext[(size_t)b * GH + kk] : 0.f;
      }
      for (int e = tid; e < KC * UB; e += 256) {
        const int k = e / UB, c = e - k * UB;
        const int kk = k0 + k, j = j0 + c;
        ws[k * (UB + 1) + c] = (kk < GH && j < H) ? p.whh[(size_t)kk * H + j] : 0.f;
      }
      __syncthreads();
#pragma unroll
      for (int kk = 0; kk < KC; kk += 8) {
        const float a0 = as[(wid * 16 + (lane & 15)) * PITCH + kk + (lane >> 4)];
        const float w0 = ws[(kk + (lane >> 4)) * (UB + 1) + (lane & 15)];
        acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, w0, acc0, 0, 0, 0);
        const float a1 = as[(wid * 16 + (lane & 15)) * PITCH + kk + 4 + (lane >> 4)];
        const float w1 = ws[(kk + 4 + (lane >> 4)) * (UB + 1) + (lane & 15)];
        acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, w1, acc1, 0, 0, 0);
      }
      __syncthreads();
    }
  }
  const int j = j0 + (lane & 15);
  if (j >= H) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + wid * 16 + 4 * (lane >> 4) + r;
    if (b >= B) continue;
    const size_t bj = (size_t)b * H + j;
    float dh = acc0[r] + acc1[r] + p.dpass[bj];
    if (p.s < 0) {   // gradient of the initial state
      p.dh0[bj] = dh;
      continue;
    }
    const bool valid = !p.lens || p.t < p.lens[b];
    if (valid && p.dy) dh += p.dy[((size_t)p.t * B + b) * H + j];
    float* gx = p.dgx + ((size_t)p.s * B + b) * GH;
    float* gh = p.dgh + ((size_t)p.s * B + b) * GH;
    if (!valid) {   // the state passed through: all of dh (and dc) goes on to step s - 1
#pragma unroll
      for (int g = 0; g < G; ++g) gx[g * H + j] = gh[g * H + j] = 0.f;
      p.dpass[bj] = dh;
      continue;
    }
    const float* sv = S ? p.save + ((size_t)p.s * B + b) * (S * H) : nullptr;
    if constexpr (MODE == M_LSTM) {
      const float ig = sv[j], fg = sv[H + j], gg = sv[2 * H + j], og = sv[3 * H + j];
      const float cp = p.call[(size_t)p.s * B * H + bj], cn = p.call[(size_t)(p.s + 1) * B * H + bj];
      const float tc = tanh_f(cn);
      const float dcv = dh * og * (1.f - tc * tc) + p.dc[bj];
      const float da_i = dcv * gg * ig * (1.f - ig);
      const float da_f = dcv * cp * fg * (1.f - fg);
      const float da_g = dcv * ig * (1.f - gg * gg);
      const float da_o = dh * tc * og * (1.f - og);
      gx[j] = gh[j] = da_i;
      gx[H + j] = gh[H + j] = da_f;
      gx[2 * H + j] = gh[2 * H + j] = da_g;
      gx[3 * H + j] = gh[3 * H + j] = da_o;
      p.dc[bj] = dcv * fg;
      p.dpass[bj] = 0.f;
    } else if constexpr (MODE == M_GRU) {
      const float rg = sv[j], zg = sv[H + j], ng = sv[2 * H + j], hc = sv[3 * H + j];
      const float hp = p.hall[(size_t)p.s * B * H + bj];
      const float dz = dh * (hp - ng);
      const float dan = dh * (1.f - zg) * (1.f - ng * ng);
      const float dar = dan * hc * rg * (1.f - rg);
      const float daz = dz * zg * (1.f - zg);
      gx[j] = gh[j] = dar;
      gx[H + j] = gh[H + j] = daz;
      gx[2 * H + j] = dan;
      gh[2 * H + j] = dan * rg;
      p.dpass[bj] = dh * zg;
    } else {
      const float hn = p.hall[(size_t)(p.s + 1) * B * H + bj];
      const float da = MODE == M_TANH ? dh * (1.f - hn * hn) : (hn > 0.f ? dh : 0.f);
      gx[j] = gh[j] = da;
      p.dpass[bj] = 0.f;
    }
  }
}

// ---- v2 step kernels --------------------------------------------------------------------------
// Forward: a workgroup owns UPW hidden units (4 for LSTM / GRU: MFMA column c = gate * 4 + unit;
// 16 for SimpleRNN) x 64 batch rows (16 per wave), so H = 512 gives 128 workgroups instead of 32.
// Its 16 W_hh rows are staged in LDS once per step in 512-deep chunks (16-B loads); the h rows go
// straight from L2 into registers, 16 B per lane per 16-deep k block, and the k order inside a
// block is permuted identically for both operands (lane group q, k-step i <-> element 4q + i), so
// one 16-B load feeds four MFMAs. Two accumulators alternate (the f32 MFMA's dependent latency is
// above its issue interval). The gates of a (row, unit) then meet in one lane through a small LDS
// transpose of the wave's 16 x 16 result.
constexpr int KCH = 512;

template <typename T> __device__ __forceinline__ f32x4 ld4(const T* p) { return *reinterpret_cast<const f32x4*>(p); }

template <int MODE, bool VEC>
__global__ __launch_bounds__(256) void rnn_fwd_step2(FwdArgs p) {
  constexpr int G = Gates<MODE>::G, S = Saved<MODE>::S;
  constexpr int UPW = G == 1 ? 16 : 4;
  __shared__ __attribute__((aligned(16))) float ws[16 * (KCH + 4)];
  __shared__ float dt[4 * 16 * 17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4;
  const int j0 = blockIdx.x * UPW, b0 = blockIdx.y * BB;
  const int B = p.B, H = p.H, GH = G * H;
  const float* hprev = p.hall + (size_t)p.s * B * H;
  const int arow = b0 + wid * 16 + (lane & 15);
  const float* hr = hprev + (size_t)min(arow, B - 1) * H;
  const bool arow_ok = arow < B;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < H; k0 += KCH) {
    const int kc = min(KCH, H - k0);
    const int kcp = (kc + 15) & ~15;
    // W rows of the 16 columns (zero for unused columns and past kc)
    if constexpr (VEC) {
      for (int e = tid; e < 16 * (kcp >> 2); e += 256) {
        const int c = e / (kcp >> 2), k = (e - c * (kcp >> 2)) * 4;
        const int g = c / UPW, u = c - g * UPW;
        f32x4 v = {0.f, 0.f, 0.f, 0.f};
        if (g < G && j0 + u < H && k < kc) v = ld4(p.whh + (size_t)(g * H + j0 + u) * H + k0 + k);
        *reinterpret_cast<f32x4*>(&ws[c * (KCH + 4) + k]) = v;
      }
    } else {
      for (int e = tid; e < 16 * kcp; e += 256) {
        const int c = e / kcp, k = e - c * kcp;
        const int g = c / UPW, u = c - g * UPW;
        ws[c * (KCH + 4) + k] = (g < G && j0 + u < H && k < kc) ? p.whh[(size_t)(g * H + j0 + u) * H + k0 + k] : 0.f;
      }
    }
    __syncthreads();
    const float* wr = &ws[(lane & 15) * (KCH + 4) + 4 * q];
    for (int blk = 0; blk < (kcp >> 4); ++blk) {
      const int k = k0 + blk * 16 + 4 * q;
      f32x4 a;
      if constexpr (VEC) {
        a = (arow_ok && k < H) ? ld4(hr + k) : f32x4{0.f, 0.f, 0.f, 0.f};
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) a[i] = (arow_ok && k + i < H) ? hr[k + i] : 0.f;
      }
      const f32x4 b = *reinterpret_cast<const f32x4*>(wr + blk * 16);
      if (blk & 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], acc1, 0, 0, 0);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[i], acc0, 0, 0, 0);
      }
    }
    __syncthreads();
  }
  const f32x4 acc = acc0 + acc1;   // D[row 4q + r][col lane & 15] of the wave's 16 rows
  const size_t tBG = (size_t)p.t * B;
  auto cell = [&](int b, int j, const float (&pre)[4]) {   // pre: the G hidden-side products
    const bool valid = !p.lens || p.t < p.lens[b];
    const float hp = hprev[(size_t)b * H + j];
    float hn = hp, cn = 0.f;
    const float* gxr = p.gx + (tBG + b) * GH;
    float* sv = S ? p.save + ((size_t)p.s * B + b) * (S * H) : nullptr;
    float bh[G];
#pragma unroll
    for (int g = 0; g < G; ++g) bh[g] = p.bhh ? p.bhh[g * H + j] : 0.f;
    if constexpr (MODE == M_LSTM) {
      const float cp = p.call[(size_t)p.s * B * H + (size_t)b * H + j];
      cn = cp;
      if (valid) {
        const float ig = sigm(gxr[j] + pre[0] + bh[0]);
        const float fg = sigm(gxr[H + j] + pre[1] + bh[1]);
        const float gg = tanh_f(gxr[2 * H + j] + pre[2] + bh[2]);
        const float og = sigm(gxr[3 * H + j] + pre[3] + bh[3]);
        cn = fg * cp + ig * gg;
        hn = og * tanh_f(cn);
        sv[j] = ig; sv[H + j] = fg; sv[2 * H + j] = gg; sv[3 * H + j] = og;
      }
      p.call[(size_t)(p.s + 1) * B * H + (size_t)b * H + j] = cn;
    } else if constexpr (MODE == M_GRU) {
      if (valid) {
        const float rg = sigm(gxr[j] + pre[0] + bh[0]);
        const float zg = sigm(gxr[H + j] + pre[1] + bh[1]);
        const float hc = pre[2] + bh[2];
        const float ng = tanh_f(gxr[2 * H + j] + rg * hc);
        hn = zg * hp + (1.f - zg) * ng;
        sv[j] = rg; sv[H + j] = zg; sv[2 * H + j] = ng; sv[3 * H + j] = hc;
      }
    } else {
      if (valid) {
        const float a = gxr[j] + pre[0] + bh[0];
        hn = MODE == M_TANH ? tanh_f(a) : fmaxf(a, 0.f);
      }
    }
    p.hall[(size_t)(p.s + 1) * B * H + (size_t)b * H + j] = hn;
    p.y[(tBG + b) * H + j] = valid ? hn : 0.f;
  };
  if constexpr (G == 1) {   // SimpleRNN: the D layout is already (row, unit) per lane
    const int j = j0 + (lane & 15);
    if (j >= H) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int b = b0 + wid * 16 + 4 * q + r;
      if (b < B) {
        const float pre[4] = {acc[r], 0.f, 0.f, 0.f};
        cell(b, j, pre);
      }
    }
  } else {   // the 16 x 16 tile through LDS: lane -> (row lane >> 2, unit lane & 3)
    float* d = dt + wid * 16 * 17;
#pragma unroll
    for (int r = 0; r < 4; ++r) d[(4 * q + r) * 17 + (lane & 15)] = acc[r];
    __syncthreads();
    const int row = lane >> 2, u = lane & 3;
    const int b = b0 + wid * 16 + row, j = j0 + u;
    if (b < B && j < H) {
      float pre[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int g = 0; g < G; ++g) pre[g] = d[row * 17 + g * 4 + u];
      cell(b, j, pre);
    }
  }
}

// Backward: 16 hidden units x 64 rows per workgroup of 8 waves; waves w and w + 4 share a 16-row
// block and take alternate 16-deep k blocks of the K = G*H reduction dG_h(s+1) W_hh (W_hh's rows
// k, columns of the 16 units, staged in LDS 512 rows at a time), then add through LDS.
template <int MODE, bool VEC>
__global__ __launch_bounds__(512) void rnn_bwd_step2(BwdArgs p) {
  constexpr int G = Gates<MODE>::G, S = Saved<MODE>::S;
  __shared__ float ws[KCH * 17];
  __shared__ float red[4 * 16 * 17];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, q = lane >> 4;
  const int rb = wid & 3, kh = wid >> 2;
  const int j0 = blockIdx.x * UB, b0 = blockIdx.y * BB;
  const int B = p.B, H = p.H, GH = G * H;
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  if (p.s + 1 < p.T) {
    const float* gnext = p.dgh + (size_t)(p.s + 1) * B * GH;
    const int arow = b0 + rb * 16 + (lane & 15);
    const float* ar = gnext + (size_t)min(arow, B - 1) * GH;
    const bool arow_ok = arow < B;
    for (int k0 = 0; k0 < GH; k0 += KCH) {
      const int kc = min(KCH, GH - k0);
      const int kcp = (kc + 15) & ~15;
      if constexpr (VEC) {   // 16 contiguous floats per W row (j0 % 16 == 0, H % 4 == 0)
        for (int e = tid; e < kcp * 4; e += 512) {
          const int k = e >> 2, c = (e & 3) * 4;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (k < kc && j0 + c < H) v = ld4(p.whh + (size_t)(k0 + k) * H + j0 + c);
#pragma unroll
          for (int i = 0; i < 4; ++i) ws[k * 17 + c + i] = v[i];
        }
      } else {
        for (int e = tid; e < kcp * 16; e += 512) {
          const int k = e >> 4, c = e & 15;
          ws[k * 17 + c] = (k < kc && j0 + c < H) ? p.whh[(size_t)(k0 + k) * H + j0 + c] : 0.f;
        }
      }
      __syncthreads();
      for (int blk = kh; blk < (kcp >> 4); blk += 2) {
        const int k = k0 + blk * 16 + 4 * q;
        f32x4 a;
        if constexpr (VEC) {
          a = (arow_ok && k < GH) ? ld4(ar + k) : f32x4{0.f, 0.f, 0.f, 0.f};
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[i] = (arow_ok && k + i < GH) ? ar[k + i] : 0.f;
        }
        const float* wr = &ws[(blk * 16 + 4 * q) * 17 + (lane & 15)];
        if ((blk >> 1) & 1) {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], wr[i * 17], acc1, 0, 0, 0);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], wr[i * 17], acc0, 0, 0, 0);
        }
      }
      __syncthreads();
    }
  }
  f32x4 acc = acc0 + acc1;
  float* rd = red + rb * 16 * 17;
  if (kh == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) rd[(4 * q + r) * 17 + (lane & 15)] = acc[r];
  }
  __syncthreads();
  if (kh == 1) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] += rd[(4 * q + r) * 17 + (lane & 15)];
  const int j = j0 + (lane & 15);
  if (j >= H) return;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int b = b0 + rb * 16 + 4 * q + r;
    if (b >= B) continue;
    const size_t bj = (size_t)b * H + j;
    float dh = acc[r] + p.dpass[bj];
    if (p.s < 0) {
      p.dh0[bj] = dh;
      continue;
    }
    const bool valid = !p.lens || p.t < p.lens[b];
    if (valid && p.dy) dh += p.dy[((size_t)p.t * B + b) * H + j];
    float* gx = p.dgx + ((size_t)p.s * B + b) * GH;
    float* gh = p.dgh + ((size_t)p.s * B + b) * GH;
    if (!valid) {
#pragma unroll
      for (int g = 0; g < G; ++g) gx[g * H + j] = gh[g * H + j] = 0.f;
      p.dpass[bj] = dh;
      continue;
    }
    const float* sv = S ? p.save + ((size_t)p.s * B + b) * (S * H) : nullptr;
    if constexpr (MODE == M_LSTM) {
      const float ig = sv[j], fg = sv[H + j], gg = sv[2 * H + j], og = sv[3 * H + j];
      const float cp = p.call[(size_t)p.s * B * H + bj], cn = p.call[(size_t)(p.s + 1) * B * H + bj];
      const float tc = tanh_f(cn);
      const float dcv = dh * og * (1.f - tc * tc) + p.dc[bj];
      const float da_i = dcv * gg * ig * (1.f - ig);
      const float da_f = dcv * cp * fg * (1.f - fg);
      const float da_g = dcv * ig * (1.f - gg * gg);
      const float da_o = dh * tc * og * (1.f - og);
      gx[j] = gh[j] = da_i;
      gx[H + j] = gh[H + j] = da_f;
      gx[2 * H + j] = gh[2 * H + j] = da_g;
      gx[3 * H + j] = gh[3 * H + j] = da_o;
      p.dc[bj] = dcv * fg;
      p.dpass[bj] = 0.f;
    } else if constexpr (MODE == M_GRU) {
      const float rg = sv[j], zg = sv[H + j], ng = sv[2 * H + j], hc = sv[3 * H + j];
      const float hp = p.hall[(size_t)p.s * B * H + bj];
      const float dz = dh * (hp - ng);
      const float dan = dh * (1.f - zg) * (1.f - ng * ng);
      const float dar = dan * hc * rg * (1.f - rg);
      const float daz = dz * zg * (1.f - zg);
      gx[j] = gh[j] = dar;
      gx[H + j] = gh[H + j] = daz;
      gx[2 * H + j] = dan;
      gh[2 * H + j] = dan * rg;
      p.dpass[bj] = dh * zg;
    } else {
      const float hn = p.hall[(size_t)(p.s + 1) * B * H + bj];
      const float da = MODE == M_TANH ? dh * (1.f - hn * hn) : (hn > 0.f ? dh : 0.f);
      gx[j] = gh[j] = da;
      p.dpass[bj] = 0.f;
    }
  }
}

// PHA_RNN_V1=1: the first (32 workgroups at H = 512) step kernels, for A/B measurements
static bool use_v1() {
  static const bool v = [] {
    const char* e = getenv("PHA_RNN_V1");
    return e && e[0] == '1';
  }();
  return v;
}

template <int MODE>
int fwd(const FwdArgs& a0, int reverse, hipStream_t st) {
  FwdArgs a = a0;
  constexpr int UPW = Gates<MODE>::G == 1 ? 16 : 4;
  const bool vec = a.H % 4 == 0 && ((size_t)a.hall & 15) == 0 && ((size_t)a.whh & 15) == 0;
  const bool v1 = use_v1();
  const dim3 grid1((a.H + UB - 1) / UB, (a.B + BB - 1) / BB), grid2((a.H + UPW - 1) / UPW, (a.B + BB - 1) / BB);
  for (int s = 0; s < a.T; ++s) {
    a.s = s;
    a.t = reverse ? a.T - 1 - s : s;
    if (v1) hipLaunchKernelGGL(rnn_fwd_step<MODE>, grid1, dim3(256), 0, st, a);
    else if (vec) hipLaunchKernelGGL((rnn_fwd_step2<MODE, true>), grid2, dim3(256), 0, st, a);
    else hipLaunchKernelGGL((rnn_fwd_step2<MODE, false>), grid2, dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

template <int MODE>
int bwd(const BwdArgs& a0, int reverse, hipStream_t st) {
  BwdArgs a = a0;
  const bool vec = a.H % 4 == 0 && ((size_t)a.dgh & 15) == 0 && ((size_t)a.whh & 15) == 0;
  const bool v1 = use_v1();
  const dim3 grid((a.H + UB - 1) / UB, (a.B + BB - 1) / BB);
  for (int s = a.T - 1; s >= -1; --s) {
    a.s = s;
    a.t = s < 0 ? 0 : (reverse ? a.T - 1 - s : s);
    if (v1) hipLaunchKernelGGL(rnn_bwd_step<MODE>, grid, dim3(256), 0, st, a);
    else if (vec) hipLaunchKernelGGL((rnn_bwd_step2<MODE, true>), grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL((rnn_bwd_step2<MODE, false>), grid, dim3(512), 0, st, a);
  }
  return (int)hipGetLastError();
}

}  // namespace rnn
}  // namespace pha

using namespace pha;

// One (layer, direction) forward over T steps, fp32. mode: 0 tanh, 1 relu, 2 LSTM, 3 GRU.
// gx [T][B][G*H] (x W_ih^T + b_ih, time order); hall [T+1][B][H] with hall[0] = h0 on entry;
// call likewise (LSTM, else null); save [T][B][4H] (LSTM / GRU, else null); y [T][B][H]; lens [B]
// int32 or null; reverse: step s processes time T-1-s. All buffers contiguous.
PHA_API int pha_rnn_fwd(int mode, int T, int B, int H, const float* gx, const float* whh, const float* bhh,
                        const int* lens, float* y, float* hall, float* call, float* save, int reverse,
                        hipStream_t st) {
  if (T <= 0 || B <= 0 || H <= 0 || !gx || !whh || !y || !hall) return (int)hipErrorInvalidValue;
  if ((mode == rnn::M_LSTM && (!call || !save)) || (mode == rnn::M_GRU && !save) || mode < 0 || mode > 3)
    return (int)hipErrorInvalidValue;
  if ((long)B > 65535L * rnn::BB) return (int)hipErrorInvalidValue;
  rnn::FwdArgs a{gx, whh, bhh, lens, y, hall, call, save, T, B, H, 0, 0};
  switch (mode) {
    case rnn::M_TANH: return rnn::fwd<rnn::M_TANH>(a, reverse, st);
    case rnn::M_RELU: return rnn::fwd<rnn::M_RELU>(a, reverse, st);
    case rnn::M_LSTM: return rnn::fwd<rnn::M_LSTM>(a, reverse, st);
    default: return rnn::fwd<rnn::M_GRU>(a, reverse, st);
  }
}

// Backward of pha_rnn_fwd. dy [T][B][H] (time order, or null); dpass [B][H] holds dh of the final
// state on entry (in place), dc [B][H] dc of the final cell (LSTM, in place; dc0 on exit);
// dgx / dgh [T][B][G*H] (step order) receive the gate gradients; dh0 [B][H].
PHA_API int pha_rnn_bwd(int mode, int T, int B, int H, const float* dy, const float* whh, const int* lens,
                        const float* hall, const float* call, const float* save, float* dgx, float* dgh,
                        float* dpass, float* dc, float* dh0, int reverse, hipStream_t st) {
  if (T <= 0 || B <= 0 || H <= 0 || !whh || !hall || !dgx || !dgh || !dpass || !dh0) return (int)hipErrorInvalidValue;
  if ((mode == rnn::M_LSTM && (!call || !save || !dc)) || (mode == rnn::M_GRU && !save) || mode < 0 || mode > 3)
    return (int)hipErrorInvalidValue;
  if ((long)B > 65535L * rnn::BB) return (int)hipErrorInvalidValue;
  rnn::BwdArgs a{dy, whh, lens, hall, call, save, dgx, dgh, dpass, dc, dh0, T, B, H, 0, 0};
  switch (mode) {
    case rnn::M_TANH: return rnn::bwd<rnn::M_TANH>(a, reverse, st);
    case rnn::M_RELU: return rnn::bwd<rnn::M_RELU>(a, reverse, st);
    case rnn::M_LSTM: return rnn::bwd<rnn::M_LSTM>(a, reverse, st);
    default: return rnn::bwd<rnn::M_GRU>(a, reverse, st);
  }
}
