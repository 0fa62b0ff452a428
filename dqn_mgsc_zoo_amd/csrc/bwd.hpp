// bwd.hpp — backward kernels specialised for the NatureQNetwork at small B.
#pragma once
#include "common.hpp"
#include "fwd.hpp"

namespace dqz {

// ---- fc1 backward: dX + dW + centered RMSProp in one pass over W1 ----------
// grid = 196 blocks of 16 rows of W1 [3136][512].  A block
//   * computes dy3[:, rows] = (dz1 @ W1[rows]^T) * relu'(y3) with the OLD W1
//     rows (M = B samples, N = 16 rows, K = 512 split over the 4 waves), and
//   * accumulates dW1[rows][:] = y3[:, rows]^T @ dz1 (M = 16 rows, N = 512
//     columns, wave w owns columns [128 w, 128 w + 128), K = B), then
//   * applies RMSProp to its rows (or writes the gradient in gradient-output
//     mode).  No other block touches these rows, so reading the old weights
//     for dX and updating them in the same kernel is race-free.
// W1, mu and nu are each read once and written once: the fc1 step is
// HBM-bound at 6 x 6.4 MB.
struct Fc1BwdArgs {
  const float* dz1;  // [B][512]
  const float* y3;   // [B][3136] online activations
  float *th, *mu, *nu;
  int64_t w_off;
  Rms rms;
  int B;
  float* dy3;  // [B][3136]
};

__global__ __launch_bounds__(256) void fc1_bwd_kernel(Fc1BwdArgs a) {
  DQZ_STAMP(5, 0);
  __shared__ float s_red[4][2][256];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  const int k0 = 16 * blockIdx.x;
  const float* W1 = a.th + a.w_off;
  float4 wv[8];  // W1[k0 + n][128 w + 16 j + 4 kq + e]
#pragma unroll
  for (int j = 0; j < 8; ++j)
    wv[j] = *reinterpret_cast<const float4*>(W1 + (int64_t)(k0 + n) * HID + 128 * w + 16 * j + 4 * kq);
  // The RMSProp operands of this lane's 32 dW entries, loaded up front so
  // their latency hides under the GEMMs.  Entry (q, r): row k0 + 4 kq + r,
  // column 128 w + 16 q + n (the C layout of the dW tiles).
  const int64_t e0 = a.w_off + (int64_t)(k0 + 4 * kq) * HID + 128 * w + n;
  float o_th[32], o_mu[32], o_nu[32];
  if (!a.rms.gout) {
#pragma unroll
    for (int q = 0; q < 8; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t i = e0 + r * HID + 16 * q;
        o_th[4 * q + r] = a.th[i];
        o_mu[4 * q + r] = a.mu[i];
        o_nu[4 * q + r] = a.nu[i];
      }
  }
  f32x4 gacc[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) gacc[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c = 0; c < a.B; c += 32) {
    // dX rows of samples [c, c + 32)
    f32x4 xacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const int row = min(c + 16 * mt + n, a.B - 1);
      const float* d = a.dz1 + (int64_t)row * HID + 128 * w + 4 * kq;
      float4 av[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) av[j] = *reinterpret_cast<const float4*>(d + 16 * j);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xacc[mt] = mfma4(av[j].x, wv[j].x, xacc[mt]);
        xacc[mt] = mfma4(av[j].y, wv[j].y, xacc[mt]);
        xacc[mt] = mfma4(av[j].z, wv[j].z, xacc[mt]);
        xacc[mt] = mfma4(av[j].w, wv[j].w, xacc[mt]);
      }
    }
    // dW over the chunk's samples: A = y3[b][k0 + m], B = dz1[b][128 w + 16 q + n]
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int b = c + 4 * kk + kq;
      const int bb = min(b, a.B - 1);
      const float yv = a.y3[(int64_t)bb * FLAT + k0 + n];
      const float av = b < a.B ? yv : 0.f;
      const float* d = a.dz1 + (int64_t)bb * HID + 128 * w + n;
#pragma unroll
      for (int q = 0; q < 8; ++q) gacc[q] = mfma4(av, d[16 * q], gacc[q]);
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_red[w][mt][(4 * kq + r) * 16 + n] = xacc[mt][r];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int sample = c + 16 * h + (t >> 4);
      const float v = (s_red[0][h][t] + s_red[1][h][t]) + (s_red[2][h][t] + s_red[3][h][t]);
      if (sample < a.B) {
        const int64_t i = (int64_t)sample * FLAT + k0 + (t & 15);
        a.dy3[i] = a.y3[i] > 0.f ? v : 0.f;
      }
    }
    __syncthreads();
  }
  DQZ_STAMP(5, 2);
  const Rms& R = a.rms;
#pragma unroll
  for (int q = 0; q < 8; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t i = e0 + r * HID + 16 * q;
      const float g = gacc[q][r];
      if (R.gout) {
        R.gout[i] = g;
      } else {
        const float m = R.c1 * g + R.decay * o_mu[4 * q + r];
        const float v = R.c1 * (g * g) + R.decay * o_nu[4 * q + r];
        a.mu[i] = m;
        a.nu[i] = v;
        a.th[i] = o_th[4 * q + r] + (-R.lr) * (g * rsqrtf(v - m * m + R.eps));
      }
    }
  DQZ_STAMP(5, 3);
}

// ---- conv3 backward: dX and per-sample dW partials -----------------------
// grid (12, B).  Jobs 0..7: dX of input-channel quarter (job & 3) for output
// rows half (job >> 2): dy2 = conv_transpose(dy3, W3) * relu'(y2), computed
// as a correlation of dy3 zero-padded by 2 with the flipped kernel.  Jobs
// 8..11: dW partial of output-channel quarter (job - 8) for this sample:
// part[b][(kh*3 + kw)*64 + ci][co] = sum_p y2[b][oh+kh][ow+kw][ci] dy3[b][p][co],
// bias row 576 = sum_p dy3[b][p][co].  The update kernel sums the B slabs.
constexpr int C3X_S = 66, C3X_RS = 754, C3X_WIN = 11 * C3X_RS;  // padded dy3 window, 8294 floats
constexpr int C3W_S = 80, C3W_RS = 720, C3W_WIN = 9 * C3W_RS;   // y2 window for dW, 6480 floats

struct Conv3BwdArgs {
  const float* dy3;  // [B][49][64]
  const float* y2;   // [B][81][64] online
  const float* w3;   // online W3 [3][3][64][64]
  float* dy2;        // [B][81][64]
  float* part;       // [B][577][64]
  int B;
};

__device__ __forceinline__ void conv3_bwd_dx(const Conv3BwdArgs& a, float* s_win, int b, int nq, int mh) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  // B operand: flipped kernel, k = (tap' = kh'*3 + kw', co), wave w owns co [16w, 16w + 16)
  float wr[36];
#pragma unroll
  for (int kk = 0; kk < 36; ++kk) {
    const int tap = 8 - (kk >> 2);  // (2 - kh')*3 + (2 - kw')
    wr[kk] = a.w3[(tap * C3CI + 16 * nq + n) * C3CO + 16 * w + 4 * (kk & 3) + kq];
  }
  // padded dy3 window: (ph, pw) in 11 x 11, interior [2, 9)
  const float4* src = reinterpret_cast<const float4*>(a.dy3 + (int64_t)b * FLAT);
  constexpr int NW4 = 121 * 16;  // 1936
  float4 r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = min(t + 256 * q, NW4 - 1);
    const int pix = i >> 4, ph = pix / 11 - 2, pw = pix % 11 - 2;
    const bool in = ph >= 0 && ph < C3O && pw >= 0 && pw < C3O;
    const float4 v = src[(in ? ph * C3O + pw : 0) * 16 + (i & 15)];
    r[q] = in ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = t + 256 * q;
    if (i < NW4) {
      const int pix = i >> 4;
      float* d = s_win + (pix / 11) * C3X_RS + (pix % 11) * C3X_S + (i & 15) * 4;
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  __syncthreads();
  int base[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int p = min(48 * mh + 16 * m + n, C2M - 1);
    base[m] = (p / C2O) * C3X_RS + (p % C2O) * C3X_S + 16 * w + kq;
  }
  f32x4 acc[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 36; ++kk) {
    const int tp = kk >> 2;  // tap' = kh'*3 + kw'
    const int off = (tp / 3) * C3X_RS + (tp % 3) * C3X_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < 3; ++m) acc[m] = mfma4(s_win[base[m] + off], wr[kk], acc[m]);
  }
  __syncthreads();
  float* s_red = s_win;  // [4][48][16]
#pragma unroll
  for (int m = 0; m < 3; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * 768 + (16 * m + 4 * kq + rr) * 16 + n] = acc[m][rr];
  __syncthreads();
  for (int i = t; i < 768; i += 256) {
    const int p = 48 * mh + (i >> 4);
    if (p < C2M) {
      const float v = (s_red[i] + s_red[768 + i]) + (s_red[1536 + i] + s_red[2304 + i]);
      const int64_t o = ((int64_t)b * C2M + p) * C2CO + 16 * nq + (i & 15);
      a.dy2[o] = a.y2[o] > 0.f ? v : 0.f;
    }
  }
}

__device__ __forceinline__ void conv3_bwd_dw(const Conv3BwdArgs& a, float* s_win, int b, int nq) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  // B operand: dy3[b][p = 4 kk + kq][16 nq + n], zero for p >= 49
  float dr[13];
#pragma unroll
  for (int kk = 0; kk < 13; ++kk) {
    const int p = 4 * kk + kq;
    const float v = a.dy3[((int64_t)b * C3M + min(p, C3M - 1)) * C3CO + 16 * nq + n];
    dr[kk] = p < C3M ? v : 0.f;
  }
  const float4* src = reinterpret_cast<const float4*>(a.y2 + (int64_t)b * (C2M * C2CO));
  constexpr int NQ4 = C2M * C2CO / 4;  // 1296
  float4 r[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) r[q] = src[min(t + 256 * q, NQ4 - 1)];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 4;
      *reinterpret_cast<float4*>(s_win + (pix / C2O) * C3W_RS + (pix % C2O) * C3W_S + (i & 15) * 4) = r[q];
    }
  }
  __syncthreads();
  // A operand: y2 window at (oh + kh, ow + kw), ci = 16 w + n; position p = 4 kk + kq
  int pb[13];
#pragma unroll
  for (int kk = 0; kk < 13; ++kk) {
    const int p = min(4 * kk + kq, C3M - 1);
    pb[kk] = (p / C3O) * C3W_RS + (p % C3O) * C3W_S + 16 * w + n;
  }
  f32x4 acc[9];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp) acc[tp] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 13; ++kk)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int off = (tp / 3) * C3W_RS + (tp % 3) * C3W_S;
      acc[tp] = mfma4(s_win[pb[kk] + off], dr[kk], acc[tp]);
    }
  // C layout: row = 4 kq + r -> ci = 16 w + 4 kq + r of tap tp; col = co = n
  float* part = a.part + (int64_t)b * (C3KK + 1) * C3CO + 16 * nq + n;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) part[(tp * C3CI + 16 * w + 4 * kq + rr) * C3CO] = acc[tp][rr];
  if (w == 0) {  // bias row: sum over positions, lanes kq = 0..3 hold p = 4 kk + kq
    float sb = 0.f;
#pragma unroll
    for (int kk = 0; kk < 13; ++kk) sb += dr[kk];
    sb += __shfl_xor(sb, 16, 64);
    sb += __shfl_xor(sb, 32, 64);
    if (kq == 0) part[C3KK * C3CO] = sb;
  }
}

__global__ __launch_bounds__(256) void conv3_bwd_kernel(Conv3BwdArgs a) {
  DQZ_STAMP(6, 0);
  __shared__ float s_win[C3X_WIN];
  const int job = blockIdx.x, b = blockIdx.y;
  if (job < 8)
    conv3_bwd_dx(a, s_win, b, job & 3, job >> 2);
  else
    conv3_bwd_dw(a, s_win, b, job - 8);
  DQZ_STAMP(6, 3);
}

// ---- conv2 backward: dX by stride phase and per-sample dW partials --------
// grid (12, B).  Jobs 0..7: dX of stride phase (ph, pw) = (job & 3) >> 1,
// job & 1 for input-channel half job >> 2: output pixels (2a + ph, 2c + pw),
// a, c in [0, 10), are a 2x2-tap correlation of dy2 zero-padded by 1 with
// W2[ph + 2(1 - u)][pw + 2(1 - v)] (K = 4 taps x 64 co), masked by relu'(y1).
// Jobs 8..11: dW partial of output-channel quarter (job - 8):
// part[b][(kh*4 + kw)*32 + ci][co] = sum_p y1[b][2oh+kh][2ow+kw][ci] dy2[b][p][co]
// (bias row 512 = sum_p dy2).  Wave w of a dW job owns kh = w.
constexpr int C2X_S = 66, C2X_RS = 756, C2X_WIN = 11 * C2X_RS;  // padded dy2 window, 8316 floats
constexpr int C2W_S = 40, C2W_RS = 808, C2W_WIN = 20 * C2W_RS;  // y1 window for dW, 16160 floats

struct Conv2BwdArgs {
  const float* dy2;  // [B][81][64]
  const float* y1;   // [B][400][32] online
  const float* w2;   // online W2 [4][4][32][64]
  float* dy1;        // [B][400][32]
  float* part;       // [B][513][64]
  int B;
};

__device__ __forceinline__ void conv2_bwd_dx(const Conv2BwdArgs& a, float* s_win, int b, int ph, int pw, int hh) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  float wr[16];
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int tp = kk >> 2, u = tp >> 1, v = tp & 1;
    const int kh = ph + 2 * (1 - u), kw = pw + 2 * (1 - v);
    wr[kk] = a.w2[((kh * C2K + kw) * C2CI + 16 * hh + n) * C2CO + 16 * w + 4 * (kk & 3) + kq];
  }
  const float4* src = reinterpret_cast<const float4*>(a.dy2 + (int64_t)b * (C2M * C2CO));
  constexpr int NW4 = 121 * 16;  // 1936
  float4 r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = min(t + 256 * q, NW4 - 1);
    const int pix = i >> 4, oh = pix / 11 - 1, ow = pix % 11 - 1;
    const bool in = oh >= 0 && oh < C2O && ow >= 0 && ow < C2O;
    const float4 v = src[(in ? oh * C2O + ow : 0) * 16 + (i & 15)];
    r[q] = in ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = t + 256 * q;
    if (i < NW4) {
      const int pix = i >> 4;
      float* d = s_win + (pix / 11) * C2X_RS + (pix % 11) * C2X_S + (i & 15) * 4;
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  __syncthreads();
  int base[7];
#pragma unroll
  for (int m = 0; m < 7; ++m) {
    const int p = min(16 * m + n, 99);  // p = 10 a + c
    base[m] = (p / 10) * C2X_RS + (p % 10) * C2X_S + 16 * w + kq;
  }
  f32x4 acc[7];
#pragma unroll
  for (int m = 0; m < 7; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) {
    const int tp = kk >> 2;  // (u', v') = (tp >> 1, tp & 1)
    const int off = (tp >> 1) * C2X_RS + (tp & 1) * C2X_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < 7; ++m) acc[m] = mfma4(s_win[base[m] + off], wr[kk], acc[m]);
  }
  __syncthreads();
  float* s_red = s_win;  // [4][112][16]
#pragma unroll
  for (int m = 0; m < 7; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * 1792 + (16 * m + 4 * kq + rr) * 16 + n] = acc[m][rr];
  __syncthreads();
  for (int i = t; i < 1600; i += 256) {
    const int p = i >> 4, ah = p / 10, cw = p % 10;
    const float v = (s_red[i] + s_red[1792 + i]) + (s_red[3584 + i] + s_red[5376 + i]);
    const int64_t o = ((int64_t)b * C1M + (2 * ah + ph) * C1O + 2 * cw + pw) * C1CO + 16 * hh + (i & 15);
    a.dy1[o] = a.y1[o] > 0.f ? v : 0.f;
  }
}

__device__ __forceinline__ void conv2_bwd_dw(const Conv2BwdArgs& a, float* s_win, int b, int nq) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;  // w = kh
  const int n = lane & 15, kq = lane >> 4;
  float dr[21];
#pragma unroll
  for (int kk = 0; kk < 21; ++kk) {
    const int p = 4 * kk + kq;
    const float v = a.dy2[((int64_t)b * C2M + min(p, C2M - 1)) * C2CO + 16 * nq + n];
    dr[kk] = p < C2M ? v : 0.f;
  }
  const float4* src = reinterpret_cast<const float4*>(a.y1 + (int64_t)b * (C1M * C1CO));
  constexpr int NQ4 = C1M * C1CO / 4;  // 3200
  float4 r[13];
#pragma unroll
  for (int q = 0; q < 13; ++q) r[q] = src[min(t + 256 * q, NQ4 - 1)];
#pragma unroll
  for (int q = 0; q < 13; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 3;
      *reinterpret_cast<float4*>(s_win + (pix / C1O) * C2W_RS + (pix % C1O) * C2W_S + (i & 7) * 4) = r[q];
    }
  }
  __syncthreads();
  int pb[21];
#pragma unroll
  for (int kk = 0; kk < 21; ++kk) {
    const int p = min(4 * kk + kq, C2M - 1);
    pb[kk] = (2 * (p / C2O) + w) * C2W_RS + 2 * (p % C2O) * C2W_S + n;
  }
  f32x4 acc[8];  // tile = (kw, ci half)
#pragma unroll
  for (int m = 0; m < 8; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 21; ++kk)
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int off = (m >> 1) * C2W_S + 16 * (m & 1);
      acc[m] = mfma4(s_win[pb[kk] + off], dr[kk], acc[m]);
    }
  float* part = a.part + (int64_t)b * (C2KK + 1) * C2CO + 16 * nq + n;
#pragma unroll
  for (int m = 0; m < 8; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr)
      part[((w * C2K + (m >> 1)) * C2CI + 16 * (m & 1) + 4 * kq + rr) * C2CO] = acc[m][rr];
  if (w == 0) {
    float sb = 0.f;
#pragma unroll
    for (int kk = 0; kk < 21; ++kk) sb += dr[kk];
    sb += __shfl_xor(sb, 16, 64);
    sb += __shfl_xor(sb, 32, 64);
    if (kq == 0) part[C2KK * C2CO] = sb;
  }
}

__global__ __launch_bounds__(256) void conv2_bwd_kernel(Conv2BwdArgs a) {
  DQZ_STAMP(7, 0);
  __shared__ float s_win[C2W_WIN];
  const int job = blockIdx.x, b = blockIdx.y;
  if (job < 8)
    conv2_bwd_dx(a, s_win, b, (job & 3) >> 1, job & 1, job >> 2);
  else
    conv2_bwd_dw(a, s_win, b, job - 8);
  DQZ_STAMP(7, 3);
}

}  // namespace dqz
