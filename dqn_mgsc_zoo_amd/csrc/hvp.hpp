// hvp.hpp — Hessian-vector product of one sample's Q-value for the
// second-order MGSC meta-gradient (dqn_mgsc_batched_reservoir/agent.py: its
// meta_loss_fn has no stop_gradient on theta'', so d theta''/d theta' brings
// in the Hessian of the online transition's loss).
//
// Forward-over-reverse for a single sample (B = 1), ReLU masks held fixed:
//   tangent forward  zdot_l = Wdot_l * y_{l-1} + W_l * ydot_{l-1} + bdot_l,
//                    ydot_l = relu'(y_l) zdot_l;
//   tangent backward ddot_l = relu'(y_l) (Wdot_{l+1}^T d_{l+1} + W_{l+1}^T ddot_{l+1});
//   d/deps grad     dW_l = sum_p (ydot_{l-1} (x) d_l + y_{l-1} (x) ddot_l), db_l = sum_p ddot_l,
// with d_l the unit-cotangent backward signals of q[a] (d_5 = e_a).
//
// Eight launches, one per dependent stage (t1 t2 t3 t4 b3 b2 b1, then every
// parameter-gradient block in one launch).  Each stage splits its reduction
// over the threads of a workgroup and sums the splits through LDS in a fixed
// order (deterministic, no partial-sum launches); the two passes over fc1's
// 3136 x 512 weights (t4, b3) read whole rows with coalesced 8- / 16-byte
// loads over hundreds of workgroups (they are the chain's HBM traffic:
// 2 x 2 x 6.4 MB).  t4's K-chunk partials are summed by the gradient launch,
// the only consumer of the fc1 tangent output.
#pragma once
#include "common.hpp"

namespace dqz {

struct HvpArgs {
  // x: the online transition's s_tm1 from a one-slot frame store
  const uint8_t* frames;
  const int32_t* fidx;
  const int32_t* slot;
  const int32_t* action;  // store action table (a = action[slot])
  const float* th;        // primal params theta'
  const float* tw;        // tangent params w (same layout)
  int64_t off[10];
  int A;
  // primal activations and unit-cotangent backward signals at theta'
  const float *y1, *y2, *y3, *h;  // [400*32], [81*64], [3136], [512]
  const float *d1, *d2, *d3, *d4; // same shapes (pre-activation grads of q[a])
  // tangent scratch
  float *ty1, *ty2, *ty3, *td4, *td3, *td2, *td1;
  float* hq;    // output, parameter layout
  float* part;  // [HVP_T4_CHUNKS][512] fc1 tangent K-chunk partials
  // grad q . w: the meta_second_kernel partials, summed once (t1's last block)
  const float* s1_part;
  int s1_nparts;
  float* s1;  // [1]
  // meta_combine in hvp_g_kernel's epilogue (vout != null): instead of H_q w
  // -> hq, v = v_dir + J (alpha s1 grad q - clip(td') H_q w) -> vout,
  // alpha = [|td'| < bound]
  const float *vdir, *J, *gq, *td;
  float bound;
  float* vout;
};

// One element of hvp_g_kernel's output: H_q w itself, or meta_combine's v.
struct HqOut {
  float a_s1, clip;  // alpha s1, clip(td')
  __device__ __forceinline__ HqOut(const HvpArgs& a) {
    if (a.vout) {
      const float td = a.td[0];
      a_s1 = fabsf(td) < a.bound ? a.s1[0] : 0.f;
      clip = fminf(fmaxf(td, -a.bound), a.bound);
    } else {
      a_s1 = clip = 0.f;
    }
  }
  __device__ __forceinline__ void put(const HvpArgs& a, int64_t i, float hq) const {
    if (a.vout)
      a.vout[i] = a.vdir[i] + a.J[i] * (a_s1 * a.gq[i] - clip * hq);
    else
      a.hq[i] = hq;
  }
};

constexpr int HVP_T4_KC = 16, HVP_T4_CHUNKS = FLAT / HVP_T4_KC;  // 196 chunks of 16 rows

__device__ __forceinline__ float hvp_x(const HvpArgs& a, int ih, int iw, int ci) {
  const int f = a.fidx[(int64_t)a.slot[0] * 8 + ci];
  return f < 0 ? 0.f : u8n(a.frames[(int64_t)f * FB + ih * FW + iw]);
}

// 1. conv1 tangent: ty1[p][co] = relu'(y1) (bdot1[co] + sum_k x_p[k] Wdot1[k][co]).
// Block p (400), thread (kh = t / 32, co = t % 32) sums kw, ci; the 8 kh
// partials are summed in order.  Block 400 sums the s1 partials.
__global__ __launch_bounds__(256) void hvp_t1_kernel(HvpArgs a) {
  __shared__ float s_x[C1KK];
  __shared__ float s_r[C1K][C1CO];
  __shared__ float s_w[4];
  const int t = threadIdx.x;
  if (blockIdx.x == C1M) {
    float v = 0.f;
    for (int j = t; j < a.s1_nparts; j += 256) v += a.s1_part[j];
    v = block_sum256(v, s_w);
    if (t == 0) a.s1[0] = v;
    return;
  }
  const int p = blockIdx.x, oh = p / C1O, ow = p % C1O;
  {
    const int kh = t >> 5, kw = (t >> 2) & 7, ci = t & 3;
    s_x[t] = hvp_x(a, C1S * oh + kh, C1S * ow + kw, ci);
  }
  __syncthreads();
  const int kh = t >> 5, co = t & 31;
  const float* W = a.tw + a.off[0];
  float z = 0.f;
#pragma unroll
  for (int j = 0; j < C1K * FC; ++j) {
    const int k = kh * C1K * FC + j;  // (kh, kw = j / 4, ci = j % 4)
    z += s_x[k] * W[k * C1CO + co];
  }
  s_r[kh][co] = z;
  __syncthreads();
  if (t < C1CO) {
    float s = a.tw[a.off[1] + t];
#pragma unroll
    for (int k = 0; k < C1K; ++k) s += s_r[k][t];
    a.ty1[p * C1CO + t] = a.y1[p * C1CO + t] > 0.f ? s : 0.f;
  }
}

// 2. conv2 tangent: ty2 = relu'(y2) (bdot2 + conv(y1, Wdot2) + conv(ty1, W2)).
// Block (p, 16-channel group g); thread (tap = t / 16 = kh * 4 + kw, co).
__global__ __launch_bounds__(256) void hvp_t2_kernel(HvpArgs a) {
  __shared__ float s_r[16][16];
  const int t = threadIdx.x, p = blockIdx.x, g = blockIdx.y;
  const int oh = p / C2O, ow = p % C2O, tap = t >> 4, kh = tap >> 2, kw = tap & 3;
  const int co = 16 * g + (t & 15);
  const int src = ((oh * C2S + kh) * C1O + ow * C2S + kw) * C1CO;
  const float *W = a.th + a.off[2] + tap * C2CI * C2CO + co, *Wd = a.tw + a.off[2] + tap * C2CI * C2CO + co;
  float z = 0.f;
#pragma unroll 8
  for (int ci = 0; ci < C2CI; ++ci) z += a.y1[src + ci] * Wd[ci * C2CO] + a.ty1[src + ci] * W[ci * C2CO];
  s_r[tap][t & 15] = z;
  __syncthreads();
  if (t < 16) {
    const int c = 16 * g + t;
    float s = a.tw[a.off[3] + c];
#pragma unroll
    for (int k = 0; k < 16; ++k) s += s_r[k][t];
    a.ty2[p * C2CO + c] = a.y2[p * C2CO + c] > 0.f ? s : 0.f;
  }
}

// 3. conv3 tangent: ty3 = relu'(y3) (bdot3 + conv(y2, Wdot3) + conv(ty2, W3)).
// Block (p, 16-channel group g); thread (input-channel quad s = t / 16, co)
// over the 9 taps.
__global__ __launch_bounds__(256) void hvp_t3_kernel(HvpArgs a) {
  __shared__ float s_r[16][16];
  const int t = threadIdx.x, p = blockIdx.x, g = blockIdx.y;
  const int oh = p / C3O, ow = p % C3O, s = t >> 4;
  const int co = 16 * g + (t & 15);
  const float *W = a.th + a.off[4] + co, *Wd = a.tw + a.off[4] + co;
  float z = 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const int src = ((oh + kh) * C2O + ow + kw) * C2CO + 4 * s;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int wi = (tap * C3CI + 4 * s + e) * C3CO;
      z += a.y2[src + e] * Wd[wi] + a.ty2[src + e] * W[wi];
    }
  }
  s_r[s][t & 15] = z;
  __syncthreads();
  if (t < 16) {
    const int c = 16 * g + t;
    float v = a.tw[a.off[5] + c];
#pragma unroll
    for (int k = 0; k < 16; ++k) v += s_r[k][t];
    a.ty3[p * C3CO + c] = a.y3[p * C3CO + c] > 0.f ? v : 0.f;
  }
}

// 4. fc1 tangent K-chunk partials: part[c][n] = sum_{k in chunk c} y3[k]
// Wdot1[k][n] + ty3[k] W1[k][n] (thread t: columns 2t, 2t + 1; whole-row
// float2 loads), and the fc2-level backward tangent ddot4 = relu'(h)
// Wdot2[:, a] (block 0).
__global__ __launch_bounds__(256) void hvp_t4_kernel(HvpArgs a) {
  const int t = threadIdx.x, c = blockIdx.x;
  const float *W = a.th + a.off[6], *Wd = a.tw + a.off[6];
  float2 z = make_float2(0.f, 0.f);
#pragma unroll
  for (int j = 0; j < HVP_T4_KC; ++j) {
    const int k = c * HVP_T4_KC + j;
    const float2 w = *reinterpret_cast<const float2*>(W + (int64_t)k * HID + 2 * t);
    const float2 wd = *reinterpret_cast<const float2*>(Wd + (int64_t)k * HID + 2 * t);
    const float y = a.y3[k], ty = a.ty3[k];
    z.x += y * wd.x + ty * w.x;
    z.y += y * wd.y + ty * w.y;
  }
  *reinterpret_cast<float2*>(a.part + (int64_t)c * HID + 2 * t) = z;
  if (c == 0) {
    const int act = a.action[a.slot[0]];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int n = t + 256 * h;
      a.td4[n] = a.h[n] > 0.f ? a.tw[a.off[8] + n * a.A + act] : 0.f;
    }
  }
}

// 5. ddot3[k] = relu'(y3[k]) sum_n (Wdot1[k][n] d4[n] + W1[k][n] ddot4[n]):
// one wave per row k (lane l: columns 8 l .. 8 l + 7, 16-byte loads).
__global__ __launch_bounds__(256) void hvp_b3_kernel(HvpArgs a) {
  const int lane = threadIdx.x & 63, k = 4 * blockIdx.x + (threadIdx.x >> 6);
  if (k >= FLAT) return;
  const float *W = a.th + a.off[6] + (int64_t)k * HID + 8 * lane, *Wd = a.tw + a.off[6] + (int64_t)k * HID + 8 * lane;
  float z = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float4 w = reinterpret_cast<const float4*>(W)[h], wd = reinterpret_cast<const float4*>(Wd)[h];
    const float4 d = reinterpret_cast<const float4*>(a.d4 + 8 * lane)[h];
    const float4 dd = reinterpret_cast<const float4*>(a.td4 + 8 * lane)[h];
    z += ((wd.x * d.x + w.x * dd.x) + (wd.y * d.y + w.y * dd.y)) + ((wd.z * d.z + w.z * dd.z) + (wd.w * d.w + w.w * dd.w));
  }
  z = wave_sum(z);
  if (lane == 0) a.td3[k] = a.y3[k] > 0.f ? z : 0.f;
}

// 6. ddot2[pix][ci] = relu'(y2) sum_{taps, co} (d3 Wdot3 + ddot3 W3) (the
// transposed conv3, stride 1).  Block (pix, 16-channel group g); thread
// (ci, output-channel quad cs = t % 16): 16-byte W loads along co.
__global__ __launch_bounds__(256) void hvp_b2_kernel(HvpArgs a) {
  __shared__ float s_r[16][17];
  const int t = threadIdx.x, pix = blockIdx.x, g = blockIdx.y;
  const int ih = pix / C2O, iw = pix % C2O, cs = t & 15, cl = t >> 4, ci = 16 * g + cl;
  float z = 0.f;
  for (int kh = 0; kh < C3K; ++kh) {
    const int oh = ih - kh;
    if (oh < 0 || oh >= C3O) continue;
    for (int kw = 0; kw < C3K; ++kw) {
      const int ow = iw - kw;
      if (ow < 0 || ow >= C3O) continue;
      const int src = (oh * C3O + ow) * C3CO + 4 * cs;
      const int64_t wi = ((kh * C3K + kw) * C3CI + ci) * C3CO + 4 * cs;
      const float4 w = *reinterpret_cast<const float4*>(a.th + a.off[4] + wi);
      const float4 wd = *reinterpret_cast<const float4*>(a.tw + a.off[4] + wi);
      const float4 d = *reinterpret_cast<const float4*>(a.d3 + src);
      const float4 dd = *reinterpret_cast<const float4*>(a.td3 + src);
      z += ((d.x * wd.x + dd.x * w.x) + (d.y * wd.y + dd.y * w.y)) + ((d.z * wd.z + dd.z * w.z) + (d.w * wd.w + dd.w * w.w));
    }
  }
  s_r[cl][cs] = z;
  __syncthreads();
  if (t < 16) {
    const int c = 16 * g + t;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) v += s_r[t][k];
    a.td2[pix * C2CO + c] = a.y2[pix * C2CO + c] > 0.f ? v : 0.f;
  }
}

// 7. ddot1[pix][ci] = relu'(y1) sum_{taps, co} (d2 Wdot2 + ddot2 W2) (the
// transposed conv2, stride 2: at most 2 x 2 live taps).  Block pix; thread
// (ci = t / 8, output-channel octet cs = t % 8).
__global__ __launch_bounds__(256) void hvp_b1_kernel(HvpArgs a) {
  __shared__ float s_r[C2CI][9];
  const int t = threadIdx.x, pix = blockIdx.x;
  const int ih = pix / C1O, iw = pix % C1O, cs = t & 7, ci = t >> 3;
  float z = 0.f;
  for (int kh = (ih & 1); kh < C2K; kh += C2S) {
    const int oh = (ih - kh) / C2S;
    if (ih < kh || oh >= C2O) continue;
    for (int kw = (iw & 1); kw < C2K; kw += C2S) {
      const int ow = (iw - kw) / C2S;
      if (iw < kw || ow >= C2O) continue;
      const int src = (oh * C2O + ow) * C2CO + 8 * cs;
      const int64_t wi = ((kh * C2K + kw) * C2CI + ci) * C2CO + 8 * cs;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const float4 w = *reinterpret_cast<const float4*>(a.th + a.off[2] + wi + 4 * h);
        const float4 wd = *reinterpret_cast<const float4*>(a.tw + a.off[2] + wi + 4 * h);
        const float4 d = *reinterpret_cast<const float4*>(a.d2 + src + 4 * h);
        const float4 dd = *reinterpret_cast<const float4*>(a.td2 + src + 4 * h);
        z += ((d.x * wd.x + dd.x * w.x) + (d.y * wd.y + dd.y * w.y)) +
             ((d.z * wd.z + dd.z * w.z) + (d.w * wd.w + dd.w * w.w));
      }
    }
  }
  s_r[ci][cs] = z;
  __syncthreads();
  if (t < C2CI) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += s_r[t][k];
    a.td1[pix * C1CO + t] = a.y1[pix * C1CO + t] > 0.f ? v : 0.f;
  }
}

// 8. Every parameter-gradient block of H_q w in one launch, grid in ranges:
//   [257] conv1 rows k (row 256 = bias): sum_p x_p[k] ddot1[p][co] over 8
//         position splits (thread (split, co));
//   [513] conv2 rows, [577] conv3 rows (last row = bias):
//         sum_p (ydot[src] d[p][co] + y[src] ddot[p][co]) over 4 position
//         splits (thread (split, co));
//   [2]   fc2 / fc1 bias / fc2 bias: hdot = relu'(h) (bdot1 + sum of t4's
//         chunk partials), the fc2 column a = hdot;
//   [...] fc1: ydot3 (x) d4 + y3 (x) ddot4, 4 elements per thread.
constexpr int HVP_G_C1 = C1KK + 1, HVP_G_C2 = C2KK + 1, HVP_G_C3 = C3KK + 1, HVP_G_H = 2;
constexpr int HVP_G_FC = FLAT * HID / 4 / 256;  // 1568
constexpr int HVP_G_BLOCKS = HVP_G_C1 + HVP_G_C2 + HVP_G_C3 + HVP_G_H + HVP_G_FC;

template <int IH, int CI, int K, int S, int CO, int OH>
__device__ __forceinline__ void hvp_g_conv_row(const HvpArgs& a, const float* y, const float* yd, const float* d,
                                               const float* dd, int k, int64_t off_w, int64_t off_b, float (*s_r)[64],
                                               const HqOut& ho) {
  const int t = threadIdx.x, co = t & 63, sp = t >> 6;  // 4 position splits
  constexpr int P = OH * OH, PS = (P + 3) / 4;
  const int p0 = sp * PS, p1 = min(P, p0 + PS);
  float g = 0.f;
  if (k == K * K * CI) {
    for (int p = p0; p < p1; ++p) g += dd[p * CO + co];
  } else {
    const int kh = k / (K * CI), kw = (k / CI) % K, ci = k % CI;
    for (int p = p0; p < p1; ++p) {
      const int src = (((p / OH) * S + kh) * IH + (p % OH) * S + kw) * CI + ci;
      g += yd[src] * d[p * CO + co] + y[src] * dd[p * CO + co];
    }
  }
  s_r[sp][co] = g;
  __syncthreads();
  if (t < CO) {
    const float v = (s_r[0][t] + s_r[1][t]) + (s_r[2][t] + s_r[3][t]);
    if (k == K * K * CI)
      ho.put(a, off_b + t, v);
    else
      ho.put(a, off_w + (int64_t)k * CO + t, v);
  }
}

__global__ __launch_bounds__(256) void hvp_g_kernel(HvpArgs a) {
  __shared__ float s_r[8][64];
  __shared__ float s_x[C1M];
  const int t = threadIdx.x;
  const HqOut ho(a);
  int i = blockIdx.x;
  if (i < HVP_G_C1) {  // conv1: thread (split = t / 32 of 50 positions, co)
    // the row's 400 patch values x_p[k] staged once (a loop of scattered
    // byte loads per thread was 11 of this launch's 20 us)
    const int k = i, co = t & 31, sp = t >> 5;
    if (k < C1KK) {
      const int kh = k / (C1K * FC), kw = (k / FC) % C1K, ci = k % FC;
      const int f = a.fidx[(int64_t)a.slot[0] * 8 + ci];
      const uint8_t* fr = a.frames + (int64_t)max(f, 0) * FB;
      for (int p = t; p < C1M; p += 256)
        s_x[p] = f < 0 ? 0.f : u8n(fr[(C1S * (p / C1O) + kh) * FW + C1S * (p % C1O) + kw]);
    } else {
      for (int p = t; p < C1M; p += 256) s_x[p] = 1.f;  // bias row: sum_p ddot1
    }
    __syncthreads();
    float g = 0.f;
#pragma unroll 10
    for (int p = 50 * sp; p < 50 * sp + 50; ++p) g += s_x[p] * a.td1[p * C1CO + co];
    s_r[sp][co] = g;
    __syncthreads();
    if (t < C1CO) {
      float v = 0.f;
#pragma unroll
      for (int s = 0; s < 8; ++s) v += s_r[s][t];
      ho.put(a, a.off[0] + (int64_t)k * C1CO + t, v);  // row 256 is the bias (off[1] = off[0] + 8192)
    }
    return;
  }
  i -= HVP_G_C1;
  if (i < HVP_G_C2) {
    hvp_g_conv_row<C1O, C1CO, C2K, C2S, C2CO, C2O>(a, a.y1, a.ty1, a.d2, a.td2, i, a.off[2], a.off[3], s_r, ho);
    return;
  }
  i -= HVP_G_C2;
  if (i < HVP_G_C3) {
    hvp_g_conv_row<C2O, C2CO, C3K, 1, C3CO, C3O>(a, a.y2, a.ty2, a.d3, a.td3, i, a.off[4], a.off[5], s_r, ho);
    return;
  }
  i -= HVP_G_C3;
  if (i < HVP_G_H) {  // hidden unit n: hdot, fc2 column, fc1 bias; fc2 bias = 0
    const int n = 256 * i + t, act = a.action[a.slot[0]];
    float z = a.tw[a.off[7] + n];
    for (int c = 0; c < HVP_T4_CHUNKS; ++c) z += a.part[(int64_t)c * HID + n];
    const float hd = a.h[n] > 0.f ? z : 0.f;
    for (int col = 0; col < a.A; ++col) ho.put(a, a.off[8] + (int64_t)n * a.A + col, col == act ? hd : 0.f);
    ho.put(a, a.off[7] + n, a.td4[n]);
    if (i == 0 && t < a.A) ho.put(a, a.off[9] + t, 0.f);
    return;
  }
  i -= HVP_G_H;
  {  // fc1 rows: 4 consecutive columns per thread
    const int64_t e = ((int64_t)i * 256 + t) * 4;
    const int k = (int)(e / HID), n = (int)(e % HID);
    const float ty = a.ty3[k], y = a.y3[k];
    const float4 d = *reinterpret_cast<const float4*>(a.d4 + n);
    const float4 dd = *reinterpret_cast<const float4*>(a.td4 + n);
    const float4 hq =
        make_float4(ty * d.x + y * dd.x, ty * d.y + y * dd.y, ty * d.z + y * dd.z, ty * d.w + y * dd.w);
    if (a.vout) {
      const int64_t j = a.off[6] + e;
      const float4 vd = *reinterpret_cast<const float4*>(a.vdir + j);
      const float4 jj = *reinterpret_cast<const float4*>(a.J + j);
      const float4 g = *reinterpret_cast<const float4*>(a.gq + j);
      *reinterpret_cast<float4*>(a.vout + j) =
          make_float4(vd.x + jj.x * (ho.a_s1 * g.x - ho.clip * hq.x), vd.y + jj.y * (ho.a_s1 * g.y - ho.clip * hq.y),
                      vd.z + jj.z * (ho.a_s1 * g.z - ho.clip * hq.z), vd.w + jj.w * (ho.a_s1 * g.w - ho.clip * hq.w));
    } else {
      *reinterpret_cast<float4*>(a.hq + a.off[6] + e) = hq;
    }
  }
}

// The second order's elementwise stages run in gradient epilogues: the
// u' / v_dir / w pieces in the one-transition backward's (common.hpp
// Rms::meta3), v = v_dir + J (alpha s1 grad q - clip(td') H_q w) in
// hvp_g_kernel's (HqOut).

}  // namespace dqz
