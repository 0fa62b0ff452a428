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
// with d_l the unit-cotangent backward signals of q[a] (d_5 = e_a).  Every
// kernel here is a plain one-thread-per-output loop: this runs once per meta
// step on one sample (~40 M MAC), off the learner's hot loop.
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
  float *ty1, *ty2, *ty3, *th4, *td4, *td3, *td2, *td1;
  float* hq;    // output, parameter layout
  float* part;  // [HVP_SPLITS][C1M * C1CO] K-split partial sums of the current stage
};

// Every stage below splits its reduction (K) over blockIdx.y and writes
// part[split][i]; hvp_fin_kernel then sums the splits in order (deterministic),
// adds the tangent bias and applies the fixed ReLU mask.  One thread per
// (output, split): thousands of waves instead of one long loop per output.
constexpr int HVP_SPLITS = 16;

__device__ __forceinline__ float hvp_x(const HvpArgs& a, int ih, int iw, int ci) {
  const int f = a.fidx[(int64_t)a.slot[0] * 8 + ci];
  return f < 0 ? 0.f : u8n(a.frames[(int64_t)f * FB + ih * FW + iw]);
}

// out[i] = mask[i] > 0 ? bias[i % nb] + sum_s part[s][i] : 0   (mask / bias optional)
__global__ void hvp_fin_kernel(const float* __restrict__ part, int S, int N, const float* __restrict__ mask,
                               const float* __restrict__ bias, int nb, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  float z = bias ? bias[i % nb] : 0.f;
  for (int s = 0; s < S; ++s) z += part[(int64_t)s * N + i];
  out[i] = (mask == nullptr || mask[i] > 0.f) ? z : 0.f;
}

// 1. conv1 tangent partial over kernel row kh = split: conv(x, Wdot1)
__global__ void hvp_t1_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, kh = blockIdx.y;
  if (i >= C1M * C1CO) return;
  const int p = i / C1CO, co = i % C1CO, oh = p / C1O, ow = p % C1O;
  const float* W = a.tw + a.off[0];
  float z = 0.f;
  for (int kw = 0; kw < C1K; ++kw)
#pragma unroll
    for (int ci = 0; ci < FC; ++ci)
      z += hvp_x(a, C1S * oh + kh, C1S * ow + kw, ci) * W[((kh * C1K + kw) * FC + ci) * C1CO + co];
  a.part[(int64_t)kh * (C1M * C1CO) + i] = z;
}

// 2./3. conv2 / conv3 tangent partial over kernel row kh: conv(y, Wdot) + conv(ydot, W)
template <int IH, int CI, int K, int S, int CO, int OH>
__device__ __forceinline__ float hvp_conv_t(const float* y, const float* yd, const float* W, const float* Wd,
                                            int p, int co, int kh) {
  const int oh = p / OH, ow = p % OH;
  float z = 0.f;
  for (int kw = 0; kw < K; ++kw)
    for (int ci = 0; ci < CI; ++ci) {
      const int src = ((oh * S + kh) * IH + ow * S + kw) * CI + ci;
      const int wi = ((kh * K + kw) * CI + ci) * CO + co;
      z += y[src] * Wd[wi] + yd[src] * W[wi];
    }
  return z;
}

__global__ void hvp_t2_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, kh = blockIdx.y;
  if (i >= C2M * C2CO) return;
  a.part[(int64_t)kh * (C2M * C2CO) + i] = hvp_conv_t<C1O, C1CO, C2K, C2S, C2CO, C2O>(
      a.y1, a.ty1, a.th + a.off[2], a.tw + a.off[2], i / C2CO, i % C2CO, kh);
}

__global__ void hvp_t3_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, kh = blockIdx.y;
  if (i >= FLAT) return;
  a.part[(int64_t)kh * FLAT + i] = hvp_conv_t<C2O, C2CO, C3K, 1, C3CO, C3O>(
      a.y2, a.ty2, a.th + a.off[4], a.tw + a.off[4], i / C3CO, i % C3CO, kh);
}

// 4. fc1 tangent partial over k in [196 s, 196 s + 196) (hdot), and the
// fc2-level backward tangent ddot4 = relu'(h) Wdot2[:, a] (split 0)
constexpr int HVP_FC_KS = FLAT / HVP_SPLITS;  // 196
__global__ void hvp_t4_kernel(HvpArgs a) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
  if (n >= HID) return;
  const float *W = a.th + a.off[6], *Wd = a.tw + a.off[6];
  float z = 0.f;
  for (int k = s * HVP_FC_KS; k < (s + 1) * HVP_FC_KS; ++k)
    z += a.y3[k] * Wd[(int64_t)k * HID + n] + a.ty3[k] * W[(int64_t)k * HID + n];
  a.part[(int64_t)s * HID + n] = z;
  if (s == 0) {
    const int act = a.action[a.slot[0]];
    a.td4[n] = a.h[n] > 0.f ? a.tw[a.off[8] + n * a.A + act] : 0.f;
  }
}

// 5. ddot3 partial over n in [32 s, 32 s + 32): Wdot1 d4 + W1 ddot4
__global__ void hvp_b3_kernel(HvpArgs a) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
  if (k >= FLAT) return;
  const float *W = a.th + a.off[6] + (int64_t)k * HID, *Wd = a.tw + a.off[6] + (int64_t)k * HID;
  constexpr int NS = HID / HVP_SPLITS;  // 32
  float z = 0.f;
  for (int n = s * NS; n < (s + 1) * NS; ++n) z += Wd[n] * a.d4[n] + W[n] * a.td4[n];
  a.part[(int64_t)s * FLAT + k] = z;
}

// 6./7. transposed-conv tangent partials over kernel row kh = split
template <int IH, int CI, int K, int S, int CO, int OH>
__device__ __forceinline__ float hvp_convT_t(const float* d, const float* dd, const float* W, const float* Wd,
                                             int ih, int iw, int ci, int kh) {
  float z = 0.f;
  const int th = ih - kh;
  if (th < 0 || th % S) return 0.f;
  const int oh = th / S;
  if (oh >= OH) return 0.f;
  for (int kw = 0; kw < K; ++kw) {
    const int tw = iw - kw;
    if (tw < 0 || tw % S) continue;
    const int ow = tw / S;
    if (ow >= OH) continue;
    for (int co = 0; co < CO; ++co) {
      const int src = (oh * OH + ow) * CO + co;
      const int wi = ((kh * K + kw) * CI + ci) * CO + co;
      z += d[src] * Wd[wi] + dd[src] * W[wi];
    }
  }
  return z;
}

__global__ void hvp_b2_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, kh = blockIdx.y;
  if (i >= C2M * C2CO) return;
  const int pix = i / C2CO, ci = i % C2CO;
  a.part[(int64_t)kh * (C2M * C2CO) + i] = hvp_convT_t<C2O, C3CI, C3K, 1, C3CO, C3O>(
      a.d3, a.td3, a.th + a.off[4], a.tw + a.off[4], pix / C2O, pix % C2O, ci, kh);
}

__global__ void hvp_b1_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, kh = blockIdx.y;
  if (i >= C1M * C1CO) return;
  const int pix = i / C1CO, ci = i % C1CO;
  a.part[(int64_t)kh * (C1M * C1CO) + i] = hvp_convT_t<C1O, C2CI, C2K, C2S, C2CO, C2O>(
      a.d2, a.td2, a.th + a.off[2], a.tw + a.off[2], pix / C1O, pix % C1O, ci, kh);
}

// 8. d/deps of conv1's weight gradient, partial over positions [25 s, 25 s + 25);
// row 256 = the bias (sum over positions of ddot1)
constexpr int HVP_C1_PS = C1M / HVP_SPLITS;  // 25
__global__ void hvp_g_conv1_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x, s = blockIdx.y;
  constexpr int N = (C1KK + 1) * C1CO;
  if (i >= N) return;
  const int k = i / C1CO, co = i % C1CO;
  float g = 0.f;
  if (k == C1KK) {
    for (int p = s * HVP_C1_PS; p < (s + 1) * HVP_C1_PS; ++p) g += a.td1[p * C1CO + co];
  } else {
    const int kh = k / (C1K * FC), kw = (k / FC) % C1K, ci = k % FC;
    for (int p = s * HVP_C1_PS; p < (s + 1) * HVP_C1_PS; ++p)
      g += hvp_x(a, C1S * (p / C1O) + kh, C1S * (p % C1O) + kw, ci) * a.td1[p * C1CO + co];
  }
  a.part[(int64_t)s * N + i] = g;
}

template <int IH, int CI, int K, int S, int CO, int OH>
__device__ __forceinline__ float hvp_dw(const float* y, const float* yd, const float* d, const float* dd, int k,
                                        int co) {
  const int kh = k / (K * CI), kw = (k / CI) % K, ci = k % CI;
  float g = 0.f;
  for (int p = 0; p < OH * OH; ++p) {
    const int src = (((p / OH) * S + kh) * IH + (p % OH) * S + kw) * CI + ci;
    g += yd[src] * d[p * CO + co] + y[src] * dd[p * CO + co];
  }
  return g;
}

__global__ void hvp_g_conv23_kernel(HvpArgs a) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int N2 = (C2KK + 1) * C2CO, N3 = (C3KK + 1) * C3CO;
  if (i < N2) {
    const int k = i / C2CO, co = i % C2CO;
    if (k == C2KK) {
      float g = 0.f;
      for (int p = 0; p < C2M; ++p) g += a.td2[p * C2CO + co];
      a.hq[a.off[3] + co] = g;
    } else {
      a.hq[a.off[2] + k * C2CO + co] = hvp_dw<C1O, C1CO, C2K, C2S, C2CO, C2O>(a.y1, a.ty1, a.d2, a.td2, k, co);
    }
  } else if (i < N2 + N3) {
    const int j = i - N2, k = j / C3CO, co = j % C3CO;
    if (k == C3KK) {
      float g = 0.f;
      for (int p = 0; p < C3M; ++p) g += a.td3[p * C3CO + co];
      a.hq[a.off[5] + co] = g;
    } else {
      a.hq[a.off[4] + k * C3CO + co] = hvp_dw<C2O, C2CO, C3K, 1, C3CO, C3O>(a.y2, a.ty2, a.d3, a.td3, k, co);
    }
  }
}

__global__ void hvp_g_fc_kernel(HvpArgs a) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n1 = (int64_t)FLAT * HID;
  if (i < n1) {
    const int k = (int)(i / HID), n = (int)(i % HID);
    a.hq[a.off[6] + i] = a.ty3[k] * a.d4[n] + a.y3[k] * a.td4[n];
  } else if (i < n1 + HID) {
    const int n = (int)(i - n1);
    a.hq[a.off[7] + n] = a.td4[n];
  } else if (i < n1 + HID + (int64_t)HID * a.A) {
    const int j = (int)(i - n1 - HID), n = j / a.A, col = j % a.A;
    a.hq[a.off[8] + j] = col == a.action[a.slot[0]] ? a.th4[n] : 0.f;
  } else if (i < n1 + HID + (int64_t)HID * a.A + a.A) {
    a.hq[a.off[9] + (i - n1 - HID - (int64_t)HID * a.A)] = 0.f;
  }
}

// Second-order u' / v pieces (meta.hpp naming): g' = -clip(td') grad q,
// mu'' = d mu' + c g', nu'' = d nu' + c g'^2, D2 = nu'' - mu''^2 + eps,
//   u'    = -lr g' D2^{-1/2}                       (loss partials: u'^2)
//   v_dir = 2 u' c d lr g' D2^{-3/2} (G - mu'')     -> written over mu1
//   w     = 2 u' (-lr) D2^{-3/2} (D2 - c g'(g' - mu''))  -> written over nu1
// and partial sums of grad q . w.
struct MetaSecondArgs {
  float lr, decay, c1, eps, bound;
  int64_t n;
  const float* td;  // [1] online transition TD at theta' (one-sample learner)
};

__global__ __launch_bounds__(256) void meta_second_kernel(MetaSecondArgs a, const float* __restrict__ gq,
                                                          const float* __restrict__ G, float* mu1, float* nu1,
                                                          float* __restrict__ loss_part, float* __restrict__ s1_part) {
  __shared__ float sbuf[4];
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  float sq = 0.f, s1 = 0.f;
  if (i < a.n) {
    const float clip = fminf(fmaxf(a.td[0], -a.bound), a.bound);
    const float gqv = gq[i];
    const float g = -clip * gqv;
    const float m = a.c1 * g + a.decay * mu1[i];
    const float v = a.c1 * (g * g) + a.decay * nu1[i];
    const float d2 = v - m * m + a.eps;
    const float rs = rsqrtf(d2);
    const float rs3 = rs * rs * rs;
    const float u = (-a.lr) * (g * rs);
    mu1[i] = 2.f * u * a.c1 * a.decay * a.lr * g * rs3 * (G[i] - m);
    const float w = 2.f * u * (-a.lr) * rs3 * (d2 - a.c1 * g * (g - m));
    nu1[i] = w;
    sq = u * u;
    s1 = gqv * w;
  }
  sq = wave_sum(sq);
  s1 = wave_sum(s1);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) sbuf[wave] = sq;
  __syncthreads();
  if (threadIdx.x == 0) loss_part[blockIdx.x] = (sbuf[0] + sbuf[1]) + (sbuf[2] + sbuf[3]);
  __syncthreads();
  if (lane == 0) sbuf[wave] = s1;
  __syncthreads();
  if (threadIdx.x == 0) s1_part[blockIdx.x] = (sbuf[0] + sbuf[1]) + (sbuf[2] + sbuf[3]);
}

// v = v_dir + J (alpha s1 grad q - clip(td') H_q w), alpha = [|td'| < bound];
// s1 = sum of the partials (every block re-sums them: deterministic).
__global__ __launch_bounds__(256) void meta_combine_kernel(MetaSecondArgs a, const float* __restrict__ vdir,
                                                           const float* __restrict__ J, const float* __restrict__ gq,
                                                           const float* __restrict__ hq,
                                                           const float* __restrict__ s1_part, int nparts,
                                                           float* __restrict__ v_out) {
  __shared__ float sbuf[4];
  __shared__ float s_s1;
  float p = 0.f;
  for (int j = threadIdx.x; j < nparts; j += blockDim.x) p += s1_part[j];
  p = wave_sum(p);
  if ((threadIdx.x & 63) == 0) sbuf[threadIdx.x >> 6] = p;
  __syncthreads();
  if (threadIdx.x == 0) s_s1 = (sbuf[0] + sbuf[1]) + (sbuf[2] + sbuf[3]);
  __syncthreads();
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n) return;
  const float td = a.td[0];
  const float alpha = fabsf(td) < a.bound ? 1.f : 0.f;
  const float clip = fminf(fmaxf(td, -a.bound), a.bound);
  v_out[i] = vdir[i] + J[i] * (alpha * s_s1 * gq[i] - clip * hq[i]);
}

}  // namespace dqz
