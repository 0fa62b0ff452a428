// learner.hip — MI355X-native DQN learner step behind the dqz C ABI.
//
// One step (dqn/agent.py:109-119, prioritized/agent.py:115-127):
//   conv1..conv3 + fc1 forward of Z network copies in one launch per layer
//     z=0 online(s_tm1), z=1 target(s_t), [z=2 online(s_t) for double-Q]
//   head: fc2, TD error (rlax q_learning / double_q_learning), loss,
//     clip_gradient backward (dq), fc2/fc1-bias grads, dz1
//   fc1 dX, then {conv3 dX, conv3 dW, fc1 dW + fused centered RMSProp},
//   {conv2 dX (stride-phase split), conv2 dW}, {conv1 dW},
//   reduce of split-K dW partials + centered RMSProp for the rest.
// The frame gather + /255 normalisation (networks.py:192) is fused into the
// conv1 A-operand loader: stacks are never materialised in HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>

#include "dqz.h"
#include "gemm.hpp"

namespace dqz {

// ---------------------------------------------------------------------------
// errors

static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
static int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define DQZ_HIP(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) return fail(DQZ_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------------------
// geometry (networks.py:181-221)

constexpr int FH = 84, FW = 84, FC = 4, FB = FH * FW;
constexpr int C1K = 8, C1S = 4, C1CO = 32, C1O = 20, C1M = C1O * C1O, C1KK = C1K * C1K * FC;       // 400, 256
constexpr int C2K = 4, C2S = 2, C2CI = 32, C2CO = 64, C2O = 9, C2M = C2O * C2O, C2KK = 16 * C2CI;  // 81, 512
constexpr int C3K = 3, C3CI = 64, C3CO = 64, C3O = 7, C3M = C3O * C3O, C3KK = 9 * C3CI;           // 49, 576
constexpr int FLAT = C3M * C3CO;                                                                  // 3136
constexpr int HID = 512;
constexpr int MAXA = 32;
constexpr int MAXB = 256;

static void param_layout(int A, int shared_bias, int64_t off[10], int64_t sz[10], int64_t* total) {
  const int64_t sizes[10] = {C1KK * C1CO, C1CO, C2KK * C2CO, C2CO, C3KK * C3CO, C3CO,
                             (int64_t)FLAT * HID, HID, (int64_t)HID * A, shared_bias ? 1 : A};
  int64_t o = 0;
  for (int i = 0; i < 10; ++i) {
    off[i] = o;
    sz[i] = sizes[i];
    o += (sizes[i] + 63) / 64 * 64;
  }
  *total = o;
}

// ---------------------------------------------------------------------------
// shapes shared by the ops

struct Shape {
  TileGrid g;
  int M, N, K, KS, BM, BN;
  __device__ __forceinline__ void coords(int t, TileCoord& tc) const {
    int z, s, tm, tn;
    g.decode(t, z, s, tm, tn);
    tc.z = z;
    tc.split = s;
    tc.m0 = tm * BM;
    tc.n0 = tn * BN;
    tc.k0 = s * KS;
    tc.k1 = min(K, (s + 1) * KS);
    tc.M = M;
    tc.N = N;
  }
  __host__ __device__ int tiles() const { return g.count(); }
};

template <class C>
static Shape make_shape(int Z, int M, int N, int K, int S) {
  Shape sh;
  int ks = (K + S - 1) / S;
  ks = (ks + C::BK - 1) / C::BK * C::BK;
  S = (K + ks - 1) / ks;
  sh.g.Z = Z;
  sh.g.S = S;
  sh.g.MT = (M + C::BM - 1) / C::BM;
  sh.g.NT_ = (N + C::BN - 1) / C::BN;
  sh.M = M;
  sh.N = N;
  sh.K = K;
  sh.KS = ks;
  sh.BM = C::BM;
  sh.BN = C::BN;
  return sh;
}

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }
__device__ __forceinline__ float u8n(unsigned v) { return (float)v / 255.0f; }  // x.astype(f32) / 255.0

// Pixel (ih, iw, ci) of stack `which` (0 = s_tm1, 1 = s_t) of replay slot.
__device__ __forceinline__ unsigned stack_pixel(const uint8_t* frames, const int32_t* fidx, int slot, int which,
                                                int ih, int iw, int ci) {
  const int f = fidx[(int64_t)slot * 8 + which * 4 + ci];
  return f < 0 ? 0u : (unsigned)frames[(int64_t)f * FB + ih * FW + iw];
}

struct NetZ {
  const float* p[3];  // parameter buffer of network copy z
  int which[3];       // input stack of copy z: 0 = s_tm1, 1 = s_t
};

// ---------------------------------------------------------------------------
// forward ops

// conv1 8x8/4 4->32 with the frame gather + normalisation in the A loader.
struct Conv1Fwd : Shape {
  static constexpr bool kAKFast = true, kBKFast = false;
  const uint8_t* frames;
  const int32_t* fidx;
  const int32_t* slots;
  const uint8_t* states;  // direct uint8 [B][84][84][4] input when non-null
  NetZ nz;
  int64_t w_off, b_off;
  float* out;  // [Z][B*400][32]
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord& tc, int m, int k) const {
    const int b = m / C1M, p = m % C1M, oh = p / C1O, ow = p % C1O;
    const int kh = k >> 5, kw = (k >> 2) & 7, ci = k & 3;
    const int ih = oh * C1S + kh, iw = ow * C1S + kw;
    unsigned v;
    if (states)
      v = states[(((int64_t)b * FH + ih) * FW + iw) * FC + ci];
    else
      v = stack_pixel(frames, fidx, slots[b], nz.which[tc.z], ih, iw, ci);
    return u8n(v);
  }
  __device__ float b(const TileCoord& tc, int k, int n) const { return nz.p[tc.z][w_off + k * C1CO + n]; }
  __device__ void store(const TileCoord& tc, int m, int n, float v) const {
    out[((int64_t)tc.z * M + m) * C1CO + n] = relu(v + nz.p[tc.z][b_off + n]);
  }
};

// Generic VALID conv over an NHWC f32 input (conv2, conv3) + bias + ReLU.
template <int IH, int CI, int KH, int S, int CO, int OH>
struct ConvFwd : Shape {
  static constexpr bool kAKFast = true, kBKFast = false;
  const float* in;  // [Z][B][IH][IH][CI]
  int B;
  NetZ nz;
  int64_t w_off, b_off;
  float* out;  // [Z][B*OH*OH][CO]
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord& tc, int m, int k) const {
    const int b = m / (OH * OH), p = m % (OH * OH), oh = p / OH, ow = p % OH;
    const int kh = k / (KH * CI), r = k % (KH * CI), kw = r / CI, ci = r % CI;
    const int ih = oh * S + kh, iw = ow * S + kw;
    return in[((((int64_t)tc.z * B + b) * IH + ih) * IH + iw) * CI + ci];
  }
  __device__ float b(const TileCoord& tc, int k, int n) const { return nz.p[tc.z][w_off + k * CO + n]; }
  __device__ void store(const TileCoord& tc, int m, int n, float v) const {
    out[((int64_t)tc.z * M + m) * CO + n] = relu(v + nz.p[tc.z][b_off + n]);
  }
};
using Conv2Fwd = ConvFwd<C1O, C1CO, C2K, C2S, C2CO, C2O>;
using Conv3Fwd = ConvFwd<C2O, C2CO, C3K, 1, C3CO, C3O>;

// fc1 3136->512, split-K partial sums (bias/ReLU applied by the reduce).
struct Fc1Fwd : Shape {
  static constexpr bool kAKFast = true, kBKFast = false;
  const float* in;  // [Z][B][3136]
  NetZ nz;
  int64_t w_off;
  float* part;  // [Z][S][B][512]
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord& tc, int m, int k) const { return in[((int64_t)tc.z * M + m) * FLAT + k]; }
  __device__ float b(const TileCoord& tc, int k, int n) const { return nz.p[tc.z][w_off + (int64_t)k * HID + n]; }
  __device__ void store(const TileCoord& tc, int m, int n, float v) const {
    part[(((int64_t)tc.z * g.S + tc.split) * M + m) * HID + n] = v;
  }
};

// ---------------------------------------------------------------------------
// backward ops (online network only, z = 0 activations)

// dflat = dz1 @ W1^T, masked by ReLU'(conv3) -> dy3
struct Fc1Dx : Shape {
  static constexpr bool kAKFast = true, kBKFast = true;
  const float* dz1;  // [B][512]
  const float* w1;   // online W1 [3136][512]
  const float* y3;   // [B][3136] online conv3 output
  float* dy3;
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord&, int m, int k) const { return dz1[m * HID + k]; }
  __device__ float b(const TileCoord&, int k, int n) const { return w1[(int64_t)n * HID + k]; }
  __device__ void store(const TileCoord&, int m, int n, float v) const {
    const int64_t i = (int64_t)m * FLAT + n;
    dy3[i] = y3[i] > 0.f ? v : 0.f;
  }
};

struct Rms {
  float lr, decay, c1, eps;
  // optax 0.1.2 scale_by_stddev + scale(-lr):
  //   mu = (1-decay) g + decay mu ; nu = (1-decay) g^2 + decay nu
  //   theta += -lr * g * rsqrt(nu - mu^2 + eps)
  __device__ __forceinline__ void apply(float* th, float* mu, float* nu, int64_t i, float g) const {
    const float m = c1 * g + decay * mu[i];
    const float v = c1 * (g * g) + decay * nu[i];
    mu[i] = m;
    nu[i] = v;
    th[i] = th[i] + (-lr) * (g * rsqrtf(v - m * m + eps));
  }
};

// dW1 = flat^T @ dz1 (K = B), RMSProp applied in the epilogue: the W1
// gradient (6.4 MB, 95% of the parameters) never touches HBM.
struct Fc1DwRms : Shape {
  static constexpr bool kAKFast = false, kBKFast = false;
  const float* y3;   // [B][3136]
  const float* dz1;  // [B][512]
  float *th, *mu, *nu;
  int64_t w_off;
  Rms rms;
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord&, int m, int k) const { return y3[(int64_t)k * FLAT + m]; }
  __device__ float b(const TileCoord&, int k, int n) const { return dz1[k * HID + n]; }
  __device__ void store(const TileCoord&, int m, int n, float v) const {
    rms.apply(th, mu, nu, w_off + (int64_t)m * HID + n, v);
  }
};

// conv3 dX (stride 1): da2[b,ih,iw,ci] = sum_{kh,kw,co} dy3[b,ih-kh,iw-kw,co] W3[kh,kw,ci,co]
struct Conv3Dx : Shape {
  static constexpr bool kAKFast = true, kBKFast = true;
  const float* dy3;  // [B][7][7][64]
  const float* w3;   // online conv3 w [3][3][64][64]
  const float* y2;   // [B][9][9][64]
  float* dy2;
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord&, int m, int k) const {
    const int b = m / C2M, p = m % C2M, ih = p / C2O, iw = p % C2O;
    const int kh = k / (C3K * C3CO), r = k % (C3K * C3CO), kw = r / C3CO, co = r % C3CO;
    const int oh = ih - kh, ow = iw - kw;
    if (oh < 0 || ow < 0 || oh >= C3O || ow >= C3O) return 0.f;
    return dy3[((b * C3O + oh) * C3O + ow) * C3CO + co];
  }
  __device__ float b(const TileCoord&, int k, int n) const {
    const int kk = k / C3CO, co = k % C3CO;  // kk = kh*3+kw
    return w3[(kk * C3CI + n) * C3CO + co];
  }
  __device__ void store(const TileCoord&, int m, int n, float v) const {
    const int64_t i = (int64_t)m * C3CI + n;
    dy2[i] = y2[i] > 0.f ? v : 0.f;
  }
};

// conv2 dX (stride 2, kernel 4), split into the 4 output-parity phases so no
// zero taps are multiplied: for ih = 2*ih2 + ph only kh in {ph, ph+2} hit.
//   z = phase (ph, pw); m = (b, ih2, iw2) over 10x10; k = (jh, jw, co).
struct Conv2DxPhased : Shape {
  static constexpr bool kAKFast = true, kBKFast = true;
  const float* dy2;  // [B][9][9][64]
  const float* w2;   // online conv2 w [4][4][32][64]
  const float* y1;   // [B][20][20][32]
  float* dy1;
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord& tc, int m, int k) const {
    const int ph = tc.z >> 1, pw = tc.z & 1;
    const int b = m / 100, p = m % 100, ih2 = p / 10, iw2 = p % 10;
    const int jh = k >> 7, jw = (k >> 6) & 1, co = k & 63;
    const int oh = ih2 - jh, ow = iw2 - jw;
    (void)ph;
    (void)pw;
    if (oh < 0 || ow < 0 || oh >= C2O || ow >= C2O) return 0.f;
    return dy2[((b * C2O + oh) * C2O + ow) * C2CO + co];
  }
  __device__ float b(const TileCoord& tc, int k, int n) const {
    const int ph = tc.z >> 1, pw = tc.z & 1;
    const int jh = k >> 7, jw = (k >> 6) & 1, co = k & 63;
    const int kh = ph + 2 * jh, kw = pw + 2 * jw;
    return w2[((kh * C2K + kw) * C2CI + n) * C2CO + co];
  }
  __device__ void store(const TileCoord& tc, int m, int n, float v) const {
    const int ph = tc.z >> 1, pw = tc.z & 1;
    const int b = m / 100, p = m % 100, ih = 2 * (p / 10) + ph, iw = 2 * (p % 10) + pw;
    const int64_t i = (((int64_t)b * C1O + ih) * C1O + iw) * C1CO + n;
    dy1[i] = y1[i] > 0.f ? v : 0.f;
  }
};

// conv dW (+ bias as an extra row of ones), split-K partials:
//   P[s][kidx][co] = sum_{positions in split s} col(pos, kidx) * dy(pos, co)
template <int IH, int CI, int KH, int S, int CO, int OH>
struct ConvDw : Shape {
  static constexpr bool kAKFast = false, kBKFast = false;
  static constexpr int KK = KH * KH * CI;
  const float* in;  // layer input (online) [B][IH][IH][CI]
  const float* dy;  // [B*OH*OH][CO]
  float* part;      // [S][KK+1][CO]
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord&, int m, int k) const {
    if (m == KK) return 1.f;
    const int kh = m / (KH * CI), r = m % (KH * CI), kw = r / CI, ci = r % CI;
    const int b = k / (OH * OH), p = k % (OH * OH), oh = p / OH, ow = p % OH;
    return in[(((int64_t)b * IH + oh * S + kh) * IH + ow * S + kw) * CI + ci];
  }
  __device__ float b(const TileCoord&, int k, int n) const { return dy[(int64_t)k * CO + n]; }
  __device__ void store(const TileCoord& tc, int m, int n, float v) const {
    part[((int64_t)tc.split * (KK + 1) + m) * CO + n] = v;
  }
};
using Conv3Dw = ConvDw<C2O, C2CO, C3K, 1, C3CO, C3O>;
using Conv2Dw = ConvDw<C1O, C1CO, C2K, C2S, C2CO, C2O>;

struct Conv1Dw : Shape {
  static constexpr bool kAKFast = false, kBKFast = false;
  const uint8_t* frames;
  const int32_t* fidx;
  const int32_t* slots;
  int which;
  const float* dy1;  // [B*400][32]
  float* part;       // [S][257][32]
  __device__ void tile_coords(int t, TileCoord& tc) const { coords(t, tc); }
  __device__ float a(const TileCoord&, int m, int k) const {
    if (m == C1KK) return 1.f;
    const int kh = m >> 5, kw = (m >> 2) & 7, ci = m & 3;
    const int b = k / C1M, p = k % C1M, oh = p / C1O, ow = p % C1O;
    return u8n(stack_pixel(frames, fidx, slots[b], which, oh * C1S + kh, ow * C1S + kw, ci));
  }
  __device__ float b(const TileCoord&, int k, int n) const { return dy1[(int64_t)k * C1CO + n]; }
  __device__ void store(const TileCoord& tc, int m, int n, float v) const {
    part[((int64_t)tc.split * (C1KK + 1) + m) * C1CO + n] = v;
  }
};

// ---------------------------------------------------------------------------
// plain kernels

// h1[z][b][n] = relu(b1 + sum_s part[z][s][b][n])
__global__ void fc1_reduce_kernel(const float* __restrict__ part, NetZ nz, int64_t b_off, int Z, int S, int B,
                                  float* __restrict__ h1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Z * B * HID) return;
  const int n = i % HID, zb = i / HID, z = zb / B, b = zb % B;
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += part[(((int64_t)z * S + s) * B + b) * HID + n];
  h1[i] = relu(acc + nz.p[z][b_off + n]);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct HeadArgs {
  const float* h1;  // [Z][B][512]
  NetZ nz;
  int64_t w2_off, b2_off;
  int Z, B, A, algo, shared_bias, fwd_only;
  // batch data
  const int32_t* slots;
  const int32_t* action;
  const float* reward;
  const float* discount;
  const float* weights;  // PER importance weights or null
  float bound;           // grad_error_bound
  // outputs
  float* q;      // [Z][B][A]
  float* td;     // [B]
  float* loss;   // [1]
  float* dz1;    // [B][512]
  float* gfc;    // fc1 b grad [512] | fc2 w grad [512*A] | fc2 b grad [A or 1]
};

// fc2 + TD loss + clip_gradient backward + fc2/fc1-bias grads + dz1.
// One workgroup of 1024 threads (16 waves).  Follows rlax 0.1.2 q_learning /
// double_q_learning (dqn/agent.py:94-106, double_q/agent.py:97-106,
// prioritized/agent.py:97-113): td = stopgrad(r + d * q_t[...]) - q_tm1[a],
// loss = mean(0.5 td^2 [* w]), and the cotangent reaching td is
// clip(w * td / B, -bound, bound) (rlax.clip_gradient clips the gradient).
__global__ __launch_bounds__(1024) void head_kernel(HeadArgs h) {
  __shared__ float s_q[3 * MAXB * MAXA];
  __shared__ float s_g[MAXB];
  __shared__ int s_a[MAXB];
  __shared__ float s_loss[MAXB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int A = h.A, B = h.B;
  // 1. q[z][b][:] = h1[z][b] @ W2_z + b2_z, one (z,b) row per wave iteration
  for (int row = wave; row < h.Z * B; row += 16) {
    const int z = row / B;
    const float* w2 = h.nz.p[z] + h.w2_off;
    const float* hr = h.h1 + (int64_t)row * HID;
    float acc[MAXA];
#pragma unroll
    for (int a = 0; a < MAXA; ++a) acc[a] = 0.f;
    for (int j = lane; j < HID; j += 64) {
      const float hv = hr[j];
#pragma unroll
      for (int a = 0; a < MAXA; ++a)
        if (a < A) acc[a] += hv * w2[j * A + a];
    }
#pragma unroll
    for (int a = 0; a < MAXA; ++a) {
      if (a < A) {
        const float s = wave_sum(acc[a]);
        if (lane == 0) {
          const float bias = h.nz.p[z][h.b2_off + (h.shared_bias ? 0 : a)];
          s_q[row * A + a] = s + bias;
        }
      }
    }
  }
  __syncthreads();
  for (int i = tid; i < h.Z * B * A; i += blockDim.x) h.q[i] = s_q[i];
  if (h.fwd_only) return;
  // 2. TD error per sample
  if (tid < B) {
    const int b = tid;
    const int slot = h.slots[b];
    const int a_tm1 = h.action[slot];
    const float r = h.reward[slot], d = h.discount[slot];
    const float* q_tm1 = s_q + (0 * B + b) * A;
    const float* q_tgt = s_q + (1 * B + b) * A;
    float v;
    if (h.algo == DQZ_ALGO_DQN) {
      v = q_tgt[0];
      for (int a = 1; a < A; ++a) v = fmaxf(v, q_tgt[a]);
    } else {
      const float* q_sel = s_q + (2 * B + b) * A;  // online Q(s_t) selects
      int am = 0;
      for (int a = 1; a < A; ++a)
        if (q_sel[a] > q_sel[am]) am = a;  // jnp.argmax: first maximum
      v = q_tgt[am];
    }
    const float target = r + d * v;
    const float td = target - q_tm1[a_tm1];
    const float w = h.weights ? h.weights[b] : 1.f;
    h.td[b] = td;
    s_loss[b] = 0.5f * td * td * w;
    float g = w * td / (float)B;  // d mean(l2(td) * w) / d td
    g = fminf(fmaxf(g, -h.bound), h.bound);
    s_g[b] = -g;  // d loss / d q_tm1[b, a_tm1]
    s_a[b] = a_tm1;
  }
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += s_loss[b];
    h.loss[0] = s / (float)B;
  }
  // 3. column j of fc2 / fc1: dW2[j][a], dz1[b][j], db1[j]
  const float* w2 = h.nz.p[0] + h.w2_off;
  float* g_b1 = h.gfc;
  float* g_w2 = h.gfc + HID;
  float* g_b2 = h.gfc + HID + HID * A;
  for (int j = tid; j < HID; j += blockDim.x) {
    float gw[MAXA];
#pragma unroll
    for (int a = 0; a < MAXA; ++a) gw[a] = 0.f;
    float gb1 = 0.f;
    for (int b = 0; b < B; ++b) {
      const float hv = h.h1[(int64_t)b * HID + j];  // z = 0
      const int ab = s_a[b];
      const float gq = s_g[b];
#pragma unroll
      for (int a = 0; a < MAXA; ++a)
        if (a == ab) gw[a] += hv * gq;
      const float dz = hv > 0.f ? gq * w2[j * A + ab] : 0.f;
      h.dz1[(int64_t)b * HID + j] = dz;
      gb1 += dz;
    }
    g_b1[j] = gb1;
#pragma unroll
    for (int a = 0; a < MAXA; ++a)
      if (a < A) g_w2[j * A + a] = gw[a];
  }
  if (tid < (h.shared_bias ? 1 : A)) {
    float gb = 0.f;
    for (int b = 0; b < B; ++b)
      if (h.shared_bias || s_a[b] == tid) gb += s_g[b];
    g_b2[tid] = gb;
  }
}

struct UpdArgs {
  float *th, *mu, *nu;
  int64_t off[10];
  int64_t sz[10];
  const float* p1;  // [S1][257][32]
  const float* p2;  // [S2][513][64]
  const float* p3;  // [S3][577][64]
  int S1, S2, S3;
  const float* gfc;  // fc1 b | fc2 w | fc2 b
  int A, nb2;
  Rms rms;
};

__device__ __forceinline__ float sum_split(const float* p, int S, int64_t stride, int64_t i) {
  float acc = 0.f;
  for (int s = 0; s < S; ++s) acc += p[s * stride + i];
  return acc;
}

// Reduce the conv dW/db split-K partials and apply centered RMSProp to every
// leaf except fc1/w (done in Fc1DwRms).
__global__ void update_kernel(UpdArgs u) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n0 = u.sz[0] + u.sz[1], n1 = n0 + u.sz[2] + u.sz[3], n2 = n1 + u.sz[4] + u.sz[5];
  const int64_t n3 = n2 + HID + (int64_t)HID * u.A + u.nb2;
  if (i >= n3) return;
  float g;
  int64_t dst;
  if (i < n0) {  // conv1: w rows 0..255, bias row 256
    const int64_t stride = (int64_t)(C1KK + 1) * C1CO;
    g = sum_split(u.p1, u.S1, stride, i);
    dst = i < u.sz[0] ? u.off[0] + i : u.off[1] + (i - u.sz[0]);
  } else if (i < n1) {
    const int64_t j = i - n0, stride = (int64_t)(C2KK + 1) * C2CO;
    g = sum_split(u.p2, u.S2, stride, j);
    dst = j < u.sz[2] ? u.off[2] + j : u.off[3] + (j - u.sz[2]);
  } else if (i < n2) {
    const int64_t j = i - n1, stride = (int64_t)(C3KK + 1) * C3CO;
    g = sum_split(u.p3, u.S3, stride, j);
    dst = j < u.sz[4] ? u.off[4] + j : u.off[5] + (j - u.sz[4]);
  } else {
    const int64_t j = i - n2;
    g = u.gfc[j];
    if (j < HID)
      dst = u.off[7] + j;
    else if (j < HID + (int64_t)HID * u.A)
      dst = u.off[8] + (j - HID);
    else
      dst = u.off[9] + (j - HID - (int64_t)HID * u.A);
  }
  u.rms.apply(u.th, u.mu, u.nu, dst, g);
}

// Philox4x32-10 (Salmon et al. 2011).
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const unsigned lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

__global__ void sample_uniform_kernel(int64_t base, int64_t size, int64_t capacity, int n, uint64_t seed,
                                      uint64_t* counter, int32_t* out) {
  const uint64_t ctr = *counter;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint4 r = philox4x32(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), (unsigned)i, 0x5EED5u),
                               make_uint2((unsigned)seed, (unsigned)(seed >> 32)));
    const uint64_t u = ((uint64_t)r.x << 32) | r.y;
    const int64_t j = (int64_t)__umul64hi(u, (uint64_t)size);  // uniform in [0, size)
    out[i] = (int32_t)((base + j) % capacity);
  }
  __syncthreads();
  if (threadIdx.x == 0) *counter = ctr + 1;
}

__global__ void gather_stacks_kernel(const uint8_t* frames, const int32_t* fidx, const int32_t* slots, int n,
                                     int which, uint8_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * FB) return;
  const int b = (int)(i / FB), p = (int)(i % FB);
  const int slot = slots[b];
  uchar4 v;
  unsigned c[4];
#pragma unroll
  for (int ci = 0; ci < 4; ++ci) {
    const int f = fidx[(int64_t)slot * 8 + which * 4 + ci];
    c[ci] = f < 0 ? 0u : frames[(int64_t)f * FB + p];
  }
  v.x = c[0];
  v.y = c[1];
  v.z = c[2];
  v.w = c[3];
  reinterpret_cast<uchar4*>(out)[i] = v;
}

}  // namespace dqz

// ---------------------------------------------------------------------------
// learner handle

using namespace dqz;

struct dqz_learner {
  dqz_learner_config cfg;
  int Z, shared_bias;
  int64_t off[10], sz[10], total;
  int S_fc1, S1, S2, S3;
  float *y1, *y2, *y3, *fc1p, *h1, *q, *dz1, *dy3, *dy2, *dy1, *p1, *p2, *p3, *gfc, *td, *loss;
  void* block;
};

// tile configurations
using CfgConv1 = Cfg<64, 32, 16, 4, 1>;
using CfgConv = Cfg<32, 64, 16, 2, 2>;
using CfgFc1 = Cfg<32, 64, 16, 2, 2>;
using CfgFc1Dx = Cfg<32, 32, 16, 2, 2>;
using CfgBwd2 = Cfg<64, 64, 16, 2, 2>;
using CfgBwd3 = Cfg<64, 32, 16, 4, 1>;

extern "C" {

const char* dqz_last_error(void) { return g_err.c_str(); }

int dqz_param_layout(int num_actions, int shared_bias, int64_t offsets[10], int64_t sizes[10], int64_t* total) {
  if (num_actions < 1 || num_actions > MAXA) return fail(DQZ_ERR_INVALID, "num_actions must be in [1, %d]", MAXA);
  if (!offsets || !sizes || !total) return fail(DQZ_ERR_INVALID, "null output pointer");
  param_layout(num_actions, shared_bias, offsets, sizes, total);
  return DQZ_OK;
}

int dqz_learner_create(const dqz_learner_config* cfg, dqz_learner** out) {
  if (!cfg || !out) return fail(DQZ_ERR_INVALID, "null argument");
  if (cfg->batch < 1 || cfg->batch > MAXB) return fail(DQZ_ERR_INVALID, "batch must be in [1, %d]", MAXB);
  if (cfg->num_actions < 1 || cfg->num_actions > MAXA)
    return fail(DQZ_ERR_INVALID, "num_actions must be in [1, %d]", MAXA);
  if (cfg->algo < DQZ_ALGO_DQN || cfg->algo > DQZ_ALGO_PER) return fail(DQZ_ERR_INVALID, "unknown algo %d", cfg->algo);
  dqz_learner* L = new dqz_learner();
  L->cfg = *cfg;
  L->Z = cfg->algo == DQZ_ALGO_DQN ? 2 : 3;
  L->shared_bias = cfg->algo == DQZ_ALGO_DQN ? 0 : 1;
  param_layout(cfg->num_actions, L->shared_bias, L->off, L->sz, &L->total);
  const int B = cfg->batch, Z = L->Z, A = cfg->num_actions;
  L->S_fc1 = 14;
  L->S1 = std::max(1, (B * C1M + 511) / 512);
  L->S2 = std::max(1, (B * C2M + 287) / 288);
  L->S3 = std::max(1, (B * C3M + 223) / 224);
  // recompute the effective split counts exactly as make_shape does
  L->S_fc1 = make_shape<CfgFc1>(Z, B, HID, FLAT, L->S_fc1).g.S;
  L->S1 = make_shape<CfgBwd3>(1, C1KK + 1, C1CO, B * C1M, L->S1).g.S;
  L->S2 = make_shape<CfgBwd3>(1, C2KK + 1, C2CO, B * C2M, L->S2).g.S;
  L->S3 = make_shape<CfgBwd2>(1, C3KK + 1, C3CO, B * C3M, L->S3).g.S;
  const int64_t n_y1 = (int64_t)Z * B * C1M * C1CO, n_y2 = (int64_t)Z * B * C2M * C2CO, n_y3 = (int64_t)Z * B * FLAT;
  const int64_t n_fc1p = (int64_t)Z * L->S_fc1 * B * HID, n_h1 = (int64_t)Z * B * HID, n_q = (int64_t)Z * B * A;
  const int64_t n_dz1 = (int64_t)B * HID, n_dy3 = (int64_t)B * FLAT, n_dy2 = (int64_t)B * C2M * C2CO,
                n_dy1 = (int64_t)B * C1M * C1CO;
  const int64_t n_p1 = (int64_t)L->S1 * (C1KK + 1) * C1CO, n_p2 = (int64_t)L->S2 * (C2KK + 1) * C2CO,
                n_p3 = (int64_t)L->S3 * (C3KK + 1) * C3CO;
  const int64_t n_gfc = HID + (int64_t)HID * A + A, n_td = B, n_loss = 1;
  const int64_t sizes[] = {n_y1, n_y2, n_y3, n_fc1p, n_h1, n_q, n_dz1, n_dy3, n_dy2, n_dy1, n_p1, n_p2, n_p3, n_gfc, n_td, n_loss};
  float** ptrs[] = {&L->y1, &L->y2, &L->y3, &L->fc1p, &L->h1, &L->q, &L->dz1, &L->dy3, &L->dy2, &L->dy1,
                    &L->p1, &L->p2, &L->p3, &L->gfc, &L->td, &L->loss};
  int64_t total = 0;
  for (int64_t s : sizes) total += (s + 63) / 64 * 64;
  if (hipMalloc(&L->block, total * sizeof(float)) != hipSuccess) {
    delete L;
    return fail(DQZ_ERR_HIP, "hipMalloc of %lld bytes failed", (long long)(total * 4));
  }
  (void)hipMemset(L->block, 0, total * sizeof(float));
  float* p = (float*)L->block;
  for (size_t i = 0; i < sizeof(sizes) / sizeof(sizes[0]); ++i) {
    *ptrs[i] = p;
    p += (sizes[i] + 63) / 64 * 64;
  }
  *out = L;
  return DQZ_OK;
}

int dqz_learner_destroy(dqz_learner* L) {
  if (!L) return DQZ_OK;
  if (L->block) (void)hipFree(L->block);
  delete L;
  return DQZ_OK;
}

static int check_store(const dqz_store* S) {
  if (!S || !S->frames || !S->fidx || !S->action || !S->reward || !S->discount)
    return fail(DQZ_ERR_INVALID, "store has a null buffer");
  if (S->capacity < 1) return fail(DQZ_ERR_INVALID, "store capacity must be positive");
  return DQZ_OK;
}

// Forward of Z network copies; leaves h1/q in the learner scratch.
// Phase markers for dqz_learner_profile: ev[i] is recorded before phase i.
struct PhaseEvents {
  hipEvent_t* ev;
  void mark(int i, hipStream_t st) const {
    if (ev) (void)hipEventRecord(ev[i], st);
  }
};

static int forward_impl(dqz_learner* L, const NetZ& nz, int Z, int B, const dqz_store* S, const int32_t* slots,
                        const uint8_t* states, hipStream_t st, PhaseEvents pe = PhaseEvents{nullptr}) {
  pe.mark(0, st);
  Conv1Fwd c1;
  static_cast<Shape&>(c1) = make_shape<CfgConv1>(Z, B * C1M, C1CO, C1KK, 1);
  c1.frames = S ? S->frames : nullptr;
  c1.fidx = S ? S->fidx : nullptr;
  c1.slots = slots;
  c1.states = states;
  c1.nz = nz;
  c1.w_off = L->off[0];
  c1.b_off = L->off[1];
  c1.out = L->y1;
  DQZ_HIP((launch_gemm<CfgConv1>(st, c1)));
  pe.mark(1, st);

  Conv2Fwd c2;
  static_cast<Shape&>(c2) = make_shape<CfgConv>(Z, B * C2M, C2CO, C2KK, 1);
  c2.in = L->y1;
  c2.B = B;
  c2.nz = nz;
  c2.w_off = L->off[2];
  c2.b_off = L->off[3];
  c2.out = L->y2;
  DQZ_HIP((launch_gemm<CfgConv>(st, c2)));
  pe.mark(2, st);

  Conv3Fwd c3;
  static_cast<Shape&>(c3) = make_shape<CfgConv>(Z, B * C3M, C3CO, C3KK, 1);
  c3.in = L->y2;
  c3.B = B;
  c3.nz = nz;
  c3.w_off = L->off[4];
  c3.b_off = L->off[5];
  c3.out = L->y3;
  DQZ_HIP((launch_gemm<CfgConv>(st, c3)));
  pe.mark(3, st);

  Fc1Fwd f1;
  static_cast<Shape&>(f1) = make_shape<CfgFc1>(Z, B, HID, FLAT, L->S_fc1);
  f1.in = L->y3;
  f1.nz = nz;
  f1.w_off = L->off[6];
  f1.part = L->fc1p;
  DQZ_HIP((launch_gemm<CfgFc1>(st, f1)));
  pe.mark(4, st);

  const int n = Z * B * HID;
  hipLaunchKernelGGL(fc1_reduce_kernel, dim3((n + 255) / 256), dim3(256), 0, st, L->fc1p, nz, L->off[7], Z,
                     f1.g.S, B, L->h1);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

static int step_impl(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                     const float* is_weights, void* stream, PhaseEvents pe) {
  if (!L || !P || !P->online || !P->target || !P->mu || !P->nu || !slots)
    return fail(DQZ_ERR_INVALID, "null argument");
  if (int rc = check_store(S)) return rc;
  if (L->cfg.algo == DQZ_ALGO_PER && !is_weights) return fail(DQZ_ERR_INVALID, "PER step needs is_weights");
  hipStream_t st = (hipStream_t)stream;
  const int B = L->cfg.batch, Z = L->Z, A = L->cfg.num_actions;
  NetZ nz;
  nz.p[0] = P->online;
  nz.p[1] = P->target;
  nz.p[2] = P->online;
  nz.which[0] = 0;
  nz.which[1] = 1;
  nz.which[2] = 1;
  if (int rc = forward_impl(L, nz, Z, B, S, slots, nullptr, st, pe)) return rc;
  pe.mark(5, st);

  Rms rms;
  rms.lr = L->cfg.learning_rate;
  rms.decay = L->cfg.decay;
  rms.c1 = (float)(1.0 - (double)L->cfg.decay);
  rms.eps = L->cfg.eps;

  HeadArgs h;
  h.h1 = L->h1;
  h.nz = nz;
  h.w2_off = L->off[8];
  h.b2_off = L->off[9];
  h.Z = Z;
  h.B = B;
  h.A = A;
  h.algo = L->cfg.algo;
  h.shared_bias = L->shared_bias;
  h.fwd_only = 0;
  h.slots = slots;
  h.action = S->action;
  h.reward = S->reward;
  h.discount = S->discount;
  h.weights = L->cfg.algo == DQZ_ALGO_PER ? is_weights : nullptr;
  h.bound = L->cfg.grad_error_bound;
  h.q = L->q;
  h.td = L->td;
  h.loss = L->loss;
  h.dz1 = L->dz1;
  h.gfc = L->gfc;
  hipLaunchKernelGGL(head_kernel, dim3(1), dim3(1024), 0, st, h);
  DQZ_HIP(hipGetLastError());
  pe.mark(6, st);

  // fc1 dX -> dy3
  Fc1Dx fdx;
  static_cast<Shape&>(fdx) = make_shape<CfgFc1Dx>(1, B, FLAT, HID, 1);
  fdx.dz1 = L->dz1;
  fdx.w1 = P->online + L->off[6];
  fdx.y3 = L->y3;
  fdx.dy3 = L->dy3;
  DQZ_HIP((launch_gemm<CfgFc1Dx>(st, fdx)));
  pe.mark(7, st);

  // {conv3 dX, conv3 dW, fc1 dW + RMSProp}
  Conv3Dx c3dx;
  static_cast<Shape&>(c3dx) = make_shape<CfgBwd2>(1, B * C2M, C3CI, C3KK, 1);
  c3dx.dy3 = L->dy3;
  c3dx.w3 = P->online + L->off[4];
  c3dx.y2 = L->y2;
  c3dx.dy2 = L->dy2;
  Conv3Dw c3dw;
  static_cast<Shape&>(c3dw) = make_shape<CfgBwd2>(1, C3KK + 1, C3CO, B * C3M, L->S3);
  c3dw.in = L->y2;
  c3dw.dy = L->dy3;
  c3dw.part = L->p3;
  Fc1DwRms f1dw;
  static_cast<Shape&>(f1dw) = make_shape<CfgBwd2>(1, FLAT, HID, B, 1);
  f1dw.y3 = L->y3;
  f1dw.dz1 = L->dz1;
  f1dw.th = P->online;
  f1dw.mu = P->mu;
  f1dw.nu = P->nu;
  f1dw.w_off = L->off[6];
  f1dw.rms = rms;
  DQZ_HIP((launch_gemm<CfgBwd2>(st, c3dx, c3dw, f1dw)));
  pe.mark(8, st);

  // {conv2 dX (phased), conv2 dW}
  Conv2DxPhased c2dx;
  static_cast<Shape&>(c2dx) = make_shape<CfgBwd3>(4, B * 100, C2CI, 4 * C2CO, 1);
  c2dx.dy2 = L->dy2;
  c2dx.w2 = P->online + L->off[2];
  c2dx.y1 = L->y1;
  c2dx.dy1 = L->dy1;
  Conv2Dw c2dw;
  static_cast<Shape&>(c2dw) = make_shape<CfgBwd3>(1, C2KK + 1, C2CO, B * C2M, L->S2);
  c2dw.in = L->y1;
  c2dw.dy = L->dy2;
  c2dw.part = L->p2;
  DQZ_HIP((launch_gemm<CfgBwd3>(st, c2dx, c2dw)));
  pe.mark(9, st);

  // conv1 dW
  Conv1Dw c1dw;
  static_cast<Shape&>(c1dw) = make_shape<CfgBwd3>(1, C1KK + 1, C1CO, B * C1M, L->S1);
  c1dw.frames = S->frames;
  c1dw.fidx = S->fidx;
  c1dw.slots = slots;
  c1dw.which = 0;
  c1dw.dy1 = L->dy1;
  c1dw.part = L->p1;
  DQZ_HIP((launch_gemm<CfgBwd3>(st, c1dw)));
  pe.mark(10, st);

  UpdArgs u;
  u.th = P->online;
  u.mu = P->mu;
  u.nu = P->nu;
  for (int i = 0; i < 10; ++i) {
    u.off[i] = L->off[i];
    u.sz[i] = L->sz[i];
  }
  u.p1 = L->p1;
  u.p2 = L->p2;
  u.p3 = L->p3;
  u.S1 = c1dw.g.S;
  u.S2 = c2dw.g.S;
  u.S3 = c3dw.g.S;
  u.gfc = L->gfc;
  u.A = A;
  u.nb2 = L->shared_bias ? 1 : A;
  u.rms = rms;
  const int64_t nupd = L->sz[0] + L->sz[1] + L->sz[2] + L->sz[3] + L->sz[4] + L->sz[5] + HID + (int64_t)HID * A + u.nb2;
  hipLaunchKernelGGL(update_kernel, dim3((unsigned)((nupd + 255) / 256)), dim3(256), 0, st, u);
  DQZ_HIP(hipGetLastError());
  pe.mark(DQZ_NUM_PHASES, st);
  return DQZ_OK;
}

int dqz_learner_step(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                     const float* is_weights, void* stream) {
  return step_impl(L, P, S, slots, is_weights, stream, PhaseEvents{nullptr});
}

int dqz_learner_profile(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                        const float* is_weights, int iters, float* phase_ms, void* stream) {
  if (!phase_ms || iters < 1) return fail(DQZ_ERR_INVALID, "phase_ms must be non-null and iters >= 1");
  hipStream_t st = (hipStream_t)stream;
  hipEvent_t ev[DQZ_NUM_PHASES + 1];
  for (int i = 0; i <= DQZ_NUM_PHASES; ++i) DQZ_HIP(hipEventCreate(&ev[i]));
  for (int i = 0; i < DQZ_NUM_PHASES; ++i) phase_ms[i] = 0.f;
  int rc = DQZ_OK;
  for (int it = 0; it < iters && rc == DQZ_OK; ++it) {
    rc = step_impl(L, P, S, slots, is_weights, stream, PhaseEvents{ev});
    if (rc) break;
    if (hipEventSynchronize(ev[DQZ_NUM_PHASES]) != hipSuccess) {
      rc = fail(DQZ_ERR_HIP, "hipEventSynchronize failed");
      break;
    }
    for (int i = 0; i < DQZ_NUM_PHASES; ++i) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, ev[i], ev[i + 1]);
      phase_ms[i] += ms / (float)iters;
    }
  }
  (void)st;
  for (int i = 0; i <= DQZ_NUM_PHASES; ++i) (void)hipEventDestroy(ev[i]);
  return rc;
}

int dqz_learner_outputs(dqz_learner* L, float* q_tm1, float* td, float* loss, void* stream) {
  if (!L) return fail(DQZ_ERR_INVALID, "null learner");
  hipStream_t st = (hipStream_t)stream;
  const int B = L->cfg.batch, A = L->cfg.num_actions;
  if (q_tm1) DQZ_HIP(hipMemcpyAsync(q_tm1, L->q, sizeof(float) * B * A, hipMemcpyDeviceToDevice, st));
  if (td) DQZ_HIP(hipMemcpyAsync(td, L->td, sizeof(float) * B, hipMemcpyDeviceToDevice, st));
  if (loss) DQZ_HIP(hipMemcpyAsync(loss, L->loss, sizeof(float), hipMemcpyDeviceToDevice, st));
  return DQZ_OK;
}

static int forward_head_only(dqz_learner* L, const NetZ& nz, int n, float* q_out, hipStream_t st) {
  HeadArgs h;
  memset(&h, 0, sizeof(h));
  h.h1 = L->h1;
  h.nz = nz;
  h.w2_off = L->off[8];
  h.b2_off = L->off[9];
  h.Z = 1;
  h.B = n;
  h.A = L->cfg.num_actions;
  h.algo = L->cfg.algo;
  h.shared_bias = L->shared_bias;
  h.fwd_only = 1;
  h.q = q_out;
  hipLaunchKernelGGL(head_kernel, dim3(1), dim3(1024), 0, st, h);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_forward(dqz_learner* L, const float* params, const uint8_t* states, int n, float* q_out, void* stream) {
  if (!L || !params || !states || !q_out) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 1 || n > L->cfg.batch) return fail(DQZ_ERR_INVALID, "n must be in [1, %d]", L->cfg.batch);
  hipStream_t st = (hipStream_t)stream;
  NetZ nz;
  nz.p[0] = nz.p[1] = nz.p[2] = params;
  nz.which[0] = nz.which[1] = nz.which[2] = 0;
  if (int rc = forward_impl(L, nz, 1, n, nullptr, nullptr, states, st)) return rc;
  return forward_head_only(L, nz, n, q_out, st);
}

int dqz_forward_slots(dqz_learner* L, const float* params, const dqz_store* S, const int32_t* slots, int n, int which,
                      float* q_out, void* stream) {
  if (!L || !params || !slots || !q_out) return fail(DQZ_ERR_INVALID, "null argument");
  if (int rc = check_store(S)) return rc;
  if (n < 1 || n > L->cfg.batch) return fail(DQZ_ERR_INVALID, "n must be in [1, %d]", L->cfg.batch);
  if (which != 0 && which != 1) return fail(DQZ_ERR_INVALID, "which must be 0 (s_tm1) or 1 (s_t)");
  hipStream_t st = (hipStream_t)stream;
  NetZ nz;
  nz.p[0] = nz.p[1] = nz.p[2] = params;
  nz.which[0] = nz.which[1] = nz.which[2] = which;
  if (int rc = forward_impl(L, nz, 1, n, S, slots, nullptr, st)) return rc;
  return forward_head_only(L, nz, n, q_out, st);
}

int dqz_sample_uniform(int64_t base, int64_t size, int64_t capacity, int n, uint64_t seed, uint64_t* counter_dev,
                       int32_t* out_slots, void* stream) {
  if (!counter_dev || !out_slots) return fail(DQZ_ERR_INVALID, "null argument");
  if (size < 1) return fail(DQZ_ERR_INVALID, "cannot sample from an empty replay (size=%lld)", (long long)size);
  if (capacity < size) return fail(DQZ_ERR_INVALID, "size exceeds capacity");
  if (n < 1 || n > 65536) return fail(DQZ_ERR_INVALID, "n out of range");
  if (base < 0) return fail(DQZ_ERR_INVALID, "base must be >= 0");
  hipLaunchKernelGGL(sample_uniform_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, base, size, capacity, n, seed,
                     counter_dev, out_slots);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_gather_stacks(const dqz_store* S, const int32_t* slots, int n, int which, uint8_t* out, void* stream) {
  if (int rc = check_store(S)) return rc;
  if (!slots || !out) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 0) return fail(DQZ_ERR_INVALID, "n must be >= 0");
  if (which != 0 && which != 1) return fail(DQZ_ERR_INVALID, "which must be 0 (s_tm1) or 1 (s_t)");
  if (n == 0) return DQZ_OK;
  const int64_t total = (int64_t)n * FB;
  hipLaunchKernelGGL(gather_stacks_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     S->frames, S->fidx, slots, n, which, out);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_target_copy(float* target, const float* online, int64_t total, void* stream) {
  if (!target || !online || total < 0) return fail(DQZ_ERR_INVALID, "bad argument");
  DQZ_HIP(hipMemcpyAsync(target, online, total * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return DQZ_OK;
}

}  // extern "C"
