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
// Three launches.  The tangent forward (t1 .. t4) and the tangent backward
// (b3 .. b1) are independent chains: b3 needs only the primal d4, the
// tangent weights and ddot4 = relu'(h) Wdot2[:, a], which each b3 wave forms
// from eight gathers.  So the chains run side by side, and two more stage
// boundaries go by recomputation or alignment:
//   L1 hvp_l1_kernel  t12 (each conv2 block recomputes the conv1 tangent of
//                     its 4 x 4 input window, then its conv2 outputs) |
//                     s1 and ddot4 | b3
//   L2 hvp_l2_kernel  t34 (conv3 block (p, g) = fc1 K-chunk 4 p + g: the 16
//                     conv3 outputs it forms are the chunk's 16 rows) | b2
//   L3 hvp_l3_kernel  b1 | every parameter block of H_q w (conv1's need
//                     all of ddot1 and wait for it in-launch).
// Round 5 ran eight launches, one per dependent stage, each ≈ 5.1 us
// (rocprofv3) for a few microseconds of latency.  Every per-element sum
// keeps the order of that form.  Each stage splits its reduction over the
// threads of a workgroup and sums the splits through LDS in a fixed order
// (deterministic, no partial-sum launches); the two passes over fc1's 3136
// x 512 weights (t4, b3) read whole rows with coalesced 8- / 16-byte loads
// over hundreds of workgroups (they are the chain's HBM traffic: 2 x 2 x
// 6.4 MB).  t4's K-chunk partials are summed by the gradient launch, the only
// consumer of the fc1 tangent output.
#pragma once
#include "common.hpp"

// Timing-only builds (tools/gpu_hvp_split.sh): DQZ_EXP_HVP_SKIP is a mask of
// block ranges that return at once (1 t12, 2 b3, 4 b1's sums — its arrival
// stays, 8 conv2 / conv3 parameter rows, 16 fc1 parameters, 32 conv1
// parameter rows, 64 t34, 128 b2).  The numerics of those builds are wrong
// by design.
#ifndef DQZ_EXP_HVP_SKIP
#define DQZ_EXP_HVP_SKIP 0
#endif


namespace dqz {

struct HvpArgs {
  // x: the online transition's s_tm1 bytes [4][84][84], copied by the theta'
  // forward's conv1 stage (Conv1Src::xout)
  const uint8_t* x;
  // the one-transition learner's batch record {a as int bits, r, d, 0}, which
  // the theta' forward copied from the store (a in one trip, not slot -> action)
  const float4* rec;
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
  // grad q . w: the meta_second_kernel partials, summed once (L1's s1 block)
  const float* s1_part;
  int s1_nparts;
  float* s1;  // [1]
  // meta_combine in the gradient blocks' epilogue (vout != null): instead of
  // H_q w -> hq, v = v_dir + J (alpha s1 grad q - clip(td') H_q w) -> vout,
  // alpha = [|td'| < bound]
  const float *vdir, *J, *gq, *td;
  float bound;
  float* vout;
  // ddot1 complete: the 400 b1 blocks arrive, the 257 conv1 parameter
  // blocks at the end of the same launch wait (sample word 0)
  Handoff td1_pub;
};

// One element of the gradient blocks' output: H_q w itself, or meta_combine's v.
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
  // the first n of N puts, every load issued before the first store
  template <int N>
  __device__ __forceinline__ void put_n(const HvpArgs& a, const int64_t* i, const float* hq, int n) const {
    if (a.vout) {
      float vd[N], jj[N], g[N];
#pragma unroll
      for (int u = 0; u < N; ++u) {
        vd[u] = a.vdir[i[u]];
        jj[u] = a.J[i[u]];
        g[u] = a.gq[i[u]];
      }
#pragma unroll
      for (int u = 0; u < N; ++u)
        if (u < n) a.vout[i[u]] = vd[u] + jj[u] * (a_s1 * g[u] - clip * hq[u]);
    } else {
#pragma unroll
      for (int u = 0; u < N; ++u)
        if (u < n) a.hq[i[u]] = hq[u];
    }
  }
};

constexpr int HVP_T4_KC = 16, HVP_T4_CHUNKS = FLAT / HVP_T4_KC;  // 196 chunks of 16 rows
constexpr int HVP_T12 = C2M * (C2CO / 16);                       // 324: (conv2 position, 16-channel group)
constexpr int HVP_T34 = C3M * (C3CO / 16);                       // 196: (conv3 position, 16-channel group)
constexpr int HVP_B3 = FLAT / 16;                                // 196: 16 fc1 rows each
constexpr int HVP_B2 = C2M * (C2CO / 16);                        // 324: (conv2 position, 16-channel group)
static_assert(HVP_T34 == HVP_T4_CHUNKS, "conv3 block i forms fc1 chunk i's rows");

// ---- L1 -----------------------------------------------------------------

// A conv2 block's conv1 window: conv1 outputs (2 oh + dy, 2 ow + dx), dy, dx
// in 0..3, read the 20 x 20 input tile at rows / columns 8 oh, 8 ow.
constexpr int T12_IN = C1S * 3 + C1K;  // 20
struct HvpT12Smem {
  float4 in[T12_IN * T12_IN];  // [row][col], the 4 channels of one pixel
  union {
    float w1[C1KK][C1CO];       // Wdot1, staged by 16-byte global_load_lds (lane-linear)
    float r[4][16][C1CO];       // then: the waves' conv1 partials [wave][position][channel]
  };
  float t1[16][C1CO];           // ty1 over the window
  float r2[64][16];             // conv2 (tap, input-channel group) partials
};

// t1 + t2: ty1 = relu'(y1) (bdot1 + sum_k x_p[k] Wdot1[k][co]) over the
// block's window (an f32 MFMA product per wave over two kh rows; the four
// wave partials summed in a fixed order), then
// ty2 = relu'(y2) (bdot2 + conv(y1, Wdot2) + conv(ty1, W2)) for 16 channels
// (thread (tap = t / 16, co quad cq = t / 4 % 4, input-channel group cg =
// t % 4): 4 output channels x 8 input channels with 16-byte loads; the 64
// (tap, cg) partials are summed in order).  Each conv1 position is stored by
// one block: channel group 0 of the conv2 position oh = min(ih / 2, 8),
// ow = min(iw / 2, 8).  Every thread issues 38 loads, most of them 16 bytes
// (a form with 130 scalar loads per thread waited for its loads in two
// rounds: a wave cannot hold more than 63 in flight).
__device__ __forceinline__ void hvp_t12_block(const HvpArgs& a, int i, HvpT12Smem& s) {
  if (DQZ_EXP_HVP_SKIP & 1) return;
  const int t = threadIdx.x, p = i >> 2, g = i & 3;
  const int oh = p / C2O, ow = p % C2O;
  const int kh = t >> 5, co = t & 31;
  // the input tile's bytes (the theta' forward's copy: one trip, no slot ->
  // frame-index -> frame chain), Wdot1 and the window's y1 (no branch among
  // the loads: a branch made the compiler drain them all)
  constexpr int N = T12_IN * T12_IN * FC, R = (N + 255) / 256;  // 1600 tile elements, 7 rounds
  unsigned xb[R];
  {
    const uint8_t* fr = a.x + (t & 3) * FB + C1S * 2 * oh * FW + C1S * 2 * ow;
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const int px = min(t + 256 * u, N - 1) >> 2;  // element e = pixel * 4 + channel, channel = t % 4
      xb[u] = fr[(px / T12_IN) * FW + px % T12_IN];
    }
  }
  // Wdot1 straight into LDS (global_load_lds, 16 bytes a lane: no registers,
  // in flight beside the tile's bytes; through registers the scheduler issued
  // them after the bytes had landed, or spilled them)
  constexpr int W1Q = C1KK * C1CO / 4 / 256;  // 8 float4 per thread
  {
    const float4* wg = reinterpret_cast<const float4*>(a.tw + a.off[0]);
    float4* wl = reinterpret_cast<float4*>(&s.w1[0][0]);
#pragma unroll
    for (int u = 0; u < W1Q; ++u)
      __builtin_amdgcn_global_load_lds((const void*)(wg + t + 256 * u),
                                       (__attribute__((address_space(3))) void*)(wl + 256 * u + 64 * (t >> 6)), 16, 0, 0);
  }
  float y1v[2];
  int p1[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pos = kh + 8 * h;
    p1[h] = (2 * oh + (pos >> 2)) * C1O + 2 * ow + (pos & 3);
    y1v[h] = a.y1[p1[h] * C1CO + co];
  }
  const float b1v = a.tw[a.off[1] + co];
  {
    float* in = reinterpret_cast<float*>(s.in);
#pragma unroll
    for (int u = 0; u < R; ++u)
      if (t + 256 * u < N) in[t + 256 * u] = u8n(xb[u]);
  }
  __syncthreads();
  DQZ_STAMP(16, 1);
  // the conv2 operands, in flight under the conv1 tangent (issued before the
  // barrier, they held it until every one had landed: 4.4 us to the staged
  // tile against 3.2 with no loads at all, profiles/r05/s35)
  const int tap = t >> 4, cq = (t >> 2) & 3, cg = t & 3;
  const int src = ((2 * oh + (tap >> 2)) * C1O + 2 * ow + (tap & 3)) * C1CO + 8 * cg;
  const int64_t wo = (int64_t)(tap * C2CI + 8 * cg) * C2CO + 16 * g + 4 * cq;
  float4 w2[8], wd2[8], yv[2];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    w2[e] = *reinterpret_cast<const float4*>(a.th + a.off[2] + wo + e * C2CO);
    wd2[e] = *reinterpret_cast<const float4*>(a.tw + a.off[2] + wo + e * C2CO);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) yv[h] = *reinterpret_cast<const float4*>(a.y1 + src + 4 * h);
  const int c2 = 16 * g + (t & 15);
  const float y2v = a.y2[p * C2CO + c2];  // used by t < 16
  const float b2v = a.tw[a.off[3] + c2];
  // conv1 tangent on v_mfma_f32_16x16x4_f32 (exact f32 products):
  // D[pos][co] = sum_k x[pos][k] Wdot1[k][co], k = (kh, kw, ci), wave w
  // summing kh = 2 w, 2 w + 1 (16 K-steps of 4), two 16-channel tiles.
  // Lane l holds A[pos = l % 16][k = 4 s + l / 16] and B[k][co = l % 16]; D
  // rows 4 (l / 16) .. + 3, column l % 16.  (VALU dot products from LDS
  // took 4.7 us of the block, s36.)
  {
    const int lane = t & 63, wv = t >> 6, mi = lane & 15, kq = lane >> 4;
    const float* inf = reinterpret_cast<const float*>(s.in);
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      const int khh = 2 * wv + (st >> 3), kw = st & 7, k = khh * C1K * FC + kw * FC + kq;
      const float av = inf[((4 * (mi >> 2) + khh) * T12_IN + 4 * (mi & 3) + kw) * 4 + kq];
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, s.w1[k][mi], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, s.w1[k][16 + mi], acc1, 0, 0, 0);
    }
    __syncthreads();  // s.r overwrites s.w1
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      s.r[wv][4 * kq + r][mi] = acc0[r];
      s.r[wv][4 * kq + r][16 + mi] = acc1[r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int pos = kh + 8 * h, dy = pos >> 2, dx = pos & 3;
    const float v = b1v + ((s.r[0][pos][co] + s.r[1][pos][co]) + (s.r[2][pos][co] + s.r[3][pos][co]));
    const float ty = y1v[h] > 0.f ? v : 0.f;
    s.t1[pos][co] = ty;
    if (g == 0 && (dy < 2 || oh == C2O - 1) && (dx < 2 || ow == C2O - 1)) a.ty1[p1[h] * C1CO + co] = ty;
  }
  __syncthreads();
  DQZ_STAMP(16, 2);
  float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  const float4* tt = reinterpret_cast<const float4*>(&s.t1[tap][8 * cg]);
  const float4 ta[2] = {tt[0], tt[1]};
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float yy = e < 4 ? (&yv[0].x)[e] : (&yv[1].x)[e - 4];
    const float ty = e < 4 ? (&ta[0].x)[e] : (&ta[1].x)[e - 4];
    z.x += yy * wd2[e].x + ty * w2[e].x;
    z.y += yy * wd2[e].y + ty * w2[e].y;
    z.z += yy * wd2[e].z + ty * w2[e].z;
    z.w += yy * wd2[e].w + ty * w2[e].w;
  }
  *reinterpret_cast<float4*>(&s.r2[4 * tap + cg][4 * cq]) = z;
  __syncthreads();
  if (t < 16) {
    float v = b2v;
#pragma unroll
    for (int k = 0; k < 64; ++k) v += s.r2[k][t];
    a.ty2[p * C2CO + c2] = y2v > 0.f ? v : 0.f;
  }
}

// s1 = sum of the grad q . w partials (eight loads in flight per round: one
// round trip per 2,048 partials), and ddot4 = relu'(h) Wdot2[:, a] stored
// for the gradient blocks.
__device__ __forceinline__ void hvp_s1_block(const HvpArgs& a, float* s_w) {
  const int t = threadIdx.x;
  const int act = __float_as_int(a.rec[0].x);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int n = t + 256 * h;
    a.td4[n] = a.h[n] > 0.f ? a.tw[a.off[8] + n * a.A + act] : 0.f;
  }
  float v = 0.f;
  for (int j0 = t; j0 < a.s1_nparts; j0 += 8 * 256) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = a.s1_part[min(j0 + 256 * u, a.s1_nparts - 1)];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (j0 + 256 * u < a.s1_nparts) v += x[u];
  }
  v = block_sum256(v, s_w);
  if (t == 0) a.s1[0] = v;
}

// b3: ddot3[k] = relu'(y3[k]) sum_n (Wdot1[k][n] d4[n] + W1[k][n] ddot4[n]):
// 16 rows per block, wave w rows 16 i + 4 w .. + 3 (lane l: columns 8 l ..
// 8 l + 7, 16-byte loads, all four rows' loads issued together); the lane's
// eight ddot4 = relu'(h) Wdot2[n][a] are formed here.  For A <= 16 the block
// stages all of Wdot2 (512 x A) in LDS beside the row loads, so a's load
// runs under them instead of before another trip (the gathers of column a).
__device__ __forceinline__ void hvp_b3_block(const HvpArgs& a, int i, float* s_w2) {
  if (DQZ_EXP_HVP_SKIP & 2) return;
  constexpr int R = 4;
  const int t = threadIdx.x, lane = t & 63, k0 = 16 * i + R * (t >> 6);
  const int act = __float_as_int(a.rec[0].x);
  const bool staged = a.A <= 16;
  float4 wq[8];  // Wdot2 as float4: 128 A elements, A / 2 per thread (A <= 16; always in range)
#pragma unroll
  for (int u = 0; u < 8; ++u) wq[u] = reinterpret_cast<const float4*>(a.tw + a.off[8])[min(t + 256 * u, HID * a.A / 4 - 1)];
  float4 w[R][2], wd[R][2], d[2], hv[2];
  float y3[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const float *W = a.th + a.off[6] + (int64_t)(k0 + r) * HID + 8 * lane,
                *Wd = a.tw + a.off[6] + (int64_t)(k0 + r) * HID + 8 * lane;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      w[r][h] = reinterpret_cast<const float4*>(W)[h];
      wd[r][h] = reinterpret_cast<const float4*>(Wd)[h];
    }
    y3[r] = a.y3[k0 + r];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    d[h] = reinterpret_cast<const float4*>(a.d4 + 8 * lane)[h];
    hv[h] = reinterpret_cast<const float4*>(a.h + 8 * lane)[h];
  }
  float g[8];
  if (staged) {
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (t + 256 * u < HID * a.A / 4) reinterpret_cast<float4*>(s_w2)[t + 256 * u] = wq[u];
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] = s_w2[(8 * lane + q) * a.A + act];
  } else {
    const float* w2 = a.tw + a.off[8] + (int64_t)(8 * lane) * a.A + act;
#pragma unroll
    for (int q = 0; q < 8; ++q) g[q] = w2[q * a.A];
  }
  float4 dd[2];
#pragma unroll
  for (int h = 0; h < 2; ++h)
    dd[h] = make_float4(hv[h].x > 0.f ? g[4 * h] : 0.f, hv[h].y > 0.f ? g[4 * h + 1] : 0.f,
                        hv[h].z > 0.f ? g[4 * h + 2] : 0.f, hv[h].w > 0.f ? g[4 * h + 3] : 0.f);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    float z = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      z += ((wd[r][h].x * d[h].x + w[r][h].x * dd[h].x) + (wd[r][h].y * d[h].y + w[r][h].y * dd[h].y)) +
           ((wd[r][h].z * d[h].z + w[r][h].z * dd[h].z) + (wd[r][h].w * d[h].w + w[r][h].w * dd[h].w));
    z = wave_sum(z);
    if (lane == 0) a.td3[k0 + r] = y3[r] > 0.f ? z : 0.f;
  }
}

constexpr int HVP_L1_BLOCKS = HVP_T12 + 1 + HVP_B3;  // 521
__global__ __launch_bounds__(256) void hvp_l1_kernel(HvpArgs a) {
  __shared__ HvpT12Smem s;
  const int i = blockIdx.x;
  DQZ_STAMP(16, 0);
  if (i < HVP_T12)
    hvp_t12_block(a, i, s);
  else if (i == HVP_T12)
    hvp_s1_block(a, &s.r2[0][0]);
  else
    hvp_b3_block(a, i - HVP_T12 - 1, &s.w1[0][0]);
  DQZ_STAMP(16, 3);
}

// ---- L2 -----------------------------------------------------------------

// t3 + t4: ty3 = relu'(y3) (bdot3 + conv(y2, Wdot3) + conv(ty2, W3)) for
// conv3 position p, channels 16 g .. 16 g + 15 (thread (input channel ci =
// t / 4, output-channel quad c4 = t % 4) over the 9 taps, 16-byte weight
// loads; the 64 input-channel partials summed in order) — flat rows 16 i ..
// 16 i + 15, which are fc1 K-chunk i: part[i][n] = sum_j y3[k] Wdot1[k][n] +
// ty3[k] W1[k][n] (thread (row half rh = t / 128, column quad cq = t % 128):
// 8 rows of 4 columns each, the two halves added in order).  56 loads per
// thread, all issued first (a form with 144 scalar conv loads per thread
// waited for them in several rounds: a wave holds at most 63 in flight).
struct HvpT34Smem {
  float r[64][16];  // conv3 input-channel partials
  float4 c[128];    // fc1 chunk: rows 8 .. 15's sums
  float ty[16];
};
__device__ __forceinline__ void hvp_t34_block(const HvpArgs& a, int i, HvpT34Smem& s) {
  if (DQZ_EXP_HVP_SKIP & 64) return;
  const int t = threadIdx.x, p = i >> 2, g = i & 3;
  const int rh = t >> 7, cq = t & 127;
  float4 fw[8], fwd[8], fy[2];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t k = (int64_t)i * HVP_T4_KC + 8 * rh + j;
    fw[j] = *reinterpret_cast<const float4*>(a.th + a.off[6] + k * HID + 4 * cq);
    fwd[j] = *reinterpret_cast<const float4*>(a.tw + a.off[6] + k * HID + 4 * cq);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) fy[h] = *reinterpret_cast<const float4*>(a.y3 + i * HVP_T4_KC + 8 * rh + 4 * h);
  const int oh = p / C3O, ow = p % C3O, ci = t >> 2, c4 = t & 3;
  float yv[9], tv[9];
  float4 wv[9], wdv[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int src = ((oh + tap / 3) * C2O + ow + tap % 3) * C2CO + ci;
    const int64_t wi = (int64_t)(tap * C3CI + ci) * C3CO + 16 * g + 4 * c4;
    yv[tap] = a.y2[src];
    tv[tap] = a.ty2[src];
    wv[tap] = *reinterpret_cast<const float4*>(a.th + a.off[4] + wi);
    wdv[tap] = *reinterpret_cast<const float4*>(a.tw + a.off[4] + wi);
  }
  const int c = 16 * g + (t & 15);
  const float y3c = a.y3[p * C3CO + c];  // used by t < 16
  const float b3 = a.tw[a.off[5] + c];
  float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    z.x += yv[tap] * wdv[tap].x + tv[tap] * wv[tap].x;
    z.y += yv[tap] * wdv[tap].y + tv[tap] * wv[tap].y;
    z.z += yv[tap] * wdv[tap].z + tv[tap] * wv[tap].z;
    z.w += yv[tap] * wdv[tap].w + tv[tap] * wv[tap].w;
  }
  *reinterpret_cast<float4*>(&s.r[ci][4 * c4]) = z;
  __syncthreads();
  DQZ_STAMP(17, 1);
  if (t < 16) {
    float v = b3;
#pragma unroll
    for (int k = 0; k < 64; ++k) v += s.r[k][t];
    const float ty = y3c > 0.f ? v : 0.f;
    a.ty3[p * C3CO + c] = ty;
    s.ty[t] = ty;
  }
  __syncthreads();
  float4 zc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float ty = s.ty[8 * rh + j], y = j < 4 ? (&fy[0].x)[j] : (&fy[1].x)[j - 4];
    zc.x += y * fwd[j].x + ty * fw[j].x;
    zc.y += y * fwd[j].y + ty * fw[j].y;
    zc.z += y * fwd[j].z + ty * fw[j].z;
    zc.w += y * fwd[j].w + ty * fw[j].w;
  }
  if (rh == 1) s.c[cq] = zc;
  __syncthreads();
  if (rh == 0) {
    const float4 u = s.c[cq];
    *reinterpret_cast<float4*>(a.part + (int64_t)i * HID + 4 * cq) =
        make_float4(zc.x + u.x, zc.y + u.y, zc.z + u.z, zc.w + u.w);
  }
}

// b2: ddot2[pix][ci] = relu'(y2) sum_{taps, co} (d3 Wdot3 + ddot3 W3) (the
// transposed conv3, stride 1).  Block (pix, 16-channel group g); thread
// (ci, output-channel quad cs = t % 16): 16-byte W loads along co.
__device__ __forceinline__ void hvp_b2_block(const HvpArgs& a, int i, float (*s_r)[17]) {
  if (DQZ_EXP_HVP_SKIP & 128) return;
  const int t = threadIdx.x, pix = i >> 2, g = i & 3;
  const int ih = pix / C2O, iw = pix % C2O, cs = t & 15, cl = t >> 4, ci = 16 * g + cl;
  // the nine taps' operands loaded together (taps outside the output are
  // clamped to a valid position and skipped in the sum, in tap order)
  float4 w[9], wd[9], d[9], dd[9];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
    const int oh = min(max(ih - kh, 0), C3O - 1), ow = min(max(iw - kw, 0), C3O - 1);
    const int src = (oh * C3O + ow) * C3CO + 4 * cs;
    const int64_t wi = ((kh * C3K + kw) * C3CI + ci) * C3CO + 4 * cs;
    w[tap] = *reinterpret_cast<const float4*>(a.th + a.off[4] + wi);
    wd[tap] = *reinterpret_cast<const float4*>(a.tw + a.off[4] + wi);
    d[tap] = *reinterpret_cast<const float4*>(a.d3 + src);
    dd[tap] = *reinterpret_cast<const float4*>(a.td3 + src);
  }
  float z = 0.f;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int oh = ih - tap / 3, ow = iw - tap % 3;
    if (oh < 0 || oh >= C3O || ow < 0 || ow >= C3O) continue;
    z += ((d[tap].x * wd[tap].x + dd[tap].x * w[tap].x) + (d[tap].y * wd[tap].y + dd[tap].y * w[tap].y)) +
         ((d[tap].z * wd[tap].z + dd[tap].z * w[tap].z) + (d[tap].w * wd[tap].w + dd[tap].w * w[tap].w));
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

constexpr int HVP_L2_BLOCKS = HVP_T34 + HVP_B2;  // 520
__global__ __launch_bounds__(256) void hvp_l2_kernel(HvpArgs a) {
  __shared__ HvpT34Smem s;
  const int i = blockIdx.x;
  DQZ_STAMP(17, 0);
  if (i < HVP_T34)
    hvp_t34_block(a, i, s);
  else
    hvp_b2_block(a, i - HVP_T34, reinterpret_cast<float(*)[17]>(&s.r[0][0]));
  DQZ_STAMP(17, 3);
}

// ---- L3 -----------------------------------------------------------------

// b1: ddot1[pix][ci] = relu'(y1) sum_{taps, co} (d2 Wdot2 + ddot2 W2) (the
// transposed conv2, stride 2: at most 2 x 2 live taps).  Block pix; thread
// (ci = t / 8, output-channel octet cs = t % 8).
__device__ __forceinline__ void hvp_b1_block(const HvpArgs& a, int pix, float (*s_r)[9]) {
  if (DQZ_EXP_HVP_SKIP & 4) {
    a.td1_pub.arrive(0);
    return;
  }
  const int t = threadIdx.x;
  const int ih = pix / C1O, iw = pix % C1O, cs = t & 7, ci = t >> 3;
  // the 2 x 2 taps of this pixel's stride phase, every operand loaded before
  // the first product (taps outside the output clamped and skipped, in order)
  float4 w[4][2], wd[4][2], d[4][2], dd[4][2];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int kh = (ih & 1) + C2S * (q >> 1), kw = (iw & 1) + C2S * (q & 1);
    const int oh = min(max((ih - kh) / C2S, 0), C2O - 1), ow = min(max((iw - kw) / C2S, 0), C2O - 1);
    const int src = (oh * C2O + ow) * C2CO + 8 * cs;
    const int64_t wi = ((kh * C2K + kw) * C2CI + ci) * C2CO + 8 * cs;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      w[q][h] = *reinterpret_cast<const float4*>(a.th + a.off[2] + wi + 4 * h);
      wd[q][h] = *reinterpret_cast<const float4*>(a.tw + a.off[2] + wi + 4 * h);
      d[q][h] = *reinterpret_cast<const float4*>(a.d2 + src + 4 * h);
      dd[q][h] = *reinterpret_cast<const float4*>(a.td2 + src + 4 * h);
    }
  }
  float z = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int kh = (ih & 1) + C2S * (q >> 1), kw = (iw & 1) + C2S * (q & 1);
    if (ih < kh || (ih - kh) / C2S >= C2O || iw < kw || (iw - kw) / C2S >= C2O) continue;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      z += ((d[q][h].x * wd[q][h].x + dd[q][h].x * w[q][h].x) + (d[q][h].y * wd[q][h].y + dd[q][h].y * w[q][h].y)) +
           ((d[q][h].z * wd[q][h].z + dd[q][h].z * w[q][h].z) + (d[q][h].w * wd[q][h].w + dd[q][h].w * w[q][h].w));
  }
  s_r[ci][cs] = z;
  __syncthreads();
  if (t < C2CI) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += s_r[t][k];
    store_sc1_f1(a.td1, C1M * C1CO * 4, pix * C1CO + t, a.y1[pix * C1CO + t] > 0.f ? v : 0.f);
  }
  a.td1_pub.arrive(0);
}

// ---- the parameter-gradient blocks of H_q w (L3) -------------------------
//   [257] conv1 rows k (row 256 = bias): sum_p x_p[k] ddot1[p][co] over 8
//         position splits (thread (split, co)), after b1's hand-off;
//   [513] conv2 rows, [577] conv3 rows (last row = bias):
//         sum_p (ydot[src] d[p][co] + y[src] ddot[p][co]) over 4 position
//         splits (thread (split, co));
//   [8]   fc2 / fc1 bias / fc2 bias: hdot = relu'(h) (bdot1 + sum of t4's
//         chunk partials), the fc2 column a = hdot; 64 hidden units per
//         block, the 196 chunk partials of each in 4 groups of 49 loads;
//   [392] fc1: ydot3 (x) d4 + y3 (x) ddot4, 16 elements per thread.
// Every per-thread sum issues all its loads before the first addition
// (round 5: the position and chunk loops waited for one round trip per
// iteration, 13-21 serial trips, and kept the gradient launch at 12.2 us).
constexpr int HVP_G_C1 = C1KK + 1, HVP_G_C2 = C2KK + 1, HVP_G_C3 = C3KK + 1, HVP_G_H = HID / 64;
constexpr int HVP_G_FC = FLAT * HID / 16 / 256;  // 392 (hvp_g_fc1: 16 elements per thread)

template <int IH, int CI, int K, int S, int CO, int OH>
__device__ __forceinline__ void hvp_g_conv_row(const HvpArgs& a, const float* y, const float* yd, const float* d,
                                               const float* dd, int k, int64_t off_w, int64_t off_b, float (*s_r)[64],
                                               const HqOut& ho) {
  if (DQZ_EXP_HVP_SKIP & 8) return;
  const int t = threadIdx.x, co = t & 63, sp = t >> 6;  // 4 position splits
  constexpr int P = OH * OH, PS = (P + 3) / 4;
  const int p0 = sp * PS;
  float g = 0.f;
  if (k == K * K * CI) {
    float v[PS];
#pragma unroll
    for (int j = 0; j < PS; ++j) v[j] = dd[min(p0 + j, P - 1) * CO + co];
#pragma unroll
    for (int j = 0; j < PS; ++j)
      if (p0 + j < P) g += v[j];
  } else {
    const int kh = k / (K * CI), kw = (k / CI) % K, ci = k % CI;
    float u0[PS], u1[PS], w0[PS], w1[PS];
#pragma unroll
    for (int j = 0; j < PS; ++j) {
      const int p = min(p0 + j, P - 1);
      const int src = (((p / OH) * S + kh) * IH + (p % OH) * S + kw) * CI + ci;
      u0[j] = yd[src];
      u1[j] = d[p * CO + co];
      w0[j] = y[src];
      w1[j] = dd[p * CO + co];
    }
#pragma unroll
    for (int j = 0; j < PS; ++j)
      if (p0 + j < P) g += u0[j] * u1[j] + w0[j] * w1[j];
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

// hidden unit n = 64 i + t % 64: hdot, fc2 column, fc1 bias; fc2 bias = 0.
// Thread (group q, unit n): chunks [49 q, +49) of unit n, summed in chunk
// order, then the four group sums in group order.
__device__ __forceinline__ void hvp_g_hidden(const HvpArgs& a, int i, float (*s_r)[64], const HqOut& ho) {
  constexpr int NG = 4, CG = HVP_T4_CHUNKS / NG;  // 49
  static_assert(NG * CG == HVP_T4_CHUNKS, "chunk groups");
  const int t = threadIdx.x, nl = t & 63, q = t >> 6, n = 64 * i + nl;
  float pv[CG];
#pragma unroll
  for (int c = 0; c < CG; ++c) pv[c] = a.part[(int64_t)(CG * q + c) * HID + n];
  float zq = 0.f;
#pragma unroll
  for (int c = 0; c < CG; ++c) zq += pv[c];
  s_r[q][nl] = zq;
  __syncthreads();
  if (q != 0) return;
  const int act = __float_as_int(a.rec[0].x);
  const float z = a.tw[a.off[7] + n] + ((s_r[0][nl] + s_r[1][nl]) + (s_r[2][nl] + s_r[3][nl]));
  const float hd = a.h[n] > 0.f ? z : 0.f;
  // the row's A fc2 entries and the fc1 bias: every put's loads before its
  // store (a put per column waited one round trip each)
  constexpr int NP = 9;
  for (int c0 = 0; c0 < a.A + 1; c0 += NP) {
    int64_t idx[NP];
    float hq[NP];
#pragma unroll
    for (int u = 0; u < NP; ++u) {
      const int col = min(c0 + u, a.A);  // col A: the fc1 bias
      idx[u] = col < a.A ? a.off[8] + (int64_t)n * a.A + col : a.off[7] + n;
      hq[u] = col < a.A ? (col == act ? hd : 0.f) : a.td4[n];
    }
    ho.put_n<NP>(a, idx, hq, min(NP, a.A + 1 - c0));
  }
  if (i == 0 && t < a.A) ho.put(a, a.off[9] + t, 0.f);
}

// fc1 rows: 4 groups of 4 consecutive columns per thread (group u: element
// ((4 i + u) 256 + t) 4), every group's loads before the first store.
constexpr int HVP_G_FCU = 4;
__device__ __forceinline__ void hvp_g_fc1(const HvpArgs& a, int i, const HqOut& ho) {
  if (DQZ_EXP_HVP_SKIP & 16) return;
  const int t = threadIdx.x;
  constexpr int U = HVP_G_FCU;
  int64_t e[U];
  float ty[U], y[U];
  float4 d[U], dd[U], vd[U], jj[U], g[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    e[u] = ((int64_t)(U * i + u) * 256 + t) * 4;
    const int k = (int)(e[u] / HID), n = (int)(e[u] % HID);
    ty[u] = a.ty3[k];
    y[u] = a.y3[k];
    d[u] = *reinterpret_cast<const float4*>(a.d4 + n);
    dd[u] = *reinterpret_cast<const float4*>(a.td4 + n);
    if (a.vout) {
      const int64_t j = a.off[6] + e[u];
      vd[u] = *reinterpret_cast<const float4*>(a.vdir + j);
      jj[u] = *reinterpret_cast<const float4*>(a.J + j);
      g[u] = *reinterpret_cast<const float4*>(a.gq + j);
    }
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const float4 hq = make_float4(ty[u] * d[u].x + y[u] * dd[u].x, ty[u] * d[u].y + y[u] * dd[u].y,
                                  ty[u] * d[u].z + y[u] * dd[u].z, ty[u] * d[u].w + y[u] * dd[u].w);
    if (a.vout)
      *reinterpret_cast<float4*>(a.vout + a.off[6] + e[u]) = make_float4(
          vd[u].x + jj[u].x * (ho.a_s1 * g[u].x - ho.clip * hq.x), vd[u].y + jj[u].y * (ho.a_s1 * g[u].y - ho.clip * hq.y),
          vd[u].z + jj[u].z * (ho.a_s1 * g[u].z - ho.clip * hq.z), vd[u].w + jj[u].w * (ho.a_s1 * g[u].w - ho.clip * hq.w));
    else
      *reinterpret_cast<float4*>(a.hq + a.off[6] + e[u]) = hq;
  }
}

// conv1 row k (thread (split = t / 32 of 50 positions, co)).  The row's
// 400 patch values x_p[k] are staged before the wait for ddot1 (a loop of
// scattered byte loads per thread was 11 of the gradient launch's 20 us in
// round 4), ddot1 is read with sc1 loads after it.
__device__ __forceinline__ void hvp_g_conv1(const HvpArgs& a, int k, float (*s_r)[64], float* s_x, const HqOut& ho) {
  if (DQZ_EXP_HVP_SKIP & 32) return;
  const int t = threadIdx.x, co = t & 31, sp = t >> 5;
  if (k < C1KK) {
    const int kh = k / (C1K * FC), kw = (k / FC) % C1K, ci = k % FC;
    const uint8_t* fr = a.x + ci * FB;
    for (int p = t; p < C1M; p += 256) s_x[p] = u8n(fr[(C1S * (p / C1O) + kh) * FW + C1S * (p % C1O) + kw]);
  } else {
    for (int p = t; p < C1M; p += 256) s_x[p] = 1.f;  // bias row: sum_p ddot1
  }
  DQZ_STAMP(18, 1);
  a.td1_pub.wait(0);  // its barrier also publishes s_x
  DQZ_STAMP(18, 2);
  float tv[50];       // this thread's ddot1 column
#pragma unroll
  for (int j = 0; j < 50; ++j) tv[j] = load_sc1_f1(a.td1, C1M * C1CO * 4, (50 * sp + j) * C1CO + co);
  float g = 0.f;
#pragma unroll
  for (int j = 0; j < 50; ++j) g += s_x[50 * sp + j] * tv[j];
  s_r[sp][co] = g;
  __syncthreads();
  if (t < C1CO) {
    float v = 0.f;
#pragma unroll
    for (int s = 0; s < 8; ++s) v += s_r[s][t];
    ho.put(a, a.off[0] + (int64_t)k * C1CO + t, v);  // row 256 is the bias (off[1] = off[0] + 8192)
  }
}

// L3: b1 first, then the conv parameter rows that do not need ddot1 (the
// fc2 / bias rows first: the longest-lived), then conv1's, which wait
// in-launch for the 400 b1 blocks (all dispatched before any of them on
// every XCD, so the wait cannot hold a b1 block out), then the streaming fc1
// range, which fills the slots while conv1's rows finish (conv1's rows last:
// span 14.2 us against 12.9, profiles/r05/s33).  With the conv1 blocks
// right after b1, 257 pollers slowed every other block of the launch (its
// span 15.6 -> 25 us, s27; polling every ~1 us instead, 30 us, s31: the b1
// blocks' arrivals queue behind the polls of the same word).
constexpr int HVP_B1 = C1M;  // 400
constexpr int HVP_L3_BLOCKS = HVP_B1 + HVP_G_H + HVP_G_C2 + HVP_G_C3 + HVP_G_FC + HVP_G_C1;  // 2,147
__global__ __launch_bounds__(256) void hvp_l3_kernel(HvpArgs a) {
  __shared__ float s_r[8][64];
  __shared__ float s_x[C1M];
  constexpr int GH = HVP_B1, G2 = GH + HVP_G_H, G3 = G2 + HVP_G_C2, G1 = G3 + HVP_G_C3, GF = G1 + HVP_G_C1;
  const int i = blockIdx.x;
  DQZ_STAMP(18, 0);
  if (i < GH) {
    hvp_b1_block(a, i, reinterpret_cast<float(*)[9]>(&s_r[0][0]));
  } else {
    const HqOut ho(a);
    if (i < G2)
      hvp_g_hidden(a, i - GH, s_r, ho);
    else if (i < G3)
      hvp_g_conv_row<C1O, C1CO, C2K, C2S, C2CO, C2O>(a, a.y1, a.ty1, a.d2, a.td2, i - G2, a.off[2], a.off[3], s_r, ho);
    else if (i < G1)
      hvp_g_conv_row<C2O, C2CO, C3K, 1, C3CO, C3O>(a, a.y2, a.ty2, a.d3, a.td3, i - G3, a.off[4], a.off[5], s_r, ho);
    else if (i < GF)
      hvp_g_conv1(a, i - G1, s_r, s_x, ho);
    else
      hvp_g_fc1(a, i - GF, ho);
  }
  DQZ_STAMP(18, 3);
}

// The second order's elementwise stages run in gradient epilogues: the
// u' / v_dir / w pieces in the one-transition backward's (common.hpp
// Rms::meta3), v = v_dir + J (alpha s1 grad q - clip(td') H_q w) in the
// gradient blocks' (HqOut).

}  // namespace dqz
