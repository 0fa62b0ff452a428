// meta.hpp — MGSC meta-update kernels (dqn_mgsc_batched/agent.py:104-220).
//
// The reference differentiates meta_loss_fn w.r.t. the M meta-batch logits
// with per-transition gradients materialised by vmap (M x 6.75 MB).  Here
// nothing per-example is stored:
//   G  = sum_i p_i g_i is ONE batched backward whose per-sample cotangent at
//        q_i[a_i] is -p_i clip(td_i)   (head meta mode + gradient-output mode);
//   v  = dL/dG = -2 u' * du/dG          (elementwise, meta_rms1/2_kernel);
//   p_i dL/dp_i = p_i v.g_i = sum_layers <dz_i^(p), V * y_i + vb>, where
//        dz^(p) are the p-weighted pre-activation gradients the batched
//        backward already produced (they are linear in the cotangent) and
//        V * y is a forward of the stored activations with the tangent v as
//        weights (meta_dot_kernel);
//   dL/dx_j = p_j dL/dp_j - p_j sum_i p_i dL/dp_i (softmax backward), then
//        optax.adam on the logits (meta_adam_kernel).
#pragma once
#include "common.hpp"
#include "conv1.hpp"
#include "fwd.hpp"
#include "sampling.hpp"

namespace dqz {

constexpr int META_THREADS = 256;

__device__ __forceinline__ float block_sum_f32(float v, float* sbuf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  v = wave_sum(v);
  if (lane == 0) sbuf[wave] = v;
  __syncthreads();
  float r = sbuf[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r += sbuf[w];
  __syncthreads();
  return r;
}

__device__ __forceinline__ float block_max_f32(float v, float* sbuf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  if (lane == 0) sbuf[wave] = v;
  __syncthreads();
  float r = sbuf[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, sbuf[w]);
  __syncthreads();
  return r;
}

// p = exp(x - (c + log(sum exp(x - c)))), c = max x  (JNPprobabilities_from_logits,
// replay_circular.py:79-86).  Block 0 strides over the M meta-batch entries
// (x gathered from logits[pos]); blocks 1.. pad the slots to the chunked meta
// batch, slots_pad[i] = slots[min(i, M - 1)] (one launch for both).
__global__ __launch_bounds__(META_THREADS) void meta_softmax_kernel(const float* __restrict__ logits,
                                                                    const int32_t* __restrict__ pos, int M,
                                                                    float* __restrict__ x_out,
                                                                    float* __restrict__ p_out,
                                                                    const int32_t* __restrict__ slots, int n_pad,
                                                                    int32_t* __restrict__ slots_pad) {
  if (blockIdx.x > 0) {
    const int i = (blockIdx.x - 1) * META_THREADS + threadIdx.x;
    if (i < n_pad) slots_pad[i] = slots[min(i, M - 1)];
    return;
  }
  __shared__ float sbuf[META_THREADS / 64];
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < M; i += META_THREADS) {
    const float x = logits[pos[i]];
    x_out[i] = x;
    mx = fmaxf(mx, x);
  }
  const float c = block_max_f32(mx, sbuf);
  float se = 0.f;
  for (int i = threadIdx.x; i < M; i += META_THREADS) se += expf(x_out[i] - c);
  const float lse = c + logf(block_sum_f32(se, sbuf));
  for (int i = threadIdx.x; i < M; i += META_THREADS) p_out[i] = expf(x_out[i] - lse);
}

// ---- MGSC meta tangent forward in one launch ------------------------------
// V * y_{l-1} + vb of every layer over the meta batch's stored primal
// activations (linear mode, the tangent v as weights): the four layers are
// independent of each other, so one launch holds them as block ranges
// [conv1 4/sample] [conv2 4/sample] [conv3 4/sample] [fc1 tiles] instead of
// four dependent launches.  Dynamic LDS = conv1's 57.6 KB.
// With one meta chunk the blocks do not store V * y + vb: each adds
// <V * y + vb, dz> over its outputs (the p-weighted pre-activation gradient
// of the same layer, TangentDot) into its slot of part[b][META_DOT_SLOTS]
// (conv1 rows rb: slots 0..3, conv2 / conv3 quarters: 4..7 / 8..11, fc1
// (column tile nt, split s): 12 + 7 nt + s), and the conv3 quarter-0 block
// of sample b also the fc1 bias and fc2 terms (slot META_EXTRA_SLOT), so
// meta_dot_kernel's pass over the stored tangents disappears.
constexpr int META_EXTRA_SLOT = 12 + (HID / 32) * FC1_S;  // 124
static_assert(META_EXTRA_SLOT < META_DOT_SLOTS, "meta dot slots");

struct MetaExtra {
  const float* dz1;   // [M][512]
  const float* h1;    // [M][512] online fc1 output
  const float* gq;    // [M]
  const int32_t* ga;  // [M]
  const float* v;     // tangent (param layout)
  int64_t b1_off, w2_off, b2_off;
  int A;
  float* part;        // [M][META_DOT_SLOTS] (null: no dot products)
};

// vb1 . dz1[b] + gq[b] (h1[b] . V2[:, a_b] + vb2[a_b])  (256 threads)
__device__ __forceinline__ void meta_extra_term(const MetaExtra& e, int b, float* s_tmp) {
  const int t = threadIdx.x, act = e.ga[b];
  float f1 = 0.f, f2 = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int n = t + 256 * h;
    f1 += e.v[e.b1_off + n] * e.dz1[(int64_t)b * HID + n];
    f2 += e.h1[(int64_t)b * HID + n] * e.v[e.w2_off + n * e.A + act];
  }
  f1 = block_sum256(f1, s_tmp);
  f2 = block_sum256(f2, s_tmp);
  if (t == 0) e.part[(int64_t)b * META_DOT_SLOTS + META_EXTRA_SLOT] = f1 + e.gq[b] * (e.v[e.b2_off + act] + f2);
}

static_assert(4 * FC1_32RW * sizeof(float) <= kConv1FwdSmem, "fc1's 32 x 32 tiles fit the tangent launch's LDS");
inline int tangent_fwd_blocks(int B, int MG) { return 3 * 4 * ((B + 7) / 8 * 8) + fc1_fwd_blocks(1, MG); }
__global__ __launch_bounds__(256) void tangent_fwd_kernel(Conv1FwdArgs c1, LayerFwdArgs c2, LayerFwdArgs c3,
                                                          Fc1FwdArgs f1, MetaExtra ex) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int n = 4 * ((c1.B + 7) / 8 * 8);
  int i = blockIdx.x;
  if (i < n) {
    const SampleJob sj = xcd_sample_job_at(i, C1_BLOCKS, c1.B);
    if (sj.valid) conv1_fwd_body<false, 0>(c1, smem, sj);
    return;
  }
  i -= n;
  if (i < n) {
    const SampleJob sj = xcd_sample_job_at(i, 4, c2.B);
    if (sj.valid) conv2_fwd_body<false, false>(c2, smem, sj);
    return;
  }
  i -= n;
  if (i < n) {
    const SampleJob sj = xcd_sample_job_at(i, 4, c3.B);
    if (!sj.valid) return;
    conv3_fwd_body<false>(c3, smem, sj);
    if (ex.part && sj.job == 0) meta_extra_term(ex, sj.s, smem);
    return;
  }
  if (f1.dot.part) fc1_fwd_block32<true>(f1, smem, i - n); else fc1_fwd_block32<false>(f1, smem, i - n);
}

// ---- the tangent's conv part from the per-sample gradient slabs -----------
// The B = M backward already leaves, per sample b, the p-weighted gradient of
// every conv layer as a dW partial slab (slab_b = p_b g_b: conv1 [4 row
// blocks][257][32], conv2 [513][64], conv3 [577][64], bias rows last, rows in
// the parameter layout, each layer's w and b leaves contiguous).  The conv
// ranges of tangent_fwd_kernel compute sum over positions of
// <dz_l, V_l y_{l-1} + vb_l>, which is <v_l, p_b g_l^b>: the same number as the
// dot product of v with those slabs.  So the tangent launch keeps only its fc1
// range (and the fc1-bias / fc2 terms) and the conv layers become 12 dot
// products per sample over 411 KB of slabs (MALL-resident, written one launch
// earlier) instead of a linear conv forward of the meta batch (1.1 GMAC at
// M = 100).  Slots as before: conv1 row block rb -> rb, conv2 / conv3 row
// quarter q -> 4 + q / 8 + q.
struct SlabDotArgs {
  const float* p1;  // [M][4][257][32]
  const float* p2;  // [M][513][64]
  const float* p3;  // [M][577][64]
  const float* v;   // tangent (param layout)
  int64_t off1, off2, off3;  // v offsets of the conv1 / conv2 / conv3 w leaves (b follows w)
  float* part;      // [M][META_DOT_SLOTS]
  int M;
};
constexpr int SLAB_DOT_JOBS = 12;

__device__ __forceinline__ void slab_dot_body(const SlabDotArgs& a, int b, int j, float* s_tmp) {
  constexpr int N1 = (C1KK + 1) * C1CO / 4, N2 = (C2KK + 1) * C2CO / 4, N3 = (C3KK + 1) * C3CO / 4;  // float4s
  const float4* src;
  const float4* vv;
  int n;
  if (j < 4) {
    src = reinterpret_cast<const float4*>(a.p1) + ((int64_t)b * C1_BLOCKS + j) * N1;
    vv = reinterpret_cast<const float4*>(a.v + a.off1);
    n = N1;
  } else if (j < 8) {
    const int q0 = (j - 4) * N2 / 4, q1 = (j - 3) * N2 / 4;
    src = reinterpret_cast<const float4*>(a.p2) + (int64_t)b * N2 + q0;
    vv = reinterpret_cast<const float4*>(a.v + a.off2) + q0;
    n = q1 - q0;
  } else {
    const int q0 = (j - 8) * N3 / 4, q1 = (j - 7) * N3 / 4;
    src = reinterpret_cast<const float4*>(a.p3) + (int64_t)b * N3 + q0;
    vv = reinterpret_cast<const float4*>(a.v + a.off3) + q0;
    n = q1 - q0;
  }
  constexpr int R = (N3 / 4 + 255) / 256;  // 10 float4 pairs per thread at most
  static_assert(N1 <= 256 * R && N2 / 4 + 1 <= 256 * R && N3 / 4 + 1 <= 256 * R, "slab part per block");
  float4 x[R], y[R];
  const int t = threadIdx.x;
#pragma unroll
  for (int r = 0; r < R; ++r) {  // every load in flight before the first product
    const int i = min(t + 256 * r, n - 1);
    x[r] = src[i];
    y[r] = vv[i];
  }
  float d = 0.f;
#pragma unroll
  for (int r = 0; r < R; ++r)
    if (t + 256 * r < n) d += (x[r].x * y[r].x + x[r].y * y[r].y) + (x[r].z * y[r].z + x[r].w * y[r].w);
  d = block_sum256(d, s_tmp);
  if (t == 0) a.part[(int64_t)b * META_DOT_SLOTS + j] = d;
}

// The tangent launch with one meta chunk: [fc1 tiles] [12 slab dots per
// sample], the fc1-bias / fc2 term (slot META_EXTRA_SLOT) by each sample's
// first slab-dot block.  Static LDS (fc1's four 32 x 32 tiles, 16.9 KB):
// every block of the grid is resident at once.
inline int tangent_slab_blocks(int M, int MG) { return fc1_fwd_blocks(1, MG) + SLAB_DOT_JOBS * M; }
__global__ __launch_bounds__(256) void tangent_slab_kernel(SlabDotArgs sd, Fc1FwdArgs f1, MetaExtra ex) {
  __shared__ __attribute__((aligned(16))) float smem[4 * FC1_32RW];
  const int nf = (HID / 32) * FC1_S * f1.MG;  // fc1_fwd_blocks(1, MG)
  int i = blockIdx.x;
  if (i < nf) {
    fc1_fwd_block32<true>(f1, smem, i);
    return;
  }
  i -= nf;
  const int b = i / SLAB_DOT_JOBS, j = i % SLAB_DOT_JOBS;
  slab_dot_body(sd, b, j, smem);
  if (j == 0) {
    __syncthreads();
    meta_extra_term(ex, b, smem);
  }
}

struct MetaRmsArgs {
  float lr, decay, c1, eps;
  int64_t n4;  // total / 4 (float4 granules)
};

// theta' = theta + u(G; mu, nu); keeps mu', nu' and J = du/dG
//   = -lr D^{-3/2} (D - c1 G (G - mu')),  D = nu' - mu'^2 + eps
// (meta batches of more than one chunk: G is complete only after the last).
__global__ __launch_bounds__(256) void meta_rms1_kernel(MetaRmsArgs a, const float4* __restrict__ G,
                                                        const float4* __restrict__ th,
                                                        const float4* __restrict__ mu,
                                                        const float4* __restrict__ nu, float4* __restrict__ thp,
                                                        float4* __restrict__ mu1, float4* __restrict__ nu1,
                                                        float4* __restrict__ J) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.n4) return;
  const float4 g4 = G[i], t4 = th[i], m4 = mu[i], v4 = nu[i];
  float4 o_t, o_m, o_v, o_j;
  auto one = [&](float g, float t, float m0, float v0, float& ot, float& om, float& ov, float& oj) {
    const float m = a.c1 * g + a.decay * m0;
    const float v = a.c1 * (g * g) + a.decay * v0;
    const float d = v - m * m + a.eps;
    const float rs = rsqrtf(d);
    ot = t + (-a.lr) * (g * rs);
    om = m;
    ov = v;
    oj = -a.lr * (d - a.c1 * g * (g - m)) * (rs * rs * rs);
  };
  one(g4.x, t4.x, m4.x, v4.x, o_t.x, o_m.x, o_v.x, o_j.x);
  one(g4.y, t4.y, m4.y, v4.y, o_t.y, o_m.y, o_v.y, o_j.y);
  one(g4.z, t4.z, m4.z, v4.z, o_t.z, o_m.z, o_v.z, o_j.z);
  one(g4.w, t4.w, m4.w, v4.w, o_t.w, o_m.w, o_v.w, o_j.w);
  thp[i] = o_t;
  mu1[i] = o_m;
  nu1[i] = o_v;
  J[i] = o_j;
}

// meta_rms2 (u' = u(g'; mu', nu'), v = dL/dG = -2 u' J, the u'^2 partials)
// runs in the one-transition backward's gradient epilogues (common.hpp
// Rms::meta2), and with one meta chunk so does meta_rms1 (Rms::meta1).

struct MetaDotArgs {
  const float* dy1;  // [M][400][32] p-weighted conv1 pre-activation grads
  const float* dy2;  // [M][81][64]
  const float* dy3;  // [M][3136]
  const float* dz1;  // [M][512]
  const float* gq;   // [M] cotangent at q[a] (= -p clip(td))
  const int32_t* ga; // [M] a_tm1
  const float* zv1;  // [M][400][32] V1 * x + vb1
  const float* zv2;  // [M][81][64]
  const float* zv3;  // [M][3136]
  const float* zvp;  // fc1 split-K partials of V_fc1 y3 [S][M][512]
  int S, M, A;
  const float* v;    // tangent (param layout)
  int64_t b1_off, w2_off, b2_off;
  const float* h1;   // [M][512] online fc1 output (z = 0)
  float* s_out;      // [M]  p_i dL/dp_i
};

// p_i dL/dp_i of sample `b` (256 threads; the block's sum in every thread).
__device__ __forceinline__ float meta_dot_sample(const MetaDotArgs& a, int b) {
  __shared__ float sbuf[4];
  __shared__ float s_fc2[4];
  const int t = threadIdx.x;
  float acc = 0.f;
  {
    const float4* d = reinterpret_cast<const float4*>(a.dy1 + (int64_t)b * C1M * C1CO);
    const float4* z = reinterpret_cast<const float4*>(a.zv1 + (int64_t)b * C1M * C1CO);
    for (int i = t; i < C1M * C1CO / 4; i += 256) {
      const float4 x = d[i], y = z[i];
      acc += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
  }
  {
    const float4* d = reinterpret_cast<const float4*>(a.dy2 + (int64_t)b * C2M * C2CO);
    const float4* z = reinterpret_cast<const float4*>(a.zv2 + (int64_t)b * C2M * C2CO);
    for (int i = t; i < C2M * C2CO / 4; i += 256) {
      const float4 x = d[i], y = z[i];
      acc += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
  }
  {
    const float4* d = reinterpret_cast<const float4*>(a.dy3 + (int64_t)b * FLAT);
    const float4* z = reinterpret_cast<const float4*>(a.zv3 + (int64_t)b * FLAT);
    for (int i = t; i < FLAT / 4; i += 256) {
      const float4 x = d[i], y = z[i];
      acc += x.x * y.x + x.y * y.y + x.z * y.z + x.w * y.w;
    }
  }
  // fc1: dz1 . (vb1 + sum_s partial); fc2: gq . (h1 . V2[:, a] + vb2[a])
  const int act = a.ga[b];
  float f2 = 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int n = t + 256 * h;
    float zf = a.v[a.b1_off + n];
    for (int s = 0; s < a.S; ++s) zf += a.zvp[((int64_t)s * a.M + b) * HID + n];
    acc += a.dz1[(int64_t)b * HID + n] * zf;
    f2 += a.h1[(int64_t)b * HID + n] * a.v[a.w2_off + n * a.A + act];
  }
  f2 = wave_sum(f2);
  if ((t & 63) == 0) s_fc2[t >> 6] = f2;
  __syncthreads();
  if (t == 0) acc += a.gq[b] * (a.v[a.b2_off + act] + ((s_fc2[0] + s_fc2[1]) + (s_fc2[2] + s_fc2[3])));
  acc = wave_sum(acc);
  if ((t & 63) == 0) sbuf[t >> 6] = acc;
  __syncthreads();
  return (sbuf[0] + sbuf[1]) + (sbuf[2] + sbuf[3]);
}

// One block (256 threads) per meta-batch sample.
__global__ __launch_bounds__(256) void meta_dot_kernel(MetaDotArgs a) {
  const float acc = meta_dot_sample(a, blockIdx.x);
  if (threadIdx.x == 0) a.s_out[blockIdx.x] = acc;
}

struct MetaAdamArgs {
  const float* x;   // [M] gathered logits
  const float* p;   // [M]
  const float* s;   // [M] p_i dL/dp_i
  const float* dot_part;  // or null: s_i = sum of the tangent launch's partials [M][META_DOT_SLOTS] (stored to s_out)
  float* s_out;
  int M;
  float* logits;
  const int32_t* pos;
  float *m, *v;
  int32_t* count;
  float lr, b1, b2, eps;
  const float* loss_part;
  int nparts;
  float* loss;
  float* dlogits;   // [M]
  LogitRun* run;    // the logit buffer's running log-sum-exp, or null
  int* dirty;       // its chunk flags (chunk_sums_kernel runs after), with run
  int64_t n_logits; // its capacity
};

// softmax backward + optax.adam (scale_by_adam, bias-corrected; scale(-lr)),
// new logits scattered back.  One block striding over the M entries.  With
// dot_part, s_i is first summed from the tangent launch's partials (fixed
// slot order) and stored; thread i handles entry i in both loops, so it
// reads back its own store.
__device__ __forceinline__ float meta_s(const MetaAdamArgs& a, int i) {
  if (!a.dot_part) return a.s[i];
  const float4* q = reinterpret_cast<const float4*>(a.dot_part + (int64_t)i * META_DOT_SLOTS);
  float4 r[META_DOT_SLOTS / 4];
#pragma unroll
  for (int k = 0; k < META_DOT_SLOTS / 4; ++k) r[k] = q[k];
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < META_DOT_SLOTS / 4; ++k) {
    acc += r[k].x;
    if (4 * k + 1 <= META_EXTRA_SLOT) acc += r[k].y;
    if (4 * k + 2 <= META_EXTRA_SLOT) acc += r[k].z;
    if (4 * k + 3 <= META_EXTRA_SLOT) acc += r[k].w;
    if (4 * k + 4 > META_EXTRA_SLOT) break;
  }
  a.s_out[i] = acc;
  return acc;
}

// Sum of the tangent launch's dot-product partials of one entry (slots
// 0 .. META_EXTRA_SLOT in order), from its row loaded as float4s.
__device__ __forceinline__ float meta_s_row(const float4 (&r)[META_DOT_SLOTS / 4]) {
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < META_DOT_SLOTS / 4; ++k) {
    acc += r[k].x;
    if (4 * k + 1 <= META_EXTRA_SLOT) acc += r[k].y;
    if (4 * k + 2 <= META_EXTRA_SLOT) acc += r[k].z;
    if (4 * k + 3 <= META_EXTRA_SLOT) acc += r[k].w;
    if (4 * k + 4 > META_EXTRA_SLOT) break;
  }
  return acc;
}

// Every global load the block needs for its first META_THREADS entries and
// the first META_ADAM_LP x META_THREADS loss partials is issued before the
// first reduction (the loops over the partials had issued one load per
// dependent iteration); entries and partials past those take the loops.
constexpr int META_ADAM_LP = 16;
__device__ __forceinline__ void meta_adam_body(const MetaAdamArgs& a) {
  __shared__ float sbuf[META_THREADS / 64];
  const int t = threadIdx.x;
  const bool own = t < a.M;
  const int i0 = own ? t : 0;
  float4 dr[META_DOT_SLOTS / 4];
  float s0 = 0.f;
  if (a.dot_part) {
    const float4* q = reinterpret_cast<const float4*>(a.dot_part + (int64_t)i0 * META_DOT_SLOTS);
#pragma unroll
    for (int k = 0; k < META_DOT_SLOTS / 4; ++k) dr[k] = q[k];
  } else {
    s0 = a.s[i0];
  }
  float lpv[META_ADAM_LP];
#pragma unroll
  for (int r = 0; r < META_ADAM_LP; ++r) lpv[r] = a.loss_part[min(t + r * META_THREADS, a.nparts - 1)];
  const float x0 = a.x[i0], p0 = a.p[i0], m0 = a.m[i0], v0 = a.v[i0];
  const int32_t pos0 = a.pos[i0];
  const int32_t cnt = *a.count + 1;
  LogitRun r{0.0, 0.f, 0};
  if (a.run) r = *a.run;
  __builtin_amdgcn_sched_barrier(0);
  if (a.dot_part) {
    s0 = meta_s_row(dr);
    if (own) a.s_out[t] = s0;
  }
  float st = own ? s0 : 0.f;
  for (int i = t + META_THREADS; i < a.M; i += META_THREADS) st += meta_s(a, i);
  const float tot = block_sum_f32(st, sbuf);
  float lp = 0.f;
#pragma unroll
  for (int k = 0; k < META_ADAM_LP; ++k)
    if (t + k * META_THREADS < a.nparts) lp += lpv[k];
  for (int j = t + META_ADAM_LP * META_THREADS; j < a.nparts; j += META_THREADS) lp += a.loss_part[j];
  lp = block_sum_f32(lp, sbuf);
  const float c1 = 1.f - powf(a.b1, (float)cnt), c2 = 1.f - powf(a.b2, (float)cnt);
  __shared__ double dbuf[META_THREADS / 64];
  __shared__ int s_far;
  if (t == 0) s_far = 0;
  __syncthreads();
  double dS = 0.0;  // running-sum change of this thread's writes (positions are distinct)
  auto entry = [&](int i, float si, float xi, float pi, float mi, float vi, int32_t posi) {
    const float g = si - pi * tot;
    const float m = (1.f - a.b1) * g + a.b1 * mi;
    const float v = (1.f - a.b2) * (g * g) + a.b2 * vi;
    const float mh = m / c1;
    const float vh = v / c2;
    a.m[i] = m;
    a.v[i] = v;
    a.dlogits[i] = g;
    const float nx = xi + (-a.lr) * (mh / (sqrtf(vh) + a.eps));
    a.logits[posi] = nx;
    if (r.valid) {
      dS += run_term(nx, r.c) - run_term(xi, r.c);
      if (nx != -INFINITY && (double)nx - (double)r.c >= 80.0) s_far = 1;
      a.dirty[posi / SM_CHUNK] = 1;
    }
  };
  if (own) entry(t, s0, x0, p0, m0, v0, pos0);
  for (int i = t + META_THREADS; i < a.M; i += META_THREADS)
    entry(i, a.dot_part ? a.s_out[i] : a.s[i], a.x[i], a.p[i], a.m[i], a.v[i], a.pos[i]);
  // the buffer's running log-sum-exp follows the M writes (what
  // dqz_logits_write does for them) and their chunks are flagged, so the next
  // add / sample needs no scan; a tripped guard re-seeds here (rare)
  if (a.run && r.valid) {
    __shared__ int s_reseed;
    dS = block_sum_f64(dS, dbuf);  // fixed order: deterministic
    if (t == 0) {
      const double before = r.S;
      r.S += dS;
      s_reseed = s_far || !run_ok(before, r.S, -INFINITY, r.c);
      *a.run = r;
    }
    __syncthreads();
    if (s_reseed) {
      block_rescan(a.logits, a.n_logits, a.run);
      const int nb = (int)((a.n_logits + SM_CHUNK - 1) / SM_CHUNK);
      for (int k = t; k < nb; k += META_THREADS) a.dirty[k] = 1;
    }
  }
  if (t == 0) {
    *a.count = cnt;
    *a.loss = lp;
  }
}

__global__ __launch_bounds__(META_THREADS) void meta_adam_kernel(MetaAdamArgs a) { meta_adam_body(a); }

// ---- meta Adam + the written chunks' sums in one launch -------------------
// (one meta chunk, M <= META_THREADS, a logit buffer whose running state the
// host vouches for).  The separate form ran meta_adam_kernel (one block) and
// then chunk_sums_kernel over the flagged chunks: two launches and a boundary
// for <= M chunk re-sums.  Here the grid is one block per logit chunk; a block
// whose chunk holds none of the M positions exits at once (the leader, the
// block of pos[0]'s chunk, never does).  Every remaining block forms the
// whole Adam step in the same fixed order (so all of them agree on tot, the
// new logits, dS and the re-seed decision bit for bit), stores the logits of
// its own chunk and re-sums that chunk from an LDS copy patched with them;
// the leader alone stores m, v, dlogits, s, the count, the loss and the
// running state.  Dirty flags stay clear: every writer re-sums what it
// writes.  A tripped guard (rare) is handled by the last of the active
// blocks to arrive, after every block's logit stores drained write-through:
// re-scan of the buffer and every chunk sum, with L2-bypassing loads.
//
// The leader's stores overwrite state every active block reads at entry (m,
// v, count, run), and nothing says the grid is resident at once (a large
// buffer has more chunk blocks than the chip holds, or other work holds the
// CUs).  So every active block, once its entry loads have returned, adds its
// number of meta entries to `enter`; the entries partition the M positions,
// so the leader stores only after `enter` reached M.  Only the leader waits,
// and every other block runs to its end without waiting, so the wait always
// ends (bounded anyway: spin_max polls, then bit 0 of `err`).

// An empty asm that the compiler must take as a new definition of x (so no
// later use waits on the load that produced it).
template <class T>
__device__ __forceinline__ void launder_v(T& x) {
  asm volatile("" : "+v"(x));
}

struct MetaAdamChunks {
  double* csum;  // [nblocks]
  int nblocks;
  int* arrive;   // re-seed arrival counter (zero between launches)
  int* enter;    // active blocks' entry loads done, in meta entries (zero between launches)
  int* err;      // bit 0: the leader's wait for `enter` gave up
  unsigned spin_max;
};

__device__ __forceinline__ float rescan_sc1(const float* x, int64_t n, LogitRun* run, double* dbuf, float* fbuf) {
  const int bytes = (int)(n * 4);
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < n; j += SM_THREADS) m = fmaxf(m, load_sc1_f1(x, bytes, (int)j));
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) fbuf[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(fbuf[0], fbuf[1]), fmaxf(fbuf[2], fbuf[3]));
  const float c = m == -INFINITY ? 0.f : m;
  double sum = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += SM_THREADS) sum += run_term(load_sc1_f1(x, bytes, (int)j), c);
  sum = block_sum_f64(sum, dbuf);
  if (threadIdx.x == 0) *run = LogitRun{sum, c, 1};
  __syncthreads();
  return c;
}

__device__ __forceinline__ double chunk_sum_sc1(const float* x, int64_t n, int k, float c, double* s_wave) {
  const int bytes = (int)(n * 4);
  const int64_t base = (int64_t)k * SM_CHUNK + threadIdx.x * SM_PER_LANE;
  float xv[SM_PER_LANE];
  if (base + SM_PER_LANE <= n) {
#pragma unroll
    for (int q = 0; q < SM_PER_LANE / 4; ++q) {
      const float4 f = load_sc1_f4(reinterpret_cast<const float4*>(x), bytes, (int)(base / 4) + q);
      xv[4 * q] = f.x;
      xv[4 * q + 1] = f.y;
      xv[4 * q + 2] = f.z;
      xv[4 * q + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < SM_PER_LANE; ++i) xv[i] = base + i < n ? load_sc1_f1(x, bytes, (int)(base + i)) : -INFINITY;
  }
  double lane = 0.0;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) lane += chunk_term(xv[i], c);
  return block_total_f64(lane, s_wave);
}

__global__ __launch_bounds__(META_THREADS) void meta_adam_chunks_kernel(MetaAdamArgs a, MetaAdamChunks ck) {
  static_assert(META_THREADS == SM_THREADS, "one thread per meta entry and per chunk lane");
  __shared__ float s_chunk[SM_CHUNK];
  __shared__ float sbuf[META_THREADS / 64];
  __shared__ double dbuf[META_THREADS / 64];
  __shared__ int s_act, s_far, s_reseed, s_last, s_mine;
  const int k = blockIdx.x, t = threadIdx.x;
  const bool own = t < a.M;
  const int i0 = own ? t : 0;
  DQZ_STAMP(19, 0);
  // Every load is issued before the block learns whether it is active (the
  // positions are loaded with the rest): one round trip instead of two, for
  // the inactive blocks' wasted loads (L2 hits but for their own chunk)
  int32_t pos0 = a.pos[i0];
  const int32_t posl = a.pos[0];
  // this chunk's logits (before the writes) into LDS, under the Adam loads
  float4 cv[SM_PER_LANE / 4];
  {
    const int64_t base = (int64_t)k * SM_CHUNK + t * SM_PER_LANE;
#pragma unroll
    for (int q = 0; q < SM_PER_LANE / 4; ++q) {
      if (base + 4 * q + 3 < a.n_logits) {
        cv[q] = *reinterpret_cast<const float4*>(a.logits + base + 4 * q);
      } else {
        float e[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) e[u] = base + 4 * q + u < a.n_logits ? a.logits[base + 4 * q + u] : -INFINITY;
        cv[q] = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
  }
  float4 dr[META_DOT_SLOTS / 4];
  {
    const float4* q = reinterpret_cast<const float4*>(a.dot_part + (int64_t)i0 * META_DOT_SLOTS);
#pragma unroll
    for (int u = 0; u < META_DOT_SLOTS / 4; ++u) dr[u] = q[u];
  }
  float lpv[META_ADAM_LP];
#pragma unroll
  for (int r = 0; r < META_ADAM_LP; ++r) lpv[r] = a.loss_part[min(t + r * META_THREADS, a.nparts - 1)];
  float x0 = a.x[i0], p0 = a.p[i0], m0 = a.m[i0], v0 = a.v[i0];
  int32_t cnt = *a.count + 1;
  LogitRun r = *a.run;
  __builtin_amdgcn_sched_barrier(0);
  if (t == 0) {
    s_act = 0;
    s_far = 0;
    s_mine = 0;
  }
  __syncthreads();
  const bool mine = own && pos0 / SM_CHUNK == k;
  if (mine) {
    s_act = 1;
    atomicAdd(&s_mine, 1);  // LDS
  }
  __syncthreads();
  const bool leader = k == posl / SM_CHUNK;
  if (!s_act) return;  // (the leader's chunk holds pos[0])
  // entry loads returned in every wave, then this block's entries arrive
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  DQZ_STAMP(19, 1);
  // The compiler's wait counts know nothing of that s_waitcnt, and the
  // atomic below is issued by one lane only: at the merge after it, a use of
  // the latest load would wait with vmcnt(0), i.e. for the atomic's reply too
  // (a device-scope RMW of one word that every active block hits, microseconds
  // in the trace).  So every loaded value is consumed or passed through an
  // empty asm (which the compiler must take as a new definition) first.
#pragma unroll
  for (int q = 0; q < SM_PER_LANE / 4; ++q) *reinterpret_cast<float4*>(s_chunk + t * SM_PER_LANE + 4 * q) = cv[q];
  float s0 = meta_s_row(dr);
  launder_v(s0);
  launder_v(x0);
  launder_v(p0);
  launder_v(m0);
  launder_v(v0);
  launder_v(cnt);
  launder_v(r.S);
  launder_v(r.c);
  launder_v(r.valid);
  launder_v(pos0);
#pragma unroll
  for (int u = 0; u < META_ADAM_LP; ++u) launder_v(lpv[u]);
  if (t == 0) __hip_atomic_fetch_add(ck.enter, s_mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DQZ_STAMP(13, 0);
  const float tot = block_sum_f32(own ? s0 : 0.f, sbuf);
  DQZ_STAMP(13, 1);
  float lp = 0.f;
  if (leader) {
#pragma unroll
    for (int u = 0; u < META_ADAM_LP; ++u)
      if (t + u * META_THREADS < a.nparts) lp += lpv[u];
    for (int j = t + META_ADAM_LP * META_THREADS; j < a.nparts; j += META_THREADS) lp += a.loss_part[j];
    lp = block_sum_f32(lp, sbuf);
  }
  const float c1 = 1.f - powf(a.b1, (float)cnt), c2 = 1.f - powf(a.b2, (float)cnt);
  double dS = 0.0;
  float nx = 0.f;
  float g = 0.f, m = 0.f, v = 0.f;
  if (own) {  // meta_adam_body's arithmetic, in the same order
    g = s0 - p0 * tot;
    m = (1.f - a.b1) * g + a.b1 * m0;
    v = (1.f - a.b2) * (g * g) + a.b2 * v0;
    const float mh = m / c1;
    const float vh = v / c2;
    nx = x0 + (-a.lr) * (mh / (sqrtf(vh) + a.eps));
  }
  DQZ_STAMP(13, 2);
  if (leader) {
    // the leader's first store of state another block reads at entry: every
    // active block's entries have arrived (the wait sits after this block's
    // own arithmetic, which overlaps it; the later stores of count and run
    // come after this point too)
    if (t == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load(ck.enter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < a.M) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > ck.spin_max) {
          __hip_atomic_fetch_or(ck.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      // every active block has arrived (or the wait gave up): reset for the next launch
      __hip_atomic_store(ck.enter, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (own) {
      a.m[t] = m;
      a.v[t] = v;
      a.dlogits[t] = g;
      a.s_out[t] = s0;
    }
  }
  if (own) {
    if (r.valid) {
      dS = run_term(nx, r.c) - run_term(x0, r.c);
      if (nx != -INFINITY && (double)nx - (double)r.c >= 80.0) s_far = 1;
    }
    if (mine) s_chunk[pos0 - k * SM_CHUNK] = nx;
  }
  if (!r.valid) {  // (the host vouches for the state, so not expected) as meta_adam_body: writes only
    if (mine) a.logits[pos0] = nx;
    if (leader && t == 0) {
      *a.count = cnt;
      *a.loss = lp;
    }
    return;
  }
  DQZ_STAMP(19, 2);
  dS = block_sum_f64(dS, dbuf);  // fixed order: the same in every block (also a barrier for s_chunk / s_far)
  if (t == 0) s_reseed = s_far || !run_ok(r.S, r.S + dS, -INFINITY, r.c);
  __syncthreads();
  DQZ_STAMP(13, 3);
  const bool reseed = s_reseed;
  if (!reseed) {
    if (mine) a.logits[pos0] = nx;
    float xv[SM_PER_LANE];
#pragma unroll
    for (int i = 0; i < SM_PER_LANE; ++i) xv[i] = s_chunk[t * SM_PER_LANE + i];
    double lane = 0.0;
#pragma unroll
    for (int i = 0; i < SM_PER_LANE; ++i) lane += chunk_term(xv[i], r.c);
    DQZ_STAMP(12, 0);
    const double ctot = block_total_f64(lane, dbuf);
    DQZ_STAMP(12, 1);
    if (t == 0) {
      ck.csum[k] = ctot;
      if (leader) {
        r.S += dS;
        *a.run = r;
        *a.count = cnt;
        *a.loss = lp;
      }
    }
    DQZ_STAMP(19, 3);
    return;
  }
  // re-seed (rare): logits out write-through, the last active block re-scans
  if (mine) store_sc1_f1(a.logits, (int)(a.n_logits * 4), (int)pos0, nx);
  if (leader && t == 0) {
    *a.count = cnt;
    *a.loss = lp;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // active blocks: the distinct chunks of pos[0 .. M)
  int first = 0;
  if (own) {
    first = 1;
    for (int j = 0; j < t; ++j)
      if (a.pos[j] / SM_CHUNK == pos0 / SM_CHUNK) first = 0;
  }
  const int nact = (int)block_sum_f32((float)first, sbuf);
  if (t == 0) s_last = __hip_atomic_fetch_add(ck.arrive, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nact - 1;
  __syncthreads();
  if (!s_last) return;
  if (t == 0) __hip_atomic_store(ck.arrive, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const float c = rescan_sc1(a.logits, a.n_logits, a.run, dbuf, sbuf);
  for (int kk = 0; kk < ck.nblocks; ++kk) {
    const double sk = chunk_sum_sc1(a.logits, a.n_logits, kk, c, dbuf);
    if (t == 0) ck.csum[kk] = sk;
  }
}

}  // namespace dqz
