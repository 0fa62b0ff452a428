// head.hpp — fc1 split-K reduce + fc2 + TD loss (one workgroup per sample),
// the optimizer update kernel, and the replay sampler / gather kernels.
#pragma once
#include "common.hpp"

namespace dqz {

struct HeadArgs {
  const float* fc1p;  // fc1 split-K partials [Z][S][B][512]
  int S;
  float* h1;  // [Z][B][512] (written)
  NetZ nz;
  int64_t b1_off, w2_off, b2_off;
  int Z, B, A, algo, shared_bias, fwd_only;
  const int32_t* slots;
  const int32_t* action;
  const float* reward;
  const float* discount;
  const float* weights;  // PER importance weights or null
  // fused PER draw (or null): the B unnormalised importance weights
  // w_b = (up / p_b)^beta conv1 published; normalised here by the batch
  // maximum if per_normalize (importance_sampling_weights,
  // replay.py:344-376), also written to per_w_out
  const double* per_wb;
  int per_normalize;
  float* per_w_out;
  const float* meta_p;   // MGSC meta mode: per-sample probabilities or null
  // MGSC meta mode with the softmax formed here (one meta chunk, M <= 512):
  // p = softmax(logits[pos[0..M)]) (meta_softmax_kernel's quantity), block b
  // writes x_out[b] = logits[pos[b]] and p_out[b]; meta_p is then unused
  const float* meta_logits;
  const int32_t* meta_pos;
  int meta_M;
  float *meta_x_out, *meta_p_out;
  const float4* rec;     // batch records {a, r, d, 0} written by conv1, or null (slot chain)
  uint64_t* advance;     // fused sampler's step counter, advanced once here (or null)
  int unit;              // 1: unit cotangent on q[a] (gradient of q itself; HVP pass)
  float bound;           // grad_error_bound
  float* q;              // [Z][B][A]
  float* td;             // [B]
  float* loss_part;      // [B] per-sample 0.5 td^2 w
  float* gq;             // [B] d loss / d q_tm1[b, a_b]
  int32_t* ga;           // [B] a_b
  float* dz1;            // [B][512] d loss / d fc1 pre-activation (online)
  // actor mode (fwd_only): eps-greedy draw per sample into act_out (or null)
  dqz_action* act_out;
  double eps;
  uint64_t act_seed, act_ctr;
};

// distrax.EpsilonGreedy(q, eps).sample as the host mirror computes it
// (parts.epsilon_greedy_probs + numpy Generator.choice): fp64 probabilities
// (1 - eps) [q_a == max] / #ties + eps / A, cdf = cumsum normalised by its
// last entry, action = first a with cdf[a] > u.
__device__ __forceinline__ dqz_action eps_greedy(const float* q, int A, double eps, double u) {
  float v = q[0];
  for (int a = 1; a < A; ++a) v = fmaxf(v, q[a]);
  int ties = 0;
  for (int a = 0; a < A; ++a) ties += q[a] == v;
  const double greedy = 1.0 / (double)ties, floor = eps / (double)A;
  double total = 0.0;
  for (int a = 0; a < A; ++a) total += (1.0 - eps) * (q[a] == v ? greedy : 0.0) + floor;
  double cum = 0.0;
  int act = A - 1;
  for (int a = 0; a < A; ++a) {
    cum += (1.0 - eps) * (q[a] == v ? greedy : 0.0) + floor;
    if (cum / total > u) {
      act = a;
      break;
    }
  }
  return dqz_action{act, v};
}

// Maximum of a wave's non-negative doubles (the PER importance weights), in
// every lane: the DPP row scan of wave_sum with max (common.hpp dpp_d; lanes
// whose DPP source is outside the row read 0, the identity here), then
// readlane 63.  Max is exact in any order, so the result equals a shuffle
// butterfly's bit for bit.
__device__ __forceinline__ double wave_max_nonneg(double m) {
  m = fmax(m, dpp_d<0x111>(m));
  m = fmax(m, dpp_d<0x112>(m));
  m = fmax(m, dpp_d<0x114>(m));
  m = fmax(m, dpp_d<0x118>(m));
  m = fmax(m, dpp_d<0x142, 0xa>(m));
  m = fmax(m, dpp_d<0x143, 0xc>(m));
  const long long b = __builtin_bit_cast(long long, m);
  const int lo = __builtin_amdgcn_readlane((int)b, 63), hi = __builtin_amdgcn_readlane((int)(b >> 32), 63);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}

// One workgroup (512 threads = hidden units) per sample b:
//   h1 = relu(b1 + sum_s partial), q = h1 @ W2 + b2 for every copy z,
//   TD error (rlax 0.1.2 q_learning / double_q_learning as called at
//   dqn/agent.py:94-106, double_q/agent.py:97-106, prioritized/agent.py:97-113):
//   td = stopgrad(r + d * v) - q_tm1[a]; loss_b = 0.5 td^2 [* w];
//   the cotangent at td is clip(w td / B, +-bound) because rlax.clip_gradient
//   clips the incoming gradient; dq[b, a_b] = -that; dz1 = dq W2[:, a_b] relu'.
// Cross-sample sums (fc2/fc1-bias grads, mean loss) happen in update_kernel.
// ZMAX: network copies this instantiation handles (2: online + target, or
// one copy; 3: double-Q's online(s_t) too), so no load is issued for a copy
// the launch does not have.
// out = false (head_dx1_kernel's blocks past the first): the same arithmetic
// with no global store; s_dzo (or null) receives the block's dz1 row.
template <int AMAX, int SMAX, int ZMAX>
__device__ __forceinline__ void head_body(const HeadArgs& h, int b, bool out = true, float* s_dzo = nullptr) {
  DQZ_STAMP(4, 0);
  __shared__ float s_red[8][3 * AMAX];
  __shared__ float s_q[3][AMAX];
  __shared__ float s_rec[5];  // {a_tm1 bits, r, d, w, p} of sample b
  const int n = threadIdx.x, lane = n & 63, wave = n >> 6;
  const int A = h.A, B = h.B, Z = h.Z, S = h.S;
  // Every global load is issued up front: the batch record chain
  // (slot -> action/reward/discount), the Z x S fc1 partials, fc1 biases,
  // the W2 rows and the fc2 bias; nothing below waits on more than one round
  // trip.  Global stores are deferred to the end: vmcnt counts stores too, so
  // a store issued before a dependent load's wait would be waited for as well.
  int a_tm1 = 0;
  float r = 0.f, d = 0.f, w = 1.f, pm = 0.f;
  const bool chain = !h.fwd_only && h.rec == nullptr;
  const int slot = chain ? h.slots[b] : 0;  // uniform load, in flight with the partials
  float4 rv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (!h.fwd_only && h.rec != nullptr && n == 0) rv = h.rec[b];
  float pv[ZMAX][SMAX], b1v[ZMAX], w2v[ZMAX][AMAX];
#pragma unroll
  for (int z = 0; z < ZMAX; ++z) {
    const int zc = min(z, Z - 1);
    const float* part = h.fc1p + ((int64_t)zc * S * B + b) * HID + n;
#pragma unroll
    for (int s = 0; s < SMAX; ++s) pv[z][s] = part[(int64_t)min(s, S - 1) * B * HID];
    b1v[z] = h.nz.p[zc][h.b1_off + n];
    const float* w2 = h.nz.p[zc] + h.w2_off + n * A;
#pragma unroll
    for (int a = 0; a < AMAX; ++a) w2v[z][a] = w2[min(a, A - 1)];
  }
  // fc2 (q = h1 W2 + b2).  AMAX <= 8: an LDS transpose-reduce — thread n
  // writes its K = Z A products h1[z][n] W2[n][a] to s_p[k = z A + a][n];
  // output k is summed by T adjacent lanes (T = 32 for K <= 16, else 16),
  // 512 / T terms each in a fixed order, then a butterfly over the T lanes:
  // one reduction chain per lane instead of one full-wave chain per output.
  // Larger action sets keep per-output wave sums.
  constexpr bool kTr = AMAX <= 8;
  constexpr int kPS = HID + 16;  // s_p row stride: rows of adjacent 16-lane groups 16 banks apart
  __shared__ float s_p[kTr ? 3 * AMAX : 1][kTr ? kPS : 1];
  const int K = Z * A, lgT = K <= 16 ? 5 : 4, T = 1 << lgT;
  const int kk = n >> lgT, jj = n & (T - 1);
  const bool qthread = kTr ? (kk < K && jj == 0) : (n < 3 * AMAX && n / AMAX < Z && n % AMAX < A);
  const int zq = kTr ? min(kk / A, 2) : n / AMAX, aq = kTr ? kk % A : n % AMAX;  // output of this q thread
  // fc2 bias of output (zq, aq): the bias of every copy is loaded (each
  // through the copy's uniform parameter pointer) and the lane's one selected
  // by value; indexing nz.p by the lane's copy would load the pointer per
  // lane, and that load's wait would also wait for every load issued above
  float b2v = 0.f;
  {
    const int a2 = h.shared_bias ? 0 : min(aq, A - 1);
    float b2z[ZMAX];
#pragma unroll
    for (int z = 0; z < ZMAX; ++z) b2z[z] = h.nz.p[min(z, Z - 1)][h.b2_off + a2];
    const int zc = min(zq, Z - 1);
#pragma unroll
    for (int z = 0; z < ZMAX; ++z) b2v = zc == z ? b2z[z] : b2v;
  }
  float wper = 1.f;
  if (h.per_wb && wave == 0) {  // the batch's IS weights (the fused PER draw)
    double m = 0.0;
    for (int j = lane; j < B; j += 64) m = fmax(m, h.per_wb[j]);
    m = wave_max_nonneg(m);
    if (lane == 0) {
      const double wb = h.per_wb[b];
      wper = (float)(h.per_normalize ? wb / m : wb);
      if (out && h.per_w_out) h.per_w_out[b] = wper;
    }
  }
  if (h.meta_logits) {
    // one thread per meta-batch logit: thread n holds pos[n], and the block
    // of sample b writes x_out[b] / p_out[b] through thread n == b, so the
    // meta batch must fit the block (launch_meta keeps M <= MAXB with one
    // chunk).  This path sums in another order than meta_softmax_kernel (the
    // K > 1 chunks): p agrees with it within f32 rounding, not bit for bit.
    static_assert(MAXB <= HID, "the head's one-chunk meta softmax needs M <= the block's threads");
    // p = exp(x - (c + log sum exp(x - c))), c = max x, over the M meta-batch
    // logits (replay_circular.py:79-86 as meta_softmax_kernel forms it; the
    // block reductions run in a fixed order)
    __shared__ float s_mx[8], s_se[8], s_pm;
    const float x = n < h.meta_M ? h.meta_logits[h.meta_pos[n]] : -INFINITY;
    float m = x;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) s_mx[wave] = m;
    __syncthreads();
    float c = s_mx[0];
#pragma unroll
    for (int w8 = 1; w8 < 8; ++w8) c = fmaxf(c, s_mx[w8]);
    const float e = wave_sum(n < h.meta_M ? expf(x - c) : 0.f);
    if (lane == 0) s_se[wave] = e;
    __syncthreads();
    const float se = ((s_se[0] + s_se[1]) + (s_se[2] + s_se[3])) + ((s_se[4] + s_se[5]) + (s_se[6] + s_se[7]));
    if (n == b) {
      const float pb = expf(x - (c + logf(se)));
      s_pm = pb;
      if (out) {
        h.meta_x_out[b] = x;
        h.meta_p_out[b] = pb;
      }
    }
    __syncthreads();
    pm = s_pm;
  }
  if (!h.fwd_only && n == 0) {  // second hop of the batch record chain, needed only for the TD
    if (chain) {
      a_tm1 = h.action[slot];
      r = h.reward[slot];
      d = h.discount[slot];
    } else {
      a_tm1 = __float_as_int(rv.x);
      r = rv.y;
      d = rv.z;
    }
    if (h.weights) w = h.weights[b];
    if (h.per_wb) w = wper;
    if (h.meta_p && !h.meta_logits) pm = h.meta_p[b];
    // broadcast for the TD below, which every thread forms (no extra barrier)
    s_rec[0] = __int_as_float(a_tm1);
    s_rec[1] = r;
    s_rec[2] = d;
    s_rec[3] = w;
    s_rec[4] = pm;
  }
  DQZ_STAMP(4, 1);
  float hz[ZMAX];
#pragma unroll
  for (int z = 0; z < ZMAX; ++z) hz[z] = 0.f;
#pragma unroll
  for (int z = 0; z < ZMAX; ++z) {
    if (z < Z) {
      float acc = b1v[z];
#pragma unroll
      for (int s = 0; s < SMAX; ++s) acc += s < S ? pv[z][s] : 0.f;
      hz[z] = relu(acc);
      if (z == 0) DQZ_STAMP(15, 0);  // fc1 partials of copy 0 have landed
      if constexpr (kTr) {
#pragma unroll
        for (int a = 0; a < AMAX; ++a)
          if (a < A) s_p[z * A + a][n] = hz[z] * w2v[z][a];
      } else {
#pragma unroll
        for (int a = 0; a < AMAX; ++a) {
          const float sa = wave_sum(hz[z] * w2v[z][a]);
          if (lane == 0) s_red[wave][z * AMAX + a] = sa;
        }
      }
    }
  }
  DQZ_STAMP(15, 1);  // products / wave sums done
  __syncthreads();
  float qv = 0.f;
  if constexpr (kTr) {
    if (kk < K) {  // every lane of output kk's group
      const float* row = &s_p[kk][jj];
      float a4[4] = {0.f, 0.f, 0.f, 0.f};
      for (int i = 0; i < (HID >> lgT); i += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) a4[u] += row[(i + u) << lgT];
      }
      float v = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      // butterfly over the T lanes: DPP within 16-lane rows (quad xor 1,
      // xor 2, half-row and row mirrors), one ds_bpermute across rows for T = 32
      v += dpp_f<0xB1>(v);
      v += dpp_f<0x4E>(v);
      v += dpp_f<0x141>(v);
      v += dpp_f<0x140>(v);
      if (T == 32) v += __shfl_xor(v, 16, 64);
      qv = v + b2v;
      if (jj == 0) s_q[zq][aq] = qv;
    }
  } else if (qthread) {
    float sa = 0.f;
#pragma unroll
    for (int ww = 0; ww < 8; ++ww) sa += s_red[ww][n];
    qv = sa + b2v;
    s_q[zq][aq] = qv;
  }
  if (!h.fwd_only) {
    __syncthreads();
    DQZ_STAMP(15, 2);  // q values in LDS
    {
      // every thread forms the TD error and its cotangent from the same LDS
      // values with the same operations (same bits in every thread), so the
      // dz1 row below needs no second barrier; thread 0 stores the outputs
      a_tm1 = __float_as_int(s_rec[0]);
      r = s_rec[1];
      d = s_rec[2];
      w = s_rec[3];
      pm = s_rec[4];
      float q0[AMAX], q1[AMAX], q2[AMAX];  // every LDS read issued before the first use
#pragma unroll
      for (int a = 0; a < AMAX; ++a) {
        q0[a] = s_q[0][min(a, A - 1)];
        q1[a] = s_q[1][min(a, A - 1)];
        q2[a] = s_q[min(2, Z - 1)][min(a, A - 1)];
      }
      float v, qa = q0[0];
#pragma unroll
      for (int a = 1; a < AMAX; ++a) qa = a == a_tm1 ? q0[a] : qa;
      if (h.algo == DQZ_ALGO_DQN) {
        v = q1[0];
#pragma unroll
        for (int a = 1; a < AMAX; ++a) v = fmaxf(v, q1[a]);  // entries past A repeat q1[A - 1]
      } else {
        int am = 0;  // online Q(s_t) selects, jnp.argmax: first maximum
        float best = q2[0];
#pragma unroll
        for (int a = 1; a < AMAX; ++a)
          if (a < A && q2[a] > best) {
            best = q2[a];
            am = a;
          }
        v = q1[0];
#pragma unroll
        for (int a = 1; a < AMAX; ++a) v = a == am ? q1[a] : v;
      }
      const float td = __fmaf_rn(d, v, r) - qa;  // explicit fma: the same bits in every kernel using head_body
      float g;
      if (h.unit) {
        g = -1.f;  // gq = d q[a] / d q[a] = 1
      } else if (h.meta_p || h.meta_logits) {
        // meta mode: p_b * grad of loss_fn on the single transition b
        // (dqn_mgsc_batched/agent.py:152-158): batch of one, clip, then weight.
        g = pm * fminf(fmaxf(td, -h.bound), h.bound);
      } else {
        g = w * td / (float)B;  // d mean(l2(td) * w) / d td
        g = fminf(fmaxf(g, -h.bound), h.bound);
      }
      if (out && n == 0) {
        h.td[b] = td;
        h.loss_part[b] = 0.5f * td * td * w;
        h.gq[b] = -g;
        h.ga[b] = a_tm1;
      }
      float wv = w2v[0][0];
#pragma unroll
      for (int a = 1; a < AMAX; ++a) wv = a == a_tm1 ? w2v[0][a] : wv;
      DQZ_STAMP(4, 2);
      const float dz = hz[0] > 0.f ? -g * wv : 0.f;
      if (s_dzo) s_dzo[n] = dz;
      if (out) h.dz1[(int64_t)b * HID + n] = dz;
    }
  } else if (h.act_out) {  // actor: eps-greedy draw b of call act_ctr
    __syncthreads();
    if (out && n == 0) {
      const uint4 r = philox4x32(make_uint4((unsigned)h.act_ctr, (unsigned)(h.act_ctr >> 32), (unsigned)b, 0xAC7u),
                                 make_uint2((unsigned)h.act_seed, (unsigned)(h.act_seed >> 32)));
      const double u = ((((uint64_t)r.x << 32) | r.y) >> 11) * 0x1.0p-53;
      h.act_out[b] = eps_greedy(s_q[0], A, h.eps, u);
    }
  }
  // deferred outputs: fc1 activations (fc2 dW in the update kernel), q values
  if (!out) return;
#pragma unroll
  for (int z = 0; z < ZMAX; ++z)
    if (z < Z) h.h1[((int64_t)z * B + b) * HID + n] = hz[z];
  if (qthread) h.q[((int64_t)zq * B + b) * A + aq] = qv;
  // the fused sampler's step counter: every conv1 block of this step has read it
  if (h.advance && b == 0 && n == 0)
    __hip_atomic_fetch_add(h.advance, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  DQZ_STAMP(4, 3);
}

template <int AMAX, int SMAX, int ZMAX>
__global__ __launch_bounds__(512) void head_kernel(HeadArgs h) {
  head_body<AMAX, SMAX, ZMAX>(h, blockIdx.x);
}

#ifdef DQZ_STEP_TU  // (the launchers instantiate the step's kernels: its TU only)
// Head launch: AMAX 8 covers Pong-style minimal action sets, 32 the rest.
template <int SMAX, int ZMAX>
inline void launch_head_z(const HeadArgs& h, int grid, hipStream_t st) {
  if (h.A <= 8)
    hipLaunchKernelGGL((head_kernel<8, SMAX, ZMAX>), dim3(grid), dim3(HID), 0, st, h);
  else
    hipLaunchKernelGGL((head_kernel<MAXA, SMAX, ZMAX>), dim3(grid), dim3(HID), 0, st, h);
}

inline hipError_t launch_head(const HeadArgs& h, int grid, hipStream_t st) {
  if (h.S > 7 || h.Z < 1 || h.Z > 3) return hipErrorInvalidValue;
  if (h.Z <= 2) {
    launch_head_z<7, 2>(h, grid, st);
  } else {
    launch_head_z<7, 3>(h, grid, st);
  }
  return hipGetLastError();
}
#endif  // DQZ_STEP_TU

struct UpdArgs {
  float *th, *mu, *nu;
  int64_t off[10];
  int64_t sz[10];
  const float* p1;  // conv1 dW partials [S1][257][32]
  const float* p2;  // conv2 dW partials [S2][513][64]
  const float* p3;  // conv3 dW partials [S3][577][64]
  int S1, S2, S3;
  const float* h1;   // [B][512] online fc1 output (z = 0)
  const float* dz1;  // [B][512]
  const float* gq;   // [B]
  const int32_t* ga; // [B]
  const float* loss_part;
  float* loss;
  int* status;  // learner health word: bit 1 set when the batch loss is not finite
  int A, B, nb2;
  Rms rms;
};

constexpr int UPD_PAIRS = 32;                  // parameter pairs per workgroup (64 parameters)
constexpr int UPD_PARAMS = 2 * UPD_PAIRS;
constexpr int UPD_GROUPS = 8;                  // threads sharing one pair's reduction

// Sum of the float2 p[s * stride + j .. +1] over s = g, g + G, ... < S, eight
// loads in flight per iteration (the slabs are written by the previous
// kernel, so every load is a cache miss; one dependent chain per slab would
// be latency-bound).
__device__ __forceinline__ float2 sum_split2(const float* p, int S, int64_t stride, int64_t j, int g) {
  constexpr int G = UPD_GROUPS;
  float2 a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = make_float2(0.f, 0.f);
  int s = g;
  for (; s + 7 * G < S; s += 8 * G) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const float2 v = *reinterpret_cast<const float2*>(p + (int64_t)(s + u * G) * stride + j);
      a[u].x += v.x;
      a[u].y += v.y;
    }
  }
  // the tail without branches: each load is unconditional (clamped to the
  // last slab) and its sum selected, so all eight are in flight together (a
  // conditional load per branch waited for each one in turn)
  float2 v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = *reinterpret_cast<const float2*>(p + (int64_t)min(s + u * G, S - 1) * stride + j);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int u = 0; u < 8; ++u)
    if (s + u * G < S) {
      a[u].x += v[u].x;
      a[u].y += v[u].y;
    }
  return make_float2(((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x)),
                     ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y)));
}

// The same sum with every load issued before the first addition, for S <=
// 8 R G slabs: R rounds of eight clamped loads, summed in sum_split2's order
// (a[u] over the rounds, then the fixed tree), so the bits are the same.  The
// loop form above issues one round of eight loads per dependent step and a
// ninth round for its tail (conv1's 4 B = 128 slabs took three serial round
// trips at B = 32; conv2 / conv3's 32 slabs one).
template <int R>
__device__ __forceinline__ float2 sum_split2_r(const float* p, int S, int64_t stride, int64_t j, int g) {
  constexpr int G = UPD_GROUPS;
  float2 v[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < 8; ++u)
      v[r][u] = *reinterpret_cast<const float2*>(p + (int64_t)min(g + (8 * r + u) * G, S - 1) * stride + j);
  __builtin_amdgcn_sched_barrier(0);
  float2 a[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = make_float2(0.f, 0.f);
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (g + (8 * r + u) * G < S) {
        a[u].x += v[r][u].x;
        a[u].y += v[r][u].y;
      }
  return make_float2(((a[0].x + a[1].x) + (a[2].x + a[3].x)) + ((a[4].x + a[5].x) + (a[6].x + a[7].x)),
                     ((a[0].y + a[1].y) + (a[2].y + a[3].y)) + ((a[4].y + a[5].y) + (a[6].y + a[7].y)));
}
// (Wider forms, up to 56 loads per lane for the M = 100 meta batch's 400
// conv1 slabs, cost that kernel 0.5 us: 162 VGPRs left its 1,276 blocks no
// longer all resident; profiles/r05/c7.)
__device__ __forceinline__ float2 sum_slabs(const float* p, int S, int64_t stride, int64_t j, int g) {
  if (S <= 8 * UPD_GROUPS) return sum_split2_r<1>(p, S, stride, j, g);
  if (S <= 16 * UPD_GROUPS) return sum_split2_r<2>(p, S, stride, j, g);
  return sum_split2(p, S, stride, j, g);
}

// One gradient element of the small head leaves (fc1/b, fc2/w, fc2/b): this
// thread's share (samples grp, grp + G, ...) and its destination offset.
// Eight samples' operands are loaded per round (unconditional, clamped to the
// last sample) before any is summed, so they are in flight together; the
// sum keeps the sample order.
__device__ __forceinline__ float small_grad(const UpdArgs& u, int64_t e, int grp, int64_t& dst) {
  constexpr int G = UPD_GROUPS, R = 8;
  float g = 0.f;
  if (e < HID) {  // fc1 bias: sum_b dz1
    const int j = (int)e;
    for (int b0 = grp; b0 < u.B; b0 += R * G) {
      float x[R];
#pragma unroll
      for (int r = 0; r < R; ++r) x[r] = u.dz1[(int64_t)min(b0 + r * G, u.B - 1) * HID + j];
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (b0 + r * G < u.B) g += x[r];
    }
    dst = u.off[7] + j;
  } else if (e < HID + (int64_t)HID * u.A) {  // fc2 w[j][a] = sum_{b: a_b = a} h1[b][j] gq[b]
    const int64_t jj = e - HID;
    const int j = (int)(jj / u.A), a = (int)(jj % u.A);
    for (int b0 = grp; b0 < u.B; b0 += R * G) {
      float h[R], q[R];
      int32_t act[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int b = min(b0 + r * G, u.B - 1);
        h[r] = u.h1[(int64_t)b * HID + j];
        q[r] = u.gq[b];
        act[r] = u.ga[b];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (b0 + r * G < u.B) {
          const float v = h[r] * q[r];
          g += act[r] == a ? v : 0.f;
        }
    }
    dst = u.off[8] + jj;
  } else if (e < HID + (int64_t)HID * u.A + u.nb2) {  // fc2 b
    const int a = (int)(e - HID - (int64_t)HID * u.A);
    for (int b0 = grp; b0 < u.B; b0 += R * G) {
      float q[R];
      int32_t act[R];
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const int b = min(b0 + r * G, u.B - 1);
        q[r] = u.gq[b];
        act[r] = u.ga[b];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (b0 + r * G < u.B) g += (u.nb2 == 1 || act[r] == a) ? q[r] : 0.f;
    }
    dst = u.off[9] + a;
  }
  return g;
}

// Reduces every gradient that crosses samples or split-K chunks and applies
// centered RMSProp to every leaf except fc1/w (fused into its dW epilogue).
// 256 threads = 32 parameter pairs x 8 reduction groups, combined through
// LDS.  Grid: the small head leaves first (their blocks run the longest
// per-sample loops), then conv1, conv2, conv3 (float2 partial loads).  The
// RMSProp operands are loaded at entry, under the reduction's latency.
__device__ __forceinline__ void update_body(const UpdArgs& u, float2 (*s_part)[UPD_PAIRS], int blk) {
  DQZ_STAMP(9, 0);
  const int pl = threadIdx.x % UPD_PAIRS, grp = threadIdx.x / UPD_PAIRS;
  const int64_t nsmall = HID + (int64_t)HID * u.A + u.nb2;
  const int small_blocks = (int)((nsmall + UPD_PARAMS - 1) / UPD_PARAMS);
  const int64_t c1 = u.sz[0] + u.sz[1], c2 = c1 + u.sz[2] + u.sz[3], c3 = c2 + u.sz[4] + u.sz[5];
  // block 0 wave 0: the batch loss partials (unconditional clamped loads,
  // summed below in sample order; a guarded loop waited for them here)
  constexpr int LR = (MAXB + 63) / 64;
  float lv[LR];
  if (blk == 0 && threadIdx.x < 64) {
#pragma unroll
    for (int r = 0; r < LR; ++r) lv[r] = u.loss_part[min((int)threadIdx.x + 64 * r, u.B - 1)];
  }
  // destination offsets first (no loads), then the RMSProp / meta operands
  // of grp 0, then the partial sums: the operands are in flight under the
  // reduction's loads instead of a round trip after them
  int64_t dst[2] = {-1, -1};
  const bool small = (int)blk < small_blocks;
  const int64_t e = small ? (int64_t)blk * UPD_PARAMS + 2 * pl
                          : (int64_t)(blk - small_blocks) * UPD_PARAMS + 2 * pl;  // even; regions are even-sized
  if (small) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t f = e + h;
      if (f < HID)
        dst[h] = u.off[7] + f;
      else if (f < HID + (int64_t)HID * u.A)
        dst[h] = u.off[8] + (f - HID);
      else if (f < nsmall)
        dst[h] = u.off[9] + (f - HID - (int64_t)HID * u.A);
    }
  } else if (e < c1) {  // conv1: w rows 0..255, bias row 256
    for (int h = 0; h < 2; ++h) dst[h] = e + h < u.sz[0] ? u.off[0] + e + h : u.off[1] + (e + h - u.sz[0]);
  } else if (e < c2) {
    const int64_t k = e - c1;
    for (int h = 0; h < 2; ++h) dst[h] = k + h < u.sz[2] ? u.off[2] + k + h : u.off[3] + (k + h - u.sz[2]);
  } else if (e < c3) {
    const int64_t k = e - c2;
    for (int h = 0; h < 2; ++h) dst[h] = k + h < u.sz[4] ? u.off[4] + k + h : u.off[5] + (k + h - u.sz[4]);
  }
  const Rms& R = u.rms;
  float o_th[2] = {0.f, 0.f}, o_mu[2] = {0.f, 0.f}, o_nu[2] = {0.f, 0.f};
  if (grp == 0 && (R.gout == nullptr || R.meta != 0)) {
    // the epilogue's operands: theta, mu, nu (RMSProp, meta_rms1), J, mu1, nu1
    // (meta_rms2) or G, mu1, nu1 (meta 3)
    const float* pt = R.meta == 2 ? R.J : R.meta == 3 ? R.G2 : u.th;
    const float* pm = R.meta >= 2 ? R.mu1 : u.mu;
    const float* pn = R.meta >= 2 ? R.nu1 : u.nu;
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (dst[h] >= 0) {
        o_th[h] = pt[dst[h]];
        o_mu[h] = pm[dst[h]];
        o_nu[h] = pn[dst[h]];
      }
  }
  float2 g = make_float2(0.f, 0.f);
  int64_t unused;
  if (small) {
    g.x = small_grad(u, e, grp, unused);
    g.y = small_grad(u, e + 1, grp, unused);
  } else if (e < c1) {
    g = sum_slabs(u.p1, u.S1, (int64_t)(C1KK + 1) * C1CO, e, grp);
  } else if (e < c2) {
    g = sum_slabs(u.p2, u.S2, (int64_t)(C2KK + 1) * C2CO, e - c1, grp);
  } else if (e < c3) {
    g = sum_slabs(u.p3, u.S3, (int64_t)(C3KK + 1) * C3CO, e - c2, grp);
  }
  s_part[grp][pl] = g;
  if (blk == 0 && threadIdx.x < 64) {
    float loss = 0.f;
#pragma unroll
    for (int r = 0; r < LR; ++r)
      if ((int)threadIdx.x + 64 * r < u.B) loss += lv[r];
    loss = wave_sum(loss);
    if (threadIdx.x == 0) {
      u.loss[0] = loss / (float)u.B;
      // NaN / inf guard: reported by dqz_learner_sync_status (bit 1)
      if (u.status && !isfinite(loss)) __hip_atomic_fetch_or(u.status, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  float sq = 0.f, s1 = 0.f;  // meta_rms2 / meta 3: this thread's u'^2 (and grad q . w)
  const float clip = R.meta == 3 ? fminf(fmaxf(R.td[0], -R.bound), R.bound) : 0.f;
  if (grp == 0) {
    float2 gs = make_float2(0.f, 0.f);
#pragma unroll
    for (int gi = 0; gi < UPD_GROUPS; ++gi) {
      gs.x += s_part[gi][pl].x;
      gs.y += s_part[gi][pl].y;
    }
    const float gv[2] = {gs.x, gs.y};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (dst[h] < 0) continue;
      const int64_t i = dst[h];
      if (R.meta == 1) {
        float t = o_th[h], m = o_mu[h], v = o_nu[h];
        const float j = R.meta1(gv[h], t, m, v);
        R.thp[i] = t;
        R.mu1[i] = m;
        R.nu1[i] = v;
        R.J[i] = j;
        if (R.gout) R.gout[i] = gv[h];
      } else if (R.meta == 2) {
        R.vout[i] = R.meta2(gv[h], o_mu[h], o_nu[h], o_th[h], sq);
      } else if (R.meta == 3) {
        float m = o_mu[h], v = o_nu[h];
        R.meta3(gv[h], o_th[h], m, v, clip, sq, s1);
        R.gout[i] = gv[h];
        R.mu1[i] = m;
        R.nu1[i] = v;
      } else if (R.gout) {
        R.gout[i] = R.gacc ? R.gout[i] + gv[h] : gv[h];
      } else {
        float t = o_th[h], m = o_mu[h], v = o_nu[h];
        R.step(gv[h], t, m, v);
        u.mu[i] = m;
        u.nu[i] = v;
        u.th[i] = t;
      }
    }
  }
  if (R.meta >= 2 && threadIdx.x < 64) {  // grp 0 is the first half of wave 0
    sq = wave_sum(sq);
    if (threadIdx.x == 0) R.sq_part[R.sq_off + blk] = sq;
    if (R.meta == 3) {
      s1 = wave_sum(s1);
      if (threadIdx.x == 0) R.s1_part[R.sq_off + blk] = s1;
    }
  }
  DQZ_STAMP(9, 3);
}

inline unsigned update_blocks(const int64_t sz[10], int A, int nb2) {
  const int64_t nconv = sz[0] + sz[1] + sz[2] + sz[3] + sz[4] + sz[5];
  const int64_t nsmall = HID + (int64_t)HID * A + nb2;
  return (unsigned)((nsmall + UPD_PARAMS - 1) / UPD_PARAMS + (nconv + UPD_PARAMS - 1) / UPD_PARAMS);
}

DQZ_STEP_KERNEL __launch_bounds__(256) void update_kernel(UpdArgs u) {
  __shared__ float2 s_part[UPD_GROUPS][UPD_PAIRS];
  update_body(u, s_part, blockIdx.x);
}

DQZ_OTHER_KERNEL void sample_uniform_kernel(int64_t base, int64_t size, int64_t capacity, int n, uint64_t seed,
                                      uint64_t* counter, int32_t* out) {
  DQZ_STAMP(10, 0);
  const uint64_t ctr = *counter;
  const UniformDraw d{base, size, capacity, seed, counter, out};
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = uniform_slot(ctr, i, d);
  __syncthreads();
  if (threadIdx.x == 0) *counter = ctr + 1;
  DQZ_STAMP(10, 3);
}

DQZ_OTHER_KERNEL void gather_stacks_kernel(const uint8_t* frames, const int32_t* fidx, const int32_t* slots, int n,
                                     int which, uint8_t* out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)n * FB) return;
  const int b = (int)(i / FB), p = (int)(i % FB);
  const int slot = slots[b];
  unsigned c[4];
#pragma unroll
  for (int ci = 0; ci < 4; ++ci) {
    const int f = fidx[(int64_t)slot * 8 + which * 4 + ci];
    c[ci] = f < 0 ? 0u : frames[(int64_t)f * FB + p];
  }
  reinterpret_cast<uchar4*>(out)[i] = make_uchar4(c[0], c[1], c[2], c[3]);
}

// One replay add (dqz_store_put): block i < t.num_frames copies new frame i
// (441 x 16 B) into its pool row; block 0 also writes the transition record.
// `frames` may be pinned host memory (read over the fabric).
DQZ_OTHER_KERNEL __launch_bounds__(256) void store_put_kernel(uint8_t* pool, int32_t* fidx, int32_t* action, float* reward,
                                                        float* discount, dqz_transition_put t,
                                                        const uint8_t* frames) {
  constexpr int Q = FB / 16;  // 441
  const int f = blockIdx.x;
  if (f < t.num_frames) {
    const uint4* src = reinterpret_cast<const uint4*>(frames + (int64_t)f * FB);
    uint4* dst = reinterpret_cast<uint4*>(pool + (int64_t)t.frame_rows[f] * FB);
    uint4 v[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) v[k] = src[min((int)threadIdx.x + 256 * k, Q - 1)];
#pragma unroll
    for (int k = 0; k < 2; ++k)
      if ((int)threadIdx.x + 256 * k < Q) dst[threadIdx.x + 256 * k] = v[k];
  }
  if (f == 0) {
    if (threadIdx.x < 8) fidx[t.slot * 8 + threadIdx.x] = t.fidx[threadIdx.x];
    if (threadIdx.x == 8) action[t.slot] = t.action;
    if (threadIdx.x == 9) reward[t.slot] = t.reward;
    if (threadIdx.x == 10) discount[t.slot] = t.discount;
  }
}

}  // namespace dqz
