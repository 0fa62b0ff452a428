// sampling.hpp — device replay samplers.
//
//  * learned-logit buffers (replay_circular.py:148-248, 500-565): f32 logits
//    in HBM (-inf = empty slot).  log-sum-exp is a two-pass online (max, sum)
//    reduction; softmax sampling forms p = exp(x - lse) in f32 exactly as the
//    reference's probabilities_from_logits, then the float64 CDF that
//    numpy's Generator.choice builds (cumsum, normalise, searchsorted right).
//  * prioritized replay (replay.py:379-559): the fp64 implicit sum tree in
//    HBM, same node layout as the host SumTree; set recomputes every touched
//    ancestor as left + right, so device and host sums are bit-identical.
#pragma once
#include "common.hpp"

namespace dqz {

constexpr int SM_THREADS = 256;
constexpr int SM_CHUNK = 4096;  // logits per block in the reduction / CDF passes

struct MaxSum {
  float m, s;  // running max and sum of exp(x - m)
};

__device__ __forceinline__ MaxSum ms_combine(MaxSum a, MaxSum b) {
  if (a.m == -INFINITY) return b;
  if (b.m == -INFINITY) return a;
  const float m = fmaxf(a.m, b.m);
  return MaxSum{m, a.s * expf(a.m - m) + b.s * expf(b.m - m)};
}

__device__ __forceinline__ MaxSum block_reduce_ms(MaxSum v, MaxSum* sbuf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = ms_combine(v, MaxSum{__shfl_xor(v.m, o, 64), __shfl_xor(v.s, o, 64)});
  if (lane == 0) sbuf[wave] = v;
  __syncthreads();
  MaxSum r = sbuf[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = ms_combine(r, sbuf[w]);
  __syncthreads();
  return r;
}

__device__ __forceinline__ double block_sum_f64(double v, double* sbuf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (lane == 0) sbuf[wave] = v;
  __syncthreads();
  double r = sbuf[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r += sbuf[w];
  __syncthreads();
  return r;
}

// Pass 1: per-block (max, sum exp) of logits[n].
__global__ __launch_bounds__(SM_THREADS) void lse_partial_kernel(const float* __restrict__ x, int64_t n,
                                                                 MaxSum* __restrict__ part) {
  __shared__ MaxSum sbuf[SM_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SM_CHUNK;
  MaxSum acc{-INFINITY, 0.f};
  for (int i = threadIdx.x; i < SM_CHUNK; i += SM_THREADS) {
    const int64_t j = base + i;
    if (j < n) {
      const float v = x[j];
      if (v != -INFINITY) acc = ms_combine(acc, MaxSum{v, 1.f});
    }
  }
  acc = block_reduce_ms(acc, sbuf);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// Pass 2 (one block): lse = m + log(s); optional logit write of a new item:
// logits[write_pos] = size == 0 ? 0 : lse - log(size)   (log-mean-exp).
__global__ __launch_bounds__(SM_THREADS) void lse_final_kernel(const MaxSum* __restrict__ part, int nparts,
                                                               float* lse_out, float* logits, int64_t write_pos,
                                                               int64_t size) {
  __shared__ MaxSum sbuf[SM_THREADS / 64];
  MaxSum acc{-INFINITY, 0.f};
  for (int i = threadIdx.x; i < nparts; i += SM_THREADS) acc = ms_combine(acc, part[i]);
  acc = block_reduce_ms(acc, sbuf);
  if (threadIdx.x == 0) {
    const float lse = acc.m == -INFINITY ? -INFINITY : acc.m + logf(acc.s);
    if (lse_out) *lse_out = lse;
    if (logits && write_pos >= 0) logits[write_pos] = size == 0 ? 0.f : lse - logf((float)size);
  }
}

// Sets logits[pos] = -inf before a log-mean-exp (MGSCReservoirDistribution.replace).
__global__ void logit_clear_kernel(float* logits, int64_t pos) {
  if (threadIdx.x == 0) logits[pos] = -INFINITY;
}

// Uniform doubles in [0, 1) from Philox (53-bit mantissa), counter advanced on device.
__global__ void philox_uniform_kernel(uint64_t seed, uint64_t* counter, int n, double* out) {
  const uint64_t ctr = *counter;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const uint4 r = philox4x32(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), (unsigned)i, 0x50F7u),
                               make_uint2((unsigned)seed, (unsigned)(seed >> 32)));
    out[i] = ((((uint64_t)r.x << 32) | r.y) >> 11) * 0x1.0p-53;
  }
  __syncthreads();
  if (threadIdx.x == 0) *counter = ctr + 1;
}

// Per-block float64 sums of p = exp(x - lse) (f32 p, widened like numpy's choice).
__global__ __launch_bounds__(SM_THREADS) void prob_block_sum_kernel(const float* __restrict__ x, int64_t n,
                                                                    const float* __restrict__ lse,
                                                                    double* __restrict__ bsum) {
  __shared__ double sbuf[SM_THREADS / 64];
  const float L = *lse;
  const int64_t base = (int64_t)blockIdx.x * SM_CHUNK;
  double acc = 0.0;
  for (int i = threadIdx.x; i < SM_CHUNK; i += SM_THREADS) {
    const int64_t j = base + i;
    if (j < n) acc += (double)expf(x[j] - L);
  }
  acc = block_sum_f64(acc, sbuf);
  if (threadIdx.x == 0) bsum[blockIdx.x] = acc;
}

// One block per query u: find the chunk whose normalised cumulative sum
// first exceeds u (block sums scanned by one lane), then inside the chunk a
// 256-way parallel prefix (16 logits per lane) and a 16-step scan by the lane
// that holds the crossing.  Returns the first index with cdf > u
// (searchsorted side='right'); cdf = cumsum(float64(p)) / total.
constexpr int SM_PER_LANE = SM_CHUNK / SM_THREADS;  // 16

__global__ __launch_bounds__(SM_THREADS) void softmax_choice_kernel(const float* __restrict__ x, int64_t n,
                                                                    const float* __restrict__ lse,
                                                                    const double* __restrict__ bsum, int nblocks,
                                                                    const double* __restrict__ uniforms,
                                                                    int64_t* __restrict__ out) {
  __shared__ double s_scan[SM_THREADS];
  __shared__ double s_tot, s_before;
  __shared__ int s_blk;
  __shared__ int64_t s_idx;
  const float L = *lse;
  const double u = uniforms[blockIdx.x];
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int b = 0; b < nblocks; ++b) tot += bsum[b];
    double run = 0.0;
    int blk = nblocks - 1;
    for (int b = 0; b < nblocks; ++b) {
      if ((run + bsum[b]) / tot > u) {
        blk = b;
        break;
      }
      run += bsum[b];
    }
    s_tot = tot;
    s_blk = blk;
    s_before = run;
    s_idx = -1;
  }
  __syncthreads();
  const int64_t base = (int64_t)s_blk * SM_CHUNK + threadIdx.x * SM_PER_LANE;
  double p[SM_PER_LANE];
  double mine = 0.0;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) {
    p[i] = base + i < n ? (double)expf(x[base + i] - L) : 0.0;
    mine += p[i];
  }
  s_scan[threadIdx.x] = mine;
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive prefix over the 256 lane sums
    double run = s_before;
    for (int t = 0; t < SM_THREADS; ++t) {
      const double v = s_scan[t];
      s_scan[t] = run;
      run += v;
    }
  }
  __syncthreads();
  const double tot = s_tot;
  double run = s_scan[threadIdx.x];
  const double next = threadIdx.x + 1 < SM_THREADS ? s_scan[threadIdx.x + 1] : run + mine;
  if (run / tot <= u && next / tot > u) {
    for (int i = 0; i < SM_PER_LANE; ++i) {
      run += p[i];
      if (run / tot > u) {
        s_idx = base + i;
        break;
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t idx = s_idx;
    if (idx < 0) {  // rounding at the chunk edge: last live slot of the chunk
      const int64_t end = min(n, (int64_t)(s_blk + 1) * SM_CHUNK);
      for (int64_t j = end - 1; j >= (int64_t)s_blk * SM_CHUNK; --j)
        if (x[j] != -INFINITY) {
          idx = j;
          break;
        }
    }
    out[blockIdx.x] = idx;
  }
}

// ---------------------------------------------------------------------------
// fp64 sum tree (storage[1] = root; node i -> 2i, 2i+1; leaves from `cap`)

__device__ __forceinline__ double load_fresh(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Single workgroup: write n leaves, then recompute their ancestors level by
// level (duplicate parents write identical values).
__global__ __launch_bounds__(1024) void sumtree_set_kernel(double* tree, int64_t cap, int levels,
                                                           const int64_t* idx, const double* vals, int n) {
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    __hip_atomic_store(&tree[cap + idx[i]], vals[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  for (int l = 1; l <= levels; ++l) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      const int64_t node = (cap + idx[i]) >> l;
      const double v = load_fresh(&tree[2 * node]) + load_fresh(&tree[2 * node + 1]);
      __hip_atomic_store(&tree[node], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
}

// Descent of SumTree._query_single for each target; -1 when out of range.
__global__ void sumtree_query_kernel(const double* __restrict__ tree, int64_t cap, const double* __restrict__ targets,
                                     int n, int64_t* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double t = targets[i];
  if (!(t >= 0.0 && t < tree[1])) {
    out[i] = -1;
    return;
  }
  int64_t node = 1;
  while (node < cap) {
    const double left = tree[2 * node];
    if (t < left) {
      node = 2 * node;
    } else {
      t -= left;
      node = 2 * node + 1;
    }
  }
  out[i] = node - cap;
}

// PrioritizedDistribution.sample + importance_sampling_weights with device
// Philox streams (replay.py:680-716, 344-376).  Tree index == replay slot.
// One block; n <= 1024.
__global__ __launch_bounds__(1024) void per_sample_kernel(const double* __restrict__ tree, int64_t cap,
                                                          int64_t live_base, int64_t size, int64_t capacity, int n,
                                                          double usp, double beta, int normalize, uint64_t seed,
                                                          uint64_t* counter, int32_t* out_slots,
                                                          float* out_weights, double* out_probs) {
  __shared__ double s_w[1024];
  const uint64_t ctr = *counter;
  const int i = threadIdx.x;
  double w = 0.0;
  if (i < n) {
    const uint4 r = philox4x32(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), (unsigned)i, 0x9E12u),
                               make_uint2((unsigned)seed, (unsigned)(seed >> 32)));
    const double u_target = ((((uint64_t)r.x << 32) | r.y) >> 11) * 0x1.0p-53;
    const double u_mix = (double)(r.z >> 8) * 0x1.0p-24;
    const int64_t uni = (live_base + (int64_t)((double)(r.w) * 0x1.0p-32 * (double)size)) % capacity;
    const double root = tree[1];
    int64_t slot = uni;
    if (root > 0.0 && !(u_mix < usp)) {
      double t = u_target * root;
      int64_t node = 1;
      while (node < cap) {
        const double left = tree[2 * node];
        if (t < left) {
          node = 2 * node;
        } else {
          t -= left;
          node = 2 * node + 1;
        }
      }
      slot = node - cap;
    }
    const double leaf = tree[cap + slot];
    const double up = 1.0 / (double)size;
    const double pp = root > 0.0 ? leaf / root : up;
    const double prob = (1.0 - usp) * pp + usp * up;
    w = pow(up / prob, beta);
    out_slots[i] = (int32_t)slot;
    if (out_probs) out_probs[i] = prob;
  }
  s_w[i] = w;
  __syncthreads();
  if (i < n) {
    double m = 0.0;
    if (normalize)
      for (int j = 0; j < n; ++j) m = fmax(m, s_w[j]);
    out_weights[i] = (float)(normalize ? w / m : w);
  }
  __syncthreads();
  if (i == 0) *counter = ctr + 1;
}

}  // namespace dqz
