// sampling.hpp — device replay samplers.
//
//  * learned-logit buffers (replay_circular.py:148-248, 500-565): f32 logits
//    in HBM (-inf = empty slot).  The log-sum-exp (the default logit of an
//    add) is a running float64 sum about a fixed shift c, seeded by a
//    two-pass (max, sum) scan.  A draw is numpy's choice (float64 CDF,
//    normalised by its last entry, searchsorted right) over the terms
//    expf(x - c): softmax(logits) up to f32 rounding of the exponent, as the
//    reference's probabilities_from_logits is.  Per-chunk sums of those terms
//    are kept at write time, so a draw reads one chunk, not the buffer.
//  * prioritized replay (replay.py:379-559): the fp64 implicit sum tree in
//    HBM, same node layout as the host SumTree; set recomputes every touched
//    ancestor as left + right, so device and host sums are bit-identical.
#pragma once
#include "common.hpp"

namespace dqz {

constexpr int SM_THREADS = 256;

__device__ __forceinline__ double load_fresh(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
constexpr int SM_CHUNK = 4096;  // logits per block in the reduction / CDF passes

__device__ __forceinline__ double run_term(float x, float c) { return x == -INFINITY ? 0.0 : exp((double)x - (double)c); }

struct MaxSum {
  float m;   // running max
  double s;  // float64 sum of exp(x - m) (the seed of the running state)
};

__device__ __forceinline__ MaxSum ms_combine(MaxSum a, MaxSum b) {
  if (a.m == -INFINITY) return b;
  if (b.m == -INFINITY) return a;
  const float m = fmaxf(a.m, b.m);
  return MaxSum{m, a.s * exp((double)a.m - (double)m) + b.s * exp((double)b.m - (double)m)};
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

// Pass 1: per-block (max, sum exp) of logits[n].  Each lane holds 16 logits
// (float4 loads), takes their max, then sums exp(x - max): one expf per logit.
// clear_pos (>= 0): that slot is set to -inf first (the reservoir replace)
// by the block that owns it, which is the only block that reads it.
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void lse_partial_kernel(float* __restrict__ x, int64_t n,
                                                                 MaxSum* __restrict__ part, int64_t clear_pos) {
  __shared__ MaxSum sbuf[SM_THREADS / 64];
  const int64_t base = (int64_t)blockIdx.x * SM_CHUNK;
  float v[SM_CHUNK / SM_THREADS];
#pragma unroll
  for (int q = 0; q < SM_CHUNK / SM_THREADS / 4; ++q) {
    const int64_t j = base + 4 * (threadIdx.x + SM_THREADS * q);
    float4 f = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
    if (j + 3 < n && (reinterpret_cast<uintptr_t>(x + j) & 15) == 0) {
      f = *reinterpret_cast<const float4*>(x + j);
    } else {
      if (j < n) f.x = x[j];
      if (j + 1 < n) f.y = x[j + 1];
      if (j + 2 < n) f.z = x[j + 2];
      if (j + 3 < n) f.w = x[j + 3];
    }
    if (clear_pos >= j && clear_pos < j + 4) {
      const int e = (int)(clear_pos - j);
      if (e == 0) f.x = -INFINITY;
      if (e == 1) f.y = -INFINITY;
      if (e == 2) f.z = -INFINITY;
      if (e == 3) f.w = -INFINITY;
      x[clear_pos] = -INFINITY;
    }
    v[4 * q] = f.x;
    v[4 * q + 1] = f.y;
    v[4 * q + 2] = f.z;
    v[4 * q + 3] = f.w;
  }
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < SM_CHUNK / SM_THREADS; ++i) m = fmaxf(m, v[i]);
  double sum = 0.0;
  if (m != -INFINITY) {
#pragma unroll
    for (int i = 0; i < SM_CHUNK / SM_THREADS; ++i) sum += run_term(v[i], m);
  }
  const MaxSum acc = block_reduce_ms(MaxSum{m, sum}, sbuf);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// (max, sum) of all block partials, every lane combining a strided subset in
// a fixed order: any block that calls it gets the same bits.
__device__ __forceinline__ MaxSum combine_parts(const MaxSum* __restrict__ part, int nparts, MaxSum* sbuf) {
  MaxSum acc{-INFINITY, 0.f};
  for (int i = threadIdx.x; i < nparts; i += SM_THREADS) acc = ms_combine(acc, part[i]);
  return block_reduce_ms(acc, sbuf);
}

// Running log-sum-exp of a logit buffer: S = sum_i exp(x_i - c) in float64
// about a fixed shift c, kept up to date by every write that goes through
// the library (the add / reservoir replace / popleft / explicit writes of
// replay_circular.py:166-190, 209-215, 526-545), so an add costs O(1)
// instead of a scan of the whole buffer.  A full scan re-seeds it (c = max,
// S from the scan) whenever the host-side owner cannot vouch for it (logits
// handed out for writing, e.g. to the meta-update; set_state), every
// kLogitReseed running adds (bounds the drift), and on the device when a
// removal would cancel most of S or an item lands far above c (the writer
// re-seeds in its own block before it returns, so a sampler always finds a
// valid state and chunk sums about its c).
struct LogitRun {
  double S;
  float c;
  int valid;
};

// The f32 log-sum-exp of a running state: c + log(S) in float64, rounded once.
__device__ __forceinline__ float run_lse(const LogitRun& r) {
  return r.S > 0.0 ? (float)((double)r.c + log(r.S)) : -INFINITY;
}

// The reference's default logit (replay_circular.py:171-176): the float32
// logsumexp minus np.log(size) in float64, stored back as float32.
__device__ __forceinline__ float logmeanexp_item(float lse, int64_t size) {
  return size == 0 ? 0.f : (float)((double)lse - log((double)size));
}


// Pass 2 (one block): lse = m + log(s); optional logit write of a new item:
// logits[write_pos] = size == 0 ? 0 : lse - log(size) (log-mean-exp); seeds
// the running state `run` (may be null) from the scan.
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void lse_final_kernel(const MaxSum* __restrict__ part, int nparts,
                                                               float* lse_out, float* logits, int64_t write_pos,
                                                               int64_t size, LogitRun* run) {
  __shared__ MaxSum sbuf[SM_THREADS / 64];
  const MaxSum acc = combine_parts(part, nparts, sbuf);
  if (threadIdx.x == 0) {
    // the f32 lse every sampler and add uses: c + log(S) of the running state
    const float lse = acc.m == -INFINITY ? -INFINITY : (float)((double)acc.m + log(acc.s));
    if (lse_out) *lse_out = lse;
    float item = -INFINITY;
    if (logits && write_pos >= 0) {
      item = logmeanexp_item(lse, size);
      logits[write_pos] = item;
    }
    if (run) {
      LogitRun r{acc.m == -INFINITY ? 0.0 : acc.s, acc.m == -INFINITY ? 0.f : acc.m, 1};
      r.S += run_term(item, r.c);  // the slot was -inf during the scan
      *run = r;
    }
  }
}

// Scan of one double per thread over the block in a fixed order
// (deterministic run to run): a Hillis-Steele scan inside each wave by
// shuffles, then each wave adds the totals of the waves before it, summed in
// wave order.  Returns the exclusive prefix; *tot gets the block total with
// exactly the bits the last lane's inclusive prefix has.  Two barriers; a
// caller that does not reuse s_wave afterwards may drop the second (TAIL).
template <bool TAIL = true>
__device__ __forceinline__ double block_scan_excl_f64(double v, double* s_wave, double* tot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double up = __shfl_up(incl, o, 64);
    if (lane >= o) incl += up;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  double pre = 0.0, all = 0.0;
  constexpr int W = SM_THREADS / 64;
#pragma unroll
  for (int w = 0; w < W - 1; ++w) {
    if (w < wave) pre += s_wave[w];
    all += s_wave[w];
  }
  const double last_incl = s_wave[W - 1] + all;  // the last lane's incl + pre, same operands
  double excl = __shfl_up(incl, 1, 64);
  excl = lane == 0 ? 0.0 : excl;
  excl = wave == 0 ? excl : (lane == 0 ? pre : excl + pre);
  *tot = last_incl;
  if constexpr (TAIL) __syncthreads();
  return excl;
}

// block_scan_excl_f64's *tot alone, with the same bits: each wave's total by
// the DPP fold (wave_fold63_f64: VALU moves where the scan's shuffles are
// ds_bpermute round trips), then the same wave-order combine.  All threads
// of the block (full waves).
__device__ __forceinline__ double block_total_f64(double v, double* s_wave) {
  v = wave_fold63_f64(v);
  if ((threadIdx.x & 63) == 63) s_wave[threadIdx.x >> 6] = v;
  __syncthreads();
  constexpr int W = SM_THREADS / 64;
  double all = 0.0;
#pragma unroll
  for (int w = 0; w < W - 1; ++w) all += s_wave[w];
  const double r = s_wave[W - 1] + all;
  __syncthreads();
  return r;
}

// ---------------------------------------------------------------------------
// Chunk sums of the sampling terms, kept at write time.
//
// A draw's distribution is softmax(logits) formed as terms t_i = expf(x_i - c)
// (f32, widened to float64; 0 for an empty slot) about the running state's
// shift c, and the float64 CDF over them.  The buffer keeps one float64 sum
// per chunk of SM_CHUNK logits: csum[k] = chunk_sum(k) — lane t sums its 16
// consecutive terms in index order, then block_scan_excl_f64's fixed-order
// total (block_total_f64) — a pure function of (logits, c).  Every write recomputes the chunks
// it touched (the add / put kernels in their own block; the explicit writes
// and the meta-update through dirty flags and chunk_sums_kernel), and a
// re-seed (new c) recomputes all of them.  A draw is then a two-level search
// (csum prefix -> chunk, chunk terms -> slot) whose second level re-forms
// exactly the terms csum[k] was summed from: no pass over the buffer per draw,
// where the reference forms the softmax of every slot for every sample
// (replay_circular.py:205-217, 540-545).
constexpr int SM_PER_LANE = SM_CHUNK / SM_THREADS;  // 16

__device__ __forceinline__ double chunk_term(float x, float c) { return x == -INFINITY ? 0.0 : (double)expf(x - c); }

// Lane t's 16 consecutive logits of chunk k (-inf past n): four float4 loads.
__device__ __forceinline__ void load_chunk_lane(const float* __restrict__ x, int64_t n, int k,
                                                float (&xv)[SM_PER_LANE]) {
  const int64_t base = (int64_t)k * SM_CHUNK + threadIdx.x * SM_PER_LANE;
  if (base + SM_PER_LANE <= n && (reinterpret_cast<uintptr_t>(x) & 15) == 0) {
#pragma unroll
    for (int q = 0; q < SM_PER_LANE / 4; ++q) {
      const float4 f = *reinterpret_cast<const float4*>(x + base + 4 * q);
      xv[4 * q] = f.x;
      xv[4 * q + 1] = f.y;
      xv[4 * q + 2] = f.z;
      xv[4 * q + 3] = f.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < SM_PER_LANE; ++i) xv[i] = base + i < n ? x[base + i] : -INFINITY;
  }
}

// The canonical sum of chunk k's terms (all 256 threads; every thread gets it).
__device__ __forceinline__ double chunk_sum(const float* __restrict__ x, int64_t n, int k, float c, double* s_wave) {
  float xv[SM_PER_LANE];
  load_chunk_lane(x, n, k, xv);
  double lane = 0.0;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) lane += chunk_term(xv[i], c);
  return block_total_f64(lane, s_wave);
}

// One block per chunk: csum[k] = chunk_sum(k) about the running state's c;
// with `dirty`, only the chunks flagged by a writer (flags cleared).
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void chunk_sums_kernel(const float* __restrict__ x, int64_t n,
                                                                const LogitRun* run, double* __restrict__ csum,
                                                                int* __restrict__ dirty) {
  __shared__ double s_wave[SM_THREADS / 64];
  const int k = blockIdx.x;
  if (dirty && dirty[k] == 0) return;
  const double s = chunk_sum(x, n, k, run->c, s_wave);
  if (threadIdx.x == 0) {
    csum[k] = s;
    if (dirty) dirty[k] = 0;
  }
}

// Re-seed of the running state by one block (a guard tripped inside a
// single-block writer; rare): c = max, S = float64 sum of exp(x - c).
// Returns c to every thread.
__device__ __forceinline__ float block_rescan(const float* __restrict__ x, int64_t n, LogitRun* run) {
  __shared__ float fbuf[SM_THREADS / 64];
  __shared__ double dbuf[SM_THREADS / 64];
  float m = -INFINITY;
  for (int64_t j = threadIdx.x; j < n; j += SM_THREADS) m = fmaxf(m, x[j]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) fbuf[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(fbuf[0], fbuf[1]), fmaxf(fbuf[2], fbuf[3]));
  const float c = m == -INFINITY ? 0.f : m;
  double sum = 0.0;
  for (int64_t j = threadIdx.x; j < n; j += SM_THREADS) sum += run_term(x[j], c);
  sum = block_sum_f64(sum, dbuf);
  if (threadIdx.x == 0) *run = LogitRun{sum, c, 1};
  __syncthreads();
  return c;
}

// Every chunk in turn, by one block (after block_rescan).
__device__ __forceinline__ void block_all_chunk_sums(const float* __restrict__ x, int64_t n, float c,
                                                     double* __restrict__ csum) {
  __shared__ double s_wave[SM_THREADS / 64];
  const int nb = (int)((n + SM_CHUNK - 1) / SM_CHUNK);
  for (int k = 0; k < nb; ++k) {
    const double s = chunk_sum(x, n, k, c, s_wave);
    if (threadIdx.x == 0) csum[k] = s;
  }
}

// Guard of a running update: S must stay well conditioned (no removal that
// cancels most of it) and terms within exp's range about c (the f32 sampling
// terms included: expf(80) is finite).
__device__ __forceinline__ bool run_ok(double s_before, double s_after, float x, float c) {
  return s_after >= 1e-6 * s_before && s_after > 0.0 && (x == -INFINITY || (double)x - (double)c < 80.0);
}

// add / reservoir replace with the running state (one block), then the chunk
// sums of the (at most two) chunks it wrote.  A tripped guard re-seeds the
// state and every chunk sum in this block (rare).
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void logits_add_running_kernel(float* __restrict__ x, int64_t n,
                                                                        LogitRun* run, double* __restrict__ csum,
                                                                        int64_t clear_pos, int64_t write_pos,
                                                                        int64_t size, float* lse_out) {
  __shared__ int s_valid;
  __shared__ float s_c;
  __shared__ double s_wave[SM_THREADS / 64];
  if (threadIdx.x == 0) {
    LogitRun r = *run;
    if (r.valid && clear_pos >= 0) {
      const double before = r.S;
      r.S -= run_term(x[clear_pos], r.c);
      if (!run_ok(before, r.S, -INFINITY, r.c) && r.S != 0.0) r.valid = 0;
    }
    if (clear_pos >= 0) x[clear_pos] = -INFINITY;
    s_valid = r.valid;
    *run = r;
  }
  __syncthreads();
  bool all = false;
  if (!s_valid) {
    block_rescan(x, n, run);
    all = true;
  }
  if (threadIdx.x == 0) {
    LogitRun r = *run;
    const float lse = run_lse(r);
    if (lse_out) *lse_out = lse;
    if (write_pos >= 0) {
      const float item = logmeanexp_item(lse, size);
      const double before = r.S;
      r.S += run_term(item, r.c) - run_term(x[write_pos], r.c);
      x[write_pos] = item;
      if (!run_ok(before, r.S, item, r.c)) r.valid = 0;
    }
    *run = r;
    s_valid = r.valid;
    s_c = r.c;
  }
  __syncthreads();
  if (!s_valid) {
    s_c = 0.f;  // every thread has read s_valid; block_rescan's barrier orders this store
    const float c = block_rescan(x, n, run);
    block_all_chunk_sums(x, n, c, csum);
    return;
  }
  const float c = s_c;
  if (all) {
    block_all_chunk_sums(x, n, c, csum);
    return;
  }
  const int kw = write_pos >= 0 ? (int)(write_pos / SM_CHUNK) : -1;
  const int kc = clear_pos >= 0 ? (int)(clear_pos / SM_CHUNK) : -1;
  if (kc >= 0 && kc != kw) {
    const double s = chunk_sum(x, n, kc, c, s_wave);
    if (threadIdx.x == 0) csum[kc] = s;
  }
  if (kw >= 0) {
    const double s = chunk_sum(x, n, kw, c, s_wave);
    if (threadIdx.x == 0) csum[kw] = s;
  }
}

// One write x[pos] = v passed by value (popleft's -inf), keeping the running
// state and the chunk sum (one block).
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void logits_put1_kernel(float* __restrict__ x, int64_t n, LogitRun* run,
                                                                 double* __restrict__ csum, int64_t pos, float v) {
  __shared__ int s_valid;
  __shared__ float s_c;
  __shared__ double s_wave[SM_THREADS / 64];
  if (threadIdx.x == 0) {
    LogitRun r = *run;
    if (r.valid) {
      const double before = r.S;
      r.S += run_term(v, r.c) - run_term(x[pos], r.c);
      if (!run_ok(before, r.S, v, r.c)) r.valid = 0;
    }
    x[pos] = v;
    *run = r;
    s_valid = r.valid;
    s_c = r.c;
  }
  __syncthreads();
  if (!s_valid) {
    const float c = block_rescan(x, n, run);
    block_all_chunk_sums(x, n, c, csum);
    return;
  }
  const int k = (int)(pos / SM_CHUNK);
  const double s = chunk_sum(x, n, k, s_c, s_wave);
  if (threadIdx.x == 0) csum[k] = s;
}

// Explicit writes x[pos[i]] = val[i] in order (a repeated slot keeps its last
// value, as numpy fancy assignment does), keeping the running state; the
// written chunks are flagged for chunk_sums_kernel (all of them after a
// re-seed).
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void logits_write_kernel(float* __restrict__ x, int64_t n, LogitRun* run,
                                                                  int* __restrict__ dirty,
                                                                  const int64_t* __restrict__ pos,
                                                                  const float* __restrict__ val, int m) {
  __shared__ int s_valid;
  if (threadIdx.x == 0) {
    LogitRun r = *run;
    for (int i = 0; i < m; ++i) {
      const int64_t j = pos[i];
      const float v = val[i];
      if (r.valid) {
        const double before = r.S;
        r.S += run_term(v, r.c) - run_term(x[j], r.c);
        if (!run_ok(before, r.S, v, r.c)) r.valid = 0;
      }
      x[j] = v;
      dirty[j / SM_CHUNK] = 1;
    }
    *run = r;
    s_valid = r.valid;
  }
  __syncthreads();
  if (!s_valid) {
    block_rescan(x, n, run);
    const int nb = (int)((n + SM_CHUNK - 1) / SM_CHUNK);
    for (int k = threadIdx.x; k < nb; k += SM_THREADS) dirty[k] = 1;
  }
}

// Plain writes while the host cannot vouch for the running state (the next
// use re-seeds it and every chunk sum).
DQZ_OTHER_KERNEL void logits_scatter_kernel(float* __restrict__ x, const int64_t* __restrict__ pos,
                                      const float* __restrict__ val, int m) {
  if (threadIdx.x == 0)
    for (int i = 0; i < m; ++i) x[pos[i]] = val[i];  // in order: a repeated slot keeps its last value
}

DQZ_OTHER_KERNEL void logits_scatter1_kernel(float* __restrict__ x, int64_t pos, float v) {
  if (threadIdx.x == 0) x[pos] = v;
}

// Uniform double in [0, 1) of draw q at Philox step ctr (53-bit mantissa):
// the dqz_uniform_philox stream.
__device__ __forceinline__ double philox_uniform(uint64_t seed, uint64_t ctr, int q) {
  const uint4 r = philox4x32(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), (unsigned)q, 0x50F7u),
                             make_uint2((unsigned)seed, (unsigned)(seed >> 32)));
  return ((((uint64_t)r.x << 32) | r.y) >> 11) * 0x1.0p-53;
}

// Uniform doubles in [0, 1) from Philox, counter advanced on device.
DQZ_OTHER_KERNEL void philox_uniform_kernel(uint64_t seed, uint64_t* counter, int n, double* out) {
  const uint64_t ctr = *counter;
  for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = philox_uniform(seed, ctr, i);
  __syncthreads();
  if (threadIdx.x == 0) *counter = ctr + 1;
}

// Level 1 of a draw over the chunk sums, by one wave: lane l sums
// csum[l seg, (l + 1) seg) in order (seg = ceil(nblocks / 64): 4 at 1M
// logits), an inclusive Hillis-Steele scan over the 64 lanes by shuffles
// gives each lane's exclusive prefix and the total (the draw's normaliser;
// the diagnostics form it the same way).  No LDS and no barrier.  A lane's
// first CS_SEG sums stay in registers (constant indices: no scratch), the
// rest (beyond 2M logits) are re-read.
constexpr int CS_SEG = 8;

struct CsumLevel1 {
  int blk;        // the chunk the query's u falls in
  double before;  // the normalised-cumsum mass before it
  double tot;     // total of all chunk sums
  double u;       // the query
};

// Wave-uniform result on every lane of the calling wave (a whole wave).  The
// query u comes from `uf`, called after the chunk sums' loads are issued, so
// u's own loads (the step counter, a caller's uniform) are in flight with
// them instead of ahead of them.
template <class UF>
__device__ __forceinline__ CsumLevel1 csum_level1(const double* __restrict__ csum, int nblocks, UF uf) {
  const int l = threadIdx.x & 63;
  const int seg = (nblocks + 63) / 64;
  const int b0 = min(l * seg, nblocks), b1 = min(b0 + seg, nblocks);
  double mb[CS_SEG];
#pragma unroll
  for (int j = 0; j < CS_SEG; ++j) mb[j] = csum[min(b0 + j, nblocks - 1)];
  const double u = uf();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < CS_SEG; ++j) mb[j] = b0 + j < b1 ? mb[j] : 0.0;
  double mine = 0.0;
#pragma unroll
  for (int j = 0; j < CS_SEG; ++j)
    if (b0 + j < b1) mine += mb[j];
  for (int b = b0 + CS_SEG; b < b1; ++b) mine += csum[b];
  double incl = mine;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double up = __shfl_up(incl, o, 64);
    if (l >= o) incl += up;
  }
  const double tot = __shfl(incl, 63, 64);
  double excl = __shfl_up(incl, 1, 64);
  excl = l == 0 ? 0.0 : excl;
  // this lane's first crossing chunk and the mass before it
  double acc = excl, before = 0.0, before_last = excl;
  int hit = -1;
#pragma unroll
  for (int j = 0; j < CS_SEG; ++j) {
    if (b0 + j < b1) {
      const double v = mb[j];
      if (b0 + j == nblocks - 1) before_last = acc;
      if (hit < 0 && (acc + v) / tot > u) {
        hit = b0 + j;
        before = acc;
      }
      acc += v;
    }
  }
  for (int b = b0 + CS_SEG; b < b1; ++b) {
    const double v = csum[b];
    if (b == nblocks - 1) before_last = acc;
    if (hit < 0 && (acc + v) / tot > u) {
      hit = b;
      before = acc;
    }
    acc += v;
  }
  const unsigned long long m = __ballot(hit >= 0);
  CsumLevel1 r;
  r.tot = tot;
  r.u = u;
  if (m) {  // the lowest crossing lane holds the earliest chunk
    const int src = __ffsll((long long)m) - 1;
    r.blk = __shfl(hit, src, 64);
    r.before = __shfl(before, src, 64);
  } else {  // rounding at the top: the last chunk (as numpy's searchsorted clamps)
    const int src = (nblocks - 1) / seg;
    r.blk = nblocks - 1;
    r.before = __shfl(before_last, src, 64);
  }
  return r;
}

// One query u: the first slot whose normalised cumulative term sum exceeds u
// (searchsorted side='right' on cumsum(t) / total, as numpy's choice does on
// its p).  Level 1 (wave 0, csum_level1) finds the chunk, level 2 (all 256
// lanes) the lane (16 terms each) and the slot from the chunk's re-formed
// terms, whose scan total is csum[chunk].  At most one lane sees the
// crossing, so it stores the slot directly.
// TF: the term of a logit (chunk_term about the running state's c, or the
// exact mode's np_expf(x - lse)); csum holds the chunk sums of the same terms.
template <class TF, class UF>
__device__ __forceinline__ int64_t softmax_choice_terms(const float* __restrict__ x, int64_t n, TF term,
                                                        const double* __restrict__ csum, int nblocks, UF uf) {
  __shared__ double s_wave[SM_THREADS / 64];
  __shared__ double s_before, s_tot;
  __shared__ int s_blk;
  __shared__ int64_t s_idx;
  const int t = threadIdx.x;
  __shared__ double s_u;
  if (t < 64) {
    const CsumLevel1 r = csum_level1(csum, nblocks, uf);
    if (t == 0) {
      s_blk = r.blk;
      s_before = r.before;
      s_tot = r.tot;
      s_idx = -1;
      s_u = r.u;
    }
  }
  __syncthreads();
  const int blk = s_blk;
  const double tot = s_tot, before = s_before, u = s_u;
  float xv[SM_PER_LANE];
  load_chunk_lane(x, n, blk, xv);
  double p[SM_PER_LANE];
  double lane = 0.0;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) {
    p[i] = term(xv[i]);
    lane += p[i];
  }
  double tot2;  // (s_wave is not used again in this call: no trailing barrier)
  const double lexcl = block_scan_excl_f64<false>(lane, s_wave, &tot2);
  const int64_t base = (int64_t)blk * SM_CHUNK + t * SM_PER_LANE;
  double acc = before + lexcl;
  if (acc / tot <= u && (acc + lane) / tot > u) {
    int hit2 = -1;
#pragma unroll
    for (int i = 0; i < SM_PER_LANE; ++i) {  // constant indices: p stays in registers
      if (hit2 < 0) {
        acc += p[i];
        if (acc / tot > u) hit2 = i;
      }
    }
    if (hit2 >= 0) s_idx = base + hit2;
  }
  __syncthreads();
  int64_t idx = s_idx;
  if (idx < 0) {  // rounding at the chunk edge: the last live slot of the chunk (block-uniform)
    if (t == 0) {
      const int64_t end = min(n, (int64_t)(blk + 1) * SM_CHUNK);
      for (int64_t j = end - 1; j >= (int64_t)blk * SM_CHUNK; --j)
        if (x[j] != -INFINITY) {
          idx = j;
          break;
        }
      s_idx = idx;
    }
    __syncthreads();
    idx = s_idx;
  }
  return idx;
}

template <class UF>
__device__ __forceinline__ int64_t softmax_choice_body(const float* __restrict__ x, int64_t n, const LogitRun* run,
                                                       const double* __restrict__ csum, int nblocks, UF uf) {
  const float c = run->c;
  return softmax_choice_terms(x, n, [c](float v) { return chunk_term(v, c); }, csum, nblocks, uf);
}

// Diagnostics (dqz_logits_probs / dqz_logits_terms), one block per chunk:
// p = t / total as f32 (the draw's distribution), the terms t themselves, the
// running lse and c.
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void logit_terms_kernel(const float* __restrict__ x, int64_t n,
                                                                 const LogitRun* run, const double* __restrict__ csum,
                                                                 int nblocks, float* __restrict__ p_out,
                                                                 float* __restrict__ t_out, float* lse_out,
                                                                 float* c_out) {
  __shared__ double s_tot;
  const LogitRun r = *run;
  if (threadIdx.x < 64) {
    const CsumLevel1 l1 = csum_level1(csum, nblocks, [] { return 2.0; });  // u = 2: only the total is used
    if (threadIdx.x == 0) s_tot = l1.tot;
  }
  __syncthreads();
  const double tot = s_tot;
  const int k = blockIdx.x;
  float xv[SM_PER_LANE];
  load_chunk_lane(x, n, k, xv);
  const int64_t base = (int64_t)k * SM_CHUNK + threadIdx.x * SM_PER_LANE;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) {
    if (base + i < n) {
      const double ti = chunk_term(xv[i], r.c);
      if (p_out) p_out[base + i] = (float)(ti / tot);
      if (t_out) t_out[base + i] = (float)ti;
    }
  }
  if (k == 0 && threadIdx.x == 0) {
    if (lse_out) *lse_out = run_lse(r);
    if (c_out) *c_out = r.c;
  }
}

// The learned-logit draw fused into the learner's forward launch
// (dqz_learner_step_logits): every conv1 block of sample b draws uniform b
// of step *counter (the dqz_uniform_philox stream) or takes the caller's,
// and runs the two-level search itself before its frame gather.  The head
// advances *counter once every conv1 block has read it.
struct SoftmaxDraw {
  const float* x;         // logits [n]
  int64_t n;
  const LogitRun* run;
  const double* csum;     // [nblocks] chunk sums
  int nblocks;
  uint64_t seed;
  uint64_t* counter;      // Philox step counter (null when `uniforms` is set)
  const double* uniforms;  // the caller's uniforms [B] (a host Generator's draws), or null
  int32_t* slots_out;     // [B]: block (rb 0, z 0) of sample b publishes its slot
};

__device__ __forceinline__ int32_t softmax_draw_slot(const SoftmaxDraw& d, int b) {
  return (int32_t)softmax_choice_body(d.x, d.n, d.run, d.csum, d.nblocks, [&] {
    return d.uniforms ? d.uniforms[b] : philox_uniform(d.seed, *d.counter, b);
  });
}

// Learned-logit batch draw (replay_circular.py:205-217, 540-545:
// Generator.choice(C, n, p=softmax(logits))), one block per query: the
// caller's uniform or Philox (seed, *counter, q), then the two-level search.
// The last query to finish resets the done word and advances *counter, so
// graph replays start clean.
struct SampleSync {
  static constexpr int kStride = 64;  // done / err words on their own 256-byte lines
  int* words;
};

DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void softmax_sample_kernel(
    const float* __restrict__ x, int64_t n, const LogitRun* run, const double* __restrict__ csum, int nblocks,
    SampleSync sync, uint64_t seed, uint64_t* counter, const double* __restrict__ uniforms, int nq,
    int32_t* __restrict__ out_slots, int64_t* __restrict__ out_idx) {
  int* done = sync.words + SampleSync::kStride;
  const int q = blockIdx.x;
  // the counter is loaded inside the draw (as softmax_draw_slot does), so
  // csum_level1 issues the chunk-sum loads first; wave 0, thread 0 included,
  // runs the lambda, and thread 0 keeps the value for the final increment
  uint64_t ctr = 0;
  const int64_t idx = softmax_choice_body(x, n, run, csum, nblocks, [&]() -> double {
    if (uniforms) return uniforms[q];
    ctr = *counter;
    return philox_uniform(seed, ctr, q);
  });
  if (threadIdx.x == 0) {
    if (out_slots) out_slots[q] = (int32_t)idx;
    if (out_idx) out_idx[q] = idx;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (__hip_atomic_fetch_add(done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nq - 1) {
      __hip_atomic_store(done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (!uniforms) *counter = ctr + 1;
    }
  }
}

// ---------------------------------------------------------------------------
// Exact mode of the learned-logit draw (dqz_logits_sample_exact): the
// reference's own float32 probabilities, bit for bit, and its choice.
//
// The reference forms p = exp(x - lse), lse = c + log(sum(exp(x - c))), c =
// max(x), with numpy float32 operations (replay_circular.py:69-76), then
// Generator.choice(C, n, p) = searchsorted(cumsum(float64(p)) / total, u,
// 'right') (:205-217, :540-545).  The default draw above forms its terms
// about the running state's shift instead (so a write costs O(1), not a pass
// over the buffer), which moves a draw near a CDF step by a float32 ulp of
// one term.  Here every operation is numpy's: np_expf / np_logf are its SIMD
// float32 exp and log (AVX2 / AVX-512 loops of loops_exponent_log, constants
// from its compiled module), the sum is np.sum's (pairwise summation per
// 8192-element buffer, buffer sums added in order), the subtractions and
// additions are single float32 operations (no contraction: each product is
// rounded before its sum, as there).  oracle/numpy_f32.py restates the same
// operations and tests/test_numpy_f32_cpu.py pins it against numpy.  The
// choice then sums the float64 terms in this file's chunk order, not
// numpy's sequential cumsum: the two CDFs differ by float64 rounding (~1e-16
// relative), so a draw can differ only for a uniform that close to a step.
// Passes: chunk maxima, c, per-buffer pairwise sums, lse, the exact chunk
// sums, the draws: six launches, each a pass over the buffer at most.

__device__ __forceinline__ float np_expf(float x) {
#pragma clang fp contract(off)
  if (x != x) return x;
  if (x <= -103.97208404541015625f) return 0.f;
  if (x >= 88.72283935546875f) return INFINITY;
  float q = x * 1.442695040888963407359924681001892137f;
  q = (q + 12582912.f) - 12582912.f;  // rint by the 1.5 * 2^23 magic
  float r = __fmaf_rn(q, -6.93145752e-1f, x);
  r = __fmaf_rn(q, -1.42860677e-6f, r);
  r = __fmaf_rn(q, 0.f, r);
  float num = __fmaf_rn(5.082762527590693718096e-04f, r, 6.757896990527504603057e-03f);
  num = __fmaf_rn(num, r, 5.114512081637298353406e-02f);
  num = __fmaf_rn(num, r, 2.473615434895520810817e-01f);
  num = __fmaf_rn(num, r, 7.257664613233124478488e-01f);
  num = __fmaf_rn(num, r, 1.f);
  float den = __fmaf_rn(2.159509375685829852307e-02f, r, -2.742335390411667452936e-01f);
  den = __fmaf_rn(den, r, 1.f);
  return ldexpf(num / den, (int)q);
}

// positive normal x (a sum of exponentials whose largest term is 1)
__device__ __forceinline__ float np_logf(float x) {
#pragma clang fp contract(off)
  const unsigned bits = __float_as_uint(x);
  float e = (float)(int)((bits >> 23) & 0xFFu) - 127.f;
  float m = __uint_as_float((bits & 0x7FFFFFu) | (126u << 23));
  float y;
  if (m <= __uint_as_float(0x3f3504f3u)) {  // sqrt(0.5)
    y = m + m;
  } else {
    y = m;
    e = e + 1.f;
  }
  y = y - 1.f;
  float num = __fmaf_rn(2.589979117907922693523e-02f, y, 3.808837741388407920751e-01f);
  num = __fmaf_rn(num, y, 1.480000633576506585156e+00f);
  num = __fmaf_rn(num, y, 2.112677543073053063722e+00f);
  num = __fmaf_rn(num, y, 9.999999999999998702752e-01f);
  num = __fmaf_rn(num, y, 0.f);
  float den = __fmaf_rn(__uint_as_float(0x3bc083dfu), y, 1.546476374983906719538e-01f);
  den = __fmaf_rn(den, y, 9.864942958519418960339e-01f);
  den = __fmaf_rn(den, y, 2.453006071784736363091e+00f);
  den = __fmaf_rn(den, y, 2.612677543073109236779e+00f);
  den = __fmaf_rn(den, y, 1.f);
  return __fmaf_rn(e, 0.693147180559945309417232121458176568f, num / den);
}

constexpr int NPX_BUF = 8192;   // np.getbufsize(): the reduction's buffer
constexpr int NPX_LEAF = 128;   // numpy's PW_BLOCKSIZE
constexpr int NPX_MAXLEAF = 256;

// chunk maxima (np.max is order-free)
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void npx_max_kernel(const float* __restrict__ x, int64_t n,
                                                              float* __restrict__ part) {
  __shared__ float sbuf[SM_THREADS / 64];
  float xv[SM_PER_LANE];
  load_chunk_lane(x, n, blockIdx.x, xv);
  float m = -INFINITY;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) m = fmaxf(m, xv[i]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) sbuf[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = fmaxf(fmaxf(sbuf[0], sbuf[1]), fmaxf(sbuf[2], sbuf[3]));
}

// c = max of the chunk maxima -> scal[0]
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void npx_cmax_kernel(const float* __restrict__ part, int nparts,
                                                               float* __restrict__ scal) {
  __shared__ float sbuf[SM_THREADS / 64];
  float m = -INFINITY;
  for (int k = threadIdx.x; k < nparts; k += SM_THREADS) m = fmaxf(m, part[k]);
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) sbuf[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) scal[0] = fmaxf(fmaxf(sbuf[0], sbuf[1]), fmaxf(sbuf[2], sbuf[3]));
}

// One workgroup per 8192-element buffer.  numpy's recursion over a buffer
// of length L (n <= 128 a leaf, else halves with the first rounded down to a
// multiple of 8) depends on L alone, so the host lays it out once per buffer
// length (npx_program, learner.hip): the leaves in order, then the internal
// nodes' additions (left + right) grouped by height.  Here: the program to
// LDS, the leaves in parallel (8 lanes per leaf, lane j numpy's accumulator
// r[j]), then the additions height by height -> bsum[buffer].
// Program: [nleaf, nlev, root, lo[nleaf], len[nleaf], lev_off[nlev + 1],
// (dst, a, b)[...]]; node values: leaves 0..nleaf-1, internal nodes after.
constexpr int NPX_PROG = 1024;

DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void npx_bufsum_kernel(const float* __restrict__ x, int64_t n,
                                                                 const float* __restrict__ scal,
                                                                 float* __restrict__ bsum,
                                                                 const int* __restrict__ prog_full,
                                                                 const int* __restrict__ prog_last) {
  __shared__ int sp[NPX_PROG];
  __shared__ float s_val[2 * NPX_MAXLEAF];
  const bool partial = blockIdx.x == gridDim.x - 1 && n % NPX_BUF != 0;
  const int* prog = partial ? prog_last : prog_full;
  for (int i = threadIdx.x; i < NPX_PROG; i += SM_THREADS) sp[i] = prog[i];
  __syncthreads();
  const int nleaf = sp[0], nlev = sp[1], root = sp[2];
  const int* p_lo = sp + 3;
  const int* p_len = p_lo + nleaf;
  const int* p_lev = p_len + nleaf;
  const int* p_ops = p_lev + nlev + 1;
  const int64_t base = (int64_t)blockIdx.x * NPX_BUF;
  const float c = scal[0];
  const int j = threadIdx.x & 7;
  for (int l = threadIdx.x >> 3; l < nleaf; l += SM_THREADS / 8) {
    const int64_t lo = base + p_lo[l];
    const int m = p_len[l];
    float r = 0.f;
    if (m >= 8) {
      r = np_expf(x[lo + j] - c);
      for (int i = 8 + j; i < m - m % 8; i += 8) r = r + np_expf(x[lo + i] - c);
    }
    // r[k] of this leaf's 8-lane group (8-aligned in the wave)
    const float r1 = __shfl_xor(r, 1, 8), r2 = __shfl_xor(r, 2, 8), r3 = __shfl_xor(r, 3, 8);
    const float r4 = __shfl_xor(r, 4, 8), r5 = __shfl_xor(r, 5, 8), r6 = __shfl_xor(r, 6, 8), r7 = __shfl_xor(r, 7, 8);
    if (j == 0) {
      float res;
      if (m >= 8) {
        res = ((r + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
        for (int i = m - m % 8; i < m; ++i) res = res + np_expf(x[lo + i] - c);
      } else {
        res = 0.f;
        for (int i = 0; i < m; ++i) res = res + np_expf(x[lo + i] - c);
      }
      s_val[l] = res;
    }
  }
  __syncthreads();
  for (int h = 0; h < nlev; ++h) {
    for (int k = p_lev[h] + threadIdx.x; k < p_lev[h + 1]; k += SM_THREADS)
      s_val[p_ops[3 * k]] = s_val[p_ops[3 * k + 1]] + s_val[p_ops[3 * k + 2]];
    __syncthreads();
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = s_val[root];
}

// np.sum = the buffer sums added in order; lse = c + log(sum) -> scal[1]
DQZ_OTHER_KERNEL void npx_lse_kernel(const float* __restrict__ bsum, int nbuf, float* __restrict__ scal) {
  if (threadIdx.x != 0) return;
  float s = 0.f;
  for (int k = 0; k < nbuf; ++k) s = s + bsum[k];
  scal[1] = scal[0] + np_logf(s);
}

// The exact terms p = np_expf(x - lse) per chunk: their float64 chunk sums
// (block_total_f64, the canonical order) and, if asked, p itself.
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void npx_chunk_kernel(const float* __restrict__ x, int64_t n,
                                                                const float* __restrict__ scal,
                                                                double* __restrict__ csum, float* __restrict__ p_out) {
  __shared__ double s_wave[SM_THREADS / 64];
  const int k = blockIdx.x;
  const float lse = scal[1];
  float xv[SM_PER_LANE];
  load_chunk_lane(x, n, k, xv);
  const int64_t base = (int64_t)k * SM_CHUNK + threadIdx.x * SM_PER_LANE;
  double lane = 0.0;
#pragma unroll
  for (int i = 0; i < SM_PER_LANE; ++i) {
    const float p = np_expf(xv[i] - lse);
    lane += (double)p;
    if (p_out && base + i < n) p_out[base + i] = p;
  }
  const double tot = block_total_f64(lane, s_wave);
  if (threadIdx.x == 0) csum[k] = tot;
}

// The reference's default logit of an add (replay_circular.py:166-179,
// :518-533): 0 into an empty buffer, else logsumexp(logits) - np.log(size),
// the float32 lse minus a float64 log (numpy promotes to float64), stored as
// float32.  clear_pos >= 0: the reservoir `replace` clears that slot first
// (npx_clear_kernel, ahead of the lse passes).
DQZ_OTHER_KERNEL void npx_clear_kernel(float* __restrict__ x, int64_t pos) {
  if (threadIdx.x == 0) x[pos] = -INFINITY;
}
DQZ_OTHER_KERNEL void npx_add_kernel(float* __restrict__ x, int64_t pos, int64_t size,
                                     const float* __restrict__ scal) {
  if (threadIdx.x != 0) return;
  x[pos] = size == 0 ? 0.f : (float)((double)scal[1] - log((double)size));
}

// One query per block: the two-level search over the exact terms.
DQZ_OTHER_KERNEL __launch_bounds__(SM_THREADS) void npx_sample_kernel(const float* __restrict__ x, int64_t n,
                                                                 const float* __restrict__ scal,
                                                                 const double* __restrict__ csum, int nblocks,
                                                                 const double* __restrict__ uniforms,
                                                                 int64_t* __restrict__ out_idx) {
  const int q = blockIdx.x;
  const float lse = scal[1];
  const int64_t idx = softmax_choice_terms(
      x, n, [lse](float v) { return (double)np_expf(v - lse); }, csum, nblocks, [&] { return uniforms[q]; });
  if (threadIdx.x == 0) out_idx[q] = idx;
}

// ---------------------------------------------------------------------------
// fp64 sum tree (storage[1] = root; node i -> 2i, 2i+1; leaves from `cap`)

// Single workgroup: write n leaves, then recompute their ancestors level by
// level (duplicate parents write identical values).
DQZ_OTHER_KERNEL __launch_bounds__(1024) void sumtree_set_kernel(double* tree, int64_t cap, int levels,
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

// Fast path for small updates (n <= 256, the PER write-back of one batch):
// every sibling on every leaf's path is fetched in one batch up front, then
// the ancestors are rebuilt level by level in LDS.  Leaves a and b have
// sibling ancestors exactly at level msb(a ^ b), so one O(n) pass tells each
// leaf at which levels its sibling is itself being updated and by whom; each
// level then costs two LDS reads and two barriers instead of a global round
// trip.  Same left + right sums as sumtree_set_kernel (bit-identical).
// Caller passes distinct leaves.
constexpr int ST_FAST = 256;

// Thread i < n owns leaf `leaf` (tree index, or -1: this thread sets nothing)
// with new value v; live leaves are distinct.
__device__ __forceinline__ void sumtree_set_small_body(double* tree, int levels, int n, int64_t leaf, double v) {
  __shared__ int64_t s_leaf[ST_FAST];
  __shared__ double s_val[ST_FAST];
  __shared__ double s_sib[32][ST_FAST];  // old sibling per level; later the new ancestor values
  __shared__ short s_rep[32][ST_FAST];   // updated leaf whose ancestor is my sibling at level l, or -1
  const int i = threadIdx.x;
  const bool live = i < n && leaf >= 0;
  if (!live) leaf = -1;
  const double leaf_v = v;
  constexpr int kBatch = 24;  // every sibling of a 2^24-leaf path in one round trip
  for (int l0 = 0; l0 < levels; l0 += kBatch) {
    double tb[kBatch];
#pragma unroll
    for (int j = 0; j < kBatch; ++j) tb[j] = live && l0 + j < levels ? tree[(leaf >> (l0 + j)) ^ 1] : 0.0;
#pragma unroll
    for (int j = 0; j < kBatch; ++j)
      if (l0 + j < levels) s_sib[l0 + j][i] = tb[j];
  }
  for (int l = 0; l < levels; ++l) s_rep[l][i] = -1;
  s_leaf[i] = leaf;
  s_val[i] = v;
  __syncthreads();
  if (live)
    for (int j = 0; j < n; ++j) {
      const int64_t o = s_leaf[j];
      const uint64_t d = (uint64_t)(leaf ^ o);
      if (o >= 0 && d != 0) s_rep[63 - __builtin_clzll(d)][i] = (short)j;
    }
  __syncthreads();
  for (int l = 0; l < levels; ++l) {
    const int r = s_rep[l][i];
    const double other = r >= 0 ? s_val[r] : s_sib[l][i];
    const double parent = ((leaf >> l) & 1) ? other + v : v + other;
    __syncthreads();
    v = parent;
    s_val[i] = v;
    s_sib[l][i] = v;  // this level's sibling is consumed -> the new level-(l + 1) value
    __syncthreads();
  }
  // stores last: a barrier would otherwise wait for every pending store
  if (live) {
    tree[leaf] = leaf_v;
    for (int l = 0; l < levels; ++l) tree[leaf >> (l + 1)] = s_sib[l][i];
  }
}

DQZ_OTHER_KERNEL __launch_bounds__(ST_FAST) void sumtree_set_small_kernel(double* tree, int64_t cap, int levels,
                                                                    const int64_t* idx, const double* vals, int n) {
  const int i = threadIdx.x;
  sumtree_set_small_body(tree, levels, n, i < n ? cap + idx[i] : -1, i < n ? vals[i] : 0.0);
}

// PrioritizedDqn priority write-back (prioritized/agent.py:201-206 +
// PrioritizedDistribution.update_priorities, replay.py:620-630 + _power,
// :336-341) for the learner's last batch, on device: p = |td|,
// *max_seen = max(*max_seen, max p), leaf = p^alpha (0 -> 0), sum-tree
// set.  A slot drawn twice keeps its last draw's value (numpy fancy
// assignment order in SumTree.set).  n <= ST_FAST.
DQZ_OTHER_KERNEL __launch_bounds__(ST_FAST) void per_write_back_kernel(double* tree, int64_t cap, int levels,
                                                                 const int32_t* slots, const float* td, double alpha,
                                                                 int n, double* max_seen) {
  __shared__ double s_max[ST_FAST / 64];
  __shared__ int32_t s_slot[ST_FAST];
  const int i = threadIdx.x;
  int64_t leaf = -1;
  double p = 0.0;
  const int32_t s = i < n ? slots[i] : -1;
  if (i < n) p = fabs((double)td[i]);
  s_slot[i] = s;
  __syncthreads();
  if (i < n) {
    bool last = true;  // the last draw of a repeated slot wins (SumTree.set order)
    for (int j = i + 1; j < n; ++j) last &= s_slot[j] != s;
    if (last) leaf = cap + s;
  }
  double m = p;
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  if ((i & 63) == 0) s_max[i >> 6] = m;
  const double v = p == 0.0 ? 0.0 : pow(p, alpha);
  sumtree_set_small_body(tree, levels, n, leaf, v);  // its barriers publish s_max
  if (i == 0) {
    double mm = *max_seen;
    for (int w = 0; w < ST_FAST / 64; ++w) mm = fmax(mm, s_max[w]);
    *max_seen = mm;
  }
}

// The PER priority write-back run by ONE wave inside another launch
// (bwd_bc_kernel's first workgroup, dqz_learner_step_per): the same
// arithmetic as per_write_back_kernel (|td| -> max_seen, p^alpha, the last
// draw of a repeated slot wins, ancestors rebuilt as left + right through the
// levels where another updated leaf's path joins), for n <= 64 leaves, with
// its LDS carved from the host launch's buffer (`lds`, >= PWB_LDS_BYTES), so
// the host kernel's LDS footprint does not grow.  Lanes are the draws; one
// wave runs in lockstep, so LDS writes of one level are read by the next
// after a wave barrier.
constexpr int PWB_LEVELS = 24;  // trees of up to 2^24 leaves
constexpr int PWB_LDS_BYTES = 64 * (8 * PWB_LEVELS + 8 + 8 + 4 + 2 * PWB_LEVELS);

struct PerWbArgs {
  double* tree;          // null: no write-back in this launch
  int64_t cap;
  int levels;
  const int32_t* slots;  // tree indices of the batch (dqz_per_sample's out_indices)
  const float* td;       // the learner's TD errors of this step
  double alpha;
  int n;
  double* max_seen;
};

__device__ __forceinline__ void per_write_back_wave(const PerWbArgs& a, char* lds) {
  double* s_sib = reinterpret_cast<double*>(lds);      // [PWB_LEVELS][64]
  double* s_val = s_sib + PWB_LEVELS * 64;             // [64]
  int64_t* s_leaf = reinterpret_cast<int64_t*>(s_val + 64);  // [64]
  int32_t* s_slot = reinterpret_cast<int32_t*>(s_leaf + 64); // [64]
  short* s_rep = reinterpret_cast<short*>(s_slot + 64);       // [PWB_LEVELS][64]
  const int i = threadIdx.x & 63;
  const int n = a.n, levels = a.levels;
  const int32_t sl = i < n ? a.slots[i] : -1;
  const double p = i < n ? fabs((double)a.td[i]) : 0.0;
  s_slot[i] = sl;
  __builtin_amdgcn_wave_barrier();
  int64_t leaf = -1;
  if (i < n) {
    bool last = true;
    for (int j = i + 1; j < n; ++j) last &= s_slot[j] != sl;
    if (last) leaf = a.cap + sl;
  }
  const bool live = leaf >= 0;
  double tb[PWB_LEVELS];
#pragma unroll
  for (int l = 0; l < PWB_LEVELS; ++l) tb[l] = live && l < levels ? a.tree[(leaf >> l) ^ 1] : 0.0;
  double m = p;
  for (int o = 32; o > 0; o >>= 1) m = fmax(m, __shfl_xor(m, o, 64));
  double v = p == 0.0 ? 0.0 : pow(p, a.alpha);
  const double leaf_v = v;
  s_leaf[i] = leaf;
  s_val[i] = v;
  for (int l = 0; l < levels; ++l) s_rep[l * 64 + i] = -1;
  __builtin_amdgcn_wave_barrier();
  if (live)
    for (int j = 0; j < n; ++j) {
      const int64_t o = s_leaf[j];
      const uint64_t d = (uint64_t)(leaf ^ o);
      if (o >= 0 && d != 0) s_rep[(63 - __builtin_clzll(d)) * 64 + i] = (short)j;
    }
#pragma unroll
  for (int l = 0; l < PWB_LEVELS; ++l)
    if (l < levels) s_sib[l * 64 + i] = tb[l];
  __builtin_amdgcn_wave_barrier();
  for (int l = 0; l < levels; ++l) {
    const int r = s_rep[l * 64 + i];
    const double other = r >= 0 ? s_val[r] : s_sib[l * 64 + i];
    const double parent = ((leaf >> l) & 1) ? other + v : v + other;
    __builtin_amdgcn_wave_barrier();  // every lane has read level l before any writes level l + 1
    v = parent;
    s_val[i] = v;
    s_sib[l * 64 + i] = v;
    __builtin_amdgcn_wave_barrier();
  }
  if (live) {
    a.tree[leaf] = leaf_v;
    for (int l = 0; l < levels; ++l) a.tree[leaf >> (l + 1)] = s_sib[l * 64 + i];
  }
  if (i == 0) *a.max_seen = fmax(*a.max_seen, m);
}

// Descent of SumTree._query_single (replay.py:539-559) by one half-wave (32
// lanes), four tree levels per global round trip.  In the implicit layout
// the descendants of `node` at relative depth k are the contiguous indices
// node * 2^k .. node * 2^k + 2^k - 1, so a round loads the 2 + 4 + 8 + 16 = 30
// nodes below the current one (lane l: depth k = floor(log2(l + 2)),
// j = l + 2 - 2^k) and takes the four left/right decisions from registers with
// the reference's own fp64 arithmetic (compare with the left sum, subtract it
// on the way right): the same node sequence as the serial descent, bit for
// bit, in ceil(levels / 4) dependent loads instead of `levels`.  The first
// round also fetches the root (nodes 1 .. 31, lane l holds node l + 1), so
// callers that scale their target by the root pay no extra round trip:
// `scale` >= 0 -> t = scale * root (PER), scale < 0 -> t as given, and the
// slot is -1 when t is not in [0, root).  Returns the slot and its leaf.
struct Descent {
  int64_t slot;
  double leaf, root;
};

__device__ __forceinline__ Descent halfwave_descend(const double* tree, int64_t cap, int levels, double t,
                                                    double scale, int l) {
  // round 0: nodes 1..31 (depths 0..4), clamped to the tree
  const int64_t top = min((int64_t)31, 2 * cap - 1);
  const double v0 = l < top ? tree[1 + l] : 0.0;
  const double root = __shfl(v0, 0, 32);
  Descent d{-1, 0.0, root};
  if (scale >= 0.0)
    t = scale * root;  // u in [0, 1): u * root < root in fp64 (no range check, as the serial descent)
  else if (!(t >= 0.0 && t < root))
    return d;
  int64_t node = 1;
  int depth = 0;
  double v = v0;
  int base = -1;  // lane of relative depth k, j = 0 is base + 2^k (round 0: lane = node - 1)
  while (true) {
    const int K = min(4, levels - depth);
    int64_t pos = 0;
    for (int k = 1; k <= K; ++k) {
      const double left = __shfl(v, base + (1 << k) + 2 * (int)pos, 32);
      if (t < left) {
        pos = 2 * pos;
      } else {
        t -= left;
        pos = 2 * pos + 1;
      }
    }
    node = (node << K) + pos;
    depth += K;
    if (depth >= levels) {
      d.slot = node - cap;
      d.leaf = K > 0 ? __shfl(v, base + (1 << K) + (int)pos, 32) : root;
      return d;
    }
    // next round: the 30 nodes below `node`
    const int k = 31 - __builtin_clz(l + 2), j = l + 2 - (1 << k);
    const int kmax = min(4, levels - depth);
    v = (l < (2 << kmax) - 2) ? tree[(node << k) + j] : 0.0;
    base = -2;
  }
}

// One half-wave per target; -1 when out of range.
DQZ_OTHER_KERNEL __launch_bounds__(256) void sumtree_query_kernel(const double* __restrict__ tree, int64_t cap,
                                                            int levels, const double* __restrict__ targets, int n,
                                                            int64_t* __restrict__ out) {
  const int i = blockIdx.x * 8 + (threadIdx.x >> 5), l = threadIdx.x & 31;
  if (i >= n) return;  // half-wave uniform
  const Descent d = halfwave_descend(tree, cap, levels, targets[i], -1.0, l);
  if (l == 0) out[i] = d.slot;
}

// PrioritizedDistribution.sample + importance_sampling_weights
// (replay.py:680-716, 344-376).  Draws either from device Philox streams or,
// when `inj_u` is set, injected from the caller's RandomState in the
// reference's order: inj_uniform[i] = active_indices[randint] (a tree index),
// inj_u[i] = the target uniform, inj_u[n + i] = the usp-mix uniform; the
// counter is then neither read nor advanced.  Philox mode: tree index ==
// replay slot, uniform picks over the live window (live_base + j) % capacity.
// Tree index -> replay slot through `index_to_slot` when set.  One block of
// 32 half-waves; half-wave h handles draws h, h + 32, ...; n <= 1024.
// Probabilities are formed without contraction, as numpy evaluates them:
// (1 - usp) * (leaf / root) + usp * (1 / size).
struct PerSampleArgs {
  const double* tree;
  int64_t cap;
  int levels;
  int64_t live_base, size, capacity;
  int n;
  double usp, beta;
  int normalize;
  uint64_t seed;
  uint64_t* counter;
  const int32_t* inj_uniform;
  const double* inj_u;
  const int32_t* index_to_slot;
  int32_t* out_indices;
  int32_t* out_slots;
  float* out_weights;
  double* out_probs;
  double* out_wb;  // fused draw only: the unnormalised IS weight (up / p)^beta of each draw
};

// Depths 0 .. PS_TOPD of the tree (2047 nodes, 16 KB) are staged in LDS once
// per launch and shared by every draw; below them a half-wave descends five
// levels per global round trip (lane l holds relative nodes l and l + 32 of
// the 62 below the current node: depth k = floor(log2(q + 2)), j = q + 2 -
// 2^k) and takes the decisions from registers.  At 2^20 leaves: one shared
// 16 KB load + two dependent rounds instead of five.  Same compare-and-
// subtract arithmetic as SumTree._query_single (replay.py:539-559), so the
// same node sequence bit for bit.
constexpr int PS_TOPD = 10;
constexpr int PS_TOP_NODES = 2 << PS_TOPD;  // LDS doubles of the staged top

// Stages tree nodes 1 .. 2^(dtop + 1) - 1 into s_top[1 ..] (whole block) and
// returns dtop.
// The top is staged in two halves so a caller can issue other loads between
// them: per_top_load issues every load of the thread (a guarded loop left to
// the compiler loaded, waited and stored one node per thread at a time: eight
// dependent round trips per 256-thread block), per_top_store writes them.
constexpr int PS_TOP_R = (PS_TOP_NODES + 255) / 256;  // nodes per thread of a 256-thread block
struct PerTop {
  double v[PS_TOP_R];
  int dtop, ntop;
};
__device__ __forceinline__ PerTop per_top_load(const PerSampleArgs& a) {
  PerTop t;
  t.dtop = min(a.levels, PS_TOPD);
  t.ntop = (2 << t.dtop) - 1;
  const int nb = blockDim.x;
#pragma unroll
  for (int r = 0; r < PS_TOP_R; ++r) t.v[r] = a.tree[1 + min((int)threadIdx.x + r * nb, t.ntop - 1)];
  return t;
}
__device__ __forceinline__ int per_top_store(const PerSampleArgs& a, const PerTop& t, double* s_top) {
  const int nb = blockDim.x;
#pragma unroll
  for (int r = 0; r < PS_TOP_R; ++r) {
    const int q = threadIdx.x + r * nb;
    if (q < t.ntop) s_top[1 + q] = t.v[r];
  }
  for (int q = threadIdx.x + PS_TOP_R * nb; q < t.ntop; q += nb) s_top[1 + q] = a.tree[1 + q];  // blocks under 256 threads
  __syncthreads();
  return t.dtop;
}
// Stages tree nodes 1 .. 2^(dtop + 1) - 1 into s_top[1 ..] (whole block) and
// returns dtop.
__device__ __forceinline__ int per_stage_top(const PerSampleArgs& a, double* s_top) {
  const PerTop t = per_top_load(a);
  __builtin_amdgcn_sched_barrier(0);
  return per_top_store(a, t, s_top);
}

// Draw i of PrioritizedDistribution.sample (replay.py:680-716) by one
// half-wave (lane l): the tree index and its sampling probability.
struct PerPick {
  int64_t idx;
  double prob;
};

// The draw's three random inputs: injected from the caller's RandomState, or
// Philox (seed, ctr, i).  Separate from the descent so a caller can issue
// their loads before it stages the tree top.
struct PerDrawInput {
  double u_target, u_mix;
  int64_t uni;
};

// Injected inputs as loaded (u_target, u_mix, uni) or, in Philox mode, the
// step counter in `uni` (per_draw_input turns it into the draw's inputs).
__device__ __forceinline__ PerDrawInput per_draw_load(const PerSampleArgs& a, int i) {
  if (a.inj_u) return PerDrawInput{a.inj_u[i], a.inj_u[a.n + i], a.inj_uniform[i]};
  return PerDrawInput{0.0, 0.0, (int64_t)*a.counter};
}

__device__ __forceinline__ PerDrawInput per_draw_input(const PerSampleArgs& a, int i, uint64_t ctr) {
  PerDrawInput d;
  if (a.inj_u) {
    d.u_target = a.inj_u[i];
    d.u_mix = a.inj_u[a.n + i];
    d.uni = a.inj_uniform[i];
  } else {
    const uint4 r = philox4x32(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), (unsigned)i, 0x9E12u),
                               make_uint2((unsigned)a.seed, (unsigned)(a.seed >> 32)));
    d.u_target = ((((uint64_t)r.x << 32) | r.y) >> 11) * 0x1.0p-53;
    d.u_mix = (double)(r.z >> 8) * 0x1.0p-24;
    d.uni = (a.live_base + (int64_t)((double)(r.w) * 0x1.0p-32 * (double)a.size)) % a.capacity;
  }
  return d;
}

__device__ __forceinline__ PerPick per_pick(const PerSampleArgs& a, int l, const double* s_top, int dtop,
                                            const PerDrawInput& in) {
  const double root = s_top[1];
  const double u_target = in.u_target, u_mix = in.u_mix;
  const int64_t uni = in.uni;
  const bool use_uniform = u_mix < a.usp;
  int64_t idx = uni;
  double leaf;
  if (root > 0.0 && !use_uniform) {
    double t = u_target * root;  // u in [0, 1): t < root in fp64 (no range check, as the serial descent)
    int64_t node = 1;
    int depth = 0;
    for (; depth < dtop; ++depth) {
      const double left = s_top[2 * node];
      if (t < left) {
        node = 2 * node;
      } else {
        t -= left;
        node = 2 * node + 1;
      }
    }
    double lv = s_top[node];  // the leaf itself when the whole tree sits in LDS
    while (depth < a.levels) {
      const int K = min(5, a.levels - depth);
      double v0 = 0.0, v1 = 0.0;
      {
        const int k0 = 31 - __builtin_clz(l + 2), k1 = 31 - __builtin_clz(l + 34);
        if (k0 <= K) v0 = a.tree[(node << k0) + (l + 2 - (1 << k0))];
        if (k1 <= K) v1 = a.tree[(node << k1) + (l + 34 - (1 << k1))];
      }
      int64_t pos = 0;
      for (int k = 1; k <= K; ++k) {
        const int q = (1 << k) - 2 + 2 * (int)pos;  // left child at relative depth k
        const double left = q < 32 ? __shfl(v0, q, 32) : __shfl(v1, q - 32, 32);
        if (t < left) {
          pos = 2 * pos;
        } else {
          t -= left;
          pos = 2 * pos + 1;
        }
      }
      const int q = (1 << K) - 2 + (int)pos;
      lv = q < 32 ? __shfl(v0, q, 32) : __shfl(v1, q - 32, 32);
      node = (node << K) + pos;
      depth += K;
    }
    idx = node - a.cap;
    leaf = lv;
  } else {
    leaf = a.tree[a.cap + idx];
  }
  const double up = 1.0 / (double)a.size;
  const double pp = root > 0.0 ? leaf / root : up;
  double prob;
  {
    // numpy rounds the product and the sum separately: no fma (hipcc
    // contracts even __dmul_rn + __dadd_rn under its default fp-contract)
#pragma clang fp contract(off)
    const double x1 = (1.0 - a.usp) * pp;
    const double x2 = a.usp * up;
    prob = x1 + x2;
  }
  return PerPick{idx, prob};
}

// importance_sampling_weights (replay.py:344-376) of one draw, unnormalised.
__device__ __forceinline__ double per_weight(double up, double prob, double beta) { return pow(up / prob, beta); }

DQZ_OTHER_KERNEL __launch_bounds__(1024) void per_sample_kernel(PerSampleArgs a) {
  __shared__ double s_top[PS_TOP_NODES];  // node i at s_top[i], i in [1, 2^(dtop + 1))
  __shared__ double s_w[1024];
  const bool inj = a.inj_u != nullptr;
  const uint64_t ctr = inj ? 0 : *a.counter;
  const int dtop = per_stage_top(a, s_top);
  const int h = threadIdx.x >> 5, l = threadIdx.x & 31;
  const double up = 1.0 / (double)a.size;
  for (int i = h; i < a.n; i += 32) {
    const PerPick pk = per_pick(a, l, s_top, dtop, per_draw_input(a, i, ctr));
    const double w = per_weight(up, pk.prob, a.beta);
    if (l == 0) {
      if (a.out_indices) a.out_indices[i] = (int32_t)pk.idx;
      a.out_slots[i] = a.index_to_slot ? a.index_to_slot[pk.idx] : (int32_t)pk.idx;
      if (a.out_probs) a.out_probs[i] = pk.prob;
      s_w[i] = w;
    }
  }
  __syncthreads();
  double m = 0.0;
  if (a.normalize)
    for (int j = 0; j < a.n; ++j) m = fmax(m, s_w[j]);
  for (int i = threadIdx.x; i < a.n; i += blockDim.x) a.out_weights[i] = (float)(a.normalize ? s_w[i] / m : s_w[i]);
  __syncthreads();
  if (threadIdx.x == 0 && !inj) *a.counter = ctr + 1;
}

// PER draw b fused into the learner's conv1 workgroups (dqz_learner_step_per_draw):
// the block stages the tree's top in `lds` (conv1's input buffer, before its
// frame gather), its first half-wave descends, and the block gets the slot;
// the publishing block (rb 0, z 0) writes the tree index, slot and
// probability of draw b (the head turns the B probabilities into normalised
// IS weights, the backward's write-back uses the indices).  The Philox
// counter is advanced by the head once every conv1 block has read it.
struct PerDrawOut {
  int32_t slot;  // every thread
  double prob;   // thread 0
};

__device__ __forceinline__ PerDrawOut per_draw_slot(const PerSampleArgs& a, int b, double* lds, bool publish) {
  __shared__ int32_t s_slot;
  double prob = 0.0;
  // the tree top's loads and the draw's inputs (the counter or the injected
  // values: block-uniform loads) are all in flight before the first wait
  const PerTop top = per_top_load(a);
  const PerDrawInput raw = per_draw_load(a, b);
  __builtin_amdgcn_sched_barrier(0);
  const int dtop = per_top_store(a, top, lds);
  if (threadIdx.x < 32) {
    const PerDrawInput in = a.inj_u ? raw : per_draw_input(a, b, (uint64_t)raw.uni);
    const PerPick pk = per_pick(a, threadIdx.x, lds, dtop, in);
    if (threadIdx.x == 0) {
      const int32_t slot = a.index_to_slot ? a.index_to_slot[pk.idx] : (int32_t)pk.idx;
      s_slot = slot;
      prob = pk.prob;
      if (publish) {
        a.out_indices[b] = (int32_t)pk.idx;
        a.out_slots[b] = slot;
        a.out_probs[b] = pk.prob;
      }
    }
  }
  __syncthreads();  // s_slot published; every read of lds done before the frame gather reuses it
  return PerDrawOut{s_slot, prob};
}

// The publishing block's IS weight of draw b, (1/size / p)^beta unnormalised
// (per_sample_kernel's per_weight, the same bits), for the head's batch
// normalisation; called by thread 0 with the probability per_draw_slot left it.
__device__ __forceinline__ void per_publish_weight(const PerSampleArgs& a, int b, double prob) {
  if (a.out_wb) a.out_wb[b] = per_weight(1.0 / (double)a.size, prob, a.beta);
}

// PrioritizedTransitionReplay.add on device (replay.py:1068-1096 with
// PrioritizedDistribution.remove_priorities / add_priorities): the evicted
// tree index (or -1) gets 0, the new one (priority >= 0 ? priority :
// *max_seen) ** alpha (0 -> 0, _power), ancestors rebuilt, and
// index_to_slot[add] = slot.  One launch of ST_FAST threads, two live.
DQZ_OTHER_KERNEL __launch_bounds__(ST_FAST) void per_add_kernel(double* tree, int64_t cap, int levels, int32_t remove_idx,
                                                          int32_t add_idx, double priority, const double* max_seen,
                                                          double alpha, int32_t* index_to_slot, int32_t slot) {
  const int i = threadIdx.x;
  int64_t leaf = -1;
  double v = 0.0;
  if (i == 0 && remove_idx >= 0 && remove_idx != add_idx) leaf = cap + remove_idx;
  if (i == 1) {
    const double p = priority >= 0.0 ? priority : *max_seen;
    v = p == 0.0 ? 0.0 : (alpha == 1.0 ? p : pow(p, alpha));  // alpha 1: host-exponentiated
    leaf = cap + add_idx;
  }
  sumtree_set_small_body(tree, levels, 2, leaf, v);
  if (i == 0 && index_to_slot) index_to_slot[add_idx] = slot;
}

}  // namespace dqz
