// learner.hip — everything of libdqz but the learner step's kernels (those
// are learner_step.hip's code object; common.hpp, "Two translation units"):
// the replay-side device code (frame store puts and gathers, the uniform,
// learned-logit and prioritized samplers, sum trees), the MGSC meta-update
// and its HVP, Atari preprocessing, and the C-ABI entries that drive them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <functional>
#include <cmath>
#include <vector>
#include <cstdlib>
#include <cstring>

#include "learner_impl.hpp"
#include "meta.hpp"
#include "hvp.hpp"
#include "preprocess.hpp"

using namespace dqz;

// the meta-update's tangent launch takes conv1's dynamic LDS
static int g_meta_attr_done = 0;

static int init_meta_attrs() {
  if (g_meta_attr_done) return DQZ_OK;
  DQZ_HIP(hipFuncSetAttribute((const void*)tangent_fwd_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)kConv1FwdSmem));
  g_meta_attr_done = 1;
  return DQZ_OK;
}

extern "C" {

const char* dqz_last_error(void) { return err_buf().c_str(); }

#ifndef DQZ_BUILD_ID
#define DQZ_BUILD_ID "unset"
#endif
const char* dqz_build_id(void) { return DQZ_BUILD_ID; }

int dqz_store_put(const dqz_store* S, const dqz_transition_put* t, const uint8_t* frames, void* stream) {
  if (int rc = check_store(S)) return rc;
  if (!t) return fail(DQZ_ERR_INVALID, "null transition");
  if (t->slot < 0 || t->slot >= S->capacity)
    return fail(DQZ_ERR_INVALID, "slot %lld out of range [0, %lld)", (long long)t->slot, (long long)S->capacity);
  if (t->num_frames < 0 || t->num_frames > 8) return fail(DQZ_ERR_INVALID, "num_frames must be in [0, 8]");
  for (int i = 0; i < 8; ++i)
    if (t->fidx[i] < -1 || t->fidx[i] >= S->num_frames) return fail(DQZ_ERR_INVALID, "fidx[%d] out of range", i);
  for (int i = 0; i < t->num_frames; ++i)
    if (t->frame_rows[i] < 0 || t->frame_rows[i] >= S->num_frames)
      return fail(DQZ_ERR_INVALID, "frame_rows[%d] out of range", i);
  const void* dframes = nullptr;
  if (t->num_frames > 0) {
    if (!frames) return fail(DQZ_ERR_INVALID, "null frames");
    if (int rc = device_view(frames, &dframes, "frames")) return rc;
    if (reinterpret_cast<uintptr_t>(dframes) % 16) return fail(DQZ_ERR_INVALID, "frames must be 16-byte aligned");
  }
  hipLaunchKernelGGL(store_put_kernel, dim3(t->num_frames > 0 ? t->num_frames : 1), dim3(256), 0,
                     (hipStream_t)stream, const_cast<uint8_t*>(S->frames), const_cast<int32_t*>(S->fidx),
                     const_cast<int32_t*>(S->action), const_cast<float*>(S->reward),
                     const_cast<float*>(S->discount), *t, static_cast<const uint8_t*>(dframes));
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_sample_uniform(int64_t base, int64_t size, int64_t capacity, int n, uint64_t seed, uint64_t* counter_dev,
                       int32_t* out_slots, void* stream) {
  if (!counter_dev || !out_slots) return fail(DQZ_ERR_INVALID, "null argument");
  if (size < 1) return fail(DQZ_ERR_INVALID, "cannot sample from an empty replay (size=%lld)", (long long)size);
  if (capacity < size) return fail(DQZ_ERR_INVALID, "size exceeds capacity");
  if (n < 1 || n > 65536) return fail(DQZ_ERR_INVALID, "n out of range");
  if (base < 0) return fail(DQZ_ERR_INVALID, "base must be >= 0");
  hipLaunchKernelGGL(sample_uniform_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, base % capacity, size, capacity, n, seed,
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

// ---------------------------------------------------------------------------
// learned-logit and prioritized samplers

struct dqz_logit_buffer {
  int64_t capacity;
  int nblocks, max_queries;
  void* block;  // double csum[nblocks] | MaxSum part[nblocks] | int dirty[nblocks] | float lse | LogitRun | sync
  double* csum;    // per-chunk sums of the sampling terms (sampling.hpp chunk_sum)
  MaxSum* part;
  int* dirty;      // chunks a writer changed, for chunk_sums_kernel
  float* lse;
  LogitRun* run;   // running log-sum-exp (sampling.hpp)
  int* sync;       // softmax_sample_kernel's done word (SampleSync)
  // exact mode (dqz_logits_sample_exact): chunk sums of the exact terms,
  // chunk maxima, numpy-buffer sums, {c, lse}
  int nbuf;
  double* csum_x;
  float *part_x, *bsum_x, *scal_x;
  int *prog_full, *prog_last;  // npx_program of a full and of the last buffer
  bool run_known;  // host side: every write since the last scan went through the library
  int run_adds;    // running adds since the last scan
};

// numpy's pairwise-summation recursion over one buffer of length L
// (sampling.hpp npx_bufsum_kernel's program): the leaves in order, then the
// internal additions grouped by height, each (dst, left, right).
static std::vector<int> npx_program(int L) {
  std::vector<int> lo, len;
  std::vector<std::array<int, 4>> ops;  // height, dst, a, b
  int nleaf = 0;
  std::function<void(int, int)> leaves = [&](int l, int m) {
    if (m <= NPX_LEAF) {
      lo.push_back(l);
      len.push_back(m);
      return;
    }
    int m2 = m / 2;
    m2 -= m2 % 8;
    leaves(l, m2);
    leaves(l + m2, m - m2);
  };
  leaves(0, L);
  nleaf = (int)lo.size();
  int next_leaf = 0, next = nleaf;
  std::function<std::pair<int, int>(int)> build = [&](int m) -> std::pair<int, int> {
    if (m <= NPX_LEAF) return {next_leaf++, 0};
    int m2 = m / 2;
    m2 -= m2 % 8;
    const auto a = build(m2);
    const auto b = build(m - m2);
    const int h = std::max(a.second, b.second) + 1, d = next++;
    ops.push_back({h, d, a.first, b.first});
    return {d, h};
  };
  const int root = build(L).first;
  std::stable_sort(ops.begin(), ops.end(), [](const std::array<int, 4>& x, const std::array<int, 4>& y) { return x[0] < y[0]; });
  const int nlev = ops.empty() ? 0 : ops.back()[0];
  std::vector<int> prog = {nleaf, nlev, root};
  prog.insert(prog.end(), lo.begin(), lo.end());
  prog.insert(prog.end(), len.begin(), len.end());
  size_t k = 0;
  for (int h = 1; h <= nlev + 1; ++h) {  // lev_off[h - 1] = first op of height h
    prog.push_back((int)k);
    while (k < ops.size() && ops[k][0] == h) ++k;
  }
  for (const auto& o : ops) prog.insert(prog.end(), {o[1], o[2], o[3]});
  if (prog.size() > (size_t)NPX_PROG || next > 2 * NPX_MAXLEAF) std::abort();
  return prog;
}

// Running adds between full re-scans of a logit buffer (bounds the running
// sum's drift; each scan reads the whole buffer once).
constexpr int kLogitReseed = 4096;

int dqz_logit_buffer_create(int64_t capacity, int max_queries, dqz_logit_buffer** out) {
  if (!out || capacity < 1 || max_queries < 1) return fail(DQZ_ERR_INVALID, "bad logit buffer arguments");
  if (capacity > ((int64_t)INT32_MAX + 1) * SM_CHUNK / 2) return fail(DQZ_ERR_INVALID, "capacity too large");
  dqz_logit_buffer* b = new dqz_logit_buffer();
  b->capacity = capacity;
  b->max_queries = max_queries;
  b->nblocks = (int)((capacity + SM_CHUNK - 1) / SM_CHUNK);
  const size_t head = (size_t)b->nblocks * (sizeof(MaxSum) + sizeof(double) + sizeof(int));
  const size_t sync_off = (head + 64 + sizeof(LogitRun) + 255) / 256 * 256;
  b->nbuf = (int)((capacity + NPX_BUF - 1) / NPX_BUF);
  const size_t x_off = sync_off + 3 * SampleSync::kStride * sizeof(int);  // 256-aligned
  const size_t prog_off = (x_off + (size_t)b->nblocks * (sizeof(double) + sizeof(float)) + (size_t)b->nbuf * sizeof(float) +
                            64 + 255) / 256 * 256;
  const size_t bytes = prog_off + 2 * NPX_PROG * sizeof(int);
  if (hipMalloc(&b->block, bytes) != hipSuccess) {
    delete b;
    return fail(DQZ_ERR_HIP, "hipMalloc of logit scratch failed");
  }
  if (hipMemset(b->block, 0, bytes) != hipSuccess) {
    (void)hipFree(b->block);
    delete b;
    return fail(DQZ_ERR_HIP, "hipMemset of logit scratch failed");
  }
  char* p = (char*)b->block;
  b->csum = (double*)p;
  b->part = (MaxSum*)(p + (size_t)b->nblocks * sizeof(double));
  b->dirty = (int*)(p + (size_t)b->nblocks * (sizeof(double) + sizeof(MaxSum)));
  b->lse = (float*)(p + head);
  b->run = (LogitRun*)(p + head + 64);
  b->sync = (int*)(p + sync_off);
  b->csum_x = (double*)(p + x_off);
  b->part_x = (float*)(p + x_off + (size_t)b->nblocks * sizeof(double));
  b->bsum_x = b->part_x + b->nblocks;
  b->scal_x = b->bsum_x + b->nbuf;
  b->prog_full = (int*)(p + prog_off);
  b->prog_last = b->prog_full + NPX_PROG;
  {
    const std::vector<int> full = npx_program(NPX_BUF), last = npx_program((int)(capacity - (int64_t)(b->nbuf - 1) * NPX_BUF));
    if (hipMemcpy(b->prog_full, full.data(), full.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(b->prog_last, last.data(), last.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess) {
      (void)hipFree(b->block);
      delete b;
      return fail(DQZ_ERR_HIP, "hipMemcpy of the exact-mode programs failed");
    }
  }
  b->run_known = false;
  b->run_adds = 0;
  *out = b;
  return DQZ_OK;
}

int dqz_logit_buffer_destroy(dqz_logit_buffer* b) {
  if (!b) return DQZ_OK;
  if (b->block) (void)hipFree(b->block);
  delete b;
  return DQZ_OK;
}

// csum of the flagged chunks (dirty != null) or of all of them.
static int chunk_sums(dqz_logit_buffer* b, const float* logits, bool dirty_only, hipStream_t st) {
  hipLaunchKernelGGL(chunk_sums_kernel, dim3(b->nblocks), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run,
                     b->csum, dirty_only ? b->dirty : nullptr);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

// Full two-pass log-sum-exp over the buffer (re-seeds the running state),
// then every chunk sum about the new shift.
static int logits_lse(dqz_logit_buffer* b, float* logits, int64_t clear_pos, int64_t write_pos, int64_t size,
                      float* lse_out, hipStream_t st) {
  hipLaunchKernelGGL(lse_partial_kernel, dim3(b->nblocks), dim3(SM_THREADS), 0, st, logits, b->capacity, b->part,
                     clear_pos);
  DQZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(lse_final_kernel, dim3(1), dim3(SM_THREADS), 0, st, b->part, b->nblocks, lse_out ? lse_out : b->lse,
                     logits, write_pos, size, b->run);
  DQZ_HIP(hipGetLastError());
  if (int rc = chunk_sums(b, logits, false, st)) return rc;
  b->run_known = true;
  b->run_adds = 0;
  return DQZ_OK;
}

int dqz_logits_add(dqz_logit_buffer* b, float* logits, int64_t clear_pos, int64_t write_pos, int64_t size,
                   float* lse_out, void* stream) {
  if (!b || !logits) return fail(DQZ_ERR_INVALID, "null argument");
  if (write_pos < 0 || write_pos >= b->capacity || clear_pos >= b->capacity)
    return fail(DQZ_ERR_INVALID, "position out of range");
  if (size < 0) return fail(DQZ_ERR_INVALID, "size must be >= 0");
  hipStream_t st = (hipStream_t)stream;
  if (!b->run_known || b->run_adds >= kLogitReseed) {
    // the reservoir `replace` clear (logits[clear_pos] = -inf) happens inside pass 1
    if (int rc = logits_lse(b, logits, clear_pos, write_pos, size, lse_out, st)) return rc;
  } else {
    hipLaunchKernelGGL(logits_add_running_kernel, dim3(1), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run,
                       b->csum, clear_pos, write_pos, size, lse_out ? lse_out : b->lse);
    DQZ_HIP(hipGetLastError());
    ++b->run_adds;
  }
  if (lse_out) DQZ_HIP(hipMemcpyAsync(b->lse, lse_out, sizeof(float), hipMemcpyDeviceToDevice, st));
  return DQZ_OK;
}

int dqz_logits_write(dqz_logit_buffer* b, float* logits, const int64_t* positions, const float* values, int n,
                     void* stream) {
  if (!b || !logits || (n > 0 && (!positions || !values))) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 0) return fail(DQZ_ERR_INVALID, "n must be >= 0");
  if (n == 0) return DQZ_OK;
  hipStream_t st = (hipStream_t)stream;
  if (!b->run_known) {  // no running state to keep: write, and the next use re-seeds
    hipLaunchKernelGGL(logits_scatter_kernel, dim3(1), dim3(64), 0, st, logits, positions, values, n);
    DQZ_HIP(hipGetLastError());
    return DQZ_OK;
  }
  hipLaunchKernelGGL(logits_write_kernel, dim3(1), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run, b->dirty,
                     positions, values, n);
  DQZ_HIP(hipGetLastError());
  return chunk_sums(b, logits, true, st);
}

int dqz_logits_put(dqz_logit_buffer* b, float* logits, int64_t position, float value, void* stream) {
  if (!b || !logits) return fail(DQZ_ERR_INVALID, "null argument");
  if (position < 0 || position >= b->capacity) return fail(DQZ_ERR_INVALID, "position out of range");
  hipStream_t st = (hipStream_t)stream;
  if (!b->run_known) {
    hipLaunchKernelGGL(logits_scatter1_kernel, dim3(1), dim3(64), 0, st, logits, position, value);
    DQZ_HIP(hipGetLastError());
    return DQZ_OK;
  }
  hipLaunchKernelGGL(logits_put1_kernel, dim3(1), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run, b->csum,
                     position, value);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

__global__ void logits_run_set_kernel(LogitRun* run, LogitRun v) {
  if (threadIdx.x == 0) *run = v;
}

int dqz_logits_run_get(dqz_logit_buffer* b, double* S, float* c, int* valid, int* known, int* adds, void* stream) {
  if (!b || !S || !c || !valid || !known || !adds) return fail(DQZ_ERR_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  LogitRun r{0.0, 0.f, 0};
  DQZ_HIP(hipMemcpyAsync(&r, b->run, sizeof(LogitRun), hipMemcpyDeviceToHost, st));
  DQZ_HIP(hipStreamSynchronize(st));
  *S = r.S;
  *c = r.c;
  *valid = r.valid;
  *known = b->run_known ? 1 : 0;
  *adds = b->run_adds;
  return DQZ_OK;
}

int dqz_logits_run_set(dqz_logit_buffer* b, const float* logits, double S, float c, int valid, int known, int adds,
                       void* stream) {
  if (!b || !logits) return fail(DQZ_ERR_INVALID, "null argument");
  if (adds < 0) return fail(DQZ_ERR_INVALID, "adds must be >= 0");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(logits_run_set_kernel, dim3(1), dim3(64), 0, st, b->run, LogitRun{S, c, valid ? 1 : 0});
  DQZ_HIP(hipGetLastError());
  b->run_known = known != 0 && valid != 0;
  b->run_adds = adds;
  // the chunk sums are a function of (logits, c): the restored state's
  if (b->run_known) return chunk_sums(b, logits, false, st);
  return DQZ_OK;
}

int dqz_logits_invalidate(dqz_logit_buffer* b) {
  if (!b) return fail(DQZ_ERR_INVALID, "null argument");
  b->run_known = false;
  return DQZ_OK;
}

// The samplers use the running state and its chunk sums: seed both with a
// scan first when the host cannot vouch for them.
static int ensure_run(dqz_logit_buffer* b, const float* logits, hipStream_t st) {
  if (b->run_known) return DQZ_OK;
  return logits_lse(b, const_cast<float*>(logits), -1, -1, 0, nullptr, st);
}

static int logits_sample_impl(dqz_logit_buffer* b, const float* logits, uint64_t seed, uint64_t* counter_dev,
                              const double* uniforms, int n, int32_t* out_slots, int64_t* out_idx, hipStream_t st) {
  if (!b || !logits || (!uniforms && !counter_dev) || (!out_slots && !out_idx))
    return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 1 || n > 65535) return fail(DQZ_ERR_INVALID, "n out of range");
  if (out_slots && b->capacity > INT32_MAX) return fail(DQZ_ERR_INVALID, "int32 slots need capacity < 2^31");
  if (int rc = ensure_run(b, logits, st)) return rc;
  hipLaunchKernelGGL(softmax_sample_kernel, dim3(n), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run, b->csum,
                     b->nblocks, SampleSync{b->sync}, seed, counter_dev, uniforms, n, out_slots, out_idx);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_logits_sample(dqz_logit_buffer* b, const float* logits, const double* uniforms, int n, int64_t* out_idx,
                      void* stream) {
  if (!uniforms || !out_idx) return fail(DQZ_ERR_INVALID, "null argument");
  return logits_sample_impl(b, logits, 0, nullptr, uniforms, n, nullptr, out_idx, (hipStream_t)stream);
}

int dqz_logits_sample_slots(dqz_logit_buffer* b, const float* logits, uint64_t seed, uint64_t* counter_dev,
                            const double* uniforms, int n, int32_t* out_slots, int64_t* out_idx, void* stream) {
  return logits_sample_impl(b, logits, seed, counter_dev, uniforms, n, out_slots, out_idx, (hipStream_t)stream);
}

// numpy's float32 logsumexp of the whole buffer -> b->scal_x[1] (c in [0])
static int npx_lse(dqz_logit_buffer* b, const float* logits, hipStream_t st) {
  hipLaunchKernelGGL(npx_max_kernel, dim3(b->nblocks), dim3(SM_THREADS), 0, st, logits, b->capacity, b->part_x);
  DQZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(npx_cmax_kernel, dim3(1), dim3(SM_THREADS), 0, st, b->part_x, b->nblocks, b->scal_x);
  DQZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(npx_bufsum_kernel, dim3(b->nbuf), dim3(SM_THREADS), 0, st, logits, b->capacity, b->scal_x,
                     b->bsum_x, b->prog_full, b->prog_last);
  DQZ_HIP(hipGetLastError());
  hipLaunchKernelGGL(npx_lse_kernel, dim3(1), dim3(64), 0, st, b->bsum_x, b->nbuf, b->scal_x);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_logits_add_exact(dqz_logit_buffer* b, float* logits, int64_t clear_pos, int64_t write_pos, int64_t size,
                         void* stream) {
  if (!b || !logits) return fail(DQZ_ERR_INVALID, "null argument");
  if (write_pos < 0 || write_pos >= b->capacity || clear_pos >= b->capacity)
    return fail(DQZ_ERR_INVALID, "position out of range");
  if (size < 0) return fail(DQZ_ERR_INVALID, "size must be >= 0");
  hipStream_t st = (hipStream_t)stream;
  if (clear_pos >= 0) {
    hipLaunchKernelGGL(npx_clear_kernel, dim3(1), dim3(64), 0, st, logits, clear_pos);
    DQZ_HIP(hipGetLastError());
  }
  if (size > 0)
    if (int rc = npx_lse(b, logits, st)) return rc;
  hipLaunchKernelGGL(npx_add_kernel, dim3(1), dim3(64), 0, st, logits, write_pos, size, b->scal_x);
  DQZ_HIP(hipGetLastError());
  b->run_known = false;  // the running state did not follow this write
  return DQZ_OK;
}

int dqz_logits_sample_exact(dqz_logit_buffer* b, const float* logits, const double* uniforms, int n, int64_t* out_idx,
                            float* p_out, void* stream) {
  if (!b || !logits) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 0 || n > 65535) return fail(DQZ_ERR_INVALID, "n out of range");
  if (n > 0 && (!uniforms || !out_idx)) return fail(DQZ_ERR_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  if (int rc = npx_lse(b, logits, st)) return rc;
  hipLaunchKernelGGL(npx_chunk_kernel, dim3(b->nblocks), dim3(SM_THREADS), 0, st, logits, b->capacity, b->scal_x,
                     b->csum_x, p_out);
  DQZ_HIP(hipGetLastError());
  if (n > 0) {
    hipLaunchKernelGGL(npx_sample_kernel, dim3(n), dim3(SM_THREADS), 0, st, logits, b->capacity, b->scal_x, b->csum_x,
                       b->nblocks, uniforms, out_idx);
    DQZ_HIP(hipGetLastError());
  }
  return DQZ_OK;
}

int dqz_logits_probs(dqz_logit_buffer* b, const float* logits, float* p_out, float* lse_out, void* stream) {
  if (!b || !logits || !p_out) return fail(DQZ_ERR_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  if (int rc = ensure_run(b, logits, st)) return rc;
  hipLaunchKernelGGL(logit_terms_kernel, dim3(b->nblocks), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run,
                     b->csum, b->nblocks, p_out, (float*)nullptr, lse_out, (float*)nullptr);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_logits_terms(dqz_logit_buffer* b, const float* logits, float* t_out, double* csum_out, float* c_out,
                     void* stream) {
  if (!b || !logits || !t_out) return fail(DQZ_ERR_INVALID, "null argument");
  hipStream_t st = (hipStream_t)stream;
  if (int rc = ensure_run(b, logits, st)) return rc;
  hipLaunchKernelGGL(logit_terms_kernel, dim3(b->nblocks), dim3(SM_THREADS), 0, st, logits, b->capacity, b->run,
                     b->csum, b->nblocks, (float*)nullptr, t_out, (float*)nullptr, c_out);
  DQZ_HIP(hipGetLastError());
  if (csum_out)
    DQZ_HIP(hipMemcpyAsync(csum_out, b->csum, sizeof(double) * b->nblocks, hipMemcpyDeviceToDevice, st));
  return DQZ_OK;
}

int dqz_learner_step_logits(dqz_learner* L, const dqz_params* P, const dqz_store* S, dqz_logit_buffer* buf,
                            const float* logits, uint64_t seed, uint64_t* counter_dev, const double* uniforms,
                            int32_t* slots_out, void* stream) {
  if (!L || !buf || !logits || (!counter_dev && !uniforms) || !slots_out)
    return fail(DQZ_ERR_INVALID, "null argument");
  if (L->cfg.algo == DQZ_ALGO_PER) return fail(DQZ_ERR_INVALID, "PER samples by priority, not by learned logits");
  if (buf->capacity > INT32_MAX) return fail(DQZ_ERR_INVALID, "int32 slots need capacity < 2^31");
  hipStream_t st = (hipStream_t)stream;
  if (int rc = ensure_run(buf, logits, st)) return rc;
  SoftmaxDraw sm{logits, buf->capacity, buf->run, buf->csum, buf->nblocks,
                 seed,   uniforms ? nullptr : counter_dev,    uniforms,  slots_out};
  return step_impl(L, P, S, slots_out, nullptr, stream, kNoProfile, nullptr, nullptr, nullptr, 0, 0, nullptr, &sm);
}

int dqz_uniform_philox(uint64_t seed, uint64_t* counter_dev, int n, double* out, void* stream) {
  if (!counter_dev || !out || n < 1 || n > 65536) return fail(DQZ_ERR_INVALID, "bad argument");
  hipLaunchKernelGGL(philox_uniform_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, seed, counter_dev, n, out);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

static int tree_levels(int64_t cap) {
  int l = 0;
  while ((int64_t(1) << l) < cap) ++l;
  return l;
}

int dqz_sumtree_set(double* tree, int64_t cap, const int64_t* idx, const double* values, int n, void* stream) {
  if (!tree || !idx || !values) return fail(DQZ_ERR_INVALID, "null argument");
  if (cap < 1 || (cap & (cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two");
  if (n < 0 || n > 65536) return fail(DQZ_ERR_INVALID, "n out of range");
  if (n == 0) return DQZ_OK;
  const int levels = tree_levels(cap);
  if (n <= ST_FAST && levels <= 32)
    hipLaunchKernelGGL(sumtree_set_small_kernel, dim3(1), dim3(ST_FAST), 0, (hipStream_t)stream, tree, cap, levels,
                       idx, values, n);
  else
    hipLaunchKernelGGL(sumtree_set_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, tree, cap, levels, idx,
                       values, n);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_per_write_back(dqz_learner* L, double* tree, int64_t cap, const int32_t* slots, double alpha,
                       double* max_seen_dev, void* stream) {
  if (!L || !tree || !slots || !max_seen_dev) return fail(DQZ_ERR_INVALID, "null argument");
  if (cap < 1 || (cap & (cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two");
  const int n = L->cfg.batch;
  const int levels = tree_levels(cap);
  if (n > ST_FAST || levels > 32) return fail(DQZ_ERR_INVALID, "batch must be <= %d and cap <= 2^32", ST_FAST);
  hipLaunchKernelGGL(per_write_back_kernel, dim3(1), dim3(ST_FAST), 0, (hipStream_t)stream, tree, cap, levels, slots,
                     L->td, alpha, n, max_seen_dev);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_sumtree_query(const double* tree, int64_t cap, const double* targets, int n, int64_t* out, void* stream) {
  if (!tree || !targets || !out) return fail(DQZ_ERR_INVALID, "null argument");
  if (cap < 1 || (cap & (cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two");
  if (n < 0) return fail(DQZ_ERR_INVALID, "n must be >= 0");
  if (n == 0) return DQZ_OK;
  hipLaunchKernelGGL(sumtree_query_kernel, dim3((n + 7) / 8), dim3(256), 0, (hipStream_t)stream, tree, cap,
                     tree_levels(cap), targets, n, out);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_per_sample(const double* tree, int64_t cap, int64_t live_base, int64_t size, int64_t capacity, int n,
                   double usp, double beta, int normalize, uint64_t seed, uint64_t* counter_dev,
                   const int32_t* injected_uniform, const double* injected_u, const int32_t* index_to_slot,
                   int32_t* out_indices, int32_t* out_slots, float* out_weights, double* out_probs, void* stream) {
  if (!tree || !out_slots || !out_weights) return fail(DQZ_ERR_INVALID, "null argument");
  if (!injected_u && !counter_dev) return fail(DQZ_ERR_INVALID, "Philox draws need counter_dev");
  if ((injected_u == nullptr) != (injected_uniform == nullptr))
    return fail(DQZ_ERR_INVALID, "injected_uniform and injected_u go together");
  if (cap < capacity || (cap & (cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two >= capacity");
  if (size < 1) return fail(DQZ_ERR_INVALID, "No IDs to sample.");
  if (n < 1 || n > 1024) return fail(DQZ_ERR_INVALID, "n must be in [1, 1024]");
  if (!(beta >= 0.0 && beta <= 1.0)) return fail(DQZ_ERR_INVALID, "Require 0 <= exponent <= 1.");
  if (!(usp >= 0.0 && usp <= 1.0)) return fail(DQZ_ERR_INVALID, "Require 0 <= uniform_sample_probability <= 1.");
  PerSampleArgs a{};
  a.tree = tree;
  a.cap = cap;
  a.levels = tree_levels(cap);
  a.live_base = live_base;
  a.size = size;
  a.capacity = capacity;
  a.n = n;
  a.usp = usp;
  a.beta = beta;
  a.normalize = normalize;
  a.seed = seed;
  a.counter = counter_dev;
  a.inj_uniform = injected_uniform;
  a.inj_u = injected_u;
  a.index_to_slot = index_to_slot;
  a.out_indices = out_indices;
  a.out_slots = out_slots;
  a.out_weights = out_weights;
  a.out_probs = out_probs;
  hipLaunchKernelGGL(per_sample_kernel, dim3(1), dim3(1024), 0, (hipStream_t)stream, a);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_learner_step_per_draw(dqz_learner* L, const dqz_params* P, const dqz_store* S, const dqz_per_draw* d,
                              void* stream) {
  if (!L || !d || !d->tree || !d->out_indices || !d->out_slots || !d->out_probs || !d->max_seen_dev)
    return fail(DQZ_ERR_INVALID, "null argument");
  if (L->cfg.algo != DQZ_ALGO_PER) return fail(DQZ_ERR_INVALID, "the learner is not a PER learner");
  if (!d->injected_u && !d->counter_dev) return fail(DQZ_ERR_INVALID, "Philox draws need counter_dev");
  if ((d->injected_u == nullptr) != (d->injected_uniform == nullptr))
    return fail(DQZ_ERR_INVALID, "injected_uniform and injected_u go together");
  if (d->cap < d->capacity || (d->cap & (d->cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two >= capacity");
  if (d->size < 1) return fail(DQZ_ERR_INVALID, "No IDs to sample.");
  const double beta = d->importance_sampling_exponent, usp = d->uniform_sample_probability;
  if (!(beta >= 0.0 && beta <= 1.0)) return fail(DQZ_ERR_INVALID, "Require 0 <= exponent <= 1.");
  if (!(usp >= 0.0 && usp <= 1.0)) return fail(DQZ_ERR_INVALID, "Require 0 <= uniform_sample_probability <= 1.");
  const int levels = tree_levels(d->cap);
  if (L->cfg.batch > 64 || levels > PWB_LEVELS)
    return fail(DQZ_ERR_INVALID, "the fused PER step takes batch <= 64 and cap <= 2^%d", PWB_LEVELS);
  PerSampleArgs a{};
  a.tree = d->tree;
  a.cap = d->cap;
  a.levels = levels;
  a.live_base = d->live_base;
  a.size = d->size;
  a.capacity = d->capacity;
  a.n = L->cfg.batch;
  a.usp = usp;
  a.beta = beta;
  a.normalize = d->normalize_weights;
  a.seed = d->seed;
  a.counter = d->counter_dev;
  a.inj_uniform = d->injected_uniform;
  a.inj_u = d->injected_u;
  a.index_to_slot = d->index_to_slot;
  a.out_indices = d->out_indices;
  a.out_slots = d->out_slots;
  a.out_weights = d->out_weights;
  a.out_probs = d->out_probs;
  PerWbArgs wb{d->tree, d->cap, levels, d->out_indices, nullptr, d->alpha, 0, d->max_seen_dev};
  return step_impl(L, P, S, d->out_slots, nullptr, stream, kNoProfile, nullptr, nullptr, nullptr, 0, 0, &wb, nullptr,
                   &a);
}

int dqz_per_add(double* tree, int64_t cap, int32_t remove_index, int32_t add_index, double priority,
                const double* max_seen_dev, double alpha, int32_t* index_to_slot, int32_t slot, void* stream) {
  if (!tree) return fail(DQZ_ERR_INVALID, "null tree");
  if (cap < 1 || (cap & (cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two");
  const int levels = tree_levels(cap);
  if (levels > 32) return fail(DQZ_ERR_INVALID, "cap must be <= 2^32");
  if (add_index < 0 || add_index >= cap || remove_index >= cap) return fail(DQZ_ERR_INVALID, "index out of range");
  if (priority < 0.0 && !max_seen_dev) return fail(DQZ_ERR_INVALID, "priority < 0 needs max_seen_dev");
  if (priority >= 0.0 && !std::isfinite(priority)) return fail(DQZ_ERR_INVALID, "value must be finite and positive.");
  if (alpha < 0.0) return fail(DQZ_ERR_INVALID, "Require priority_exponent >= 0.");
  hipLaunchKernelGGL(per_add_kernel, dim3(1), dim3(ST_FAST), 0, (hipStream_t)stream, tree, cap, levels, remove_index,
                     add_index, priority, max_seen_dev, alpha, index_to_slot, slot);
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_target_copy(float* target, const float* online, int64_t total, void* stream) {
  if (!target || !online || total < 0) return fail(DQZ_ERR_INVALID, "bad argument");
  DQZ_HIP(hipMemcpyAsync(target, online, total * sizeof(float), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return DQZ_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// MGSC meta-update (meta.hpp)


struct dqz_meta {
  dqz_meta_config cfg;
  // Meta batches larger than the learner's MAXB run in K chunks of C samples
  // (the last one padded with p = 0 samples): G accumulates over the chunks,
  // and once v is known each chunk's backward signals are recomputed for the
  // tangent pass (K = 1 keeps them from the first pass).
  int C, K;
  dqz_learner* lm;   // meta batch learner (B = C)
  dqz_learner* l1;   // one-transition learner (B = 1)
  int64_t total;
  float *G, *thp, *mu1, *nu1, *J;  // [total] each; G also holds g', thp also holds v
  float *zv1, *zv2, *zv3, *zvp;    // tangent forward outputs
  float *x, *p, *s, *dl, *loss, *loss_part, *td;  // p, s, td: [K C] (p = 0 past M)
  int32_t* slots_pad;                                // [K C]
  float* Gs;                                         // [total] scratch gradient of the recompute pass (K > 1)
  int nparts;
  // second-order (reservoir) meta-gradient
  float *GQ, *HQ, *s1_part, *hpart;
  float *ty1, *ty2, *ty3, *td4, *td3, *td2, *td1, *s1;
  uint8_t* x1;  // [4][84][84] the online transition's s_tm1 bytes (written by the theta' forward)
  float* dotp;  // [C][META_DOT_SLOTS] the tangent launch's dot-product partials (one chunk)
  int* arrive;  // (x Handoff::kStride) [0] meta_adam_chunks_kernel's re-seed arrival counter, [1, 3) the
                // HVP's ddot1 hand-off words, [3] the Adam entry counter (all zero between launches),
                // [4] the meta-level error word (dqz_meta_sync_status)
  unsigned spin_max = 1u << 24;  // polls before the Adam leader's entry wait gives up
  int nparts2;
  void* block;
};

extern "C" {

int dqz_meta_create(const dqz_meta_config* cfg, dqz_meta** out) {
  if (!cfg || !out) return fail(DQZ_ERR_INVALID, "null argument");
  if (cfg->meta_batch < 1 || cfg->meta_batch > (1 << 26))
    return fail(DQZ_ERR_INVALID, "meta_batch must be in [1, 2^26]");
  if (int rc = init_meta_attrs()) return rc;
  const int C = std::min(cfg->meta_batch, MAXB), K = (cfg->meta_batch + C - 1) / C;
  dqz_learner_config lc;
  lc.batch = C;
  lc.num_actions = cfg->num_actions;
  lc.algo = DQZ_ALGO_DQN;
  lc.learning_rate = cfg->learning_rate;
  lc.decay = cfg->decay;
  lc.eps = cfg->eps;
  lc.grad_error_bound = cfg->grad_error_bound;
  dqz_meta* H = new dqz_meta();
  H->cfg = *cfg;
  H->C = C;
  H->K = K;
  if (int rc = dqz_learner_create(&lc, &H->lm)) {
    delete H;
    return rc;
  }
  lc.batch = 1;
  if (int rc = dqz_learner_create(&lc, &H->l1)) {
    dqz_learner_destroy(H->lm);
    delete H;
    return rc;
  }
  const int M = cfg->meta_batch;
  const int64_t KC = (int64_t)K * C, multi = K > 1 ? 1 : 0;
  H->total = H->lm->total;
  H->nparts = (int)((H->total / 4 + 255) / 256);
  H->nparts2 = (int)((H->total + 255) / 256);
  const int64_t so = cfg->second_order ? 1 : 0;
  const int64_t sizes[] = {H->total, H->total, H->total, H->total, H->total,
                           (int64_t)C * C1M * C1CO, (int64_t)C * C2M * C2CO, (int64_t)C * FLAT,
                           (int64_t)H->lm->S_fc1 * C * HID,
                           M, KC, KC, M, 1, H->nparts2, KC, KC, multi * H->total,
                           so * H->total, so * H->total, so * H->nparts2,
                           so * C1M * C1CO, so * C2M * C2CO, so * FLAT, so * HID, so * FLAT,
                           so * C2M * C2CO, so * C1M * C1CO, so, so * HVP_T4_CHUNKS * HID,
                           (int64_t)C * META_DOT_SLOTS, 5 * Handoff::kStride, so * FC * FB / 4};
  float** ptrs[] = {&H->G, &H->thp, &H->mu1, &H->nu1, &H->J, &H->zv1, &H->zv2, &H->zv3, &H->zvp,
                    &H->x, &H->p, &H->s, &H->dl, &H->loss, &H->loss_part, &H->td,
                    reinterpret_cast<float**>(&H->slots_pad), &H->Gs,
                    &H->GQ, &H->HQ, &H->s1_part,
                    &H->ty1, &H->ty2, &H->ty3, &H->td4, &H->td3, &H->td2, &H->td1, &H->s1, &H->hpart,
                    &H->dotp, reinterpret_cast<float**>(&H->arrive), reinterpret_cast<float**>(&H->x1)};
  static_assert(sizeof(sizes) / sizeof(sizes[0]) == sizeof(ptrs) / sizeof(ptrs[0]), "meta scratch table");
  int64_t tot = 0;
  for (int64_t n : sizes) tot += (n + 63) / 64 * 64;
  if (hipMalloc(&H->block, tot * sizeof(float)) != hipSuccess || hipMemset(H->block, 0, tot * sizeof(float)) != hipSuccess) {
    if (H->block) (void)hipFree(H->block);
    dqz_learner_destroy(H->lm);
    dqz_learner_destroy(H->l1);
    delete H;
    return fail(DQZ_ERR_HIP, "hipMalloc of %lld bytes of meta scratch failed", (long long)(tot * 4));
  }
  float* q = (float*)H->block;
  for (size_t i = 0; i < sizeof(sizes) / sizeof(sizes[0]); ++i) {
    *ptrs[i] = q;
    q += (sizes[i] + 63) / 64 * 64;
  }
  *out = H;
  return DQZ_OK;
}

int dqz_meta_destroy(dqz_meta* H) {
  if (!H) return DQZ_OK;
  dqz_learner_destroy(H->lm);
  dqz_learner_destroy(H->l1);
  if (H->block) (void)hipFree(H->block);
  delete H;
  return DQZ_OK;
}

int dqz_meta_update(dqz_meta* H, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                    const dqz_store* S1, const int32_t* online_slot, float* logits, const int32_t* pos,
                    float* adam_mu, float* adam_nu, int32_t* adam_count, dqz_logit_buffer* logit_buf,
                    void* stream) {
  if (!H || !P || !P->online || !P->target || !P->mu || !P->nu || !slots || !online_slot || !logits || !pos ||
      !adam_mu || !adam_nu || !adam_count)
    return fail(DQZ_ERR_INVALID, "null argument");
  if (int rc = check_store(S)) return rc;
  if (int rc = check_store(S1)) return rc;
  hipStream_t st = (hipStream_t)stream;
  dqz_learner* L = H->lm;
  const int M = H->cfg.meta_batch, A = H->cfg.num_actions;

  const int C = H->C, K = H->K;

  // p = softmax(logits[pos]); slots padded to K C with slots[M - 1] (p = 0
  // there).  One chunk (K C = M): no padding, and the batch learner's head
  // forms p itself (HeadArgs::meta_logits), so no launch of its own.
  const int32_t* mslots = K == 1 ? slots : H->slots_pad;
  if (K > 1) {
    hipLaunchKernelGGL(meta_softmax_kernel, dim3(1 + (unsigned)((K * C + META_THREADS - 1) / META_THREADS)),
                       dim3(META_THREADS), 0, st, logits, pos, M, H->x, H->p, slots, K * C, H->slots_pad);
    DQZ_HIP(hipGetLastError());
  }

  // G = sum_i p_i g_i: batched backwards with p-weighted cotangents, one per
  // chunk of C samples, accumulated in chunk order (deterministic).  With one
  // chunk, meta_rms1 (theta' = theta + u(G), mu', nu', J) runs in the
  // backward's gradient epilogues (Rms::meta1) instead of its own launch; G
  // itself is stored only for the second order (meta_second_kernel reads it).
  const bool so = H->cfg.second_order != 0;
  Rms epi{};
  epi.thp = H->thp;
  epi.mu1 = H->mu1;
  epi.nu1 = H->nu1;
  epi.J = H->J;
  epi.sq_part = H->loss_part;
  if (K == 1) {
    epi.meta = 1;
    HeadArgs msm{};
    msm.meta_logits = logits;
    msm.meta_pos = pos;
    msm.meta_M = M;
    msm.meta_x_out = H->x;
    msm.meta_p_out = H->p;
    if (int rc = step_impl(L, P, S, mslots, nullptr, stream, kNoProfile, so ? H->G : nullptr, H->p, nullptr, 0, 0,
                           nullptr, nullptr, nullptr, &epi, &msm))
      return rc;
    // (the batch learner's td stays current until the next update,
    // dqz_meta_outputs copies it from there)
  } else {
    for (int k = 0; k < K; ++k) {
      if (int rc = step_impl(L, P, S, H->slots_pad + (int64_t)k * C, nullptr, stream, kNoProfile, H->G,
                             H->p + (int64_t)k * C, nullptr, 0, k > 0 ? 1 : 0))
        return rc;
      DQZ_HIP(hipMemcpyAsync(H->td + (int64_t)k * C, L->td, sizeof(float) * C, hipMemcpyDeviceToDevice, st));
    }
  }

  MetaRmsArgs ra{};
  ra.lr = H->cfg.learning_rate;
  ra.decay = H->cfg.decay;
  ra.c1 = (float)(1.0 - (double)H->cfg.decay);
  ra.eps = H->cfg.eps;
  ra.n4 = H->total / 4;
  const dim3 eg((unsigned)((ra.n4 + 255) / 256));
  if (K > 1) {
    hipLaunchKernelGGL(meta_rms1_kernel, eg, dim3(256), 0, st, ra, (const float4*)H->G, (const float4*)P->online,
                       (const float4*)P->mu, (const float4*)P->nu, (float4*)H->thp, (float4*)H->mu1,
                       (float4*)H->nu1, (float4*)H->J);
    DQZ_HIP(hipGetLastError());
  }

  dqz_params P1;
  P1.online = H->thp;
  P1.target = P->online;
  P1.mu = nullptr;
  P1.nu = nullptr;
  int nloss = H->nparts;
  const float* v = H->thp;
  if (!so) {
    // g' = grad loss_fn(theta', target = theta, online transition), consumed
    // where it is formed by meta_rms2 (Rms::meta2): v = -2 u' du/dG -> the G
    // buffer (free in the first order), per-block partial sums of u'^2 (the
    // fc1 dW blocks' then the update's).
    epi.meta = 2;
    epi.vout = H->G;
    if (int rc = step_impl(H->l1, &P1, S1, online_slot, nullptr, stream, kNoProfile, nullptr, nullptr, nullptr, 0, 0,
                           nullptr, nullptr, nullptr, &epi))
      return rc;
    v = H->G;
    nloss = 4 * (FLAT / 16) + (int)update_blocks(H->l1->sz, A, H->l1->shared_bias ? 1 : A);
  } else {
    // grad q[a] at theta' (unit cotangent) -> GQ; the one-sample learner keeps
    // the primal activations, the unit-cotangent backward signals and td'.
    dqz_learner* L1 = H->l1;
    // ... consumed where it is formed (Rms::meta3, meta_second_kernel's
    // stage): v_dir -> mu1, w -> nu1, block sums of u'^2 and grad q . w
    epi.meta = 3;
    epi.G2 = H->G;
    epi.td = L1->td;
    epi.bound = H->cfg.grad_error_bound;
    epi.s1_part = H->s1_part;
    if (int rc = step_impl(L1, &P1, S1, online_slot, nullptr, stream, kNoProfile, H->GQ, nullptr, nullptr, 1, 0,
                           nullptr, nullptr, nullptr, &epi, nullptr, H->x1))
      return rc;
    const int nparts1 = 4 * (FLAT / 16) + (int)update_blocks(L1->sz, A, L1->shared_bias ? 1 : A);
    HvpArgs hv{};
    hv.x = H->x1;
    hv.rec = reinterpret_cast<const float4*>(L1->rec);
    hv.th = H->thp;
    hv.tw = H->nu1;
    for (int i = 0; i < 10; ++i) hv.off[i] = L1->off[i];
    hv.A = A;
    hv.y1 = L1->y1;
    hv.y2 = L1->y2;
    hv.y3 = L1->y3;
    hv.h = L1->h1;
    hv.d1 = L1->dy1;
    hv.d2 = L1->dy2;
    hv.d3 = L1->dy3;
    hv.d4 = L1->dz1;
    hv.ty1 = H->ty1;
    hv.ty2 = H->ty2;
    hv.ty3 = H->ty3;
    hv.td4 = H->td4;
    hv.td3 = H->td3;
    hv.td2 = H->td2;
    hv.td1 = H->td1;
    hv.hq = H->HQ;
    hv.part = H->hpart;
    hv.s1_part = H->s1_part;
    hv.s1_nparts = nparts1;
    hv.s1 = H->s1;
    // meta_combine in hvp_g's epilogue: v = v_dir + J (alpha s1 grad q -
    // clip(td') H w) -> thp (theta' is no longer needed)
    hv.vdir = H->mu1;
    hv.J = H->J;
    hv.gq = H->GQ;
    hv.td = L1->td;
    hv.bound = H->cfg.grad_error_bound;
    hv.vout = H->thp;
    // ddot1's in-launch hand-off: words after the Adam re-seed counter, the
    // one-transition learner's error word (dqz_learner_sync_status)
    hv.td1_pub = Handoff{H->arrive + Handoff::kStride, H->arrive + 2 * Handoff::kStride,
                         L1->sync + 16 * Handoff::kStride, HVP_B1, HVP_G_C1, L1->spin_max};
    // three launches (hvp.hpp): the tangent forward and backward side by
    // side, then the parameter blocks of H_q w
    hipLaunchKernelGGL(hvp_l1_kernel, dim3(HVP_L1_BLOCKS), dim3(256), 0, st, hv);
    hipLaunchKernelGGL(hvp_l2_kernel, dim3(HVP_L2_BLOCKS), dim3(256), 0, st, hv);
    hipLaunchKernelGGL(hvp_l3_kernel, dim3(HVP_L3_BLOCKS), dim3(256), 0, st, hv);
    DQZ_HIP(hipGetLastError());
    nloss = nparts1;
  }

  // Tangent forward over the stored online activations: V * y + vb per layer,
  // chunk by chunk (K > 1: the chunk's forward / backward is recomputed first
  // so L holds its activations and p-weighted backward signals).
  NetZ nv{};
  nv.p[0] = nv.p[1] = nv.p[2] = v;
  nv.which[0] = nv.which[1] = nv.which[2] = 0;
  for (int k = 0; k < K; ++k) {
    const int32_t* ks = mslots + (int64_t)k * C;
    if (K > 1) {
      if (int rc = step_impl(L, P, S, ks, nullptr, stream, kNoProfile, H->Gs, H->p + (int64_t)k * C)) return rc;
    }
    Conv1FwdArgs c1{};
    c1.src = Conv1Src{S->frames, S->fidx, ks, nullptr, 0, UniformDraw{}};
    c1.nz = nv;
    c1.w_off = L->off[0];
    c1.b_off = L->off[1];
    c1.B = C;
    c1.Z = 1;
    c1.linear = 1;
    c1.out = H->zv1;
    LayerFwdArgs c2{};
    c2.in = L->y1;
    c2.nz = nv;
    c2.w_off = L->off[2];
    c2.b_off = L->off[3];
    c2.B = C;
    c2.Z = 1;
    c2.linear = 1;
    c2.out = H->zv2;
    LayerFwdArgs c3 = c2;
    c3.in = L->y2;
    c3.w_off = L->off[4];
    c3.b_off = L->off[5];
    c3.out = H->zv3;
    Fc1FwdArgs f1{};
    f1.in = L->y3;
    f1.nz = nv;
    f1.w_off = L->off[6];
    f1.B = C;
    f1.MG = (C + 31) / 32;
    f1.part = H->zvp;
    MetaExtra ex{};
    if (K == 1) {  // dot products in the tangent epilogues (meta.hpp)
      c1.dot = TangentDot{L->dy1, H->dotp, 0};
      c2.dot = TangentDot{L->dy2, H->dotp, 4};
      c3.dot = TangentDot{L->dy3, H->dotp, 8};
      f1.dot = TangentDot{L->dz1, H->dotp, 12};
      ex = MetaExtra{L->dz1, L->h1, L->gq, L->ga, v, L->off[7], L->off[8], L->off[9], A, H->dotp};
    }
    if (K == 1) {
      // the conv layers' dot products from the batch backward's per-sample
      // gradient slabs, beside the fc1 tangent range (meta.hpp SlabDotArgs)
      SlabDotArgs sd{};
      sd.p1 = L->p1;
      sd.p2 = L->p2;
      sd.p3 = L->p3;
      sd.v = v;
      sd.off1 = L->off[0];
      sd.off2 = L->off[2];
      sd.off3 = L->off[4];
      sd.part = H->dotp;
      sd.M = C;
      hipLaunchKernelGGL(tangent_slab_kernel, dim3((unsigned)tangent_slab_blocks(C, f1.MG)), dim3(256), 0, st, sd,
                         f1, ex);
      DQZ_HIP(hipGetLastError());
      break;
    }
    // the four layers' tangent outputs are independent: one launch
    hipLaunchKernelGGL(tangent_fwd_kernel, dim3((unsigned)tangent_fwd_blocks(C, f1.MG)), dim3(256), kConv1FwdSmem,
                       st, c1, c2, c3, f1, ex);
    DQZ_HIP(hipGetLastError());
    if (K == 1) break;

    MetaDotArgs md{};
    md.dy1 = L->dy1;
    md.dy2 = L->dy2;
    md.dy3 = L->dy3;
    md.dz1 = L->dz1;
    md.gq = L->gq;
    md.ga = L->ga;
    md.zv1 = H->zv1;
    md.zv2 = H->zv2;
    md.zv3 = H->zv3;
    md.zvp = H->zvp;
    md.S = FC1_S;
    md.M = C;
    md.A = A;
    md.v = v;
    md.b1_off = L->off[7];
    md.w2_off = L->off[8];
    md.b2_off = L->off[9];
    md.h1 = L->h1;
    md.s_out = H->s + (int64_t)k * C;
    hipLaunchKernelGGL(meta_dot_kernel, dim3(C), dim3(256), 0, st, md);
    DQZ_HIP(hipGetLastError());
  }

  MetaAdamArgs ad{};
  ad.x = H->x;
  ad.p = H->p;
  ad.s = H->s;
  ad.dot_part = K == 1 ? H->dotp : nullptr;
  ad.s_out = H->s;
  ad.M = M;
  ad.logits = logits;
  ad.pos = pos;
  ad.m = adam_mu;
  ad.v = adam_nu;
  ad.count = adam_count;
  ad.lr = H->cfg.meta_learning_rate;
  ad.b1 = H->cfg.b1;
  ad.b2 = H->cfg.b2;
  ad.eps = H->cfg.meta_eps;
  ad.loss_part = H->loss_part;
  ad.nparts = nloss;
  ad.loss = H->loss;
  ad.dlogits = H->dl;
  // keep the buffer's running log-sum-exp current (the host keeps vouching
  // for it: every write went through the library)
  const bool keep = logit_buf && logit_buf->run_known;
  ad.run = keep ? logit_buf->run : nullptr;
  ad.dirty = keep ? logit_buf->dirty : nullptr;
  ad.n_logits = keep ? logit_buf->capacity : 0;
  // (the fused form's re-seed path addresses the buffer with 32-bit byte offsets)
  if (keep && K == 1 && M <= META_THREADS && logit_buf->capacity * 4 <= INT32_MAX) {
    // Adam and the re-sums of the chunks it writes in one launch
    MetaAdamChunks ck{logit_buf->csum, logit_buf->nblocks, H->arrive, H->arrive + 3 * Handoff::kStride,
                      H->arrive + 4 * Handoff::kStride, H->spin_max};
    hipLaunchKernelGGL(meta_adam_chunks_kernel, dim3(logit_buf->nblocks), dim3(META_THREADS), 0, st, ad, ck);
    DQZ_HIP(hipGetLastError());
    return DQZ_OK;
  }
  hipLaunchKernelGGL(meta_adam_kernel, dim3(1), dim3(META_THREADS), 0, st, ad);
  DQZ_HIP(hipGetLastError());
  if (keep) return chunk_sums(logit_buf, logits, true, st);
  return DQZ_OK;
}

int dqz_meta_sync_status(dqz_meta* H, int* status) {
  if (!H || !status) return fail(DQZ_ERR_INVALID, "null argument");
  int s_lm = 0, s_l1 = 0, s_own = 0;
  // (each learner's check clears that learner's words when its word is set)
  if (int rc = dqz_learner_sync_status(H->lm, &s_lm)) return rc;
  if (int rc = dqz_learner_sync_status(H->l1, &s_l1)) return rc;
  DQZ_HIP(hipMemcpy(&s_own, H->arrive + 4 * Handoff::kStride, sizeof(int), hipMemcpyDeviceToHost));
  *status = s_lm | s_l1 | s_own;
  if (*status != 0) {
    // a wait gave up somewhere in the meta-update: late arrivals may have
    // left counts behind after a reset, so clear every word the meta handle
    // owns (its learners' words are cleared just above only when their own
    // word is set: the HVP's ddot1 timeout lands in l1's word)
    DQZ_HIP(hipMemset(H->arrive, 0, sizeof(int) * 5 * Handoff::kStride));
    for (dqz_learner* L : {H->lm, H->l1})
      DQZ_HIP(hipMemset(L->sync, 0, sizeof(int) * ((16 * L->cfg.batch + 3) * Handoff::kStride + 64)));
    DQZ_HIP(hipDeviceSynchronize());
  }
  return DQZ_OK;
}

int dqz_meta_debug_stall(dqz_meta* H, int poison, unsigned spin_max) {
  if (!H) return fail(DQZ_ERR_INVALID, "null meta handle");
  const unsigned sm = spin_max ? spin_max : 1u << 24;
  H->spin_max = sm;
  H->lm->spin_max = sm;
  H->l1->spin_max = sm;
  if (poison) {
    const int32_t p = -(1 << 30);
    DQZ_HIP(hipDeviceSynchronize());
    DQZ_HIP(hipMemcpy(H->arrive + Handoff::kStride, &p, sizeof(p), hipMemcpyHostToDevice));      // ddot1 cnt
    DQZ_HIP(hipMemcpy(H->arrive + 3 * Handoff::kStride, &p, sizeof(p), hipMemcpyHostToDevice));  // Adam entry
  }
  return DQZ_OK;
}

int dqz_meta_outputs(dqz_meta* H, float* probs, float* dlogits, float* td, float* loss, void* stream) {
  if (!H) return fail(DQZ_ERR_INVALID, "null meta handle");
  hipStream_t st = (hipStream_t)stream;
  const int M = H->cfg.meta_batch;
  if (probs) DQZ_HIP(hipMemcpyAsync(probs, H->p, sizeof(float) * M, hipMemcpyDeviceToDevice, st));
  if (dlogits) DQZ_HIP(hipMemcpyAsync(dlogits, H->dl, sizeof(float) * M, hipMemcpyDeviceToDevice, st));
  if (td)
    DQZ_HIP(hipMemcpyAsync(td, H->K > 1 ? H->td : H->lm->td, sizeof(float) * M, hipMemcpyDeviceToDevice, st));
  if (loss) DQZ_HIP(hipMemcpyAsync(loss, H->loss, sizeof(float), hipMemcpyDeviceToDevice, st));
  return DQZ_OK;
}

}  // extern "C"

#ifdef DQZ_TRACE
// Diagnostic builds only (not part of include/dqz.h): copy / clear this
// code object's in-kernel timeline stamps (the HVP's; common.hpp DQZ_STAMP).
extern "C" int dqz_debug_trace_other(unsigned long long* host_out, int clear) {
  const size_t bytes = sizeof(unsigned long long) * TRACE_KERNELS * TRACE_BLOCKS * TRACE_SLOTS;
  if (host_out) DQZ_HIP(hipMemcpyFromSymbol(host_out, HIP_SYMBOL(g_dqz_trace), bytes));
  if (clear) {
    void* p = nullptr;
    DQZ_HIP(hipGetSymbolAddress(&p, HIP_SYMBOL(g_dqz_trace)));
    DQZ_HIP(hipMemset(p, 0, bytes));
  }
  return DQZ_OK;
}
#endif

// ---------------------------------------------------------------------------
// Atari observation preprocessing (processors.py:488-497)

struct dqz_frame_plan {
  FramePlan p{};
  void* block;
};

// Pillow's precompute_coeffs + normalize_coeffs_8bpc for the BILINEAR
// filter (support 1) on one axis with box (0, in_size): bounds[2 * o] =
// first source index, bounds[2 * o + 1] = count; k[o * ksize + i] = int32
// weights with 22 fractional bits.
static int pil_bilinear_coeffs(int in_size, int out_size, std::vector<int32_t>& bounds, std::vector<int32_t>& k) {
  const double scale = (double)((float)in_size - 0.0f) / out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const int ksize = (int)std::ceil(support) * 2 + 1;
  const double ss = 1.0 / filterscale;
  bounds.assign(2 * out_size, 0);
  k.assign((size_t)out_size * ksize, 0);
  std::vector<double> w(ksize);
  for (int xx = 0; xx < out_size; ++xx) {
    const double center = 0.0 + (xx + 0.5) * scale;
    int xmin = (int)(center - support + 0.5);
    if (xmin < 0) xmin = 0;
    int xmax = (int)(center + support + 0.5);
    if (xmax > in_size) xmax = in_size;
    xmax -= xmin;
    double ww = 0.0;
    for (int x = 0; x < xmax; ++x) {
      double t = (x + xmin - center + 0.5) * ss;
      if (t < 0.0) t = -t;
      w[x] = t < 1.0 ? 1.0 - t : 0.0;
      ww += w[x];
    }
    for (int x = 0; x < xmax; ++x) {
      const double v = ww != 0.0 ? w[x] / ww : w[x];
      k[(size_t)xx * ksize + x] = v < 0 ? (int32_t)(-0.5 + v * (1 << FR_PREC)) : (int32_t)(0.5 + v * (1 << FR_PREC));
    }
    bounds[2 * xx] = xmin;
    bounds[2 * xx + 1] = xmax;
  }
  return ksize;
}

extern "C" {

int dqz_frame_plan_create(int in_h, int in_w, int out_h, int out_w, dqz_frame_plan** out) {
  if (!out) return fail(DQZ_ERR_INVALID, "null argument");
  if (in_h < 1 || in_w < 1 || out_h < 1 || out_w < 1 || in_h > 4096 || in_w > 4096 || out_h > 4096 || out_w > 4096)
    return fail(DQZ_ERR_INVALID, "frame sizes must be in [1, 4096]");
  std::vector<int32_t> hb, hk, vb, vk;
  const int kh = pil_bilinear_coeffs(in_w, out_w, hb, hk);
  const int kv = pil_bilinear_coeffs(in_h, out_h, vb, vk);
  int max_band = 0;
  for (int yy0 = 0; yy0 < out_h; yy0 += FR_ROWS) {
    const int yy1 = std::min(yy0 + FR_ROWS, out_h);
    max_band = std::max(max_band, vb[2 * (yy1 - 1)] + vb[2 * (yy1 - 1) + 1] - vb[2 * yy0]);
  }
  const size_t smem = (size_t)max_band * (in_w + out_w);
  if (smem > 64 * 1024) return fail(DQZ_ERR_INVALID, "frame too large for one workgroup's band (%zu B of LDS)", smem);
  const size_t n = hb.size() + hk.size() + vb.size() + vk.size();
  dqz_frame_plan* P = new dqz_frame_plan();
  if (hipMalloc(&P->block, n * sizeof(int32_t)) != hipSuccess) {
    delete P;
    return fail(DQZ_ERR_HIP, "hipMalloc of the resize tables failed");
  }
  std::vector<int32_t> all;
  all.reserve(n);
  all.insert(all.end(), hb.begin(), hb.end());
  all.insert(all.end(), hk.begin(), hk.end());
  all.insert(all.end(), vb.begin(), vb.end());
  all.insert(all.end(), vk.begin(), vk.end());
  if (hipMemcpy(P->block, all.data(), n * sizeof(int32_t), hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(P->block);
    delete P;
    return fail(DQZ_ERR_HIP, "upload of the resize tables failed");
  }
  const int32_t* d = static_cast<const int32_t*>(P->block);
  P->p = FramePlan{in_h, in_w, out_h, out_w, kh, kv, max_band, d, d + hb.size(), d + hb.size() + hk.size(),
                   d + hb.size() + hk.size() + vb.size()};
  *out = P;
  return DQZ_OK;
}

int dqz_frame_plan_destroy(dqz_frame_plan* P) {
  if (!P) return DQZ_OK;
  if (P->block) (void)hipFree(P->block);
  delete P;
  return DQZ_OK;
}

int dqz_atari_frame(const dqz_frame_plan* P, const uint8_t* rgb, int n, uint8_t* out, void* stream) {
  if (!P || !rgb || !out) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 1 || n > 8) return fail(DQZ_ERR_INVALID, "n must be in [1, 8]");
  const void *drgb = nullptr, *dout = nullptr;
  if (int rc = device_view(rgb, &drgb, "rgb")) return rc;
  if (int rc = device_view(out, &dout, "out")) return rc;
  if (P->p.in_w % 4 == 0 && reinterpret_cast<uintptr_t>(drgb) % 4)
    return fail(DQZ_ERR_INVALID, "rgb must be 4-byte aligned");
  const int64_t stride = (int64_t)P->p.in_h * P->p.in_w * 3;
  const size_t smem = (size_t)P->p.max_band * (P->p.in_w + P->p.out_w);
  hipLaunchKernelGGL(atari_frame_kernel, dim3((P->p.out_h + FR_ROWS - 1) / FR_ROWS), dim3(256), smem,
                     (hipStream_t)stream, P->p, static_cast<const uint8_t*>(drgb), n, stride,
                     static_cast<uint8_t*>(const_cast<void*>(dout)));
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

}  // extern "C"

