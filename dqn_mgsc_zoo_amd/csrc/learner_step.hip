// learner_step.hip — the MI355X-native DQN learner step behind the dqz C ABI,
// in a code object of its own (common.hpp, "Two translation units").
//
// One step (dqn/agent.py:109-119, prioritized/agent.py:115-127), in launch order:
//   0 conv1 -> conv2 -> conv3 fwd as one hand-off launch (fwd_conv_kernel;
//     frame gather fused; z = online(s_tm1), target(s_t) [, online(s_t) for
//     double-Q])                                                  conv1.hpp, fwd.hpp
//   3 fc1 fwd (split-K)                                           fwd.hpp
//   4 head: fc1 reduce + fc2 + TD loss + dq + dz1, per sample    head.hpp
//   5 fc1 dX -> dy3 (+ the dX-ordered W3 / W2 copies)            bwd.hpp
//   6 the rest of the backward in one launch (bwd_bc_kernel): conv3 dX ->
//     conv2 dX -> conv1 dW hand-offs, fc1 dW + fused RMSProp, conv3 / conv2
//     dW partials                                                 bwd.hpp
//   7 reduce of every cross-sample / split-K gradient + centered RMSProp
#define DQZ_STEP_TU 1
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "learner_impl.hpp"

using namespace dqz;

static int g_attr_done = 0;

static int init_kernel_attrs() {
  if (g_attr_done) return DQZ_OK;
  const void* fwd_kernels[] = {(const void*)fwd_conv_kernel<0>, (const void*)fwd_conv_kernel<1>,
                               (const void*)fwd_conv_kernel<2>, (const void*)fwd_conv_kernel<3>};
  for (const void* k : fwd_kernels)
    DQZ_HIP(hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kConv1FwdSmem));
  g_attr_done = 1;
  return DQZ_OK;
}

extern "C" {

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
  if (int rc = init_kernel_attrs()) return rc;
  dqz_learner* L = new dqz_learner();
  L->cfg = *cfg;
  L->Z = cfg->algo == DQZ_ALGO_DQN ? 2 : 3;
  L->shared_bias = cfg->algo == DQZ_ALGO_DQN ? 0 : 1;
  param_layout(cfg->num_actions, L->shared_bias, L->off, L->sz, &L->total);
  const int B = cfg->batch, Z = L->Z, A = cfg->num_actions;
  L->S_fc1 = FC1_S;
  L->S2 = B;  // per-sample conv2 dW partials (conv2_bwd_kernel)
  L->S3 = B;  // per-sample conv3 dW partials (conv3_bwd_kernel)
  const int64_t n_y1 = (int64_t)Z * B * C1M * C1CO, n_y2 = (int64_t)Z * B * C2M * C2CO, n_y3 = (int64_t)Z * B * FLAT;
  const int64_t n_fc1p = (int64_t)Z * L->S_fc1 * B * HID, n_h1 = (int64_t)Z * B * HID, n_q = (int64_t)Z * B * A;
  const int64_t n_dz1 = (int64_t)B * HID, n_dy3 = (int64_t)B * FLAT, n_dy2 = (int64_t)B * C2M * C2CO,
                n_dy1 = (int64_t)B * C1M * C1CO;
  const int64_t n_p1 = (int64_t)B * C1_BLOCKS * (C1KK + 1) * C1CO, n_p2 = (int64_t)L->S2 * (C2KK + 1) * C2CO,
                n_p3 = (int64_t)L->S3 * (C3KK + 1) * C3CO;
  const int64_t sizes[] = {n_y1, n_y2, n_y3, n_fc1p, n_h1, n_q, n_dz1, n_dy3, n_dy2, n_dy1,
                           n_p1, n_p2, n_p3, B,      1,    B,   B,     B,  4 * B, (16 * B + 3) * Handoff::kStride + 64, W3P_N, W2P_N,
                           2 * (int64_t)B};
  float** ptrs[] = {&L->y1,  &L->y2,  &L->y3,  &L->fc1p, &L->h1,   &L->q,         &L->dz1, &L->dy3,
                    &L->dy2, &L->dy1, &L->p1,  &L->p2,   &L->p3,   &L->td,        &L->loss, &L->loss_part,
                    &L->gq,  reinterpret_cast<float**>(&L->ga), &L->rec, reinterpret_cast<float**>(&L->sync), &L->w3p, &L->w2p,
                    reinterpret_cast<float**>(&L->per_wb)};
  static_assert(sizeof(sizes) / sizeof(sizes[0]) == sizeof(ptrs) / sizeof(ptrs[0]), "scratch table");
  int64_t total = 0;
  for (int64_t s : sizes) total += (s + 63) / 64 * 64;
  if (hipMalloc(&L->block, total * sizeof(float)) != hipSuccess) {
    delete L;
    return fail(DQZ_ERR_HIP, "hipMalloc of %lld bytes failed", (long long)(total * 4));
  }
  if (hipMemset(L->block, 0, total * sizeof(float)) != hipSuccess) {
    (void)hipFree(L->block);
    delete L;
    return fail(DQZ_ERR_HIP, "hipMemset of learner scratch failed");
  }
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

}  // extern "C"

#define DQZ_PHASE(i, ...)                                                   \
  do {                                                                      \
    if (!pe.on()) {                                                         \
      __VA_ARGS__;                                                          \
    } else {                                                                \
      /* best of three trials: a stalled launching thread lets the queue */ \
      /* drain, and the idle device time would count as the phase's      */ \
      float best_ = 0.f;                                                    \
      for (int t_ = 0; t_ < 3; ++t_) {                                      \
        DQZ_HIP(hipEventRecord(pe.e0, st));                                 \
        for (int r_ = 0; r_ < pe.reps; ++r_) {                              \
          __VA_ARGS__;                                                      \
        }                                                                   \
        DQZ_HIP(hipEventRecord(pe.e1, st));                                 \
        DQZ_HIP(hipEventSynchronize(pe.e1));                                \
        float ms_ = 0.f;                                                    \
        (void)hipEventElapsedTime(&ms_, pe.e0, pe.e1);                      \
        if (t_ == 0 || ms_ < best_) best_ = ms_;                            \
      }                                                                     \
      pe.ms[i] = best_ / (float)pe.reps;                                    \
    }                                                                       \
  } while (0)

// conv1..fc1 forward of Z network copies (phases 0-3): conv1 -> conv2 ->
// conv3 as one hand-off launch (fwd_conv_kernel; since conv1 runs on bf16
// MFMA: 15,590 -> 16,050 steps/s against three launches, which round 4
// removed), then the split-K fc1.  Used by the learner step and the actor.
// (Round 5: fc1 inside the forward launch for launches of at most 16
// samples, its W1 loads issued at dispatch and y3 handed over per sample,
// measured slower at B = 1: the W1 stream stretched the conv chain by 0.9-1.6
// us, profiles/r05/s8, s9; removed.)
static int forward_impl(dqz_learner* L, const NetZ& nz, int Z, int B, const Conv1Src& src, hipStream_t st,
                        PhaseEvents pe) {
  Conv1FwdArgs c1{};
  c1.src = src;
  c1.nz = nz;
  c1.w_off = L->off[0];
  c1.b_off = L->off[1];
  c1.B = B;
  c1.Z = Z;
  c1.linear = 0;
  c1.out = L->y1;

  LayerFwdArgs c2{};
  c2.in = L->y1;
  c2.nz = nz;
  c2.w_off = L->off[2];
  c2.b_off = L->off[3];
  c2.B = B;
  c2.Z = Z;
  c2.linear = 0;
  c2.out = L->y2;

  LayerFwdArgs c3 = c2;
  c3.in = L->y2;
  c3.w_off = L->off[4];
  c3.b_off = L->off[5];
  c3.out = L->y3;
  // y1 / y2 hand-offs: 4 producer and 4 consumer blocks per sample.  The
  // word layout follows the learner's configured batch, not this call's n
  // (the actor's forward has n = 1): Z * n <= 3 * cfg.batch samples, and
  // every launch shares the one error word dqz_learner_sync_status reads.
  const int Bc = L->cfg.batch;
  int* hw = L->sync + 2 * Bc * Handoff::kStride;
  int* err = L->sync + 16 * Bc * Handoff::kStride;
  const int jobs = fwd_conv_jobs(Z * B);
  c2.jobs = c3.jobs = jobs;
  c1.pub = Handoff{hw, hw + 3 * Bc * Handoff::kStride, err, 4, jobs};
  c2.wait = c1.pub;
  c2.pub = Handoff{hw + 6 * Bc * Handoff::kStride, hw + 9 * Bc * Handoff::kStride, err, jobs, jobs};
  c3.wait = c2.pub;
  const dim3 grid(xcd_grid(4, Z * B).x + 2 * xcd_grid(jobs, Z * B).x);
  DQZ_PHASE(0, switch (src.fused) {
    case 1: hipLaunchKernelGGL(fwd_conv_kernel<1>, grid, dim3(256), kConv1FwdSmem, st, c1, c2, c3); break;
    case 2: hipLaunchKernelGGL(fwd_conv_kernel<2>, grid, dim3(256), kConv1FwdSmem, st, c1, c2, c3); break;
    case 3: hipLaunchKernelGGL(fwd_conv_kernel<3>, grid, dim3(256), kConv1FwdSmem, st, c1, c2, c3); break;
    default: hipLaunchKernelGGL(fwd_conv_kernel<0>, grid, dim3(256), kConv1FwdSmem, st, c1, c2, c3); break;
  } DQZ_HIP(hipGetLastError()));
  if (pe.on()) pe.ms[1] = pe.ms[2] = 0.f;

  Fc1FwdArgs f1{};
  f1.in = L->y3;
  f1.nz = nz;
  f1.w_off = L->off[6];
  f1.B = B;
  f1.MG = (B + 31) / 32;
  f1.part = L->fc1p;
  DQZ_PHASE(3, if (B <= FC1_GEMV_MAXB)
                 hipLaunchKernelGGL(fc1_gemv_kernel, dim3(fc1_fwd_blocks(Z, 1)), dim3(256), 0, st, f1);
               else
                 hipLaunchKernelGGL(fc1_fwd32_kernel, dim3(fc1_fwd_blocks(Z, f1.MG)), dim3(256), 0, st, f1);
            DQZ_HIP(hipGetLastError()));
  return DQZ_OK;
}

static HeadArgs make_head(dqz_learner* L, const NetZ& nz, int Z, int B) {
  HeadArgs h{};
  memset(&h, 0, sizeof(h));
  h.fc1p = L->fc1p;
  h.S = L->S_fc1;
  h.h1 = L->h1;
  h.nz = nz;
  h.b1_off = L->off[7];
  h.w2_off = L->off[8];
  h.b2_off = L->off[9];
  h.Z = Z;
  h.B = B;
  h.A = L->cfg.num_actions;
  h.algo = L->cfg.algo;
  h.shared_bias = L->shared_bias;
  h.q = L->q;
  return h;
}

// One learner step.  gout == null: centered RMSProp on P->online/mu/nu.
// gout != null: gradient-output mode — the full gradient is written to gout
// (dqz parameter layout) and P->online/mu/nu are left untouched.
// meta_p != null: per-sample cotangents p_b * (-clip(td_b)) (MGSC meta mode).
int dqz::step_impl(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                   const float* is_weights, void* stream, PhaseEvents pe, float* gout, const float* meta_p,
                   const UniformDraw* draw, int unit, int gacc, const PerWbArgs* wb, const SoftmaxDraw* sm,
                   const PerSampleArgs* pd, const Rms* meta_epi, const HeadArgs* meta_sm, uint8_t* xout) {
  if (!L || !P || !P->online || !P->target || !slots) return fail(DQZ_ERR_INVALID, "null argument");
  if (!gout && !meta_epi && (!P->mu || !P->nu)) return fail(DQZ_ERR_INVALID, "null optimizer state");
  if (meta_epi && meta_epi->meta == 1 && (!P->mu || !P->nu)) return fail(DQZ_ERR_INVALID, "null optimizer state");
  if (int rc = check_store(S)) return rc;
  if (L->cfg.algo == DQZ_ALGO_PER && !is_weights && !pd) return fail(DQZ_ERR_INVALID, "PER step needs is_weights");
  hipStream_t st = (hipStream_t)stream;
  const int B = L->cfg.batch, Z = L->Z, A = L->cfg.num_actions;
  NetZ nz{};
  nz.p[0] = P->online;
  nz.p[1] = P->target;
  nz.p[2] = P->online;
  nz.which[0] = 0;
  nz.which[1] = 1;
  nz.which[2] = 1;
  Conv1Src src{S->frames, S->fidx, slots, nullptr, 0, UniformDraw{}};
  src.action = S->action;
  src.reward = S->reward;
  src.discount = S->discount;
  src.rec = reinterpret_cast<float4*>(L->rec);
  src.xout = xout;
  if (draw || sm || pd) {  // conv1 draws the batch itself; later kernels read the published slots
    Conv1Src fsrc = src;
    if (draw) {
      fsrc.fused = 1;
      fsrc.draw = *draw;
    } else if (pd) {
      fsrc.fused = 3;
      fsrc.per = *pd;
      fsrc.per.out_wb = L->per_wb;
    } else {
      fsrc.fused = 2;
      fsrc.sm = *sm;
    }
    if (int rc = forward_impl(L, nz, Z, B, fsrc, st, pe)) return rc;
  } else {
    if (int rc = forward_impl(L, nz, Z, B, src, st, pe)) return rc;
  }

  // an MGSC meta stage applied in the gradient epilogues (Rms), or plain
  // RMSProp / gradient output: every field set (value-initialised first)
  Rms rms{};
  if (meta_epi) rms = *meta_epi;
  rms.lr = L->cfg.learning_rate;
  rms.decay = L->cfg.decay;
  rms.c1 = (float)(1.0 - (double)L->cfg.decay);
  rms.eps = L->cfg.eps;
  rms.gout = gout;
  rms.gacc = gacc;
  rms.sq_off = 0;

  HeadArgs h = make_head(L, nz, Z, B);
  h.fwd_only = 0;
  h.slots = slots;
  h.action = S->action;
  h.reward = S->reward;
  h.discount = S->discount;
  h.weights = L->cfg.algo == DQZ_ALGO_PER && !pd ? is_weights : nullptr;
  if (pd) {
    h.per_wb = L->per_wb;
    h.per_normalize = pd->normalize;
    h.per_w_out = pd->out_weights;
  }
  h.meta_p = meta_p;
  if (meta_sm) {  // the meta batch's softmax formed by the head (one meta chunk)
    h.meta_logits = meta_sm->meta_logits;
    h.meta_pos = meta_sm->meta_pos;
    h.meta_M = meta_sm->meta_M;
    h.meta_x_out = meta_sm->meta_x_out;
    h.meta_p_out = meta_sm->meta_p_out;
  }
  h.rec = reinterpret_cast<const float4*>(L->rec);
  h.advance = draw ? draw->counter : sm ? sm->counter : pd ? (pd->inj_u ? nullptr : pd->counter) : nullptr;
  h.unit = unit;
  h.bound = L->cfg.grad_error_bound;
  h.td = L->td;
  h.loss_part = L->loss_part;
  h.gq = L->gq;
  h.ga = L->ga;
  h.dz1 = L->dz1;

  // Backward: fc1 dX, then the merged launch that pairs the dX chain with the
  // independent dW job sets (bwd.hpp).
  Fc1BwdArgs fb{};
  fb.dz1 = L->dz1;
  fb.y3 = L->y3;
  fb.th = P->online;
  fb.mu = P->mu;
  fb.nu = P->nu;
  fb.w_off = L->off[6];
  fb.rms = rms;
  fb.B = B;
  fb.dy3 = L->dy3;
  fb.w3 = P->online + L->off[4];
  fb.w2 = P->online + L->off[2];
  fb.w3p = L->w3p;
  fb.w2p = L->w2p;
  if (B == 1 && !pe.on()) {
    // one sample (the MGSC pass at theta', the HVP's unit-cotangent pass):
    // the head and fc1 dX in one launch, every block forming the head itself
    DQZ_HIP(launch_head_dx1(h, fb, st));
  } else {
    DQZ_PHASE(4, DQZ_HIP(launch_head(h, B, st)));
    DQZ_PHASE(5, hipLaunchKernelGGL(fc1_dx_kernel, dim3(fc1_dx_blocks(B)), dim3(256), 0, st, fb);
              DQZ_HIP(hipGetLastError()));
  }

  Conv3BwdArgs c3b{};
  c3b.dy3 = L->dy3;
  c3b.y2 = L->y2;
  c3b.w3 = P->online + L->off[4];
  c3b.w3p = L->w3p;
  c3b.dy2 = L->dy2;
  c3b.part = L->p3;
  c3b.B = B;
  // hand-off words (units of Handoff::kStride ints): dy2 cnt [0, B), ack [B, 2B);
  // forward y1 / y2 [2B, 14B); dy1 cnt [14B, 15B), ack [15B, 16B); err at 16B
  int* const herr = L->sync + 16 * B * Handoff::kStride;
  c3b.sync = Handoff{L->sync, L->sync + B * Handoff::kStride, herr, 8, 16, L->spin_max};
  Conv2BwdArgs c2b{};
  c2b.dy2 = L->dy2;
  c2b.y1 = L->y1;
  c2b.w2 = P->online + L->off[2];
  c2b.w2p = L->w2p;
  c2b.dy1 = L->dy1;
  c2b.part = L->p2;
  c2b.B = B;
  c2b.sync = c3b.sync;
  Conv1DwArgs c1dw{};
  c1dw.src = src;
  c1dw.src.rec = nullptr;
  c1dw.src.xout = nullptr;
  c1dw.which = 0;
  c1dw.B = B;
  c1dw.dy1 = L->dy1;
  c1dw.part = L->p1;
  c1dw.sync1 = Handoff{L->sync + 14 * B * Handoff::kStride, L->sync + 15 * B * Handoff::kStride, herr, 8, 8,
                       L->spin_max};
  c2b.sync1 = c1dw.sync1;
  const int B8 = (B + 7) / 8 * 8;
  PerWbArgs wbk{};
  if (wb) {
    wbk = *wb;
    wbk.td = L->td;
    wbk.n = B;
  }
  const int grid = (wb ? 8 : 0) + 8 * B8 + 4 * (FLAT / 16) + 8 * B8 + 4 * B8 + 8 * B8 + 8 * B8;
  DQZ_PHASE(6, if (wb) hipLaunchKernelGGL(bwd_bc_kernel<true>, dim3(grid), dim3(256), 0, st, c3b, fb, c2b, c1dw, wbk);
            else hipLaunchKernelGGL(bwd_bc_kernel<false>, dim3(grid), dim3(256), 0, st, c3b, fb, c2b, c1dw, wbk);
            DQZ_HIP(hipGetLastError()));
  if (pe.on()) pe.ms[7] = pe.ms[8] = 0.f;

  UpdArgs u{};
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
  u.S1 = B * C1_BLOCKS;
  u.S2 = L->S2;  // one dW partial slab per sample
  u.S3 = L->S3;
  u.h1 = L->h1;
  u.dz1 = L->dz1;
  u.gq = L->gq;
  u.ga = L->ga;
  u.loss_part = L->loss_part;
  u.loss = L->loss;
  u.status = herr;
  u.A = A;
  u.B = B;
  u.nb2 = L->shared_bias ? 1 : A;
  u.rms = rms;
  u.rms.sq_off = 4 * (FLAT / 16);  // meta_rms2 partials: the fc1 dW blocks' first, then the update's
  const unsigned nblk = update_blocks(L->sz, A, u.nb2);
  DQZ_PHASE(9, hipLaunchKernelGGL(update_kernel, dim3(nblk), dim3(256), 0, st, u);
            DQZ_HIP(hipGetLastError()));
  return DQZ_OK;
}

extern "C" {

int dqz_learner_step(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                     const float* is_weights, void* stream) {
  return step_impl(L, P, S, slots, is_weights, stream, kNoProfile);
}

int dqz_learner_step_per(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                         const float* is_weights, double* tree, int64_t cap, const int32_t* indices, double alpha,
                         double* max_seen_dev, void* stream) {
  if (!L || !tree || !indices || !max_seen_dev) return fail(DQZ_ERR_INVALID, "null argument");
  if (L->cfg.batch > 64) return fail(DQZ_ERR_INVALID, "the fused write-back takes batch <= 64 (use dqz_per_write_back)");
  if (cap < 1 || (cap & (cap - 1))) return fail(DQZ_ERR_INVALID, "cap must be a power of two");
  int levels = 0;
  while (((int64_t)1 << levels) < cap) ++levels;
  if (levels > PWB_LEVELS) return fail(DQZ_ERR_INVALID, "cap must be <= 2^%d for the fused write-back", PWB_LEVELS);
  PerWbArgs wb{tree, cap, levels, indices, nullptr, alpha, 0, max_seen_dev};
  return step_impl(L, P, S, slots, is_weights, stream, kNoProfile, nullptr, nullptr, nullptr, 0, 0, &wb);
}

int dqz_learner_step_uniform(dqz_learner* L, const dqz_params* P, const dqz_store* S, int64_t base, int64_t size,
                             int64_t capacity, uint64_t seed, uint64_t* counter_dev, int32_t* slots_out,
                             void* stream) {
  if (!counter_dev || !slots_out) return fail(DQZ_ERR_INVALID, "null argument");
  if (size < 1) return fail(DQZ_ERR_INVALID, "cannot sample from an empty replay (size=%lld)", (long long)size);
  if (capacity < size || base < 0) return fail(DQZ_ERR_INVALID, "bad replay geometry");
  if (L && L->cfg.algo == DQZ_ALGO_PER) return fail(DQZ_ERR_INVALID, "PER samples by priority, not uniformly");
  const UniformDraw d{base % capacity, size, capacity, seed, counter_dev, slots_out};
  return step_impl(L, P, S, slots_out, nullptr, stream, kNoProfile, nullptr, nullptr, &d);
}

int dqz_learner_grad(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                     const float* is_weights, float* grad_out, void* stream) {
  if (!grad_out) return fail(DQZ_ERR_INVALID, "null grad_out");
  return step_impl(L, P, S, slots, is_weights, stream, kNoProfile, grad_out);
}

int dqz_learner_profile(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
                        const float* is_weights, int iters, float* phase_ms, void* stream) {
  if (!phase_ms || iters < 1) return fail(DQZ_ERR_INVALID, "phase_ms must be non-null and iters >= 1");
  for (int i = 0; i < DQZ_NUM_PHASES; ++i) phase_ms[i] = 0.f;
  PhaseEvents pe{nullptr, nullptr, iters, phase_ms};
  DQZ_HIP(hipEventCreate(&pe.e0));
  DQZ_HIP(hipEventCreate(&pe.e1));
  const int rc = step_impl(L, P, S, slots, is_weights, stream, pe);
  (void)hipEventDestroy(pe.e0);
  (void)hipEventDestroy(pe.e1);
  return rc;
}

int dqz_learner_sync_status(dqz_learner* L, int* status) {
  if (!L || !status) return fail(DQZ_ERR_INVALID, "null argument");
  DQZ_HIP(hipDeviceSynchronize());
  DQZ_HIP(hipMemcpy(status, L->sync + 16 * L->cfg.batch * Handoff::kStride, sizeof(int), hipMemcpyDeviceToHost));
  if (*status != 0) {
    // A wait gave up: its consumers ran on partial payloads and producers may
    // have arrived after the last consumer reset the words, which would let
    // later launches pass their waits early.  Clear every hand-off word (and
    // the error word) so the next step starts clean; the caller must treat
    // the steps since the previous check as invalid.
    DQZ_HIP(hipMemset(L->sync, 0, sizeof(int) * ((16 * L->cfg.batch + 3) * Handoff::kStride + 64)));
    DQZ_HIP(hipDeviceSynchronize());
  }
  return DQZ_OK;
}

int dqz_learner_debug_stall(dqz_learner* L, int sample, unsigned spin_max) {
  if (!L) return fail(DQZ_ERR_INVALID, "null learner");
  if (sample >= L->cfg.batch) return fail(DQZ_ERR_INVALID, "sample out of range");
  L->spin_max = spin_max ? spin_max : 1u << 24;
  if (sample >= 0) {  // sample's dy2 arrival counter far below its 8 arrivals: its waits run out
    const int32_t poison = -(1 << 30);
    DQZ_HIP(hipDeviceSynchronize());
    DQZ_HIP(hipMemcpy(L->sync + (int64_t)sample * Handoff::kStride, &poison, sizeof(poison),
                      hipMemcpyHostToDevice));
  }
  return DQZ_OK;
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

static int forward_q(dqz_learner* L, const float* params, const Conv1Src& src, int which, int n, float* q_out,
                     hipStream_t st) {
  NetZ nz{};
  nz.p[0] = nz.p[1] = nz.p[2] = params;
  nz.which[0] = nz.which[1] = nz.which[2] = which;
  if (int rc = forward_impl(L, nz, 1, n, src, st, kNoProfile)) return rc;
  HeadArgs h = make_head(L, nz, 1, n);
  h.fwd_only = 1;
  h.q = q_out;
  DQZ_HIP(launch_head(h, n, st));
  DQZ_HIP(hipGetLastError());
  return DQZ_OK;
}

int dqz_forward(dqz_learner* L, const float* params, const uint8_t* states, int n, float* q_out, void* stream) {
  if (!L || !params || !states || !q_out) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 1 || n > L->cfg.batch) return fail(DQZ_ERR_INVALID, "n must be in [1, %d]", L->cfg.batch);
  if (reinterpret_cast<uintptr_t>(states) % 16) return fail(DQZ_ERR_INVALID, "states must be 16-byte aligned");
  Conv1Src src{nullptr, nullptr, nullptr, states, 0, UniformDraw{}};
  return forward_q(L, params, src, 0, n, q_out, (hipStream_t)stream);
}

int dqz_forward_slots(dqz_learner* L, const float* params, const dqz_store* S, const int32_t* slots, int n, int which,
                      float* q_out, void* stream) {
  if (!L || !params || !slots || !q_out) return fail(DQZ_ERR_INVALID, "null argument");
  if (int rc = check_store(S)) return rc;
  if (n < 1 || n > L->cfg.batch) return fail(DQZ_ERR_INVALID, "n must be in [1, %d]", L->cfg.batch);
  if (which != 0 && which != 1) return fail(DQZ_ERR_INVALID, "which must be 0 (s_tm1) or 1 (s_t)");
  Conv1Src src{S->frames, S->fidx, slots, nullptr, 0, UniformDraw{}};
  return forward_q(L, params, src, which, n, q_out, (hipStream_t)stream);
}

int dqz_act(dqz_learner* L, const float* params, const uint8_t* states, int n, double epsilon, uint64_t seed,
            uint64_t counter, dqz_action* out, void* stream) {
  if (!L || !params || !states || !out) return fail(DQZ_ERR_INVALID, "null argument");
  if (n < 1 || n > L->cfg.batch) return fail(DQZ_ERR_INVALID, "n must be in [1, %d]", L->cfg.batch);
  if (!(epsilon >= 0.0 && epsilon <= 1.0)) return fail(DQZ_ERR_INVALID, "epsilon must be in [0, 1]");
  const void *dstates = nullptr, *dout = nullptr;
  if (int rc = device_view(states, &dstates, "states")) return rc;
  if (int rc = device_view(out, &dout, "out")) return rc;
  if (reinterpret_cast<uintptr_t>(dstates) % 16) return fail(DQZ_ERR_INVALID, "states must be 16-byte aligned");
  hipStream_t st = (hipStream_t)stream;
  NetZ nz{};
  nz.p[0] = nz.p[1] = nz.p[2] = params;
  nz.which[0] = nz.which[1] = nz.which[2] = 0;
  Conv1Src src{nullptr, nullptr, nullptr, static_cast<const uint8_t*>(dstates), 0, UniformDraw{}};
  if (int rc = forward_impl(L, nz, 1, n, src, st, kNoProfile)) return rc;
  HeadArgs h = make_head(L, nz, 1, n);
  h.fwd_only = 1;
  h.q = L->q;
  h.act_out = static_cast<dqz_action*>(const_cast<void*>(dout));
  h.eps = epsilon;
  h.act_seed = seed;
  h.act_ctr = counter;
  DQZ_HIP(launch_head(h, n, st));
  return DQZ_OK;
}

}  // extern "C"

#ifdef DQZ_TRACE
// Diagnostic builds only (not part of include/dqz.h): copy / clear the
// in-kernel timeline stamps (common.hpp DQZ_STAMP).
extern "C" int dqz_debug_trace(unsigned long long* host_out, int clear) {
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

