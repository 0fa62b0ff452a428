/*
 * dqz.h — C ABI of the MI355X-native DQN learner step (libdqz.so).
 *
 * Plain C: raw pointers, sizes and a hipStream_t passed as void*.  No torch
 * types cross this boundary.  Every function returns DQZ_OK (0) on success or
 * a negative status; dqz_last_error() returns a thread-local message.
 *
 * Ownership: the caller owns every device buffer that holds
 * state (parameters, optimizer moments, frame pool, transition table, sampled
 * slot buffers).  The library borrows those pointers for the duration of an
 * enqueue and owns only the opaque learner handle and its scratch.  All work
 * is enqueued on the given stream; no call synchronises the device except
 * where it documents a host output.
 *
 * Each entry point names the reference interface it replaces (file:line in
 * Stalfoes/dqn_mgsc_zoo).
 */
#ifndef DQZ_H_
#define DQZ_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DQZ_OK 0
#define DQZ_ERR_INVALID (-1)
#define DQZ_ERR_HIP (-2)
#define DQZ_ERR_UNSUPPORTED (-3)

/* Learner algorithm: which TD loss and which network head.
 *  DQN     : rlax.q_learning, dqn_atari_network          (dqn/agent.py:85-107)
 *  DOUBLE  : rlax.double_q_learning, double_dqn_atari_network (shared bias)
 *            (double_q/agent.py:85-107, networks.py:338-349)
 *  PER     : DOUBLE + importance weights, |td| returned   (prioritized/agent.py:86-127)
 */
#define DQZ_ALGO_DQN 0
#define DQZ_ALGO_DOUBLE 1
#define DQZ_ALGO_PER 2

/* Frame geometry (processors.py:488-505): 84x84 grayscale frames, 4-stack,
 * HWC layout, channel order oldest -> newest, trailing zero padding. */
#define DQZ_FRAME_H 84
#define DQZ_FRAME_W 84
#define DQZ_STACK 4
#define DQZ_FRAME_BYTES (DQZ_FRAME_H * DQZ_FRAME_W)
#define DQZ_NUM_LEAVES 10

/* Thread-local message for the last failing call on this thread. */
const char* dqz_last_error(void);

/* Source hash this library was compiled from: the first 16 hex digits of the
 * SHA-256 over csrc/ (every .hip / .hpp) and include/dqz.h, baked in at build
 * time (__graft_entry__.build()).  The Python loader refuses a library whose
 * id differs from the sources beside it, so a GPU run proves which kernels it
 * tested.  "unset" when built without the id. */
const char* dqz_build_id(void);

/* Flat parameter layout of the NatureQNetwork (networks.py:181-221,352-363):
 * leaves in Haiku order
 *   0 conv2_d/w [8,8,4,32]   1 conv2_d/b [32]
 *   2 conv2_d_1/w [4,4,32,64] 3 conv2_d_1/b [64]
 *   4 conv2_d_2/w [3,3,64,64] 5 conv2_d_2/b [64]
 *   6 linear/w [3136,512]    7 linear/b [512]
 *   8 linear_1/w [512,A]     9 linear_1/b [A]   (shared_bias: [1])
 * Each leaf starts on a 64-float boundary; padding stays zero.
 * offsets/sizes are in floats; total is the padded buffer length. */
int dqz_param_layout(int num_actions, int shared_bias, int64_t offsets[DQZ_NUM_LEAVES],
                     int64_t sizes[DQZ_NUM_LEAVES], int64_t* total);

/* Replay storage in HBM (replaces the snappy-compressed per-transition
 * storage of replay.py:163-206 / replay_circular.py:90-146).
 *   frames   uint8 [num_frames][84*84]         frame pool
 *   fidx     int32 [capacity][8]               frame index of each stack
 *                                              channel: 0..3 = s_tm1, 4..7 = s_t,
 *                                              -1 = zero padding
 *   action   int32 [capacity]   reward f32 [capacity]   discount f32 [capacity]
 * A transition lives in a slot; slots are what the samplers return. */
typedef struct dqz_store {
  const uint8_t* frames;
  const int32_t* fidx;
  const int32_t* action;
  const float* reward;
  const float* discount;
  int64_t capacity;
  int64_t num_frames;
} dqz_store;

/* Online/target parameters and centered-RMSProp moments, all [total] f32
 * in the dqz_param_layout order (optax.rmsprop(centered=True) state,
 * dqn/run_atari.py:208-213). */
typedef struct dqz_params {
  float* online;
  float* target;
  float* mu;
  float* nu;
} dqz_params;

typedef struct dqz_learner_config {
  int batch;            /* B (replay.sample(batch_size)), 1..256 */
  int num_actions;      /* A, 1..32 */
  int algo;             /* DQZ_ALGO_* */
  float learning_rate;  /* dqn/run_atari.py:81 */
  float decay;          /* 0.95 */
  float eps;            /* dqn/run_atari.py:82 */
  float grad_error_bound; /* dqn/run_atari.py:80 (rlax.clip_gradient bound) */
} dqz_learner_config;

typedef struct dqz_learner dqz_learner;

/* Allocates the learner's scratch (activations, split-K partials). */
int dqz_learner_create(const dqz_learner_config* cfg, dqz_learner** out);
int dqz_learner_destroy(dqz_learner* learner);

/* One learner step = jitted `update` of dqn/agent.py:109-119
 * (prioritized/agent.py:115-127 for PER): forward online(s_tm1),
 * target(s_t) [+ online(s_t)], TD loss with clip_gradient, backward,
 * centered RMSProp, in place on params->online / mu / nu.
 * slots: device int32 [B] replay slots of the minibatch (from a sampler or
 * injected by the caller).  is_weights: device f32 [B] or NULL (PER only). */
int dqz_learner_step(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                     const int32_t* slots, const float* is_weights, void* stream);

/* Sampling fused into the step: the batch is `size` uniform draws
 * (base + floor(u * size)) mod capacity with Philox(counter, i; seed), as
 * dqz_sample_uniform would draw them, computed inside the conv1 kernel (no
 * separate sampler launch); the drawn slots are written to slots_out (device
 * int32 [B]) and *counter_dev advances by one.  Uniform FIFO / reservoir
 * replays (replay.py:119-125, 246-296). */
int dqz_learner_step_uniform(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                             int64_t base, int64_t size, int64_t capacity, uint64_t seed,
                             uint64_t* counter_dev, int32_t* slots_out, void* stream);

/* PER learner step with the priority write-back folded in
 * (prioritized/agent.py:187-206): dqz_learner_step on `slots` with the IS
 * weights, then — inside the same backward launch, in its first workgroup,
 * beside the backward pass — what dqz_per_write_back(tree, cap, indices,
 * alpha, max_seen_dev) does after it: p = |td|, *max_seen_dev = max(...,
 * max p), leaf[indices[i]] = p^alpha with the last draw of a repeated index
 * winning, ancestors rebuilt (bit-identical sums).  indices: device int32
 * [B] tree indices (dqz_per_sample's out_indices).  cap: a power of two <=
 * 2^24; batch <= 64.  Saves the write-back's own launch. */
int dqz_learner_step_per(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                         const int32_t* slots, const float* is_weights, double* tree, int64_t cap,
                         const int32_t* indices, double alpha, double* max_seen_dev, void* stream);

/* MGSC learner step with the batch drawn inside the learner's forward
 * launch (dqn_mgsc_batched/agent.py:341-360: replay.sample(batch) from
 * softmax(logits), then the DQN update): the draw is exactly
 * dqz_logits_sample_slots(buf, logits, seed, counter_dev, NULL, B,
 * slots_out, ...) — Philox uniform b of step *counter_dev (or uniforms[b]
 * when `uniforms`, device f64 [B], is given: the replay Generator's own
 * draws), the CDF search of dqz_logits_sample — computed by each of the
 * forward's conv1 workgroups before its frame gather (no sampler launch);
 * slots_out (device int32 [B]) receives the slots and *counter_dev advances
 * by one (Philox mode).  buf / logits: the replay's learned-logit buffer. */
typedef struct dqz_logit_buffer dqz_logit_buffer;
int dqz_learner_step_logits(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                            dqz_logit_buffer* buf, const float* logits, uint64_t seed, uint64_t* counter_dev,
                            const double* uniforms, int32_t* slots_out, void* stream);

/* Gradient only: d loss / d params of the same step into grad_out (device
 * f32, dqz_param_layout order, padding untouched); params->online / mu / nu
 * are not modified and mu / nu may be NULL.  = jax.grad(loss_fn) at
 * dqn/agent.py:112-116. */
int dqz_learner_grad(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                     const int32_t* slots, const float* is_weights, float* grad_out, void* stream);

/* Phases of one learner step, in launch order (dqz_learner_profile):
 *  0 conv1 fwd (uniform draw + frame gather fused)   1 conv2 fwd
 *  2 conv3 fwd   3 fc1 fwd (split-K)
 *  4 head: fc1 reduce + fc2 + TD loss + dq + dz1 (one workgroup per sample);
 *    with DQZ_FUSED_HEAD=1 also fc1 dX behind an in-launch dz1 hand-off
 *    (one launch, head_dx_kernel) and 5 reports 0
 *  5 fc1 dX
 *  6 conv3 dX -> conv2 dX -> conv1 dW and conv3 dX -> conv2 dW (in-launch
 *    per-sample hand-offs of dy2 / dy1) + fc1 dW and RMSProp of fc1/w +
 *    conv3 dW partials (one launch, bwd_bc_kernel)
 *  7 0 (merged into 6); in the DQZ_FUSED_BWD=0 debug layout 6 is conv3 dX +
 *    fc1 dW and 7 is conv2 dX + conv3 dW partials
 *  8 0 (merged into 6); with DQZ_FUSED_BWD=0 or DQZ_DW_LATE=1: conv1 dW
 *    partials (frame gather fused) + conv2 dW partials
 *  9 gradient reductions + RMSProp (all leaves but fc1/w) */
#define DQZ_NUM_PHASES 10

/* Per-phase kernel time: runs one learner step in which every phase's
 * launch is repeated `iters` times back to back between two hipEvents on
 * `stream`, three times; phase_ms[i] = the best trial's average
 * milliseconds per launch (the kernel's duration in a saturated stream,
 * comparable to rocprofv3 --kernel-trace; the best of three drops a trial
 * whose launching thread stalled and let the device idle).  Phases that
 * update state (4, 6, 9) apply their update 3 x `iters` times: call it on a
 * scratch copy or after the timed work.  Synchronises the stream. */
int dqz_learner_profile(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                        const int32_t* slots, const float* is_weights, int iters, float* phase_ms,
                        void* stream);

/* Device-to-device copies of the last step's outputs (any may be NULL):
 * q_tm1 [B][A] online Q(s_tm1), td [B] TD errors, loss [1] mean loss. */
int dqz_learner_outputs(dqz_learner* learner, float* q_tm1, float* td, float* loss, void* stream);

/* Health word of the learner since the previous check: *status = 0 when
 * every in-launch hand-off wait of the backward pass completed and every
 * batch loss was finite; bit 0 (1): a wait gave up (a bounded spin expired;
 * the step's results are then invalid); bit 1 (2): a step's mean loss was
 * NaN or infinite (the update still ran, as the reference's jitted update
 * would).  Synchronises the device.  A non-zero status also clears every
 * hand-off word and the status, so the next step starts clean; callers treat
 * the steps since their previous check as invalid. */
int dqz_learner_sync_status(dqz_learner* learner, int* status);

/* Diagnostic (tests): the bounded hand-off spin gives up after `spin_max`
 * polls from the next step on (0 restores the default 2^24), and if sample
 * >= 0 that sample's dy2 arrival counter is poisoned so the next step's
 * waits on it run out — the timeout path of dqz_learner_sync_status,
 * exercised.  Synchronises the device. */
int dqz_learner_debug_stall(dqz_learner* learner, int sample, unsigned spin_max);

/* Q-values of the NatureQNetwork for uint8 HWC states [n][84][84][4]
 * (network.apply(...).q_values, networks.py:352-363; used by select_action,
 * dqn/agent.py:121-131).  q_out: device f32 [n][A]. n <= learner batch. */
int dqz_forward(dqz_learner* learner, const float* params, const uint8_t* states, int n,
                float* q_out, void* stream);

/* Q-values for replay slots without materialising stacks:
 * which = 0 -> s_tm1, 1 -> s_t. */
int dqz_forward_slots(dqz_learner* learner, const float* params, const dqz_store* store,
                      const int32_t* slots, int n, int which, float* q_out, void* stream);

/* ---- actor path (dqn/agent.py:121-131, 169-177) -------------------------
 * select_action on device: q = Q(params, states[i]), v = max_a q,
 * a ~ distrax.EpsilonGreedy(q, epsilon): P(a) = (1 - eps) [q_a == v] / #ties
 * + eps / A (fp64, as parts.epsilon_greedy_probs), drawn by inverting the
 * CDF the way numpy's Generator.choice does (cumsum, normalised by its last
 * entry, first entry > u) with u = Philox4x32-10(key = seed, counter =
 * (counter, i)).  `states` (uint8 [n][84][84][4]) and `out` may be device
 * memory or pinned (hipHostMalloc / torch pin_memory) host memory, which
 * the kernels read and write in place: one call, no staging copies.  Host
 * results are valid after the stream is synchronised.  n <= learner batch. */
typedef struct dqz_action {
  int32_t action;
  float value; /* max_a q: the agent's statistics['state_value'] */
} dqz_action;
int dqz_act(dqz_learner* learner, const float* params, const uint8_t* states, int n, double epsilon,
            uint64_t seed, uint64_t counter, dqz_action* out, void* stream);

/* One replay add into the HBM store in one launch (TransitionReplay.add,
 * replay.py:182-192): copies `num_frames` new frames (uint8 [num_frames][7056]
 * at `frames`, device or pinned host memory) into pool rows frame_rows[i],
 * then writes the transition record {fidx, a, r, d} at `slot`.  Writes
 * through the store's (caller-owned, writable) buffers. */
typedef struct dqz_transition_put {
  int64_t slot;
  int32_t fidx[8];       /* pool rows of s_tm1 / s_t channels, -1 = zero padding */
  int32_t action;
  float reward, discount;
  int32_t num_frames;    /* <= 8 */
  int32_t frame_rows[8]; /* destination pool row of each new frame */
} dqz_transition_put;
int dqz_store_put(const dqz_store* store, const dqz_transition_put* t, const uint8_t* frames,
                  void* stream);

/* Uniform sampling with replacement over live transitions, on device
 * (UniformDistribution.sample, replay.py:119-125; replay_circular.py:283-289).
 * Live slots are (base + j) mod capacity for j in [0, size).  FIFO replay:
 * base = t - size; reservoir replay: base = 0.  Philox4x32-10 keyed by seed,
 * counter = (*counter_dev, lane); *counter_dev is incremented on device, so
 * the call is hipGraph-replayable. */
int dqz_sample_uniform(int64_t base, int64_t size, int64_t capacity, int n, uint64_t seed,
                       uint64_t* counter_dev, int32_t* out_slots, void* stream);

/* Materialise stacked uint8 states [n][84][84][4] for the given slots
 * (the np.stack of TransitionReplay.sample, replay.py:200-206).
 * which = 0 -> s_tm1, 1 -> s_t. */
int dqz_gather_stacks(const dqz_store* store, const int32_t* slots, int n, int which,
                      uint8_t* out, void* stream);

/* ---- learned-logit replay sampling (dqn_mgsc_batched replays) ----------
 * logits: device f32 [capacity], -inf marks an empty slot
 * (CircularLogitBuffer / MGSCReservoirDistribution, replay_circular.py:148-248,
 * 500-565).  A dqz_logit_buffer owns the running log-sum-exp state and one
 * float64 sum of the sampling terms per chunk of 4096 slots, both kept
 * current by every write through the library (capacity <= 2^42). */
int dqz_logit_buffer_create(int64_t capacity, int max_queries, dqz_logit_buffer** out);
int dqz_logit_buffer_destroy(dqz_logit_buffer* buf);

/* Default logit of an added item (replay_circular.py:166-179, :518-533):
 * if clear_pos >= 0, logits[clear_pos] = -inf first (the reservoir
 * `replace`); then logits[write_pos] = size == 0 ? 0
 *   : logsumexp(logits[0:capacity]) - log(size).  lse_out (device f32) may be NULL.
 * The buffer keeps a running float64 sum of exp(x - c), so an add is O(1);
 * it is re-seeded by a full scan after dqz_logits_invalidate, every 4096
 * running adds, or when a removal would cancel most of it.  Every write to
 * `logits` must go through dqz_logits_add / dqz_logits_write, or be followed
 * by dqz_logits_invalidate. */
int dqz_logits_add(dqz_logit_buffer* buf, float* logits, int64_t clear_pos, int64_t write_pos,
                   int64_t size, float* lse_out, void* stream);

/* logits[positions[i]] = values[i] for i in order (a repeated position keeps
 * its last value), keeping the running sum (popleft's -inf, __setitem__,
 * update_priorities: replay_circular.py:180-215).  positions: device int64
 * [n], values: device f32 [n]. */
int dqz_logits_write(dqz_logit_buffer* buf, float* logits, const int64_t* positions, const float* values, int n,
                     void* stream);

/* One write logits[position] = value (by value: popleft's -inf), keeping the
 * running sum and the chunk sum. */
int dqz_logits_put(dqz_logit_buffer* buf, float* logits, int64_t position, float value, void* stream);

/* Running log-sum-exp state of a logit buffer, for checkpoints
 * (parts.py:517-561): S = float64 sum of exp(x - c) over the buffer, the
 * shift c, the device-side valid flag, and the host bookkeeping (known: every
 * write since the last scan went through the library; adds: running adds
 * since that scan).  get synchronises `stream`; set restores all five and
 * recomputes the chunk sums from `logits` about c (they are a function of
 * the two), so a restored buffer continues with the saver's bits (no re-scan
 * on either side). */
int dqz_logits_run_get(dqz_logit_buffer* buf, double* S, float* c, int* valid, int* known, int* adds,
                       void* stream);
int dqz_logits_run_set(dqz_logit_buffer* buf, const float* logits, double S, float c, int valid, int known,
                       int adds, void* stream);

/* The logits were written outside the library (e.g. the meta-update's Adam
 * step, a state restore): the next dqz_logits_add re-scans the buffer. */
int dqz_logits_invalidate(dqz_logit_buffer* buf);

/* Softmax sampling with replacement (CircularLogitBuffer.sample,
 * replay_circular.py:205-217 = Generator.choice(capacity, n, p=softmax)):
 * terms t = expf(x - c) about the running shift c (softmax up to f32
 * rounding of the exponent), cdf = cumsum(float64 t) / total, out_idx[i] =
 * first slot with cdf > uniforms[i].  Reads the chunk sums and one chunk of
 * 4096 logits per query.  uniforms: device f64 [n] in [0,1) (host Generator
 * draws for parity, or dqz_uniform_philox). */
int dqz_logits_sample(dqz_logit_buffer* buf, const float* logits, const double* uniforms, int n,
                      int64_t* out_idx, void* stream);

/* Learner-batch draw in one launch: n uniforms — the caller's `uniforms`
 * (device f64, NULL for Philox) or Philox4x32 (seed, *counter_dev, q), the
 * stream dqz_uniform_philox produces, *counter_dev then advanced on device —
 * and the softmax-CDF choice of dqz_logits_sample, written as int32 slots
 * (out_slots, for dqz_learner_step) and/or int64 (out_idx); either may be
 * NULL.  Replaces Generator.choice(C, n, p=softmax(logits)) +
 * the batch's slot lookup (replay_circular.py:205-217, 540-545) without the
 * uniform launch or an int64 -> int32 copy. */
int dqz_logits_sample_slots(dqz_logit_buffer* buf, const float* logits, uint64_t seed, uint64_t* counter_dev,
                            const double* uniforms, int n, int32_t* out_slots, int64_t* out_idx, void* stream);

/* Diagnostic: the sampling probability of every slot, p = t / total as f32
 * (p_out: device f32 [capacity]; probabilities_from_logits,
 * replay_circular.py:69-76) and the running log-sum-exp (lse_out: device
 * f32, may be NULL). */
/* Exact mode of the learned-logit draw: the reference's own float32
 * probabilities p = probabilities_from_logits(logits) (replay_circular.py:69-76,
 * numpy's float32 exp / log / sum operation for operation, bit for bit) into
 * p_out (capacity floats, or NULL), and n draws for the caller's uniforms
 * (the Generator's random() stream) as Generator.choice(C, n, p) makes them
 * (replay_circular.py:205-217, :540-545): searchsorted(cumsum(p) / total, u,
 * 'right'), the cumsum in float64 in chunk order (a draw can differ from
 * numpy's sequential cumsum only for a uniform within float64 rounding of a
 * CDF step).  Six passes over the buffer; independent of the running state.
 * n = 0: p_out only.  Replaces the reference's `self._rng_state.choice(
 * self._capacity, size=size, p=self.as_probs())` (replay_circular.py:208). */
int dqz_logits_sample_exact(dqz_logit_buffer* buf, const float* logits, const double* uniforms, int n,
                            int64_t* out_idx, float* p_out, void* stream);
/* Exact mode of the default-logit add (replay_circular.py:166-179 add, :518-533
 * add / replace): logits[clear_pos] = -inf first when clear_pos >= 0, then
 * logits[write_pos] = 0 for size 0, else float32(logsumexp(logits) -
 * log(size)) with numpy's float32 logsumexp (as dqz_logits_sample_exact forms
 * it) and a float64 log.  Five small launches, four passes over the buffer;
 * the running state is left unknown (the next default-mode call re-seeds). */
int dqz_logits_add_exact(dqz_logit_buffer* buf, float* logits, int64_t clear_pos, int64_t write_pos, int64_t size,
                         void* stream);
int dqz_logits_probs(dqz_logit_buffer* buf, const float* logits, float* p_out, float* lse_out, void* stream);

/* Diagnostic: the exact terms a draw's CDF is built from, t = expf(x - c)
 * (t_out: device f32 [capacity]), the chunk sums (csum_out: device f64
 * [ceil(capacity / 4096)], may be NULL) and c (c_out: device f32, may be
 * NULL).  Lets a checker separate the index search (bit-exact against numpy's
 * sequential-cumsum choice given the same t) from the last-ulp differences of
 * f32 exp between numpy and the device. */
int dqz_logits_terms(dqz_logit_buffer* buf, const float* logits, float* t_out, double* csum_out, float* c_out,
                     void* stream);

/* n uniform doubles in [0,1) from Philox4x32-10 (counter advanced on device). */
int dqz_uniform_philox(uint64_t seed, uint64_t* counter_dev, int n, double* out, void* stream);

/* Priority write-back of the learner's last step (prioritized/agent.py:201-206,
 * replay.py:620-630): p = |td| (fp64 of the f32 TD errors), *max_seen_dev =
 * max(*max_seen_dev, max p), leaf[slots[i]] = p^alpha (0 -> 0) with the sum
 * tree's ancestors rebuilt (a tree index drawn twice keeps its last draw;
 * `slots` holds tree indices, dqz_per_sample's out_indices).  All
 * device pointers; one launch, no host synchronisation.  Batch <= 256. */
int dqz_per_write_back(dqz_learner* learner, double* tree, int64_t cap, const int32_t* slots, double alpha,
                       double* max_seen_dev, void* stream);

/* ---- prioritized replay: fp64 sum tree in HBM (replay.py:379-559) -------
 * tree: device f64 [2*cap], cap a power of two, node i has children 2i, 2i+1,
 * root at 1, leaves at [cap, 2cap) -- the layout of the host SumTree.
 * set: leaves idx[k] = values[k] (k < n <= 65536), ancestors recomputed as
 * left + right (bit-identical to SumTree.set).  query: SumTree._query_single
 * per target; out = -1 when target is outside [0, root). */
int dqz_sumtree_set(double* tree, int64_t cap, const int64_t* idx, const double* values, int n,
                    void* stream);
int dqz_sumtree_query(const double* tree, int64_t cap, const double* targets, int n, int64_t* out,
                      void* stream);

/* PrioritizedDistribution.sample + importance_sampling_weights on device
 * (replay.py:680-716, 344-376).  Draws: injected_u == NULL -> device Philox
 * (seed, *counter_dev; the counter is advanced), tree leaf index = replay
 * slot, uniform picks over the live window (live_base + j) mod capacity.
 * injected_u != NULL -> the caller's RandomState draws in the reference's
 * order: injected_uniform[i] = active_indices[randint(size)[i]] (a tree
 * index), injected_u[i] = uniform target fraction, injected_u[n + i] = the
 * usp-mix uniform; counter_dev is ignored.  index_to_slot (device int32
 * [cap], or NULL for identity) maps tree indices to replay slots.
 * out_indices (tree indices) and out_probs (f64) may be NULL.  n <= 1024. */
int dqz_per_sample(const double* tree, int64_t cap, int64_t live_base, int64_t size, int64_t capacity,
                   int n, double uniform_sample_probability, double importance_exponent,
                   int normalize_weights, uint64_t seed, uint64_t* counter_dev,
                   const int32_t* injected_uniform, const double* injected_u, const int32_t* index_to_slot,
                   int32_t* out_indices, int32_t* out_slots, float* out_weights, double* out_probs,
                   void* stream);

/* A whole prioritized learn (prioritized/agent.py:187-206) in one learner
 * step: the draw of dqz_per_sample (same streams: Philox (seed,
 * *counter_dev) or the caller's RandomState draws injected, same node
 * sequence, same fp64 probabilities) computed by the forward's conv1
 * workgroups, the IS weights (importance_sampling_weights, normalised by the
 * batch maximum if normalize_weights) formed by the head, the double-Q step
 * with them, and the |td|^alpha write-back inside the backward launch
 * (dqz_learner_step_per).  Outputs: out_indices (tree indices), out_slots,
 * out_probs (f64), out_weights (f32, may be NULL), all device [B].  Batch
 * <= 64, cap a power of two <= 2^24. */
typedef struct dqz_per_draw {
  double* tree;
  int64_t cap;
  int64_t live_base, size, capacity;
  double uniform_sample_probability;
  double importance_sampling_exponent;
  int normalize_weights;
  uint64_t seed;
  uint64_t* counter_dev;
  const int32_t* injected_uniform;
  const double* injected_u;
  const int32_t* index_to_slot;
  double alpha;
  double* max_seen_dev;
  int32_t* out_indices;
  int32_t* out_slots;
  double* out_probs;
  float* out_weights;
} dqz_per_draw;
int dqz_learner_step_per_draw(dqz_learner* learner, const dqz_params* params, const dqz_store* store,
                              const dqz_per_draw* draw, void* stream);

/* PrioritizedTransitionReplay.add on device (replay.py:1068-1096 ->
 * PrioritizedDistribution.remove_priorities / add_priorities, :642-678): the
 * evicted tree index remove_index (-1: none) is set to 0, add_index to
 * _power(priority, alpha) -- priority < 0 reads the agent's running
 * max_seen_priority from max_seen_dev (prioritized/agent.py:155) -- and
 * index_to_slot[add_index] = slot.  One launch, no host synchronisation. */
int dqz_per_add(double* tree, int64_t cap, int32_t remove_index, int32_t add_index, double priority,
                const double* max_seen_dev, double alpha, int32_t* index_to_slot, int32_t slot, void* stream);

/* Target sync: target <- online (dqn/agent.py:155-156; hard copy, not Polyak). */
int dqz_target_copy(float* target, const float* online, int64_t total, void* stream);

/* ---- MGSC meta-update (dqn_mgsc_batched/agent.py:104-220) -------------- */

typedef struct dqz_meta_config {
  int meta_batch;          /* M (meta_batch_size, run_atari.py:101), any size: batches past 256 run in chunks */
  int num_actions;         /* A; the network is dqn_atari_network (per-action bias) */
  float learning_rate;     /* inner optax.rmsprop(centered) lr, run_atari.py:218-223 */
  float decay;             /* 0.95 */
  float eps;               /* optimizer_epsilon */
  float grad_error_bound;  /* rlax.clip_gradient bound */
  float meta_learning_rate; /* optax.adam lr, run_atari.py:241-243 */
  float b1, b2, meta_eps;  /* optax.adam defaults 0.9, 0.999, 1e-8 */
  int second_order;        /* 0: theta'' = stop_gradient(...) (dqn_mgsc_batched/agent.py:191);
                              1: no stop_gradient (dqn_mgsc_batched_reservoir/agent.py):
                              d theta''/d theta' through the online transition's Hessian */
} dqz_meta_config;

typedef struct dqz_meta dqz_meta;

int dqz_meta_create(const dqz_meta_config* cfg, dqz_meta** out);
int dqz_meta_destroy(dqz_meta* meta);

/* One jitted `meta_update` + `replay.update_priorities` (agent.py:211-220,
 * 302-334); written for the stop-gradient variant, cfg.second_order adds the
 * reservoir variant's d theta''/d theta' term (Hessian-vector product):
 *   p = softmax(logits[pos]) (replay_circular.py:79-86); G = sum_i p_i g_i
 *   (per-transition grads of loss_fn, agent.py:152-172); theta' = theta +
 *   RMSProp(G; mu, nu); g' = grad loss_fn(theta', target=theta, online
 *   transition); theta'' = stop_grad(theta' + RMSProp(g'; mu', nu'));
 *   L = sum |theta' - theta''|^2; Adam on the M logits, written back to
 *   logits[pos[i]].
 * params: online / target / mu / nu are read only (the agent's opt_state is
 * not advanced by meta_update).  slots: device int32 [M] meta-batch replay
 * slots in `store`.  online_store/online_slot: the newest transition (device
 * int32 [1]).  logits: the replay's device logit buffer; pos: device int32
 * [M] absolute positions (distinct).  adam_mu/adam_nu: device f32 [M];
 * adam_count: device int32 [1] (ScaleByAdamState).  logit_buf (may be
 * NULL): the dqz_logit_buffer owning `logits`; its running log-sum-exp is
 * then updated for the M writes (positions distinct), so the buffer's next
 * add / sample needs no re-scan; with NULL the caller must call
 * dqz_logits_invalidate. */
int dqz_meta_update(dqz_meta* meta, const dqz_params* params, const dqz_store* store,
                    const int32_t* slots, const dqz_store* online_store, const int32_t* online_slot,
                    float* logits, const int32_t* pos, float* adam_mu, float* adam_nu,
                    int32_t* adam_count, dqz_logit_buffer* logit_buf, void* stream);

/* Device copies of the last meta-update's intermediates (any may be NULL):
 * probs [M], dlogits [M] (d L / d logits), td [M] meta-batch TD errors,
 * loss [1] = sum |theta' - theta''|^2. */
int dqz_meta_outputs(dqz_meta* meta, float* probs, float* dlogits, float* td, float* loss,
                     void* stream);

/* Health word of the meta-update since the previous check (the meta-level
 * counterpart of dqz_learner_sync_status): the OR of the batch learner's
 * and the one-transition learner's words (bit 0: an in-launch hand-off wait
 * gave up, among them the HVP's ddot1 wait; bit 1: a non-finite loss) and of
 * the meta-update's own word (bit 0: the fused Adam leader's wait for the
 * other chunk blocks gave up).  Synchronises the device.  A non-zero status
 * clears every hand-off word of the meta handle (both learners' and its own
 * arrival counters) and the status; callers treat the meta-updates since
 * their previous check as invalid. */
int dqz_meta_sync_status(dqz_meta* meta, int* status);

/* Diagnostic (tests): from the next meta-update on, every bounded wait of the
 * meta handle gives up after `spin_max` polls (0 restores 2^24); poison != 0
 * sets the HVP's ddot1 arrival counter far below its arrivals (second order)
 * and the Adam entry counter far below M, so the next update's waits on them
 * run out — the timeout path of dqz_meta_sync_status, exercised.
 * Synchronises the device. */
int dqz_meta_debug_stall(dqz_meta* meta, int poison, unsigned spin_max);

/* ---- Atari observation preprocessing (processors.py:421-505) -----------
 * The observation branch of processors.atari on device: element-wise max of
 * the last n RGB frames (np.max over the pooled frames), rgb2y
 * (processors.py:367-371, numpy's float64 evaluation, truncated to uint8)
 * and PIL's BILINEAR resize (processors.py:374-387; Pillow's 8-bit
 * fixed-point two-pass resampler), in one launch.  A dqz_frame_plan holds
 * the resize coefficient tables of one (in_h, in_w) -> (out_h, out_w). */
typedef struct dqz_frame_plan dqz_frame_plan;
int dqz_frame_plan_create(int in_h, int in_w, int out_h, int out_w, dqz_frame_plan** out);
int dqz_frame_plan_destroy(dqz_frame_plan* plan);
/* rgb: n frames uint8 [n][in_h][in_w][3], contiguous; out: uint8
 * [out_h][out_w].  Either may be device memory or pinned host memory. */
int dqz_atari_frame(const dqz_frame_plan* plan, const uint8_t* rgb, int n, uint8_t* out, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DQZ_H_ */
