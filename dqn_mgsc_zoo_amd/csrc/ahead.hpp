// ahead.hpp — the target network's forward of the NEXT step's batch, run in
// the spare workgroup slots of this step's launches (the target lookahead of
// dqz_learner_step_uniform_ahead).
//
// q_learning needs max_a Q(theta-, s_t) of the batch (dqn/agent.py:94-106).
// theta- only changes at a target sync (:155-156, every 2,500 learner steps)
// and the next batch is known in advance: its slots are the Philox draws of
// step counter + 1 (UniformDraw::ctr_offset).  So in a learner-only loop over
// an unchanged replay the target copy's conv1 -> conv2 -> conv3 forward of
// step t + 1 can run during step t, beside work that leaves most of the chip
// idle, and step t + 1's forward launch carries only the online copy:
//   fc1 launch    [fc1 of both copies: 224 blocks][conv1 of target(s_t'): 4/sample]
//   fc1 dX launch [fc1 dX: 196 blocks + 4 pad][conv2 of target(s_t'): 4/sample]
//   update launch [update blocks, padded to 8][conv3 of target(s_t'): 4/sample]
// writing the target copy's activation sections y1[1], y2[1], y3[1] (which
// the backward never reads: it uses the online copy's), and the next batch's
// slots into the learner's slots_next, which the next forward launch reads
// and publishes (Conv1Src::fused == 4).  The update launch advances the
// sampler's counter (the head does not: the conv1 lookahead reads it in the
// fc1 launch).  Each range starts at a multiple of 8, so a sample's blocks
// keep its XCD (xcd_sample_job_at).  The layer bodies are the forward
// launch's own, so the target activations are the same bits.
#pragma once
#include "bwd.hpp"
#include "common.hpp"
#include "conv1.hpp"
#include "fwd.hpp"
#include "head.hpp"

namespace dqz {

__host__ __device__ inline int pad8(int n) { return (n + 7) / 8 * 8; }

// fc1 (nf blocks, both copies) + conv1 of the next batch's target copy.
// Dynamic LDS = conv1's 57.6 KB (2 blocks per CU: all 352 resident).
__global__ __launch_bounds__(256) void fc1_ahead_kernel(Fc1FwdArgs f1, int nf, Conv1FwdArgs c1) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int i = blockIdx.x;
  if (i < nf) {
    DQZ_STAMP(3, 0);
    fc1_fwd_block32(f1, smem, i);
    DQZ_STAMP(3, 3);
    return;
  }
  const SampleJob sj = xcd_sample_job_at(i - nf, C1_BLOCKS, c1.B);
  if (sj.valid) conv1_fwd_body<false, 1>(c1, smem, sj);
}

// fc1 dX (+ the dX-ordered W3 / W2 copies) + conv2 of the next batch's
// target copy.  fc1 dX's 75 KB of LDS holds conv2's 53 KB window.
static_assert(C2L_WIN <= FC1X_SMEM, "conv2's window fits fc1 dX's LDS");
__global__ __launch_bounds__(256) void fc1_dx_ahead_kernel(Fc1BwdArgs a, LayerFwdArgs c2) {
  __shared__ __attribute__((aligned(16))) float smem[FC1X_SMEM];
  const int i = blockIdx.x;
  if (i < FC1X_BLOCKS) {
    fc1_dx_block(a, smem, i);
    return;
  }
  const int j = i - pad8(FC1X_BLOCKS);
  if (j < 0) return;
  const SampleJob sj = xcd_sample_job_at(j, 4, c2.B);
  if (sj.valid) conv2_fwd_body<false, false>(c2, smem, sj);
}

// The optimizer update (nupd blocks) + conv3 of the next batch's target
// copy; block 0 advances the sampler's step counter (every conv1 draw of this
// step and of the lookahead has read it by now).
__global__ __launch_bounds__(256) void update_ahead_kernel(UpdArgs u, int nupd, LayerFwdArgs c3,
                                                           uint64_t* advance) {
  __shared__ __attribute__((aligned(16))) float smem[C3L_WIN];
  static_assert(sizeof(float2) * UPD_GROUPS * UPD_PAIRS <= sizeof(float) * C3L_WIN, "update partials fit");
  const int i = blockIdx.x;
  if (i < nupd) {
    update_body(u, reinterpret_cast<float2(*)[UPD_PAIRS]>(smem), i);
    if (i == 0 && threadIdx.x == 0)
      __hip_atomic_fetch_add(advance, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  const int j = i - pad8(nupd);
  if (j < 0) return;
  const SampleJob sj = xcd_sample_job_at(j, 4, c3.B);
  if (sj.valid) conv3_fwd_body<false>(c3, smem, sj);
}

}  // namespace dqz
