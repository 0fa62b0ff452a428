// learner_impl.hpp — host-side internals shared by libdqz's two translation
// units (common.hpp, "Two translation units, two code objects"): the learner
// handle, its parameter layout, argument checks, and the learner step's entry
// (step_impl, defined in learner_step.hip) that the MGSC meta-update and the
// fused samplers in learner.hip call.
#pragma once
#include <hip/hip_runtime.h>

#include <cstring>

#include "common.hpp"
#include "conv1.hpp"
#include "fwd.hpp"
#include "head.hpp"
#include "bwd.hpp"
#include "sampling.hpp"

namespace dqz {

inline void param_layout(int A, int shared_bias, int64_t off[10], int64_t sz[10], int64_t* total) {
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

}  // namespace dqz

struct dqz_learner {
  dqz_learner_config cfg;
  int Z, shared_bias;
  int64_t off[10], sz[10], total;
  int S_fc1, S2, S3;
  float *y1, *y2, *y3, *fc1p, *h1, *q, *dz1, *dy3, *dy2, *dy1, *p1, *p2, *p3, *td, *loss, *loss_part, *gq, *rec;
  float *w3p, *w2p;  // dX-ordered weight copies written by fc1_dx_kernel each step
  double* per_wb;    // [B] the fused PER draw's unnormalised IS weights (conv1 -> head)
  int32_t* ga;
  int32_t* sync;  // hand-off words (x Handoff::kStride): dy2 cnt/ack [B] each, fwd y1/y2 cnt/ack [3B] each,
                  // dy1 cnt/ack [B] each, then the error word (dqz_learner_sync_status)
  unsigned spin_max = 1u << 24;  // hand-off polls before a wait gives up
  void* block;
};


namespace dqz {

inline int check_store(const dqz_store* S) {
  if (!S || !S->frames || !S->fidx || !S->action || !S->reward || !S->discount)
    return fail(DQZ_ERR_INVALID, "store has a null buffer");
  if (S->capacity < 1) return fail(DQZ_ERR_INVALID, "store capacity must be positive");
  return DQZ_OK;
}

// Device address of p: device memory as is, pinned host memory through its
// mapped device pointer.  Pageable host memory is refused (a kernel access
// would fault).
inline int device_view(const void* p, const void** out, const char* what) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return fail(DQZ_ERR_INVALID, "%s must be device memory or pinned host memory", what);
  }
  if (attr.type == hipMemoryTypeHost) {
    void* d = attr.devicePointer;
    if (!d && hipHostGetDevicePointer(&d, const_cast<void*>(p), 0) != hipSuccess) {
      (void)hipGetLastError();
      return fail(DQZ_ERR_INVALID, "%s: pinned host memory without a device mapping", what);
    }
    *out = d;
  } else if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged ||
             attr.type == hipMemoryTypeUnified) {
    *out = p;
  } else {
    return fail(DQZ_ERR_INVALID, "%s must be device memory or pinned host memory", what);
  }
  return DQZ_OK;
}

// dqz_learner_profile: each phase's launch is repeated `reps` times back to
// back between two events on the launch stream, so ms[i] is that kernel's
// average duration in a saturated stream (what rocprofv3's kernel trace
// reports), not a single launch plus its dispatch gap.
struct PhaseEvents {
  hipEvent_t e0, e1;
  int reps;
  float* ms;
  bool on() const { return ms != nullptr; }
};
inline const PhaseEvents kNoProfile{nullptr, nullptr, 0, nullptr};


// One learner step (learner_step.hip; the arguments are documented there).
int step_impl(dqz_learner* L, const dqz_params* P, const dqz_store* S, const int32_t* slots,
              const float* is_weights, void* stream, PhaseEvents pe, float* gout = nullptr,
              const float* meta_p = nullptr, const UniformDraw* draw = nullptr, int unit = 0,
              int gacc = 0, const PerWbArgs* wb = nullptr, const SoftmaxDraw* sm = nullptr,
              const PerSampleArgs* pd = nullptr, const Rms* meta_epi = nullptr,
              const HeadArgs* meta_sm = nullptr, uint8_t* xout = nullptr);

}  // namespace dqz
