// common.hpp — geometry of the NatureQNetwork, error plumbing, small device
// helpers shared by the libdqz kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <string>

#include "dqz.h"

namespace dqz {

// MFMA operand / accumulator vectors (v_mfma_f32_16x16x4f32 / 32x32x2f32).
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define DQZ_STR(x) #x
#define DQZ_XSTR(x) DQZ_STR(x)
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// Two translation units, two code objects.  learner_step.hip (DQZ_STEP_TU
// defined) holds the learner step's kernels and their launchers; learner.hip
// holds every other kernel (samplers, logit buffers, the MGSC meta-update and
// HVP, preprocessing).  Each TU is compiled to its own code object, so the
// learner step's code is laid out by its own sources alone: no edit to another
// kernel can move it ("Code layout").  A kernel defined in a
// header both TUs include is a plain kernel in the TU it belongs to and an
// uninstantiated template (never emitted) in the other.
#ifdef DQZ_STEP_TU
#define DQZ_STEP_KERNEL __global__
#define DQZ_OTHER_KERNEL template <int = 0> __global__
#else
#define DQZ_STEP_KERNEL template <int = 0> __global__
#define DQZ_OTHER_KERNEL __global__
#endif

// ---------------------------------------------------------------------------
// errors (thread-local message behind dqz_last_error; one instance for both
// translation units: an inline function's static)

inline std::string& err_buf() {
  static thread_local std::string s;
  return s;
}

inline int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
inline int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  err_buf() = buf;
  return code;
}

#define DQZ_HIP(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) return fail(DQZ_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// ---------------------------------------------------------------------------
// geometry (networks.py:181-221): NHWC activations, HWIO weights

constexpr int FH = 84, FW = 84, FC = 4, FB = FH * FW;
constexpr int C1K = 8, C1S = 4, C1CO = 32, C1O = 20, C1M = C1O * C1O, C1KK = C1K * C1K * FC;       // 400, 256
constexpr int C2K = 4, C2S = 2, C2CI = 32, C2CO = 64, C2O = 9, C2M = C2O * C2O, C2KK = 16 * C2CI;  // 81, 512
constexpr int C3K = 3, C3CI = 64, C3CO = 64, C3O = 7, C3M = C3O * C3O, C3KK = 9 * C3CI;           // 49, 576
constexpr int FLAT = C3M * C3CO;                                                                  // 3136
constexpr int HID = 512;
constexpr int MAXA = 32;
constexpr int MAXB = 256;

// conv1 work unit: 5 output rows (100 positions) of one sample; its input
// window is 24 rows x 84 columns x 4 channels.
constexpr int C1_ROWS = 5;
constexpr int C1_BLOCKS = C1O / C1_ROWS;          // 4
constexpr int C1_POS = C1_ROWS * C1O;             // 100
constexpr int C1_IN_ROWS = C1S * C1_ROWS + 4;     // 24
constexpr int C1_PLANE = C1_IN_ROWS * FW;         // 2016 floats per channel
constexpr int C1_IN_FLOATS = FC * C1_PLANE;       // 8064

__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

// LDS windows of 64-channel activations with a 66-float pixel stride (conv3
// forward, conv3 / conv2 dX): channels 32..63 sit 2 floats later than in the
// plain layout.  The staging stores four channels per lane (ds_write_b64
// pairs, 8-byte aligned), 16 lanes per pixel; with channel k at k, lanes c and
// c + 8 of a pixel hit the same banks (4c = 4 (c + 8) mod 32): a 2-way
// conflict in every access.  The MFMA reads add the same constant per wave
// (a wave's 16 channels lie in one half), so their bank pattern is unchanged.
__device__ __forceinline__ int win64_ch(int ch) { return ch + 2 * (ch >> 5); }
// networks.py:192: x.astype(jnp.float32) / 255.0 (IEEE division, not a reciprocal multiply)
// x / 255.0f correctly rounded (networks.py:192) without the IEEE division
// sequence: q = x * (1/255) plus one FMA residual correction.  Checked in
// exact arithmetic to equal the rounded quotient for every x in [0, 255].
__device__ __forceinline__ float u8n(unsigned v) {
  constexpr float r = 1.0f / 255.0f;
  const float x = (float)v;
  const float q = x * r;
  return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, x), r, q);
}

// MGSC tangent forward with the meta-update's dot products in its epilogues
// (meta.hpp): instead of storing V * y + vb, a block adds <output, dy> over
// the outputs it owns and writes one partial at part[b * META_DOT_SLOTS +
// slot].  part == null: the outputs are stored as usual.
constexpr int META_DOT_SLOTS = 128;
struct TangentDot {
  const float* dy;  // the layer's p-weighted pre-activation gradients, laid out as its output
  float* part;      // [M][META_DOT_SLOTS]
  int slot0;        // the layer's first slot
};

struct NetZ {
  const float* p[3];  // parameter buffer of network copy z
  int which[3];       // input stack of copy z: 0 = s_tm1, 1 = s_t
};

// optax 0.1.2 scale_by_stddev + scale(-lr) (dqn/run_atari.py:208-213):
//   mu = (1-decay) g + decay mu ; nu = (1-decay) g^2 + decay nu
//   theta += -lr * g * rsqrt(nu - mu^2 + eps)
// The epilogue that consumes each parameter's gradient g where it is formed
// (the fc1 dW blocks of bwd_bc_kernel, update_kernel for every other leaf):
// centered RMSProp in place, or — gradient-output mode, `gout` set — the
// gradient stored at gout[i], or one of the MGSC meta-update's elementwise
// stages (meta.hpp) applied to it instead of in a launch of its own:
//   meta == 1 (meta_rms1): theta' = theta + u(g; mu, nu) -> thp, the updated
//             moments -> mu1, nu1, J = du/dg -> J (and g -> gout when set);
//   meta == 2 (meta_rms2): u' = u(g; mu1, nu1), v = -2 u' J -> vout, and the
//             block's sum of u'^2 -> sq_part[sq_off + block];
//   meta == 3 (meta_second_kernel, second order): g = grad q (-> gout), with
//             g' = -clip(td) g: v_dir -> mu1, w -> nu1 (from G2, mu1, nu1),
//             the block's sums of u'^2 and of g . w -> sq_part / s1_part.
struct Rms {
  float lr, decay, c1, eps;
  float* gout;
  int gacc;  // gradient-output mode: 1 adds into gout (meta-batch chunks), 0 overwrites
  int meta;  // 0 .. 3 (above)
  float *thp, *mu1, *nu1, *J, *vout, *sq_part;
  int sq_off;
  const float* G2;  // meta 3: the meta batch's gradient G
  const float* td;  // meta 3: td' of the one-transition step (device scalar)
  float bound;      // meta 3: grad_error_bound
  float* s1_part;   // meta 3: block sums of grad q . w
  __device__ __forceinline__ bool update() const { return gout == nullptr && meta == 0; }
  // One centered RMSProp step (optax 0.1.2 scale_by_stddev, eps inside the
  // sqrt).  Every multiply-add is an explicit fma: hipcc contracts a*b + c*d
  // either way round depending on the surrounding code, and fc1/w is updated
  // by this function in different kernels of the launch layouts, which must
  // agree bit for bit.
  __device__ __forceinline__ void step(float g, float& th, float& mu, float& nu) const {
    mu = __fmaf_rn(c1, g, decay * mu);
    nu = __fmaf_rn(c1, g * g, decay * nu);
    th = __fmaf_rn(-lr, g * rsqrtf(__fmaf_rn(-mu, mu, nu) + eps), th);
  }
  // meta_rms1 on one parameter: theta' (th), mu' (mu), nu' (nu), J (returned)
  //   J = du/dg = -lr D^{-3/2} (D - c1 g (g - mu')),  D = nu' - mu'^2 + eps
  __device__ __forceinline__ float meta1(float g, float& th, float& mu, float& nu) const {
    const float m = c1 * g + decay * mu;
    const float v = c1 * (g * g) + decay * nu;
    const float d = v - m * m + eps;
    const float rs = rsqrtf(d);
    th = th + (-lr) * (g * rs);
    mu = m;
    nu = v;
    return -lr * (d - c1 * g * (g - m)) * (rs * rs * rs);
  }
  // The second order's u' / v pieces on one parameter: gq = grad q[a],
  // g' = -clip(td') gq, mu'' = d mu1 + c g', nu'' = d nu1 + c g'^2,
  // D2 = nu'' - mu''^2 + eps, u' = -lr g' D2^{-1/2} (sq += u'^2),
  // v_dir = 2 u' c d lr g' D2^{-3/2} (G - mu'') -> mu,
  // w = 2 u' (-lr) D2^{-3/2} (D2 - c g' (g' - mu'')) -> nu (s1 += gq w)
  __device__ __forceinline__ void meta3(float gq, float G, float& mu, float& nu, float clip, float& sq,
                                        float& s1) const {
    const float g = -clip * gq;
    const float m = c1 * g + decay * mu;
    const float v = c1 * (g * g) + decay * nu;
    const float d2 = v - m * m + eps;
    const float rs = rsqrtf(d2);
    const float rs3 = rs * rs * rs;
    const float u = (-lr) * (g * rs);
    mu = 2.f * u * c1 * decay * lr * g * rs3 * (G - m);
    const float w = 2.f * u * (-lr) * rs3 * (d2 - c1 * g * (g - m));
    nu = w;
    sq += u * u;
    s1 += gq * w;
  }
  // meta_rms2 on one parameter: u' = u(g; mu1, nu1); returns v = -2 u' J
  __device__ __forceinline__ float meta2(float g, float m0, float v0, float j, float& sq) const {
    const float m = c1 * g + decay * m0;
    const float v = c1 * (g * g) + decay * v0;
    const float u = (-lr) * (g * rsqrtf(v - m * m + eps));
    sq += u * u;
    return -2.f * u * j;
  }
};

// In-kernel timeline stamps (diagnostic builds only: -DDQZ_TRACE).  Wave 0 of
// every workgroup records s_memrealtime (100 MHz, chip-wide) at named points;
// tools/trace_step.py reads them back with dqz_debug_trace().
#ifdef DQZ_TRACE
constexpr int TRACE_KERNELS = 20, TRACE_BLOCKS = 4096, TRACE_SLOTS = 4;
static __device__ unsigned long long g_dqz_trace[TRACE_KERNELS * TRACE_BLOCKS * TRACE_SLOTS];
#define DQZ_STAMP(kid, slot)                                                                              \
  do {                                                                                                    \
    if (threadIdx.x == 0) {                                                                               \
      const unsigned bl_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                \
      if (bl_ < (unsigned)dqz::TRACE_BLOCKS)                                                              \
        dqz::g_dqz_trace[((kid) * dqz::TRACE_BLOCKS + bl_) * dqz::TRACE_SLOTS + (slot)] =                \
            __builtin_amdgcn_s_memrealtime();                                                             \
    }                                                                                                     \
  } while (0)
#else
#define DQZ_STAMP(kid, slot) \
  do {                       \
  } while (0)
#endif

// Wave64 sum with DPP (VALU-only cross-lane moves; __shfl_xor lowers to
// ds_bpermute, an LDS round trip per step): row_shr 1/2/4/8 leaves each
// 16-lane row's sum in its lane 15, row_bcast 15 / 31 fold the rows into lane
// 63, readlane broadcasts it.  Masked-off lanes read 0 (update_dpp old = 0).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK, 0xf, false));
}

__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0x111>(v);
  v += dpp_f<0x112>(v);
  v += dpp_f<0x114>(v);
  v += dpp_f<0x118>(v);
  v += dpp_f<0x142, 0xa>(v);
  v += dpp_f<0x143, 0xc>(v);
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// The same fold on a double (each 32-bit half moved by the same DPP
// control), left in lane 63 without the broadcast.  Lane 63's additions are
// exactly those a Hillis-Steele inclusive scan performs there (step o adds
// the value lane 63 - o held before the step; the lanes a row_shr leaves
// unread are never on lane 63's path), so the result has the bits of that
// scan's last lane.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ double dpp_d(double v) {
  const unsigned long long b = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)b, CTRL, ROW_MASK, 0xf, false);
  const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp(0, (int)(unsigned)(b >> 32), CTRL, ROW_MASK, 0xf, false);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ double wave_fold63_f64(double v) {
  v += dpp_d<0x111>(v);
  v += dpp_d<0x112>(v);
  v += dpp_d<0x114>(v);
  v += dpp_d<0x118>(v);
  v += dpp_d<0x142, 0xa>(v);
  v += dpp_d<0x143, 0xc>(v);
  return v;
}

// Sum of a 256-thread block's values v (wave sums in a fixed order),
// deterministic, result in every thread.  s: 4 floats of LDS.
__device__ __forceinline__ float block_sum256(float v, float* s) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) s[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = (s[0] + s[1]) + (s[2] + s[3]);
  __syncthreads();
  return r;
}

// Philox4x32-10 (Salmon et al., SC'11).
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const unsigned lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}

// XCD-aware decode of a 1-D grid for per-sample kernels.  Workgroups are
// dispatched round-robin over the 8 XCDs (block i -> XCD i % 8), each with its
// own L2.  Sending every job of sample s to XCD s % 8 in every kernel keeps a
// sample's activations in one L2 from the kernel that writes them to the
// kernel that reads them.  Grid = J * ceil8(nsamp) blocks; padding blocks exit.
struct SampleJob {
  int s, job;
  bool valid;
};

__device__ __forceinline__ SampleJob xcd_sample_job_at(int i, int J, int nsamp) {
  const int x = i & 7, slot = i >> 3;
  const int s = 8 * (slot / J) + x;
  return SampleJob{s, slot % J, s < nsamp};
}

__device__ __forceinline__ SampleJob xcd_sample_job(int J, int nsamp) {
  const int i = blockIdx.x, x = i & 7, slot = i >> 3;
  const int s = 8 * (slot / J) + x;
  return SampleJob{s, slot % J, s < nsamp};
}

inline dim3 xcd_grid(int J, int nsamp) { return dim3((unsigned)(J * ((nsamp + 7) / 8) * 8)); }

// In-launch per-sample hand-off (fwd_conv_kernel: conv1 -> conv2 -> conv3;
// bwd_bc_kernel: conv3 dX -> conv2 dX), the
// form of MI355X_MICROARCH.md's visibility table row 1: producers store the
// payload write-through (sc1), drain (vmcnt(0)) in every storing wave, meet
// at the workgroup barrier, and one lane adds to the sample's counter
// (agent-scope atomic); one consumer lane polls the counter with sc1 loads,
// the workgroup barrier releases the other waves, and every payload load is
// an sc1 load.  The last of `consumers` consumers to pass resets the
// sample's words, so every launch starts from zero (the learner scratch is
// zeroed at creation).  A spin that outlives ~2^24 polls sets *err and gives
// up rather than hang the GPU.
struct Handoff {
  static constexpr int kStride = 64;  // one 256-byte line pair per sample word: pollers of
                                      // different samples never share a line
  int* cnt;  // [B * kStride] producer arrivals
  int* ack;  // [B * kStride] consumers past the wait
  int* err;  // timeout word (0 = ok)
  int need, consumers;
  unsigned spin_max = 1u << 24;  // polls before a wait gives up (dqz_learner_debug_stall shortens it)
  __device__ __forceinline__ void arrive(int b) const {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt + b * kStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __device__ __forceinline__ void wait(int b) const {
    if (threadIdx.x == 0) {
      unsigned spins = 0;
      while (__hip_atomic_load(cnt + b * kStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
        __builtin_amdgcn_s_sleep(4);
        if (++spins > spin_max) {
          __hip_atomic_fetch_or(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
      }
      if (__hip_atomic_fetch_add(ack + b * kStride, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == consumers - 1) {
        __hip_atomic_store(cnt + b * kStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ack + b * kStride, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    __syncthreads();
  }
};

// 16-byte sc1 (L1-bypassing) load of element e of a float4 array of `bytes`
// bytes whose base is wave-uniform (buffer_load_dwordx4 ... sc1).
__device__ __forceinline__ float4 load_sc1_f4(const float4* base, int bytes, int e) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, e * 16, 0, 16));
}

// 4-byte sc1 load of element e of a float array of `bytes` bytes whose base
// is wave-uniform (buffer_load_dword ... sc1).
__device__ __forceinline__ float load_sc1_f1(const float* base, int bytes, int e) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, e * 4, 0, 16));
}

// 16-byte write-through (sc1) store of v at byte offset `off` of a buffer of
// `bytes` bytes whose base is wave-uniform (buffer_store_dwordx4 ... sc1).
__device__ __forceinline__ void store_sc1_f4(float* base, int bytes, int off, f32x4 v) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);
}

// 4-byte write-through (sc1) store of element e (small hand-offs and the
// fused meta Adam's rare re-seed path: 4-byte sc1 stores cost ~6x the
// 16-byte ones per byte).
__device__ __forceinline__ void store_sc1_f1(float* base, int bytes, int e, float v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, e * 4, 0, 16);
}

// Uniform replay draw of the device sampler (replay.py:119-125 distribution):
// draw i of step `ctr` -> live slot (base + floor(u * size)) mod capacity,
// u from Philox(counter = (ctr, i), key = seed).
struct UniformDraw {
  int64_t base, size, capacity;  // base in [0, capacity): callers pass base % capacity
  uint64_t seed;
  uint64_t* counter;  // device step counter (read by the sampling kernel, advanced later)
  int32_t* slots_out;
};

__device__ __forceinline__ int32_t uniform_slot(uint64_t ctr, int i, const UniformDraw& d) {
  const uint4 r = philox4x32(make_uint4((unsigned)ctr, (unsigned)(ctr >> 32), (unsigned)i, 0x5EED5u),
                             make_uint2((unsigned)d.seed, (unsigned)(d.seed >> 32)));
  const uint64_t u = ((uint64_t)r.x << 32) | r.y;
  const int64_t j = (int64_t)__umul64hi(u, (uint64_t)d.size);  // uniform in [0, size)
  const int64_t k = d.base + j;  // base < capacity (host-normalised), j < size <= capacity
  return (int32_t)(k >= d.capacity ? k - d.capacity : k);
}

}  // namespace dqz
