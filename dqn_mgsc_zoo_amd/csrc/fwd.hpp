// fwd.hpp — conv2 / conv3 / fc1 forward as per-sample LDS-window kernels.
//
// B = 32 makes every layer a tiny GEMM (M = 32 x 81 rows at most), so a
// generic tiled GEMM leaves most of the 256 CUs idle and spends its time on
// im2col address arithmetic.  These kernels instead give each workgroup one
// sample (one network copy z) and one 16-channel quarter of the outputs:
//   * the sample's whole input window is staged once into LDS with padded
//     pixel / row strides chosen so that the A-operand reads of a
//     v_mfma_f32_16x16x4_f32 (16 consecutive output positions x 2 k lanes
//     per 32-lane group) hit 32 distinct banks;
//   * each wave owns a quarter of K and keeps its weight slice (the B
//     operand) in registers, loaded once with plain global loads;
//   * the inner loop is fully unrolled: ds_read_b32 at immediate offsets +
//     MFMA, no VALU address math;
//   * the four K-quarter partial tiles are summed through LDS in a fixed
//     order (deterministic), then bias + ReLU (or the linear tangent mode of
//     the MGSC meta-update) and a coalesced store.
// Work per launch: Z x B x 4 workgroups (256 at B = 32, Z = 2).
#pragma once
#include "common.hpp"
#include "conv1.hpp"

namespace dqz {

// 1: the mostly-empty last MFMA row tile of conv2 / conv3 forward and conv2
// dX is replaced by VALU dot products of its few live positions
#ifndef DQZ_TRIM
#define DQZ_TRIM 1
#endif

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Cross-wave partial tiles [row][16] with 16 floats of padding after every
// 4 rows: a 16x16x4 accumulator store (lane (n, kq) writes row 4 kq + r) puts
// lanes kq = 0 / 1 (one ds_write_b32 lane group) 16 banks apart instead of on
// the same banks; a 32-lane read group covers rows 2j, 2j + 1 of one 4-row
// block, so the position-major reads stay conflict-free.
#ifndef DQZ_RED_PAD
#define DQZ_RED_PAD 1
#endif
__device__ __forceinline__ int red_idx(int row, int col) { return row * 16 + (DQZ_RED_PAD ? 16 * (row >> 2) : 0) + col; }
constexpr int red_rows(int rows) { return rows * 16 + (DQZ_RED_PAD ? 16 * ((rows + 3) / 4) : 0); }

struct LayerFwdArgs {
  const float* in;  // [Z][B][...] layer input (NHWC)
  NetZ nz;
  int64_t w_off, b_off;
  int B, Z;
  int linear;  // 1: pre-activation output, no ReLU (tangent forward)
  float* out;  // [Z][B][...]
  Handoff wait, pub;  // fwd_conv_kernel: input produced / output consumed in the same launch
};

// ---- conv2: 20x20x32 -> 9x9x64, 4x4 stride 2 -------------------------------
// LDS image: element (ih, iw, ci) at ih*C2L_RS + iw*C2L_S + ci.  Bank of the
// A read for position p = 9 oh + ow: 2*oh*RS + 2*ow*S = 2p (mod 32).
constexpr int C2L_S = 33, C2L_RS = 665, C2L_WIN = 20 * C2L_RS;  // 13300 floats

// WAIT: y1 of this sample comes from conv1 blocks of the same launch (poll,
// then sc1 window loads).  PUB: y2 stores are sc1 and the block arrives.
template <bool WAIT, bool PUB>
__device__ __forceinline__ void conv2_fwd_body(const LayerFwdArgs& a, float* s_in, const SampleJob sj) {
  DQZ_STAMP(1, 0);
  const int nq = sj.job, b = sj.s % a.B, z = sj.s / a.B;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;  // w = kh
  const int n = lane & 15, kq = lane >> 4;
  const float* W = a.nz.p[z] + a.w_off;  // [512][64], k = kh*128 + kw*32 + ci
  const float bv = a.nz.p[z][a.b_off + 16 * nq + (t & 15)];  // epilogue bias, loaded early
  float wr[32];
#pragma unroll
  for (int kk = 0; kk < 32; ++kk) wr[kk] = W[(w * 128 + 4 * kk + kq) * C2CO + 16 * nq + n];
  const float4* src = reinterpret_cast<const float4*>(a.in + ((int64_t)z * a.B + b) * (C1M * C1CO));
  constexpr int NQ4 = C1M * C1CO / 4;  // 3200
  if constexpr (WAIT) a.wait.wait(sj.s);
  float4 r[13];
#pragma unroll
  for (int q = 0; q < 13; ++q) {
    if constexpr (WAIT)
      r[q] = load_sc1_f4(src, NQ4 * 16, min(t + 256 * q, NQ4 - 1));
    else
      r[q] = src[min(t + 256 * q, NQ4 - 1)];
  }
#pragma unroll
  for (int q = 0; q < 13; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 3, ci = (i & 7) * 4;  // 8 float4 per pixel
      float* d = s_in + (pix / C1O) * C2L_RS + (pix % C1O) * C2L_S + ci;
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  DQZ_STAMP(1, 1);
  __syncthreads();
  // 81 positions = 5 MFMA row tiles + position 80, which every lane folds
  // from its own weight registers on the VALU (a 6th tile would be 1/16 live)
  constexpr int MT = DQZ_TRIM ? 5 : 6;
  int base[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = min(16 * m + n, C2M - 1);
    base[m] = (2 * (p / C2O) + w) * C2L_RS + 2 * (p % C2O) * C2L_S + kq;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float last = 0.f;  // position 80 (oh = ow = 8), this lane's k rows
  const int blast = (2 * (C2O - 1) + w) * C2L_RS + 2 * (C2O - 1) * C2L_S + kq;
#pragma unroll
  for (int kk = 0; kk < 32; ++kk) {
    const int off = (kk >> 3) * C2L_S + 4 * (kk & 7);  // kw, ci block
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma4(s_in[base[m] + off], wr[kk], acc[m]);
    if constexpr (DQZ_TRIM) last = __fmaf_rn(s_in[blast + off], wr[kk], last);
  }
  DQZ_STAMP(1, 2);
  if constexpr (DQZ_TRIM) {
    last += __shfl_xor(last, 16, 64);
    last += __shfl_xor(last, 32, 64);
  }
  __syncthreads();
  float* s_red = s_in;  // [4][96 rows, padded][16]
  constexpr int RW = red_rows(96);
  static_assert(4 * RW <= C2L_WIN, "conv2 partials fit the window");
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * RW + red_idx(16 * m + 4 * kq + rr, n)] = acc[m][rr];
  if (DQZ_TRIM && kq == 0) s_red[w * RW + red_idx(C2M - 1, n)] = last;
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * (C2M * C2CO) + 16 * nq;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  for (int i = t; i < C2M * 16; i += 256) {
    const int k = red_idx(i >> 4, i & 15);
    const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bv;
    if constexpr (PUB)
      __hip_atomic_store(out + (i >> 4) * C2CO + (i & 15), linear ? v : relu(v), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    else
      out[(i >> 4) * C2CO + (i & 15)] = linear ? v : relu(v);
  }
  if constexpr (PUB) a.pub.arrive(sj.s);
  DQZ_STAMP(1, 3);
}

__global__ __launch_bounds__(256) void conv2_fwd_kernel(LayerFwdArgs a) {
  __shared__ float s_in[C2L_WIN];
  const SampleJob sj = xcd_sample_job(4, a.Z * a.B);
  if (!sj.valid) return;
  conv2_fwd_body<false, false>(a, s_in, sj);
}

// ---- conv3: 9x9x64 -> 7x7x64, 3x3 stride 1 ---------------------------------
// Wave w owns input channels [16w, 16w + 16) of every tap.  Bank of the A read
// for p = 7 oh + ow: oh*RS + ow*S = 14 oh + 2 ow = 2p (mod 32).
constexpr int C3L_S = 66, C3L_RS = 622, C3L_WIN = 9 * C3L_RS;  // 5598 floats

template <bool WAIT>
__device__ __forceinline__ void conv3_fwd_body(const LayerFwdArgs& a, float* s_in, const SampleJob sj) {
  DQZ_STAMP(2, 0);
  const int nq = sj.job, b = sj.s % a.B, z = sj.s / a.B;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  const float* W = a.nz.p[z] + a.w_off;  // [576][64], k = (kh*3 + kw)*64 + ci
  const float bv = a.nz.p[z][a.b_off + 16 * nq + (t & 15)];  // epilogue bias, loaded early
  float wr[36];
#pragma unroll
  for (int kk = 0; kk < 36; ++kk)
    wr[kk] = W[((kk >> 2) * C3CI + 16 * w + 4 * (kk & 3) + kq) * C3CO + 16 * nq + n];
  const float4* src = reinterpret_cast<const float4*>(a.in + ((int64_t)z * a.B + b) * (C2M * C2CO));
  constexpr int NQ4 = C2M * C2CO / 4;  // 1296
  if constexpr (WAIT) a.wait.wait(sj.s);
  float4 r[6];
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    if constexpr (WAIT)
      r[q] = load_sc1_f4(src, NQ4 * 16, min(t + 256 * q, NQ4 - 1));
    else
      r[q] = src[min(t + 256 * q, NQ4 - 1)];
  }
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 4, ci = (i & 15) * 4;
      float* d = s_in + (pix / C2O) * C3L_RS + (pix % C2O) * C3L_S + ci;
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  DQZ_STAMP(2, 1);
  __syncthreads();
  // 49 positions = 3 MFMA row tiles + position 48 on the VALU (see conv2)
  constexpr int MT = DQZ_TRIM ? 3 : 4;
  int base[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = min(16 * m + n, C3M - 1);
    base[m] = (p / C3O) * C3L_RS + (p % C3O) * C3L_S + 16 * w + kq;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float last = 0.f;  // position 48 (oh = ow = 6), this lane's k rows
  const int blast = (C3O - 1) * C3L_RS + (C3O - 1) * C3L_S + 16 * w + kq;
#pragma unroll
  for (int kk = 0; kk < 36; ++kk) {
    const int tap = kk >> 2;
    const int off = (tap / 3) * C3L_RS + (tap % 3) * C3L_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma4(s_in[base[m] + off], wr[kk], acc[m]);
    if constexpr (DQZ_TRIM) last = __fmaf_rn(s_in[blast + off], wr[kk], last);
  }
  DQZ_STAMP(2, 2);
  if constexpr (DQZ_TRIM) {
    last += __shfl_xor(last, 16, 64);
    last += __shfl_xor(last, 32, 64);
  }
  __syncthreads();
  float* s_red = s_in;  // [4][64 rows, padded][16]
  constexpr int RW = red_rows(64);
  static_assert(4 * RW <= C3L_WIN, "conv3 partials fit the window");
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * RW + red_idx(16 * m + 4 * kq + rr, n)] = acc[m][rr];
  if (DQZ_TRIM && kq == 0) s_red[w * RW + red_idx(C3M - 1, n)] = last;
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * FLAT + 16 * nq;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  for (int i = t; i < C3M * 16; i += 256) {
    const int k = red_idx(i >> 4, i & 15);
    const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bv;
    out[(i >> 4) * C3CO + (i & 15)] = linear ? v : relu(v);
  }
  DQZ_STAMP(2, 3);
}

__global__ __launch_bounds__(256) void conv3_fwd_kernel(LayerFwdArgs a) {
  __shared__ float s_in[C3L_WIN];
  const SampleJob sj = xcd_sample_job(4, a.Z * a.B);
  if (!sj.valid) return;
  conv3_fwd_body<false>(a, s_in, sj);
}

// ---- conv1 -> conv2 -> conv3 forward in one launch ------------------------
// Grid, in dispatch order, over the Z x B samples s = z B + b:
//   [conv1 4/sample] [conv2 4/sample] [conv3 4/sample]
// conv2 blocks of sample s wait for the 4 conv1 blocks of s (y1 hand-off),
// conv3 blocks for the 4 conv2 blocks (y2).  Producers always have lower
// block indices (workgroups are dispatched in index order), so every wait
// terminates; each range starts at a multiple of 8, so a sample's producer
// and consumer blocks share an XCD (and its L2).  Consumers stage their
// weight slices before they poll.  Dynamic LDS = conv1's 57.6 KB (2 blocks/CU:
// conv1 and conv2 are co-resident from the start, conv3 blocks dispatch as
// conv1 blocks retire).
static_assert(C2L_WIN * sizeof(float) <= kConv1FwdSmem && C3L_WIN * sizeof(float) <= kConv1FwdSmem,
              "fwd_conv_kernel's dynamic LDS holds every body's window");
// F: the fused draw mode of the conv1 blocks (Conv1Src::fused).
template <int F>
__global__ __launch_bounds__(256) void fwd_conv_kernel(Conv1FwdArgs c1, LayerFwdArgs c2, LayerFwdArgs c3) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int zb = c1.Z * c1.B, n = 4 * ((zb + 7) / 8 * 8);
  int i = blockIdx.x;
  if (i < n) {
    const SampleJob sj = xcd_sample_job_at(i, C1_BLOCKS, zb);
    if (sj.valid) conv1_fwd_body<true, F>(c1, smem, sj);
    return;
  }
  i -= n;
  if (i < n) {
    const SampleJob sj = xcd_sample_job_at(i, 4, zb);
    if (sj.valid) conv2_fwd_body<true, true>(c2, smem, sj);
    return;
  }
  const SampleJob sj = xcd_sample_job_at(i - n, 4, zb);
  if (sj.valid) conv3_fwd_body<true>(c3, smem, sj);
}

// ---- fc1: [B][3136] x [3136][512] split-K partials ------------------------
// grid (32 column tiles of 16, FC1_S K-splits of 448, Z * ceil(B/32)); wave w
// owns k in [448 s + 112 w, +112).  K is permuted inside each 16-block so a
// lane's four k for steps e = 0..3 are contiguous: one float4 A load per
// (row tile, 16-block).  Partials [Z][FC1_S][B][512] are reduced by the head.
constexpr int FC1_S = 7, FC1_KS = FLAT / FC1_S, FC1_KW = FC1_KS / 4;  // 448, 112
constexpr int Z_MAX_FC1 = 3;  // network copies of one fc1 launch (online, target, online(s_t))

struct Fc1FwdArgs {
  const float* in;  // [Z][B][3136]
  NetZ nz;
  int64_t w_off;
  int B, MG;        // MG = ceil(B / 32) row groups
  float* part;      // [Z][FC1_S][B][512]
  // In-launch split-K reduce (or null: the head sums the FC1_S partials):
  // the last of a tile's FC1_S split blocks to arrive sums them in split
  // order into sum[Z][B][512] (pre-activation, no bias), so the head loads
  // one row per sample instead of FC1_S.
  float* sum;
  int* cnt;         // [Z * MG * 32] tile arrival counters (x Handoff::kStride ints), zero between launches
};

// The MFMA body of one fc1 block: its (z, split s, column tile nt, row group
// mg) and the four waves' [2][16 x 16] K-quarter tiles in s_red[w * FC1_RW ..]
// (row 16 mt + r, column n at [mt * FC1_RT + red_idx(r, n)]: 16 floats of
// padding after every 4 rows, so the lanes kq = 0 / 1 of one ds_write_b32
// group land 16 banks apart).
constexpr int FC1_RT = red_rows(16), FC1_RW = 2 * FC1_RT;  // 320, 640 floats
__device__ __forceinline__ void fc1_fwd_tile(const Fc1FwdArgs& a, float* s_red, int i, int& z, int& s, int& nt,
                                             int& mg) {
  // Block i -> tile map: the two 16-column tiles that share W1's 128-byte
  // lines (nt = 2 cp, 2 cp + 1) go to blocks i and i + 8, which round-robin
  // dispatch places on the same XCD, so each line is fetched into one L2.
  const int slot = i >> 3, pair = (i & 7) + 8 * (slot >> 1);
  nt = 2 * (pair % 16) + (slot & 1);
  const int rest = pair / 16;
  s = rest % FC1_S;
  const int zm = rest / FC1_S;
  z = zm / a.MG;
  mg = zm % a.MG;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  const int k0 = s * FC1_KS + w * FC1_KW;
  const float* W = a.nz.p[z] + a.w_off + 16 * nt + n;  // [3136][512]
  constexpr int J = FC1_KW / 16;                        // 7
  float wr[J][4];
#pragma unroll
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[j][e] = W[(int64_t)(k0 + 16 * j + 4 * kq + e) * HID];
  float4 av[2][J];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    const int row = min(32 * mg + 16 * mt + n, a.B - 1);
    const float* x = a.in + ((int64_t)z * a.B + row) * FLAT + k0 + 4 * kq;
#pragma unroll
    for (int j = 0; j < J; ++j) av[mt][j] = *reinterpret_cast<const float4*>(x + 16 * j);
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int j = 0; j < J; ++j) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      acc[mt] = mfma4(av[mt][j].x, wr[j][0], acc[mt]);
      acc[mt] = mfma4(av[mt][j].y, wr[j][1], acc[mt]);
      acc[mt] = mfma4(av[mt][j].z, wr[j][2], acc[mt]);
      acc[mt] = mfma4(av[mt][j].w, wr[j][3], acc[mt]);
    }
  }
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * FC1_RW + mt * FC1_RT + red_idx(4 * kq + rr, n)] = acc[mt][rr];
  __syncthreads();
}

// The block's 32 x 16 split partial (the four K-quarter tiles summed in order).
__device__ __forceinline__ void fc1_fwd_store(const Fc1FwdArgs& a, const float* s_red, int z, int s, int nt, int mg) {
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int row = 32 * mg + 16 * h + (t >> 4);
    const float* sr = s_red + h * FC1_RT + red_idx(t >> 4, t & 15);
    const float v = (sr[0] + sr[FC1_RW]) + (sr[2 * FC1_RW] + sr[3 * FC1_RW]);
    if (row < a.B) a.part[(((int64_t)z * FC1_S + s) * a.B + row) * HID + 16 * nt + (t & 15)] = v;
  }
}

// fc1 forward on v_mfma_f32_32x32x2f32 (DQZ_FC1_32, default on since round
// 3: fc1 5.8 -> 4.7 us, 15,870-15,960 -> 16,140-16,240 steps/s; 0 keeps the
// 16x16x4 fc1_fwd_kernel, which the MGSC tangent launch still uses): a block owns
// 32 columns (one 128-byte line of every W1 row it reads) x the 32 rows of
// its row group x one K split; wave w owns k in [448 s + 112 w, +112).  Lane
// l = 32 h + c: B column c, and for MFMA step (g, e), g < 14, e < 4, the k
// pair {8 g + e, 8 g + 4 + e} (half h takes the second), so the A row loads
// are float4.  Output rows (r & 3) + 8 (r >> 2) + 4 h of column c.
#ifndef DQZ_FC1_32
#define DQZ_FC1_32 1
#endif
constexpr bool kFc1M32 = DQZ_FC1_32 != 0;
constexpr int FC1_32RW = 32 * 33;  // one wave's 32 x 32 tile, row stride 33
__device__ __forceinline__ void fc1_fwd_block32(const Fc1FwdArgs& a, float* s_red, int i) {
  const int nt = i % (HID / 32);
  const int rest = i / (HID / 32);
  const int s = rest % FC1_S, zm = rest / FC1_S;
  const int z = zm / a.MG, mg = zm % a.MG;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int k0 = s * FC1_KS + w * FC1_KW + 4 * h;
  const float* W = a.nz.p[z] + a.w_off + 32 * nt + c;  // [3136][512]
  constexpr int G = FC1_KW / 8;                         // 14
  float wr[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[g][e] = W[(int64_t)(k0 + 8 * g + e) * HID];
  const int row = min(32 * mg + c, a.B - 1);
  const float* x = a.in + ((int64_t)z * a.B + row) * FLAT + k0;
  float4 av[G];
#pragma unroll
  for (int g = 0; g < G; ++g) av[g] = *reinterpret_cast<const float4*>(x + 8 * g);
  f32x16 acc = {};
#pragma unroll
  for (int g = 0; g < G; ++g) {
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[g].x, wr[g][0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[g].y, wr[g][1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[g].z, wr[g][2], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[g].w, wr[g][3], acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) s_red[w * FC1_32RW + ((r & 3) + 8 * (r >> 2) + 4 * h) * 33 + c] = acc[r];
  __syncthreads();
  // 256 threads x 4 outputs: row q = t / 8 (0..31), columns 4 (t % 8) .. + 3
  const int q = t >> 3, c4 = 4 * (t & 7);
  if (32 * mg + q < a.B) {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = q * 33 + c4 + e;
      v[e] = (s_red[k] + s_red[FC1_32RW + k]) + (s_red[2 * FC1_32RW + k] + s_red[3 * FC1_32RW + k]);
    }
    *reinterpret_cast<float4*>(a.part + (((int64_t)z * FC1_S + s) * a.B + 32 * mg + q) * HID + 32 * nt + c4) =
        make_float4(v[0], v[1], v[2], v[3]);
  }
}

__global__ __launch_bounds__(256) void fc1_fwd32_kernel(Fc1FwdArgs a) {
  DQZ_STAMP(3, 0);
  __shared__ float s_red[4 * FC1_32RW];
  fc1_fwd_block32(a, s_red, blockIdx.x);
  DQZ_STAMP(3, 3);
}

__global__ __launch_bounds__(256) void fc1_fwd_kernel(Fc1FwdArgs a) {
  DQZ_STAMP(3, 0);
  __shared__ float s_red[4 * FC1_RW];
  int z, s, nt, mg;
  fc1_fwd_tile(a, s_red, blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z), z, s, nt, mg);
  DQZ_STAMP(3, 2);
  const int t = threadIdx.x;
  if (kFc1Reduce && a.sum) {
    // 128 threads x 4 columns: row t / 4, columns 16 nt + 4 (t % 4) .. + 3.
    // Partials go out write-through (16-B sc1 stores) and are read back with
    // sc1 loads by the tile's last block (the guide's hand-off row: one lane
    // per storing workgroup adds to one counter after every wave drained;
    // the workgroup whose add came last reads).  The other blocks' tiles
    // share this block's XCD (the block -> tile map above), so the reads are
    // served from that L2's backing MALL lines at worst.
    __shared__ int s_last;
    const int row = t >> 2, c4 = 4 * (t & 3);
    const int mt = row >> 4, r16 = row & 15;
    const int64_t colo = 16 * nt + c4;
    const int64_t pbytes = (int64_t)Z_MAX_FC1 * FC1_S * a.B * HID * 4;  // buffer range for the rsrc
    if (t < 128) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = mt * FC1_RT + red_idx(r16, c4 + e);
        v[e] = (s_red[k] + s_red[FC1_RW + k]) + (s_red[2 * FC1_RW + k] + s_red[3 * FC1_RW + k]);
      }
      if (32 * mg + row < a.B) {
        const int64_t off = ((((int64_t)z * FC1_S + s) * a.B + 32 * mg + row) * HID + colo) * 4;
        store_sc1_f4(a.part, (int)min(pbytes, (int64_t)INT32_MAX), (int)off, v);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* cnt = a.cnt + ((z * a.MG + mg) * (HID / 16) + nt) * Handoff::kStride;
    if (t == 0) s_last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == FC1_S - 1;
    __syncthreads();
    if (!s_last) return;
    if (t < 128 && 32 * mg + row < a.B) {
      float4 pv[FC1_S];
#pragma unroll
      for (int ss = 0; ss < FC1_S; ++ss) {
        const int64_t e = (((int64_t)z * FC1_S + ss) * a.B + 32 * mg + row) * HID + colo;
        pv[ss] = load_sc1_f4(reinterpret_cast<const float4*>(a.part), (int)min(pbytes, (int64_t)INT32_MAX), (int)(e / 4));
      }
      float4 acc = pv[0];
#pragma unroll
      for (int ss = 1; ss < FC1_S; ++ss) {
        acc.x += pv[ss].x;
        acc.y += pv[ss].y;
        acc.z += pv[ss].z;
        acc.w += pv[ss].w;
      }
      *reinterpret_cast<float4*>(a.sum + ((int64_t)z * a.B + 32 * mg + row) * HID + colo) = acc;
    }
    if (t == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    DQZ_STAMP(3, 3);
    return;
  }
  fc1_fwd_store(a, s_red, z, s, nt, mg);
  DQZ_STAMP(3, 3);
}

// ---- MGSC meta tangent forward in one launch ------------------------------
// V * y_{l-1} + vb of every layer over the meta batch's stored primal
// activations (linear mode, the tangent v as weights; meta.hpp): the four
// layers are independent of each other, so one launch holds them as block
// ranges [conv1 4/sample] [conv2 4/sample] [conv3 4/sample] [fc1 tiles]
// instead of four dependent launches.  Dynamic LDS = conv1's 57.6 KB.
static_assert(4 * FC1_RW * sizeof(float) <= kConv1FwdSmem, "fc1's partial tiles fit the tangent launch's LDS");
inline int tangent_fwd_blocks(int B, int MG) {
  return 3 * 4 * ((B + 7) / 8 * 8) + (HID / (kFc1M32 ? 32 : 16)) * FC1_S * MG;
}
__global__ __launch_bounds__(256) void tangent_fwd_kernel(Conv1FwdArgs c1, LayerFwdArgs c2, LayerFwdArgs c3,
                                                          Fc1FwdArgs f1) {
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
    if (sj.valid) conv3_fwd_body<false>(c3, smem, sj);
    return;
  }
  i -= n;
  if constexpr (kFc1M32) {
    static_assert(4 * FC1_32RW * sizeof(float) <= kConv1FwdSmem, "fc1's 32 x 32 tiles fit the tangent launch's LDS");
    fc1_fwd_block32(f1, smem, i);
  } else {
    int z, s, nt, mg;
    fc1_fwd_tile(f1, smem, i, z, s, nt, mg);
    fc1_fwd_store(f1, smem, z, s, nt, mg);
  }
}

}  // namespace dqz
