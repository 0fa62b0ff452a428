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

// The mostly-empty last MFMA row tile of conv2 / conv3 forward and conv2 dX
// ("trim") is replaced by VALU dot products of its few live positions.

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Cross-wave partial tiles [row][16] with 16 floats of padding after every
// 4 rows: a 16x16x4 accumulator store (lane (n, kq) writes row 4 kq + r) puts
// lanes kq = 0 / 1 (one ds_write_b32 lane group) 16 banks apart instead of on
// the same banks; a 32-lane read group covers rows 2j, 2j + 1 of one 4-row
// block, so the position-major reads stay conflict-free.
__device__ __forceinline__ int red_idx(int row, int col) { return row * 16 + 16 * (row >> 2) + col; }

// Epilogues that read four channels of a reduction row per lane
// (ds_read_b128): a 64-lane wave covers 16 rows, and the LDS serves it in
// four 16-lane groups {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, ... (four
// rows each).  With row = lane / 4, two rows of a group share a bank quad in
// the padded layout (row start 16 (row + row / 4) mod 64 dwords): 2-way
// conflicts in every group.  This order gives each group four rows whose
// starts are 0, 16, 32, 48 mod 64: lane quad q of the wave's 16 takes row
// 16 (i / 64) + kEpiPerm[q].  Every row of [0, 16 ceil(rows / 16)) is visited
// once, so loops run i over that range and skip rows past the end.
__device__ __forceinline__ int epi_row(int i) {
  return ((i >> 6) << 4) + (int)((0xFBAE9DC873261540ull >> (4 * ((i >> 2) & 15))) & 15);
}
constexpr int epi_range(int rows) { return (rows + 15) / 16 * 64; }
constexpr int red_rows(int rows) { return rows * 16 + 16 * ((rows + 3) / 4); }

struct LayerFwdArgs {
  const float* in;  // [Z][B][...] layer input (NHWC)
  NetZ nz;
  int64_t w_off, b_off;
  int B, Z;
  int linear;  // 1: pre-activation output, no ReLU (tangent forward)
  float* out;  // [Z][B][...]
  Handoff wait, pub;  // fwd_conv_kernel: input produced / output consumed in the same launch
  int jobs = 4;       // fwd_conv_kernel: jobs per sample of this layer (4 or 8, fwd_conv_jobs)
  TangentDot dot = {nullptr, nullptr, 0};  // MGSC tangent: dot products instead of stores
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
  // PUB epilogue: the bias of this lane's 4 channels 4 (t & 3) .. + 3
  const float4 bias4 = PUB ? *reinterpret_cast<const float4*>(a.nz.p[z] + a.b_off + 16 * nq + 4 * (t & 3))
                           : make_float4(0.f, 0.f, 0.f, 0.f);
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
  // all 13 window loads in flight before the first LDS store (left alone the
  // scheduler issued the 13th only after ten had returned: one more round
  // trip after the hand-off)
  __builtin_amdgcn_sched_barrier(0);
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
  constexpr int MT = 5;
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
    last = __fmaf_rn(s_in[blast + off], wr[kk], last);
  }
  DQZ_STAMP(1, 2);
  {
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
  if (kq == 0) s_red[w * RW + red_idx(C2M - 1, n)] = last;
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * (C2M * C2CO) + 16 * nq;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  const bool dot = a.dot.part != nullptr;
  const float* dyp = a.dot.dy + ((int64_t)z * a.B + b) * (C2M * C2CO) + 16 * nq;
  float dacc = 0.f;
  if constexpr (PUB) {
    // y2 handed to conv3: 4 channels per lane, one 16-byte write-through store
    // each (324 per block instead of 1,296 4-byte ones, which the guide prices
    // at ~6x per byte; same values)
    for (int i = t; i < epi_range(C2M); i += 256) {
      const int p = epi_row(i), c4 = 4 * (i & 3);
      if (p >= C2M) continue;
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = red_idx(p, c4 + e);
        const float bb = e == 0 ? bias4.x : e == 1 ? bias4.y : e == 2 ? bias4.z : bias4.w;
        const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bb;
        o[e] = linear ? v : relu(v);
      }
      store_sc1_f4(out, (C2M * C2CO - 16 * nq) * 4, 4 * (p * C2CO + c4), f32x4{o[0], o[1], o[2], o[3]});
    }
    a.pub.arrive(sj.s);
  } else {
    for (int i = t; i < C2M * 16; i += 256) {
      const int k = red_idx(i >> 4, i & 15);
      const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bv;
      if (dot)
        dacc += v * dyp[(i >> 4) * C2CO + (i & 15)];
      else
        out[(i >> 4) * C2CO + (i & 15)] = linear ? v : relu(v);
    }
  }
  if (!PUB && dot) {
    __syncthreads();
    const float r = block_sum256(dacc, s_in);
    if (t == 0) a.dot.part[(int64_t)b * META_DOT_SLOTS + a.dot.slot0 + nq] = r;
  }
  DQZ_STAMP(1, 3);
}

// fwd_conv_kernel's conv2: 8 jobs per sample, job j = output rows
// [5 (j >> 2), +5 or +4) (45 / 36 positions) x output channels [16 (j & 3),
// +16).  Against the 4 channel-quarter jobs of conv2_fwd_body each job stages
// 60 % / 50 % of y1 (input rows [10 (j >> 2), +12 or +10): the bytes that
// arrive after the hand-off wait) and runs 3 MFMA row tiles instead of 5, so
// the per-sample chain after conv1 is shorter; y2 goes out as 16-byte
// write-through stores (4 channels per lane) and conv3 waits for 8 arrivals.
constexpr int C2F_ROWS0 = 5;
__device__ __forceinline__ void conv2_fwd8_body(const LayerFwdArgs& a, float* s_in, const SampleJob sj) {
  DQZ_STAMP(1, 0);
  const int rh = sj.job >> 2, nq = sj.job & 3, b = sj.s % a.B, z = sj.s / a.B;
  const int oh0 = rh * C2F_ROWS0, npos = (rh ? C2O - C2F_ROWS0 : C2F_ROWS0) * C2O;  // 45 / 36
  const int ih0 = C2S * oh0, nrows = C2S * (npos / C2O - 1) + C2K;               // 12 / 10
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;  // w = kh
  const int n = lane & 15, kq = lane >> 4;
  const float* W = a.nz.p[z] + a.w_off;  // [512][64], k = kh*128 + kw*32 + ci
  // epilogue bias of this lane's channels 16 nq + 4 (t & 3) .. + 3, loaded early
  const float4 bias4 = *reinterpret_cast<const float4*>(a.nz.p[z] + a.b_off + 16 * nq + 4 * (t & 3));
  float wr[32];
#pragma unroll
  for (int kk = 0; kk < 32; ++kk) wr[kk] = W[(w * 128 + 4 * kk + kq) * C2CO + 16 * nq + n];
  const float4* src = reinterpret_cast<const float4*>(a.in + ((int64_t)z * a.B + b) * (C1M * C1CO)) +
                      ih0 * C1O * (C1CO / 4);
  const int nq4 = nrows * C1O * (C1CO / 4);  // 1920 / 1600 float4
  a.wait.wait(sj.s);
  constexpr int NL = (2 * C2F_ROWS0 + 2) * C1O * (C1CO / 4) / 256;  // 7.5 -> 8 loads per thread at most
  float4 r[NL + 1];
#pragma unroll
  for (int q = 0; q <= NL; ++q) r[q] = load_sc1_f4(src, nq4 * 16, min(t + 256 * q, nq4 - 1));
  __builtin_amdgcn_sched_barrier(0);  // every window load in flight before the first LDS store
#pragma unroll
  for (int q = 0; q <= NL; ++q) {
    const int i = t + 256 * q;
    if (i < nq4) {
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
  constexpr int MT = 3;  // 48 rows: the tail rows clamp to the last position and are not stored
  int base[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = min(16 * m + n, npos - 1);
    base[m] = (2 * (p / C2O) + w) * C2L_RS + 2 * (p % C2O) * C2L_S + kq;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 32; ++kk) {
    const int off = (kk >> 3) * C2L_S + 4 * (kk & 7);  // kw, ci block
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma4(s_in[base[m] + off], wr[kk], acc[m]);
  }
  DQZ_STAMP(1, 2);
  __syncthreads();
  float* s_red = s_in;  // [4][48 rows, padded][16]
  constexpr int RW = red_rows(16 * MT);
  static_assert(4 * RW <= C2L_WIN, "conv2 partials fit the window");
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * RW + red_idx(16 * m + 4 * kq + rr, n)] = acc[m][rr];
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * (C2M * C2CO) + oh0 * C2O * C2CO + 16 * nq;
  const int out_bytes = (C2M * C2CO - oh0 * C2O * C2CO - 16 * nq) * 4;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  for (int i = t; i < epi_range(npos); i += 256) {
    const int p = epi_row(i), c4 = 4 * (i & 3);
    if (p >= npos) continue;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = red_idx(p, c4 + e);
      const float bb = e == 0 ? bias4.x : e == 1 ? bias4.y : e == 2 ? bias4.z : bias4.w;
      const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bb;
      o[e] = linear ? v : relu(v);
    }
    store_sc1_f4(out, out_bytes, 4 * (p * C2CO + c4), f32x4{o[0], o[1], o[2], o[3]});
  }
  a.pub.arrive(sj.s);
  DQZ_STAMP(1, 3);
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
  __builtin_amdgcn_sched_barrier(0);  // every window load in flight before the first LDS store
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 4, ci = (i & 15) * 4;
      float* d = s_in + (pix / C2O) * C3L_RS + (pix % C2O) * C3L_S + win64_ch(ci);
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  DQZ_STAMP(2, 1);
  __syncthreads();
  // 49 positions = 3 MFMA row tiles + position 48 on the VALU (see conv2)
  constexpr int MT = 3;
  int base[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = min(16 * m + n, C3M - 1);
    base[m] = (p / C3O) * C3L_RS + (p % C3O) * C3L_S + win64_ch(16 * w) + kq;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float last = 0.f;  // position 48 (oh = ow = 6), this lane's k rows
  const int blast = (C3O - 1) * C3L_RS + (C3O - 1) * C3L_S + win64_ch(16 * w) + kq;
#pragma unroll
  for (int kk = 0; kk < 36; ++kk) {
    const int tap = kk >> 2;
    const int off = (tap / 3) * C3L_RS + (tap % 3) * C3L_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma4(s_in[base[m] + off], wr[kk], acc[m]);
    last = __fmaf_rn(s_in[blast + off], wr[kk], last);
  }
  DQZ_STAMP(2, 2);
  {
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
  if (kq == 0) s_red[w * RW + red_idx(C3M - 1, n)] = last;
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * FLAT + 16 * nq;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  const bool dot = a.dot.part != nullptr;
  const float* dyp = a.dot.dy + ((int64_t)z * a.B + b) * FLAT + 16 * nq;
  float dacc = 0.f;
  for (int i = t; i < C3M * 16; i += 256) {
    const int k = red_idx(i >> 4, i & 15);
    const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bv;
    if (dot)
      dacc += v * dyp[(i >> 4) * C3CO + (i & 15)];
    else
      out[(i >> 4) * C3CO + (i & 15)] = linear ? v : relu(v);
  }
  if (dot) {
    __syncthreads();
    const float r = block_sum256(dacc, s_in);
    if (t == 0) a.dot.part[(int64_t)b * META_DOT_SLOTS + a.dot.slot0 + nq] = r;
  }
  DQZ_STAMP(2, 3);
}

// ---- conv3 forward on bf16 MFMA with three-piece operands (build option) ----
// -DDQZ_CONV3_BF16X3 (off by default; round 6, profiles/r06/bf16x3/): both
// operands of every product are f32, each the exact sum of three bf16 pieces
// (split3_bf16), and the six largest of the nine piece products (hi hi, hi
// mid, mid hi, hi lo, mid mid, lo hi) leave out terms below 2^-24 of |x w|:
// f32 accuracy on v_mfma_f32_16x16x32_bf16 (16 cycles for K = 32, against
// 8 x 32 on v_mfma_f32_16x16x4_f32).  Wave w takes the row-tile pair th =
// w & 1 (positions 32 th + [0, 32), past 48 clamped and dropped) and the K
// half kh = w >> 1 (k = (kh*3 + kw)*64 + ci in [288 kh, +288): nine K steps
// of 32 = 32 consecutive ci of one tap).  Weight fragments are split while
// the job waits for its input; the window once, at staging.  LDS image (bf16
// units): pixel (ih, iw), piece q, channel ci at ih * C3B_RS + iw * C3B_S +
// 64 q + ci; a lane's A fragment is 8 consecutive ci (one ds_read_b128); in
// dwords the pixel stride is 136 = 8 and the row stride 1272 = 56 (mod 64),
// so position p starts at 8p (mod 64) and each 16-lane group of the read
// covers the 64 banks once.  Parity-green (the learner and 50-step
// trajectory tests); the forward launch 16.06 -> 15.78 us back to back, the
// graph-replayed step within noise (16,276 against 16,336 steps/s over four
// interleaved rounds), so the default stays f32.
#ifdef DQZ_CONV3_BF16X3
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
constexpr int C3B_S = 272, C3B_RS = 2544, C3B_WIN = 9 * C3B_RS;  // bf16: 22,896 (45.8 KB)
static_assert(C3B_WIN * 2 <= (int)kConv1FwdSmem, "conv3 bf16 pieces fit the forward launch's LDS");

__device__ __forceinline__ bf16x8v pk_bf16x8(const unsigned (&v)[8]) {
  return __builtin_bit_cast(bf16x8v, make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16),
                                                v[6] | (v[7] << 16)));
}

template <bool WAIT>
__device__ __forceinline__ void conv3_fwd_body_bf3(const LayerFwdArgs& a, float* s_in, const SampleJob sj) {
  DQZ_STAMP(2, 0);
  const int nq = sj.job, b = sj.s % a.B, z = sj.s / a.B;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, g = lane >> 4;
  const int th = w & 1, kh = w >> 1;
  const float* W = a.nz.p[z] + a.w_off;  // [576][64], k = (kh*3 + kw)*64 + ci
  const float bv = a.nz.p[z][a.b_off + 16 * nq + (t & 15)];  // epilogue bias, loaded early
  // B fragments: K step s -> k0 = 288 kh + 32 s; lane (n, g): k0 + 8 g + j, co = 16 nq + n
  bf16x8v wb[9][3];
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    float wv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) wv[j] = W[(288 * kh + 32 * s + 8 * g + j) * C3CO + 16 * nq + n];
    unsigned h[8], m[8], l[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) split3_bf16(wv[j], h[j], m[j], l[j]);
    wb[s][0] = pk_bf16x8(h);
    wb[s][1] = pk_bf16x8(m);
    wb[s][2] = pk_bf16x8(l);
  }
  // split now, under the hand-off wait (the compiler would sink it into the MFMA loop)
#pragma unroll
  for (int s = 0; s < 9; ++s)
#pragma unroll
    for (int q = 0; q < 3; ++q) asm volatile("" : "+v"(wb[s][q]));
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
  __builtin_amdgcn_sched_barrier(0);  // every window load in flight before the first LDS store
  uint16_t* s16 = reinterpret_cast<uint16_t*>(s_in);
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 4, ci = (i & 15) * 4;
      uint16_t* d = s16 + (pix / C2O) * C3B_RS + (pix % C2O) * C3B_S + ci;
      unsigned h[4], m[4], l[4];
      split3_bf16(r[q].x, h[0], m[0], l[0]);
      split3_bf16(r[q].y, h[1], m[1], l[1]);
      split3_bf16(r[q].z, h[2], m[2], l[2]);
      split3_bf16(r[q].w, h[3], m[3], l[3]);
      *reinterpret_cast<uint2*>(d) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
      *reinterpret_cast<uint2*>(d + 64) = make_uint2(m[0] | (m[1] << 16), m[2] | (m[3] << 16));
      *reinterpret_cast<uint2*>(d + 128) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
    }
  }
  DQZ_STAMP(2, 1);
  __syncthreads();
  int base[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = min(32 * th + 16 * i + n, C3M - 1);
    base[i] = (p / C3O) * C3B_RS + (p % C3O) * C3B_S + 8 * g;
  }
  f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int s = 0; s < 9; ++s) {
    const int k0 = 288 * kh + 32 * s, tap = k0 >> 6;
    const int off = (tap / 3) * C3B_RS + (tap % 3) * C3B_S + (k0 & 63);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint16_t* pa = s16 + base[i] + off;
      const bf16x8v ah = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const uint4*>(pa));
      const bf16x8v am = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const uint4*>(pa + 64));
      const bf16x8v al = __builtin_bit_cast(bf16x8v, *reinterpret_cast<const uint4*>(pa + 128));
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wb[s][0], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wb[s][1], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, wb[s][0], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, wb[s][2], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, wb[s][1], acc[i], 0, 0, 0);
      acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, wb[s][0], acc[i], 0, 0, 0);
    }
  }
  DQZ_STAMP(2, 2);
  __syncthreads();
  float* s_red = s_in;  // [2 K halves][64 rows, padded][16]
  constexpr int RW = red_rows(64);
  static_assert(2 * RW <= C3L_WIN, "conv3 partials fit the window");
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) {
      const int row = 32 * th + 16 * i + 4 * g + rr;
      if (row < C3M) s_red[kh * RW + red_idx(row, n)] = acc[i][rr];
    }
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * FLAT + 16 * nq;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  const bool dot = a.dot.part != nullptr;
  const float* dyp = a.dot.dy + ((int64_t)z * a.B + b) * FLAT + 16 * nq;
  float dacc = 0.f;
  for (int i = t; i < C3M * 16; i += 256) {
    const int k = red_idx(i >> 4, i & 15);
    const float v = (s_red[k] + s_red[RW + k]) + bv;
    if (dot)
      dacc += v * dyp[(i >> 4) * C3CO + (i & 15)];
    else
      out[(i >> 4) * C3CO + (i & 15)] = linear ? v : relu(v);
  }
  if (dot) {
    __syncthreads();
    const float r = block_sum256(dacc, s_in);
    if (t == 0) a.dot.part[(int64_t)b * META_DOT_SLOTS + a.dot.slot0 + nq] = r;
  }
  DQZ_STAMP(2, 3);
}
#endif  // DQZ_CONV3_BF16X3

// fwd_conv_kernel's conv3: 8 jobs per sample, job j = output rows
// [4 (j >> 2), +4 or +3) (28 / 21 positions, 2 MFMA row tiles instead of 3 +
// the VALU position) x output channels [16 (j & 3), +16); each stages input
// rows [4 (j >> 2), +6 or +5) of y2 (67 % / 56 %) after its hand-off wait.
constexpr int C3F_ROWS0 = 4;
// fwd_conv_kernel runs conv2 / conv3 as 8 jobs per sample when the launch
// has at most kFwd8MaxSamples samples (Z x B): with every block resident from
// the start the launch is one latency chain per sample, and halving each
// job's rows shortens it (the actor's and the MGSC one-transition forward);
// at the learner's 64 samples the 4-job bodies are faster (fewer, fuller
// MFMA row tiles and every conv2 block resident from the start).
constexpr int kFwd8MaxSamples = 16;
inline int fwd_conv_jobs(int zb) { return zb <= kFwd8MaxSamples ? 8 : 4; }
__device__ __forceinline__ void conv3_fwd8_body(const LayerFwdArgs& a, float* s_in, const SampleJob sj) {
  DQZ_STAMP(2, 0);
  const int rh = sj.job >> 2, nq = sj.job & 3, b = sj.s % a.B, z = sj.s / a.B;
  const int oh0 = rh * C3F_ROWS0, npos = (rh ? C3O - C3F_ROWS0 : C3F_ROWS0) * C3O;  // 28 / 21
  const int nrows = npos / C3O + C3K - 1;                                          // 6 / 5
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  const float* W = a.nz.p[z] + a.w_off;  // [576][64], k = (kh*3 + kw)*64 + ci
  const float4 bias4 = *reinterpret_cast<const float4*>(a.nz.p[z] + a.b_off + 16 * nq + 4 * (t & 3));
  float wr[36];
#pragma unroll
  for (int kk = 0; kk < 36; ++kk)
    wr[kk] = W[((kk >> 2) * C3CI + 16 * w + 4 * (kk & 3) + kq) * C3CO + 16 * nq + n];
  const float4* src = reinterpret_cast<const float4*>(a.in + ((int64_t)z * a.B + b) * (C2M * C2CO)) +
                      oh0 * C2O * (C2CO / 4);
  const int nq4 = nrows * C2O * (C2CO / 4);  // 864 / 720 float4
  a.wait.wait(sj.s);
  constexpr int NL = ((C3F_ROWS0 + C3K - 1) * C2O * (C2CO / 4) + 255) / 256;  // 4
  float4 r[NL];
#pragma unroll
  for (int q = 0; q < NL; ++q) r[q] = load_sc1_f4(src, nq4 * 16, min(t + 256 * q, nq4 - 1));
  __builtin_amdgcn_sched_barrier(0);  // every window load in flight before the first LDS store
#pragma unroll
  for (int q = 0; q < NL; ++q) {
    const int i = t + 256 * q;
    if (i < nq4) {
      const int pix = i >> 4, ci = (i & 15) * 4;
      float* d = s_in + (pix / C2O) * C3L_RS + (pix % C2O) * C3L_S + win64_ch(ci);
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  DQZ_STAMP(2, 1);
  __syncthreads();
  constexpr int MT = 2;  // 32 rows: the tail rows clamp to the last position and are not stored
  int base[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = min(16 * m + n, npos - 1);
    base[m] = (p / C3O) * C3L_RS + (p % C3O) * C3L_S + win64_ch(16 * w) + kq;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 36; ++kk) {
    const int tap = kk >> 2;
    const int off = (tap / 3) * C3L_RS + (tap % 3) * C3L_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma4(s_in[base[m] + off], wr[kk], acc[m]);
  }
  DQZ_STAMP(2, 2);
  __syncthreads();
  float* s_red = s_in;  // [4][32 rows, padded][16]
  constexpr int RW = red_rows(16 * MT);
  static_assert(4 * RW <= C3L_WIN, "conv3 partials fit the window");
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * RW + red_idx(16 * m + 4 * kq + rr, n)] = acc[m][rr];
  __syncthreads();
  float* out = a.out + ((int64_t)z * a.B + b) * FLAT + oh0 * C3O * C3CO + 16 * nq;
  const bool linear = a.linear;  // read once (see conv1_fwd_body)
  for (int i = t; i < epi_range(npos); i += 256) {
    const int p = epi_row(i), c4 = 4 * (i & 3);
    if (p >= npos) continue;
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = red_idx(p, c4 + e);
      const float bb = e == 0 ? bias4.x : e == 1 ? bias4.y : e == 2 ? bias4.z : bias4.w;
      const float v = ((s_red[k] + s_red[RW + k]) + (s_red[2 * RW + k] + s_red[3 * RW + k])) + bb;
      o[e] = linear ? v : relu(v);
    }
    *reinterpret_cast<float4*>(out + p * C3CO + c4) = make_float4(o[0], o[1], o[2], o[3]);
  }
  DQZ_STAMP(2, 3);
}


// ---- conv1 -> conv2 -> conv3 forward in one launch ------------------------
// Grid, in dispatch order, over the Z x B samples s = z B + b:
//   [conv1 4/sample] [conv2 J/sample] [conv3 J/sample], J = fwd_conv_jobs(Z B)
// conv2 blocks of sample s wait for the 4 conv1 blocks of s (y1 hand-off),
// conv3 blocks for the J conv2 blocks (y2).  Producers always have lower
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
  const int j2 = c2.jobs, j3 = c3.jobs;  // 4 or 8 per sample (fwd_conv_jobs)
  if (i < (j2 / 4) * n) {
    const SampleJob sj = xcd_sample_job_at(i, j2, zb);
    if (sj.valid) {
      if (j2 == 8)
        conv2_fwd8_body(c2, smem, sj);
      else
        conv2_fwd_body<true, true>(c2, smem, sj);
    }
    return;
  }
  const SampleJob sj = xcd_sample_job_at(i - (j2 / 4) * n, j3, zb);
  if (sj.valid) {
    if (j3 == 8)
      conv3_fwd8_body(c3, smem, sj);
    else
#ifdef DQZ_CONV3_BF16X3
      conv3_fwd_body_bf3<true>(c3, smem, sj);
#else
      conv3_fwd_body<true>(c3, smem, sj);
#endif
  }
}

// ---- fc1: [B][3136] x [3136][512] split-K partials ------------------------
// One block per (32-column tile nt, K split s of 448, network copy z, 32-row
// group mg), on v_mfma_f32_32x32x2f32: the block owns 32 columns (one 128-byte
// line of every W1 row it reads) x the 32 rows of its row group x one K
// split; wave w owns k in [448 s + 112 w, +112).  Lane l = 32 h + c: B column
// c, and for MFMA step (g, e), g < 14, e < 4, the k pair {8 g + e, 8 g + 4 +
// e} (half h takes the second), so the A row loads are float4.  Output rows
// (r & 3) + 8 (r >> 2) + 4 h of column c.  Partials [Z][FC1_S][B][512] are
// reduced by the head.  (Round 3: fc1 5.8 -> 4.7 us against the 16 x 16 x 4
// form, whose 16-column B operand fetched 64-byte halves of W1's lines; that
// kernel and the in-launch split-K reduce variant are in git history, commit
// 1a3be58.)
constexpr int FC1_S = 7, FC1_KS = FLAT / FC1_S, FC1_KW = FC1_KS / 4;  // 448, 112
constexpr int Z_MAX_FC1 = 3;  // network copies of one fc1 launch (online, target, online(s_t))

struct Fc1FwdArgs {
  const float* in;  // [Z][B][3136]
  NetZ nz;
  int64_t w_off;
  int B, MG;        // MG = ceil(B / 32) row groups
  float* part;      // [Z][FC1_S][B][512]
  TangentDot dot = {nullptr, nullptr, 0};  // MGSC tangent: per-row dot products with dz1 instead of stores
};

constexpr int FC1_32RW = 32 * 33;  // one wave's 32 x 32 tile, row stride 33
// fc1 forward's load order: every W1 load issued before the y3 loads (round
// 3's order; round 4's interleaved order made the kernel 0.2-0.3 us slower,
// fc1 4.90-4.96 -> 4.69-4.75 us back to back and 16,171 -> 16,248 steps/s,
// three interleaved rounds, profiles/r05/c2).
// (Round 6: the same loads issued all before the first MFMA, held there by a
// sched_barrier, W1 first or y3 first — the source order alone does not do
// it, the compiler interleaves them with the MFMAs at ~10 in flight: fc1
// 4.75 -> 5.35 / 5.45 us back to back, the step -0.8 / -0.5 %, the meta-update
// +10 us; profiles/r06/fc1_order.)
// And timing-only (numerics wrong): the same W1 bytes as 16-byte loads, 14
// instead of 56 per lane: 4.72 -> 4.36 us, the step +1.6 % (part of it the
// code-layout shift of the kernels after this one), with every load ahead of
// the MFMAs 5.3 us; a correct form needs each lane's four k values of one
// column regathered (LDS staging or cross-lane moves), not built
// (profiles/r06/fc1_order).
// DOT: the MGSC tangent launches' form (per-row dot products with dz1 instead
// of partial stores); the learner's fc1_fwd32_kernel compiles without it.
// (Round 5: 8 waves per block, 56 k each, measured 4.70 -> 4.86 us and
// 16,239 -> 16,169 steps/s, profiles/r05/s8; not kept.)
template <bool DOT>
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
  const int row = min(32 * mg + c, a.B - 1);
  const float* x = a.in + ((int64_t)z * a.B + row) * FLAT + k0;
  float wr[G][4];
  float4 av[G];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[g][e] = W[(int64_t)(k0 + 8 * g + e) * HID];
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
  const bool live = 32 * mg + q < a.B;
  float v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int k = q * 33 + c4 + e;
    v[e] = (s_red[k] + s_red[FC1_32RW + k]) + (s_red[2 * FC1_32RW + k] + s_red[3 * FC1_32RW + k]);
  }
  if (DOT) {  // this split's share of <V_fc1 y3, dz1> for row q: 8 lanes x 4 columns
    float d = 0.f;
    if (live) {
      const float4 dz = *reinterpret_cast<const float4*>(a.dot.dy + (int64_t)(32 * mg + q) * HID + 32 * nt + c4);
      d = (v[0] * dz.x + v[1] * dz.y) + (v[2] * dz.z + v[3] * dz.w);
    }
    d += __shfl_xor(d, 1, 64);
    d += __shfl_xor(d, 2, 64);
    d += __shfl_xor(d, 4, 64);
    if (live && (t & 7) == 0)
      a.dot.part[(int64_t)(32 * mg + q) * META_DOT_SLOTS + a.dot.slot0 + nt * FC1_S + s] = d;
    return;
  }
  if (live)
    *reinterpret_cast<float4*>(a.part + (((int64_t)z * FC1_S + s) * a.B + 32 * mg + q) * HID + 32 * nt + c4) =
        make_float4(v[0], v[1], v[2], v[3]);
}

inline int fc1_fwd_blocks(int Z, int MG) { return (HID / 32) * FC1_S * Z * MG; }

// fc1 forward of at most FC1_GEMV_MAXB rows (the MGSC pass at theta', the HVP
// pass, the actor's single state) as VALU dot products: the 32 x 32 MFMA tile
// would spend 56 v_mfma_f32_32x32x2f32 per wave (1.5 us) on one live row.
// Same blocks and partial layout as fc1_fwd_block32; thread t owns column
// t % 32 of the block's 32 and k [56 (t / 32), +56) of its split; the split's
// y3 rows are staged in LDS, and the 8 k-group sums of each output are added
// in k-group order.  (Round 5: fc1 at B = 1 4.37 -> 2.73 us span; the MGSC
// first-order meta-update 195-197 -> 193 us, profiles/r05/s9.)
constexpr int FC1_GEMV_MAXB = 4, FC1_GEMV_KG = FC1_KS / 8;  // 56
constexpr int FC1_GEMV_SMEM = FC1_GEMV_MAXB * FC1_KS + 8 * FC1_GEMV_MAXB * 32;  // floats
__device__ __forceinline__ void fc1_gemv_block(const Fc1FwdArgs& a, float* smem, int i) {
  const int nt = i % (HID / 32);
  const int rest = i / (HID / 32);
  const int s = rest % FC1_S, z = rest / FC1_S;
  const int t = threadIdx.x, c = t & 31, kg = t >> 5;
  const int B = a.B;
  const int k0 = s * FC1_KS + kg * FC1_GEMV_KG;
  const float* W = a.nz.p[z] + a.w_off + 32 * nt + c;  // [3136][512]
  float wr[FC1_GEMV_KG];
#pragma unroll
  for (int j = 0; j < FC1_GEMV_KG; ++j) wr[j] = W[(int64_t)(k0 + j) * HID];
  float* s_x = smem;                                // [B][448]: y3 rows of the split
  float* s_red = smem + FC1_GEMV_MAXB * FC1_KS;     // [8 k groups][4 rows][32 columns]
  const float4* xz = reinterpret_cast<const float4*>(a.in + (int64_t)z * B * FLAT);
  for (int e = t; e < B * (FC1_KS / 4); e += blockDim.x) {
    const int row = e / (FC1_KS / 4), q4 = e % (FC1_KS / 4);
    const int src = (row * FLAT + s * FC1_KS) / 4 + q4;
    *reinterpret_cast<float4*>(s_x + row * FC1_KS + 4 * q4) = xz[src];
  }
  __syncthreads();
  float acc[FC1_GEMV_MAXB];
#pragma unroll
  for (int r = 0; r < FC1_GEMV_MAXB; ++r) {
    acc[r] = 0.f;
    if (r < B) {
      const float* x = s_x + r * FC1_KS + kg * FC1_GEMV_KG;
#pragma unroll
      for (int j = 0; j < FC1_GEMV_KG; ++j) acc[r] = __fmaf_rn(wr[j], x[j], acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < FC1_GEMV_MAXB; ++r)
    if (r < B) s_red[(kg * FC1_GEMV_MAXB + r) * 32 + c] = acc[r];
  __syncthreads();
  if (t < 32 * B) {
    const int r = t >> 5;
    float v = s_red[r * 32 + c];
#pragma unroll
    for (int g = 1; g < 8; ++g) v += s_red[(g * FC1_GEMV_MAXB + r) * 32 + c];
    a.part[(((int64_t)z * FC1_S + s) * B + r) * HID + 32 * nt + c] = v;
  }
}

DQZ_STEP_KERNEL __launch_bounds__(256) void fc1_gemv_kernel(Fc1FwdArgs a) {
  DQZ_STAMP(3, 0);
  __shared__ __attribute__((aligned(16))) float smem[FC1_GEMV_SMEM];
  fc1_gemv_block(a, smem, blockIdx.x);
  DQZ_STAMP(3, 3);
}

DQZ_STEP_KERNEL __launch_bounds__(256) void fc1_fwd32_kernel(Fc1FwdArgs a) {
  DQZ_STAMP(3, 0);
  __shared__ float s_red[4 * FC1_32RW];
  fc1_fwd_block32<false>(a, s_red, blockIdx.x);
  DQZ_STAMP(3, 3);
}

}  // namespace dqz
