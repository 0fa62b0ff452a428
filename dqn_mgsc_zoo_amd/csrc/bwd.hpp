// bwd.hpp — backward kernels specialised for the NatureQNetwork at small B.
#pragma once
// Timing-only probes (numerics wrong by design): DQZ_EXP_DXFAST / _DWFAST
// run a third of the conv3 / conv2 dX (dW) MFMA K steps.
#ifndef DQZ_EXP_DXFAST
#define DQZ_EXP_DXFAST 0
#endif
#ifndef DQZ_EXP_DWFAST
#define DQZ_EXP_DWFAST 0
#endif
#include "common.hpp"
#include "conv1.hpp"
#include "fwd.hpp"
#include "head.hpp"
#include "sampling.hpp"

namespace dqz {

// ---- fc1 backward ----------------------------------------------------------
// dX in fc1_dx_kernel (196 blocks of 16 rows of W1 [3136][512], below);
// dW1 = y3^T @ dz1 + centered RMSProp in bwd_bc_kernel's fc1 dW range
// (fc1_dw_body, 784 blocks of 16 rows x 128 columns), which starts after
// fc1_dx_kernel (the update overwrites the rows dX reads).  W1, mu and nu
// are each read once and written once (HBM-bound at 6 x 6.4 MB).
struct Fc1BwdArgs {
  const float* dz1;  // [B][512]
  const float* y3;   // [B][3136] online activations
  float *th, *mu, *nu;
  int64_t w_off;
  Rms rms;
  int B;
  float* dy3;  // [B][3136]
  // fc1_dx_kernel also writes the B-operand-ordered copies of W3 and W2 that
  // the conv3 / conv2 dX jobs of this step load as whole float4 lines
  // (permute_dx_weights below); null in launches that do not need them.
  const float *w3, *w2;
  float *w3p, *w2p;
};

// Permuted copies of the current W3 / W2 for the dX jobs.  A dX job's lane
// (n, kq) of wave w needs, per tap t, the four values W[t][ci = 16 q + n]
// [co = 16 w + 4 j + kq], j = 0..3 (v_mfma_f32_16x16x4 B operand, k = co):
// 64-byte-strided dwords in W's HWIO layout (one 64-lane load touches 16
// lines; 36 such loads per conv3 dX lane were the bulk of its staging
// time).  The copies store them as [job group][t][w][n][kq][j], so a wave
// reads one contiguous 1 KB run per tap (one float4 per lane).
//   w3p: [nq 4][t' 9][w 4][n 16][kq 4][j 4], t' = flipped tap (8 - t)
//   w2p: [ph 2][pw 2][hh 2][t 4][w 4][n 16][kq 4][j 4], t = (u, v): kh = ph +
//        2 (1 - u), kw = pw + 2 (1 - v)
__device__ __forceinline__ int w3p_src(int i) {
  const int j = i & 3, kq = (i >> 2) & 3, n = (i >> 4) & 15, w = (i >> 8) & 3, r = i >> 10;
  const int tp = r % 9, nq = r / 9;
  return ((8 - tp) * C3CI + 16 * nq + n) * C3CO + 16 * w + 4 * j + kq;
}
__device__ __forceinline__ int w2p_src(int i) {
  const int j = i & 3, kq = (i >> 2) & 3, n = (i >> 4) & 15, w = (i >> 8) & 3, tp = (i >> 10) & 3;
  const int hh = (i >> 12) & 1, pw = (i >> 13) & 1, ph = (i >> 14) & 1;
  const int kh = ph + 2 * (1 - (tp >> 1)), kw = pw + 2 * (1 - (tp & 1));
  return ((kh * C2K + kw) * C2CI + 16 * hh + n) * C2CO + 16 * w + 4 * j + kq;
}
constexpr int W3P_N = 4 * 9 * 1024, W2P_N = 8 * 4 * 1024;  // 36864, 32768

// LDS row stride of the dz1 chunk: the dX A fragments' ds_read_b128 (lane n
// reads row 16 mt + n at column 4 kq) are conflict-free in every 16-lane
// group only with a stride of 8 (mod 64) dwords: 520 (528 put two lanes on
// each bank quad: 4 extra LDS cycles per read, the 1.67 conflict cycles per
// LDS instruction of round 2's counters).
constexpr int FC1X_LD = 520;

// dy3 = (dz1 @ W1^T) relu'(y3), the head of the backward chain (conv3
// backward waits on it).  Block blk owns W1 rows [16 blk, 16 blk + 16) for
// all samples; wave w owns hidden units [128 w, 128 w + 128) (a quarter of
// K).  dz1 is staged 32 samples at a time into LDS, the four K-quarter
// partial tiles summed through LDS in a fixed order.
constexpr int FC1X_RED = 256 + 4 * 16;  // one padded 16 x 16 dX partial tile
constexpr int FC1X_SMEM = 32 * FC1X_LD + 4 * 2 * FC1X_RED;  // floats: dz1 chunk + dX partials

// Samples [c_beg, c_end) of the batch, in chunks of 32 (fc1_dx_block gives a
// block one chunk).
__device__ __forceinline__ void fc1_dx_body(const Fc1BwdArgs& a, float* smem, int blk, int c_beg, int c_end) {
  DQZ_STAMP(5, 0);
  constexpr int LD = FC1X_LD;
  float* s_dz = smem;
  // dX partials [wave][mt][row 4 kq + r][n], 16 floats of padding after every
  // 4 rows: the writes of lanes kq = 0 / 1 (and 2 / 3), one ds_write_b32
  // lane group, land 16 banks apart instead of on the same banks; the
  // reduction's reads stay conflict-free (a wave reads rows 4w .. 4w + 3).
  float(*s_red)[2][FC1X_RED] = reinterpret_cast<float(*)[2][FC1X_RED]>(smem + 32 * LD);
  auto red_at = [](int row, int col) { return row * 16 + 16 * (row >> 2) + col; };
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  const int k0 = 16 * blk;
  const float* W1 = a.th + a.w_off;
  float4 wv[8];  // B operand: W1[k0 + n][128 w + 16 j + 4 kq + e]
#pragma unroll
  for (int j = 0; j < 8; ++j)
    wv[j] = *reinterpret_cast<const float4*>(W1 + (int64_t)(k0 + n) * HID + 128 * w + 16 * j + 4 * kq);
  for (int c = c_beg; c < c_end; c += 32) {
    if (c > c_beg) __syncthreads();  // previous chunk's s_dz / s_red readers are done
    // stage dz1 rows [c, c + 32) (rows past B are zero)
    float4 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int f = t + 256 * i, row = f >> 7;
      const float4 x = *reinterpret_cast<const float4*>(a.dz1 + (int64_t)min(c + row, a.B - 1) * HID + 4 * (f & 127));
      v[i] = c + row < a.B ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    float ym[2];  // relu'(y3) operands of the epilogue
#pragma unroll
    for (int h = 0; h < 2; ++h)
      ym[h] = a.y3[(int64_t)min(c + 16 * h + (t >> 4), a.B - 1) * FLAT + k0 + (t & 15)];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int f = t + 256 * i;
      *reinterpret_cast<float4*>(s_dz + (f >> 7) * LD + 4 * (f & 127)) = v[i];
    }
    __syncthreads();
    // rows (samples) 16 mt + n, K = hidden [128 w, 128 w + 128)
    f32x4 xacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const float* d = s_dz + (16 * mt + n) * LD + 128 * w + 4 * kq;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float4 av = *reinterpret_cast<const float4*>(d + 16 * j);
        xacc[mt] = mfma4(av.x, wv[j].x, xacc[mt]);
        xacc[mt] = mfma4(av.y, wv[j].y, xacc[mt]);
        xacc[mt] = mfma4(av.z, wv[j].z, xacc[mt]);
        xacc[mt] = mfma4(av.w, wv[j].w, xacc[mt]);
      }
    }
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) s_red[w][mt][red_at(4 * kq + r, n)] = xacc[mt][r];
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int sample = c + 16 * h + (t >> 4);
      const int k = red_at(t >> 4, t & 15);
      const float v2 = (s_red[0][h][k] + s_red[1][h][k]) + (s_red[2][h][k] + s_red[3][h][k]);
      if (sample < a.B) a.dy3[(int64_t)sample * FLAT + k0 + (t & 15)] = ym[h] > 0.f ? v2 : 0.f;
    }
  }
  DQZ_STAMP(5, 3);
}

// ---- conv3 backward: dX and per-sample dW partials -----------------------
// grid (12, B).  Jobs 0..7: dX of input-channel quarter (job & 3) for output
// rows half (job >> 2): dy2 = conv_transpose(dy3, W3) * relu'(y2), computed
// as a correlation of dy3 zero-padded by 2 with the flipped kernel.  Jobs
// 8..11: dW partial of output-channel quarter (job - 8) for this sample:
// part[b][(kh*3 + kw)*64 + ci][co] = sum_p y2[b][oh+kh][ow+kw][ci] dy3[b][p][co],
// bias row 576 = sum_p dy3[b][p][co].  The update kernel sums the B slabs.
constexpr int C3X_S = 66, C3X_RS = 754, C3X_WIN = 11 * C3X_RS;  // padded dy3 window, 8294 floats
constexpr int C3W_S = 80, C3W_RS = 720, C3W_WIN = 9 * C3W_RS;   // y2 window for dW, 6480 floats

struct Conv3BwdArgs {
  const float* dy3;  // [B][49][64]
  const float* y2;   // [B][81][64] online
  const float* w3;   // online W3 [3][3][64][64]
  const float* w3p;  // its dX-ordered copy (permute_dx_weights)
  float* dy2;        // [B][81][64]
  float* part;       // [B][577][64]
  int B;
  Handoff sync;      // per-sample dy2 arrival counters (bwd_bc_kernel)
};

// PUB: dy2 is handed to conv2 dX inside the same launch (bwd_bc_kernel): every
// dy2 store is write-through (sc1), every storing wave drains (vmcnt(0)), and
// after the workgroup barrier one lane adds to the sample's arrival counter
// (MI355X_MICROARCH.md visibility table, row 1; the consumer loads sc1).
template <bool PUB>
__device__ __forceinline__ void conv3_bwd_dx(const Conv3BwdArgs& a, float* s_win, int b, int nq, int mh) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  // B operand: flipped kernel, k = (tap' = kh'*3 + kw', co), wave w owns co [16w, 16w + 16)
  float wr[36];  // wr[4 t' + j] = W3[8 - t'][16 nq + n][16 w + 4 j + kq]
  {
    const float4* wp = reinterpret_cast<const float4*>(a.w3p) + ((nq * 9 * 4 + w) * 16 + n) * 4 + kq;
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const float4 v = wp[tp * 256];
      wr[4 * tp] = v.x;
      wr[4 * tp + 1] = v.y;
      wr[4 * tp + 2] = v.z;
      wr[4 * tp + 3] = v.w;
    }
  }
  // relu'(y2) operands of the epilogue, loaded early: thread t < 192 owns
  // position 48 mh + t / 4, channels 16 nq + 4 (t & 3) .. +3
  const int ep = min(48 * mh + (t >> 2), C2M - 1);
  const float4 ym4 = *reinterpret_cast<const float4*>(a.y2 + ((int64_t)b * C2M + ep) * C2CO + 16 * nq + 4 * (t & 3));
  // padded dy3 window: (ph, pw) in 11 x 11, interior [2, 9)
  const float4* src = reinterpret_cast<const float4*>(a.dy3 + (int64_t)b * FLAT);
  constexpr int NW4 = 121 * 16;  // 1936
  float4 r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = min(t + 256 * q, NW4 - 1);
    const int pix = i >> 4, ph = pix / 11 - 2, pw = pix % 11 - 2;
    const bool in = ph >= 0 && ph < C3O && pw >= 0 && pw < C3O;
    const float4 v = src[(in ? ph * C3O + pw : 0) * 16 + (i & 15)];
    r[q] = in ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __builtin_amdgcn_sched_barrier(0);  // every window load in flight before the first LDS store
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = t + 256 * q;
    if (i < NW4) {
      const int pix = i >> 4;
      float* d = s_win + (pix / 11) * C3X_RS + (pix % 11) * C3X_S + win64_ch((i & 15) * 4);
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  __syncthreads();
  DQZ_STAMP(6, 1);
  int base[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) {
    const int p = min(48 * mh + 16 * m + n, C2M - 1);
    base[m] = (p / C2O) * C3X_RS + (p % C2O) * C3X_S + win64_ch(16 * w) + kq;
  }
  f32x4 acc[3];
#pragma unroll
  for (int m = 0; m < 3; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < 36; ++kk) if (!DQZ_EXP_DXFAST || kk % 3 == 0) {
    const int tp = kk >> 2;  // tap' = kh'*3 + kw'
    const int off = (tp / 3) * C3X_RS + (tp % 3) * C3X_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < 3; ++m) acc[m] = mfma4(s_win[base[m] + off], wr[kk], acc[m]);
  }
  __syncthreads();
  DQZ_STAMP(6, 2);
  float* s_red = s_win;  // [4][48][16]
#pragma unroll
  for (int m = 0; m < 3; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * 768 + (16 * m + 4 * kq + rr) * 16 + n] = acc[m][rr];
  __syncthreads();
  // 4 channels per lane: one 16-byte (write-through when PUB) store each
  if (t < 192 && 48 * mh + (t >> 2) < C2M) {
    const int i = 4 * t;  // s_red index of (position t / 4, channel 4 (t & 3))
    f32x4 v;  // (a 4-byte write-through store costs ~6x the 16-byte one per byte)
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = (s_red[i + e] + s_red[768 + i + e]) + (s_red[1536 + i + e] + s_red[2304 + i + e]);
    v[0] = ym4.x > 0.f ? v[0] : 0.f;
    v[1] = ym4.y > 0.f ? v[1] : 0.f;
    v[2] = ym4.z > 0.f ? v[2] : 0.f;
    v[3] = ym4.w > 0.f ? v[3] : 0.f;
    float* slab = a.dy2 + (int64_t)b * C2M * C2CO;
    const int off = ((48 * mh + (t >> 2)) * C2CO + 16 * nq + 4 * (t & 3)) * 4;
    if constexpr (PUB)
      store_sc1_f4(slab, C2M * C2CO * 4, off, v);
    else
      *reinterpret_cast<f32x4*>(reinterpret_cast<char*>(slab) + off) = v;
  }
  if constexpr (PUB) a.sync.arrive(b);
}

// conv3 dW job (sample b, output-channel quarter nq).  (Round 3 measured
// jobs that accumulate several samples, and a per-XCD pre-reduction of the
// per-sample slabs inside the launch: both slower, commit 1a3be58.)
__device__ __forceinline__ void conv3_bwd_dw(const Conv3BwdArgs& a, float* s_win, int b, int nq) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  constexpr int NQ4 = C2M * C2CO / 4;  // 1296
  // B operand: dy3[b][p = 4 kk + kq][16 nq + n], zero for p >= 49
  float dr[13];
#pragma unroll
  for (int kk = 0; kk < 13; ++kk) {
    const int p = 4 * kk + kq;
    const float v = a.dy3[((int64_t)b * C3M + min(p, C3M - 1)) * C3CO + 16 * nq + n];
    dr[kk] = p < C3M ? v : 0.f;
  }
  float4 r[6];
  {
    const float4* src = reinterpret_cast<const float4*>(a.y2 + (int64_t)b * (C2M * C2CO));
#pragma unroll
    for (int q = 0; q < 6; ++q) r[q] = src[min(t + 256 * q, NQ4 - 1)];
  }
  // A operand: y2 window at (oh + kh, ow + kw), ci = 16 w + n; position p = 4 kk + kq
  int pb[13];
#pragma unroll
  for (int kk = 0; kk < 13; ++kk) {
    const int p = min(4 * kk + kq, C3M - 1);
    pb[kk] = (p / C3O) * C3W_RS + (p % C3O) * C3W_S + 16 * w + n;
  }
  f32x4 acc[9];
#pragma unroll
  for (int tp = 0; tp < 9; ++tp) acc[tp] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int i = t + 256 * q;
    if (i < NQ4) {
      const int pix = i >> 4;
      *reinterpret_cast<float4*>(s_win + (pix / C2O) * C3W_RS + (pix % C2O) * C3W_S + (i & 15) * 4) = r[q];
    }
  }
  __syncthreads();
  DQZ_STAMP(12, 1);
  // A = dy3 (rows: co), B = the y2 patch (columns: ci): a lane's four
  // accumulators are four consecutive co of one (tap, ci) row, stored as one
  // float4 (the products and their k order are those of the transposed form,
  // so the values are the same bits)
#pragma unroll
  for (int kk = 0; kk < 13; ++kk) if (!DQZ_EXP_DWFAST || kk % 3 == 0)
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int off = (tp / 3) * C3W_RS + (tp % 3) * C3W_S;
      acc[tp] = mfma4(dr[kk], s_win[pb[kk] + off], acc[tp]);
    }
  float sb = 0.f;  // bias: sum over positions (lanes kq hold p = 4 kk + kq)
#pragma unroll
  for (int kk = 0; kk < 13; ++kk) sb += dr[kk];
  // C layout: row = 4 kq + r -> co = 16 nq + 4 kq + r; col = n -> ci = 16 w + n of tap tp
  float* slab = a.part + (int64_t)b * (C3KK + 1) * C3CO;
#pragma unroll
  for (int tp = 0; tp < 9; ++tp)
    *reinterpret_cast<f32x4*>(slab + (tp * C3CI + 16 * w + n) * C3CO + 16 * nq + 4 * kq) = acc[tp];
  if (w == 0) {  // bias row
    sb += __shfl_xor(sb, 16, 64);
    sb += __shfl_xor(sb, 32, 64);
    if (kq == 0) slab[C3KK * C3CO + 16 * nq + n] = sb;
  }
}

// ---- conv2 backward: dX by stride phase and per-sample dW partials --------
// grid (12, B).  Jobs 0..7: dX of stride phase (ph, pw) = (job & 3) >> 1,
// job & 1 for input-channel half job >> 2: output pixels (2a + ph, 2c + pw),
// a, c in [0, 10), are a 2x2-tap correlation of dy2 zero-padded by 1 with
// W2[ph + 2(1 - u)][pw + 2(1 - v)] (K = 4 taps x 64 co), masked by relu'(y1).
// Jobs 8..11: dW partial of output-channel quarter (job - 8):
// part[b][(kh*4 + kw)*32 + ci][co] = sum_p y1[b][2oh+kh][2ow+kw][ci] dy2[b][p][co]
// (bias row 512 = sum_p dy2).  Wave w of a dW job owns kh = w.
constexpr int C2X_S = 66, C2X_RS = 756, C2X_WIN = 11 * C2X_RS;  // padded dy2 window, 8316 floats
constexpr int C2W_S = 40, C2W_RS = 808, C2W_WIN = 20 * C2W_RS;  // y1 window for dW, 16160 floats

struct Conv2BwdArgs {
  const float* dy2;  // [B][81][64]
  const float* y1;   // [B][400][32] online
  const float* w2;   // online W2 [4][4][32][64]
  const float* w2p;  // its dX-ordered copy (permute_dx_weights)
  float* dy1;        // [B][400][32]
  float* part;       // [B][513][64]
  int B;
  Handoff sync;      // dy2 arrival counters (WAIT)
  Handoff sync1;     // dy1 arrival counters (PUB)
};

// WAIT: dy2 of sample b is produced by the 8 conv3 dX jobs of the same launch
// (bwd_bc_kernel).  Weights and relu'(y1) are loaded first, then one lane
// polls the sample's counter, and every dy2 load is an sc1 (L1-bypassing)
// buffer load.  PUB: dy1 is handed on to the conv1 dW jobs of the same launch
// (sc1 stores + arrival on sync1).
template <bool WAIT, bool PUB = false>
__device__ __forceinline__ void conv2_bwd_dx(const Conv2BwdArgs& a, float* s_win, int b, int ph, int pw, int hh) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  float wr[16];  // wr[4 t + j] = W2[kh(t)][kw(t)][16 hh + n][16 w + 4 j + kq]
  {
    const float4* wp =
        reinterpret_cast<const float4*>(a.w2p) + (((((ph * 2 + pw) * 2 + hh) * 4) * 4 + w) * 16 + n) * 4 + kq;
#pragma unroll
    for (int tp = 0; tp < 4; ++tp) {
      const float4 v = wp[tp * 256];
      wr[4 * tp] = v.x;
      wr[4 * tp + 1] = v.y;
      wr[4 * tp + 2] = v.z;
      wr[4 * tp + 3] = v.w;
    }
  }
  // relu'(y1) operands of the epilogue, loaded early: thread t owns output
  // positions q = t / 4 and q + 64 (< 100), channels 16 hh + 4 (t & 3) .. +3
  float4 ym4[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = min((t >> 2) + 64 * k, 99), ah = q / 10, cw = q % 10;
    ym4[k] = *reinterpret_cast<const float4*>(a.y1 + ((int64_t)b * C1M + (2 * ah + ph) * C1O + 2 * cw + pw) * C1CO +
                                              16 * hh + 4 * (t & 3));
  }
  const float4* src = reinterpret_cast<const float4*>(a.dy2 + (int64_t)b * (C2M * C2CO));
  constexpr int NW4 = 121 * 16;  // 1936
  if constexpr (WAIT) a.sync.wait(b);
  float4 r[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = min(t + 256 * q, NW4 - 1);
    const int pix = i >> 4, oh = pix / 11 - 1, ow = pix % 11 - 1;
    const bool in = oh >= 0 && oh < C2O && ow >= 0 && ow < C2O;
    const int e = (in ? oh * C2O + ow : 0) * 16 + (i & 15);
    float4 v;
    if constexpr (WAIT)
      v = load_sc1_f4(src, C2M * C2CO * 4, e);
    else
      v = src[e];
    r[q] = in ? v : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  __builtin_amdgcn_sched_barrier(0);  // every window load in flight before the first LDS store
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int i = t + 256 * q;
    if (i < NW4) {
      const int pix = i >> 4;
      float* d = s_win + (pix / 11) * C2X_RS + (pix % 11) * C2X_S + win64_ch((i & 15) * 4);
      d[0] = r[q].x;
      d[1] = r[q].y;
      d[2] = r[q].z;
      d[3] = r[q].w;
    }
  }
  __syncthreads();
  DQZ_STAMP(7, 1);
  // 100 pixels = 6 MFMA row tiles + pixels 96..99 on the VALU (fwd.hpp's trim)
  constexpr int MT = 6;
  int base[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    const int p = min(16 * m + n, 99);  // p = 10 a + c
    base[m] = (p / 10) * C2X_RS + (p % 10) * C2X_S + win64_ch(16 * w) + kq;
  }
  f32x4 acc[MT];
#pragma unroll
  for (int m = 0; m < MT; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  float last[4] = {0.f, 0.f, 0.f, 0.f};  // pixels 96..99 (a = 9, c = 6..9), this lane's k rows
#pragma unroll
  for (int kk = 0; kk < 16; ++kk) if (!DQZ_EXP_DXFAST || kk % 3 == 0) {
    const int tp = kk >> 2;  // (u', v') = (tp >> 1, tp & 1)
    const int off = (tp >> 1) * C2X_RS + (tp & 1) * C2X_S + 4 * (kk & 3);
#pragma unroll
    for (int m = 0; m < MT; ++m) acc[m] = mfma4(s_win[base[m] + off], wr[kk], acc[m]);
    {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        last[e] = __fmaf_rn(s_win[9 * C2X_RS + (6 + e) * C2X_S + win64_ch(16 * w) + kq + off], wr[kk], last[e]);
    }
  }
  {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      last[e] += __shfl_xor(last[e], 16, 64);
      last[e] += __shfl_xor(last[e], 32, 64);
    }
  }
  __syncthreads();
  DQZ_STAMP(7, 2);
  float* s_red = s_win;  // [4][112][16]
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int rr = 0; rr < 4; ++rr) s_red[w * 1792 + (16 * m + 4 * kq + rr) * 16 + n] = acc[m][rr];
  if (kq == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) s_red[w * 1792 + (96 + e) * 16 + n] = last[e];
  }
  __syncthreads();
  // 4 channels per lane: one 16-byte (write-through when PUB) store each
  // (a 4-byte write-through store costs ~6x the 16-byte one per byte)
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int q = (t >> 2) + 64 * k;
    if (q < 100) {
      const int i = 16 * q + 4 * (t & 3), ah = q / 10, cw = q % 10;
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        v[e] = (s_red[i + e] + s_red[1792 + i + e]) + (s_red[3584 + i + e] + s_red[5376 + i + e]);
      v[0] = ym4[k].x > 0.f ? v[0] : 0.f;
      v[1] = ym4[k].y > 0.f ? v[1] : 0.f;
      v[2] = ym4[k].z > 0.f ? v[2] : 0.f;
      v[3] = ym4[k].w > 0.f ? v[3] : 0.f;
      float* slab = a.dy1 + (int64_t)b * C1M * C1CO;
      const int off = (((2 * ah + ph) * C1O + 2 * cw + pw) * C1CO + 16 * hh + 4 * (t & 3)) * 4;
      if constexpr (PUB)
        store_sc1_f4(slab, C1M * C1CO * 4, off, v);
      else
        *reinterpret_cast<f32x4*>(reinterpret_cast<char*>(slab) + off) = v;
    }
  }
  if constexpr (PUB) a.sync1.arrive(b);
}

// conv2 dW as 8 jobs per sample for the merged backward launch: job (kh, ch)
// computes part[b][(kh*4 + kw)*32 + ci][32 ch + co'] for all kw (wave w = kw),
// ci and its 32 output channels, K = the 81 positions in a fixed k
// order.  Only the 9 input rows 2 oh + kh are staged (29 KB
// of LDS instead of 64 KB, so the job fits beside the other backward jobs);
// dy2 comes from this launch's conv3 dX jobs (wait + sc1 loads).
constexpr int C2V_WIN = 9 * C2W_RS;  // 7272 floats

// conv2 dW job (sample b, kernel row kh, output-channel half ch): y1 rows to
// LDS (loaded before the wait), the wait for the sample's dy2, the MFMAs.
__device__ __forceinline__ void conv2_bwd_dw_split(const Conv2BwdArgs& a, float* s_win, int b, int kh, int ch) {
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;  // w = kw
  const int n = lane & 15, kq = lane >> 4;
  constexpr int NV4 = 9 * C1O * C1CO / 4;  // 1440
  float4 r[6];
  {
    // y1 rows 2 oh + kh, oh = 0..8 (not handed off: plain loads)
    const float4* src = reinterpret_cast<const float4*>(a.y1 + (int64_t)b * (C1M * C1CO));
#pragma unroll
    for (int q = 0; q < 6; ++q) {
      const int i = min(t + 256 * q, NV4 - 1);
      const int oh = i / (C1O * 8), rem = i % (C1O * 8);  // 8 float4 per pixel
      r[q] = src[((2 * oh + kh) * C1O) * 8 + rem];
    }
  }
  int pb[21];
#pragma unroll
  for (int kk = 0; kk < 21; ++kk) {
    const int p = min(4 * kk + kq, C2M - 1);
    pb[kk] = (p / C2O) * C2W_RS + (2 * (p % C2O) + w) * C2W_S + n;
  }
  f32x4 acc[2][2];  // [ci tile][co tile]
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) acc[mt][ct] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the y1 rows go to LDS before the wait: held in registers across the spin
  // loop they were kept in scratch (112 bytes per lane, stored and reloaded)
#pragma unroll
  for (int q = 0; q < 6; ++q) {
    const int i = t + 256 * q;
    if (i < NV4) {
      const int oh = i / (C1O * 8), rem = i % (C1O * 8), iw = rem >> 3;
      *reinterpret_cast<float4*>(s_win + oh * C2W_RS + iw * C2W_S + (rem & 7) * 4) = r[q];
    }
  }
  a.sync.wait(b);
  float dr[21][2];
#pragma unroll
  for (int kk = 0; kk < 21; ++kk) {
    const int p = 4 * kk + kq;
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const float* gp = a.dy2 + ((int64_t)b * C2M + min(p, C2M - 1)) * C2CO + 32 * ch + 16 * ct + n;
      const float v = __hip_atomic_load(gp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dr[kk][ct] = p < C2M ? v : 0.f;
    }
  }
  __syncthreads();
  DQZ_STAMP(13, 1);
  // A = dy2 (rows: co), B = y1 (columns: ci): a lane's accumulators are four
  // consecutive co, stored as one float4 (same bits as the transposed form)
#pragma unroll
  for (int kk = 0; kk < 21; ++kk) if (!DQZ_EXP_DWFAST || kk % 3 == 0)
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
      const float av = s_win[pb[kk] + 16 * mt];
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) acc[mt][ct] = mfma4(dr[kk][ct], av, acc[mt][ct]);
    }
  float sb[2] = {0.f, 0.f};
#pragma unroll
  for (int ct = 0; ct < 2; ++ct)
#pragma unroll
    for (int kk = 0; kk < 21; ++kk) sb[ct] += dr[kk][ct];
  // C: row 4 kq + r -> co = 32 ch + 16 ct + 4 kq + r; col n -> ci = 16 mt + n
  float* slab = a.part + (int64_t)b * (C2KK + 1) * C2CO;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct)
      *reinterpret_cast<f32x4*>(slab + ((kh * C2K + w) * C2CI + 16 * mt + n) * C2CO + 32 * ch + 16 * ct + 4 * kq) =
          acc[mt][ct];
  if (kh == 0 && w == 0) {  // bias row (per lane over its kk, then over kq)
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      float v = sb[ct];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (kq == 0) slab[C2KK * C2CO + 32 * ch + 16 * ct + n] = v;
    }
  }
}

// ---- fc1 dW + RMSProp, 16 rows x 128 columns per block -------------------
// 784 light blocks (3 per CU) so they fill the gaps beside the conv3 dX
// workgroups they share a launch with.  Block (kb, nq): W1 rows
// [16 kb, 16 kb + 16), columns [128 nq, 128 nq + 128); wave w owns columns
// [128 nq + 32 w, +32) (two 16-column MFMA tiles), K = the batch.
constexpr int FC1W_LD = 144;  // LDS row stride of the dz1 slice: 144 = 16 (mod 32)
constexpr int FC1W_TLD = 36;  // row stride of a wave's 16 x 32 dW transpose tile
constexpr int FC1W_SMEM = 32 * FC1W_LD + 4 * 16 * FC1W_TLD;

__device__ __forceinline__ void fc1_dw_body(const Fc1BwdArgs& a, float* smem, int blk) {
  DQZ_STAMP(11, 0);
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int n = lane & 15, kq = lane >> 4;
  const int kb = blk >> 2, nq = blk & 3;
  const int k0 = 16 * kb, c0 = 128 * nq;
  const Rms& R = a.rms;
  const bool upd = R.update();
  // GEMM operands of a 32-sample chunk: dz1[c + row][c0 ..] (LDS) and
  // y3[c + 4 kk + kq][k0 + n] (A operand, registers).
  float4 v[4];
  float yv[8];
  auto load_chunk = [&](int c) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = t + 256 * i, row = f >> 5;  // 32 float4 per row
      const float4 x = *reinterpret_cast<const float4*>(a.dz1 + (int64_t)min(c + row, a.B - 1) * HID + c0 + 4 * (f & 31));
      v[i] = c + row < a.B ? x : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int bb = c + 4 * kk + kq;
      const float y = a.y3[(int64_t)min(bb, a.B - 1) * FLAT + k0 + n];
      yv[kk] = bb < a.B ? y : 0.f;
    }
  };
  load_chunk(0);
  // RMSProp operands in row-float4 layout: lane l owns W1[k0 + (l >> 3) + 8 h]
  // [c0 + 32 w + 4 (l & 7) .. +3], h = 0, 1, so each wave instruction reads
  // eight whole 128-byte lines.  Issued right AFTER the first chunk's GEMM
  // operands and unconditionally (gradient-output mode re-reads theta: mu /
  // nu may be null there): vmcnt is in order, so the GEMM waits for its own
  // operands only and these loads land under it.
  // (meta_rms1 reads theta, mu, nu too; meta_rms2 J, mu1, nu1; meta 3 G, mu1, nu1)
  const float* pth = R.meta == 2 ? R.J : R.meta == 3 ? R.G2 : a.th;
  const float* pmu = R.meta >= 2 ? R.mu1 : (upd || R.meta == 1) ? a.mu : a.th;
  const float* pnu = R.meta >= 2 ? R.nu1 : (upd || R.meta == 1) ? a.nu : a.th;
  const int64_t e0 = a.w_off + (int64_t)(k0 + (lane >> 3)) * HID + c0 + 32 * w + 4 * (lane & 7);
  float4 o_th[2], o_mu[2], o_nu[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int64_t e = e0 + (int64_t)8 * h * HID;
    o_th[h] = *reinterpret_cast<const float4*>(pth + e);
    o_mu[h] = *reinterpret_cast<const float4*>(pmu + e);
    o_nu[h] = *reinterpret_cast<const float4*>(pnu + e);
  }
  f32x4 gacc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  for (int c = 0;;) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int f = t + 256 * i;
      *reinterpret_cast<float4*>(smem + (f >> 5) * FC1W_LD + 4 * (f & 31)) = v[i];
    }
    __syncthreads();
    if (c == 0) DQZ_STAMP(11, 1);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const float* d = smem + (4 * kk + kq) * FC1W_LD + 32 * w + n;
      gacc[0] = mfma4(yv[kk], d[0], gacc[0]);
      gacc[1] = mfma4(yv[kk], d[16], gacc[1]);
    }
    c += 32;
    if (c >= a.B) break;
    __syncthreads();  // this chunk's LDS readers are done
    load_chunk(c);
  }
  DQZ_STAMP(11, 2);
  // C layout: row = 4 kq + r, col = 16 q + n of the wave's 16 x 32 tile ->
  // wave-private LDS tile -> row-float4 layout (same-wave LDS accesses are
  // ordered: no barrier).
  float* tile = smem + 32 * FC1W_LD + w * 16 * FC1W_TLD;
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int r = 0; r < 4; ++r) tile[(4 * kq + r) * FC1W_TLD + 16 * q + n] = gacc[q][r];
  float sq = 0.f, s1 = 0.f;  // meta_rms2 / meta 3: this thread's u'^2 (and grad q . w)
  const float clip = R.meta == 3 ? fminf(fmaxf(R.td[0], -R.bound), R.bound) : 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const float4 g = *reinterpret_cast<const float4*>(tile + ((lane >> 3) + 8 * h) * FC1W_TLD + 4 * (lane & 7));
    const int64_t e = e0 + (int64_t)8 * h * HID;
    if (R.meta == 1) {
      float4 t = o_th[h], m = o_mu[h], v = o_nu[h], j;
      j.x = R.meta1(g.x, t.x, m.x, v.x);
      j.y = R.meta1(g.y, t.y, m.y, v.y);
      j.z = R.meta1(g.z, t.z, m.z, v.z);
      j.w = R.meta1(g.w, t.w, m.w, v.w);
      *reinterpret_cast<float4*>(R.thp + e) = t;
      *reinterpret_cast<float4*>(R.mu1 + e) = m;
      *reinterpret_cast<float4*>(R.nu1 + e) = v;
      *reinterpret_cast<float4*>(R.J + e) = j;
      if (R.gout) *reinterpret_cast<float4*>(R.gout + e) = g;
    } else if (R.meta == 2) {
      float4 o;
      o.x = R.meta2(g.x, o_mu[h].x, o_nu[h].x, o_th[h].x, sq);
      o.y = R.meta2(g.y, o_mu[h].y, o_nu[h].y, o_th[h].y, sq);
      o.z = R.meta2(g.z, o_mu[h].z, o_nu[h].z, o_th[h].z, sq);
      o.w = R.meta2(g.w, o_mu[h].w, o_nu[h].w, o_th[h].w, sq);
      *reinterpret_cast<float4*>(R.vout + e) = o;
    } else if (R.meta == 3) {
      float4 m = o_mu[h], v = o_nu[h];
      R.meta3(g.x, o_th[h].x, m.x, v.x, clip, sq, s1);
      R.meta3(g.y, o_th[h].y, m.y, v.y, clip, sq, s1);
      R.meta3(g.z, o_th[h].z, m.z, v.z, clip, sq, s1);
      R.meta3(g.w, o_th[h].w, m.w, v.w, clip, sq, s1);
      *reinterpret_cast<float4*>(R.gout + e) = g;
      *reinterpret_cast<float4*>(R.mu1 + e) = m;
      *reinterpret_cast<float4*>(R.nu1 + e) = v;
    } else if (!upd) {
      float4 o = g;
      if (R.gacc) {
        const float4 prev = *reinterpret_cast<const float4*>(R.gout + e);
        o.x += prev.x;
        o.y += prev.y;
        o.z += prev.z;
        o.w += prev.w;
      }
      *reinterpret_cast<float4*>(R.gout + e) = o;
    } else {
      float4 m = o_mu[h], vv = o_nu[h], th = o_th[h];
      R.step(g.x, th.x, m.x, vv.x);
      R.step(g.y, th.y, m.y, vv.y);
      R.step(g.z, th.z, m.z, vv.z);
      R.step(g.w, th.w, m.w, vv.w);
      *reinterpret_cast<float4*>(a.mu + e) = m;
      *reinterpret_cast<float4*>(a.nu + e) = vv;
      *reinterpret_cast<float4*>(a.th + e) = th;
    }
  }
  if (R.meta >= 2) {  // the block's u'^2 (and grad q . w): each wave's sums in its own tile, then wave 0
    sq = wave_sum(sq);
    s1 = wave_sum(s1);
    if (lane == 0) {
      tile[0] = sq;
      tile[1] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      const float* t0 = smem + 32 * FC1W_LD;
      constexpr int WT = 16 * FC1W_TLD;
      R.sq_part[R.sq_off + blk] = (t0[0] + t0[WT]) + (t0[2 * WT] + t0[3 * WT]);
      if (R.meta == 3) R.s1_part[R.sq_off + blk] = (t0[1] + t0[WT + 1]) + (t0[2 * WT + 1] + t0[3 * WT + 1]);
    }
  }
  DQZ_STAMP(11, 3);
}

// ---- backward launches ----------------------------------------------------
// fc1_dx_kernel (fc1 dX), then bwd_bc_kernel: the critical-path dX job chain
// and the independent dW job sets share one launch, so the latency-bound dX
// workgroups and the dW workgroups share the CUs (no cross-stream edges).

// Grid: 196 row blocks x ceil(B / 32) sample chunks (block = kb + 196 chunk),
// so a batch of more than 32 (the MGSC meta batch) runs its chunks side by
// side instead of one after another in each block (M = 100: 12.9 -> ? us).
constexpr int FC1X_BLOCKS = FLAT / 16;  // 196
inline int fc1_dx_blocks(int B) { return FC1X_BLOCKS * ((B + 31) / 32); }
__device__ __forceinline__ void fc1_dx_block(const Fc1BwdArgs& a, float* smem, int blk) {
  // W3 / W2 dX copies: element i of the 69,632 is thread i of the grid (the
  // gathers are issued first and land under the block's own work)
  const int g = blk * 256 + threadIdx.x;
  float v3 = 0.f, v2 = 0.f;
  if (a.w3p) {
    if (g < W3P_N) v3 = a.w3[w3p_src(g)];
    if (g < W2P_N) v2 = a.w2[w2p_src(g)];
  }
  const int kb = blk % FC1X_BLOCKS, c = 32 * (blk / FC1X_BLOCKS);
  fc1_dx_body(a, smem, kb, c, min(c + 32, a.B));
  if (a.w3p) {
    if (g < W3P_N) a.w3p[g] = v3;
    if (g < W2P_N) a.w2p[g] = v2;
  }
  DQZ_STAMP(5, 3);
}

// ---- B = 1: the head and fc1 dX in one launch (head_dx1_kernel) ----------
// With one sample (the MGSC meta-update's pass at theta', the HVP's
// unit-cotangent pass) every block of the fc1 dX launch runs the head itself
// (2 x 7 split-K rows of 512, fc2, the TD error: a few microseconds of
// latency, no throughput) and takes dz1 from its own LDS; block 0 alone
// stores the head's outputs.  Each block owns 32 W1 rows (two 256-thread
// halves of 16 rows), loaded before the head, and forms dy3 = relu'(y3)
// (W1 dz1) as VALU dot products (a one-row GEMV: 16 lanes per row, 32
// columns per lane in column order, then a 16-lane sum); it also writes its
// share of the dX-ordered W3 / W2 copies, as fc1_dx_kernel does.  (Round 5's
// first form ran the head in block 0 and handed dz1 to the other blocks
// in-launch: 9.0 us; the head's round trips and the hand-off were serial.)
constexpr int FC1X1_ROWS = 32;
constexpr int FC1X1_BLOCKS = FLAT / FC1X1_ROWS;  // 98

template <int AMAX, int SMAX, int ZMAX>
__global__ __launch_bounds__(512) void head_dx1_kernel(HeadArgs h, Fc1BwdArgs a) {
  __shared__ __attribute__((aligned(16))) float s_dz[HID];
  DQZ_STAMP(5, 0);
  const int half = threadIdx.x >> 8, t = threadIdx.x & 255;
  const int row0 = FC1X1_ROWS * blockIdx.x + 16 * half;
  const int r = row0 + (t >> 4), c0 = 32 * (t & 15);
  const float* W1 = a.th + a.w_off;
  float4 wv[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) wv[j] = *reinterpret_cast<const float4*>(W1 + (int64_t)r * HID + c0 + 4 * j);
  const float ym = a.y3[r];  // relu'(y3) of the one sample
  // W3 / W2 dX copies: element g of the 69,632 by thread g of the launch
  const int g = (row0 / 16) * 256 + t;
  float v3 = 0.f, v2 = 0.f;
  if (a.w3p) {
    if (g < W3P_N) v3 = a.w3[w3p_src(g)];
    if (g < W2P_N) v2 = a.w2[w2p_src(g)];
  }
  head_body<AMAX, SMAX, ZMAX>(h, 0, blockIdx.x == 0, s_dz);
  __syncthreads();
  DQZ_STAMP(5, 1);
  float d = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float4 z = *reinterpret_cast<const float4*>(s_dz + c0 + 4 * j);
    d = __fmaf_rn(wv[j].x, z.x, d);
    d = __fmaf_rn(wv[j].y, z.y, d);
    d = __fmaf_rn(wv[j].z, z.z, d);
    d = __fmaf_rn(wv[j].w, z.w, d);
  }
  // sum over the row's 16 lanes (one DPP row): quad xor 1, xor 2, half-row and row mirrors
  d += dpp_f<0xB1>(d);
  d += dpp_f<0x4E>(d);
  d += dpp_f<0x141>(d);
  d += dpp_f<0x140>(d);
  if ((t & 15) == 0) a.dy3[r] = ym > 0.f ? d : 0.f;
  if (a.w3p) {
    if (g < W3P_N) a.w3p[g] = v3;
    if (g < W2P_N) a.w2p[g] = v2;
  }
  DQZ_STAMP(5, 3);
}

#ifdef DQZ_STEP_TU
// head_dx1_kernel's launch: the head_kernel template choice (launch_head)
inline hipError_t launch_head_dx1(const HeadArgs& h, const Fc1BwdArgs& f, hipStream_t st) {
  if (h.S > 7 || h.Z < 1 || h.Z > 3 || h.B != 1) return hipErrorInvalidValue;
  const dim3 grid(FC1X1_BLOCKS), block(512);
  if (h.A <= 8) {
    if (h.Z <= 2)
      hipLaunchKernelGGL((head_dx1_kernel<8, 7, 2>), grid, block, 0, st, h, f);
    else
      hipLaunchKernelGGL((head_dx1_kernel<8, 7, 3>), grid, block, 0, st, h, f);
  } else {
    if (h.Z <= 2)
      hipLaunchKernelGGL((head_dx1_kernel<MAXA, 7, 2>), grid, block, 0, st, h, f);
    else
      hipLaunchKernelGGL((head_dx1_kernel<MAXA, 7, 3>), grid, block, 0, st, h, f);
  }
  return hipGetLastError();
}
#endif  // DQZ_STEP_TU

DQZ_STEP_KERNEL __launch_bounds__(256) void fc1_dx_kernel(Fc1BwdArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[FC1X_SMEM];
  fc1_dx_block(a, smem, blockIdx.x);
}

// bwd_bc_kernel: the whole backward after fc1 dX in one launch.  Grid, in
// dispatch order:
//   [conv3 dX 8/sample] [fc1 dW 784] [conv2 dX 8/sample]
//   [conv3 dW 4/sample] [conv1 dW 8/sample] [conv2 dW 8/sample]
// Hand-offs inside the launch (common.hpp Handoff): dy2 from
// the 8 conv3 dX jobs of a sample to its 8 conv2 dX and 8 conv2 dW jobs, dy1
// from the 8 conv2 dX jobs to its 8 conv1 dW jobs.  Every consumer has a
// higher block index than its producers and workgroups are dispatched in
// index order, so every wait terminates.  The first two ranges fill the chip
// (4 workgroups per CU), so consumers are dispatched as conv3 dX blocks
// retire instead of spinning from the start.  Sample jobs keep the XCD-aware
// decode (each range starts at a multiple of 8, so producer and consumer
// share an L2).
// With a PER write-back (wb.tree set, dqz_learner_step_per) the grid gets 8
// leading workgroups: wave 0 of the first runs per_write_back_wave beside the
// whole backward (the TD errors are final since the head), the other seven
// exit at once (the sample ranges keep their XCD alignment).
// Timing-only experiment switches (never set in a product build; the
// numerics of a build with them are wrong): DQZ_EXP_SKIP bit 0 skips the fc1
// dW range, bit 1 conv3 dW, bit 2 conv2 dW, bit 3 conv1 dW (skipped
// consumers still pass their hand-off waits, so the words stay balanced).
#ifndef DQZ_EXP_SKIP
#define DQZ_EXP_SKIP 0
#endif
// (Round 5: the optimizer update as this launch's last range, each update
// block waiting for the dW jobs of its layers, which stored their slabs
// write-through and drained before arriving: correct, but the drains
// stretched the conv1 dW tail by 3 us, as much as the update launch's
// boundary saved (16,210 against 16,244 steps/s; first-order meta-update
// 193 -> 201 us; profiles/r05/s13).  With a thousand update blocks polling
// three shared words the launch ran 1.3x slower (s10-s12).  Removed.)
// Wave issue priority (s_setprio): the conv3 / conv2 dX waves 3, the conv1
// dW waves (the launch's tail, behind dy1) 2, every other dW wave the default
// 0, so on a SIMD shared with dW waves the chain's instructions issue first
// (round 6: +0.1 / +0.4 / +1.1 % in three interleaved A/B sessions; conv2 /
// conv3 dW at 1 as well: +0.3 %; the forward's conv2 / conv3 consumers above
// their producers: -0.8 %; profiles/r06/prio).
// (Round 6, also measured and not kept: the fc1 RMSProp outputs and the conv
// dW slabs as write-through sc1 stores, so the backward leaves 32 MB fewer
// dirty lines for the boundary before the update: -0.8 %, r06/prio; the
// XCD's dirty lines written back early instead, by an agent-scope release
// fence in the last 8 / 32 fc1 dW blocks: -1.9 / -6.6 %, r06/wbl2.)
// (Round 5, also removed: the dX chain on XCDs 0..L-1 and the dW sets on the
// other XCDs.  With L = 4 the chain ended 0.5 us sooner, but the dW side
// became the tail (+2.8 us) and the boundary after the launch grew 2.8 ->
// 5.8 us, the written lines now dirty in half the L2s: 15,873-15,901
// against 16,137-16,223 steps/s; L = 3 / 5 / 6 15,210 / 14,750 / 13,200;
// profiles/r05/split.)
template <bool WB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 8))) void bwd_bc_kernel(
    Conv3BwdArgs c3, Fc1BwdArgs f1, Conv2BwdArgs c2, Conv1DwArgs c1, PerWbArgs wb) {
  constexpr int kW = C3X_WIN > FC1W_SMEM ? C3X_WIN : FC1W_SMEM;
  constexpr int kW2 = C2X_WIN > C3W_WIN ? C2X_WIN : C3W_WIN;
  constexpr int kW3 = C2V_WIN > C1H_SMEM ? C2V_WIN : C1H_SMEM;
  constexpr int kWA = kW > kW2 ? kW : kW2;
  constexpr int kSmem = kWA > kW3 ? kWA : kW3;
  static_assert(kSmem * 4 >= PWB_LDS_BYTES, "the write-back's LDS comes out of the backward's buffer");
  __shared__ __attribute__((aligned(16))) float smem[kSmem];
  const int B8 = (c3.B + 7) / 8 * 8;
  constexpr int NF = 4 * (FLAT / 16);  // 784 fc1 dW blocks (a multiple of 8)
  int i = blockIdx.x;
  if constexpr (WB) {
    if (i < 8) {
      if (i == 0 && threadIdx.x < 64) per_write_back_wave(wb, reinterpret_cast<char*>(smem));
      return;
    }
    i -= 8;
  }
  if (i < 8 * B8) {
    const SampleJob sj = xcd_sample_job_at(i, 8, c3.B);
    if (!sj.valid) return;
    __builtin_amdgcn_s_setprio(3);  // the dX chain first (see above)
    DQZ_STAMP(6, 0);
    conv3_bwd_dx<true>(c3, smem, sj.s, sj.job & 3, sj.job >> 2);
    DQZ_STAMP(6, 3);
    return;
  }
  i -= 8 * B8;
  if (i < NF) {
    if (DQZ_EXP_SKIP & 1) return;
    fc1_dw_body(f1, smem, i);
    return;
  }
  i -= NF;
  if (i < 8 * B8) {
    const SampleJob sj = xcd_sample_job_at(i, 8, c2.B);
    if (!sj.valid) return;
    __builtin_amdgcn_s_setprio(3);  // the dX chain first (see above)
    DQZ_STAMP(7, 0);
    conv2_bwd_dx<true, true>(c2, smem, sj.s, (sj.job & 3) >> 1, sj.job & 1, sj.job >> 2);
    DQZ_STAMP(7, 3);
    return;
  }
  i -= 8 * B8;
  if (i < 4 * B8) {
    const SampleJob sj = xcd_sample_job_at(i, 4, c3.B);
    if (!sj.valid) return;
    if (DQZ_EXP_SKIP & 2) return;
    DQZ_STAMP(12, 0);
    conv3_bwd_dw(c3, smem, sj.s, sj.job);
    DQZ_STAMP(12, 3);
    return;
  }
  i -= 4 * B8;
  // conv1 dW (the launch's tail: it waits for dy1) is dispatched ahead of
  // conv2 dW (whose dy2 is ready early): 14,003-14,012 -> 14,178-14,198
  // steps/s; ahead of conv3 dW as well measured the same
  if (i < 8 * B8) {
    const SampleJob sj = xcd_sample_job_at(i, 8, c1.B);
    if (!sj.valid) return;
    if (DQZ_EXP_SKIP & 8) {
      c1.sync1.wait(sj.s);
      return;
    }
    __builtin_amdgcn_s_setprio(2);  // the launch's tail next
    conv1_dw_half(c1, smem, sj.job >> 1, sj.job & 1, sj.s);
    return;
  }
  i -= 8 * B8;
  const SampleJob sj = xcd_sample_job_at(i, 8, c2.B);
  if (!sj.valid) return;
  if (DQZ_EXP_SKIP & 4) {
    c2.sync.wait(sj.s);
    return;
  }
  DQZ_STAMP(13, 0);
  conv2_bwd_dw_split(c2, smem, sj.s, sj.job >> 1, sj.job & 1);
  DQZ_STAMP(13, 3);
}

}  // namespace dqz
