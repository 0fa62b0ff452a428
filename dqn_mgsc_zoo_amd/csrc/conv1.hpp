// conv1.hpp — conv1 (8x8 stride 4, 4->32) forward and weight-gradient
// kernels with the replay frame gather fused in.
//
// A workgroup owns 5 output rows (100 positions) of one sample.  It gathers
// the 24x84 input window of the sample's four stack channels straight from
// the HBM frame pool (16-byte loads; a channel whose frame index is -1 is
// the trailing zero padding of processors.py:57-69), normalises it with
// x / 255.0 (networks.py:192) into a [channel][row][col] f32 LDS image, and
// runs v_mfma_f32_32x32x2_f32 with both operands read from LDS by
// ds_read_b32 at compile-time immediate offsets.  Stacks never exist in HBM.
#pragma once
#include "common.hpp"
#include "sampling.hpp"

namespace dqz {

struct Conv1Src {
  const uint8_t* frames;  // frame pool (null when `states` is used)
  const int32_t* fidx;    // [capacity][8]
  const int32_t* slots;   // [B]
  const uint8_t* states;  // direct uint8 [B][84][84][4] input, or null
  int fused;              // 1: slots come from the fused uniform sampler `draw`;
                          // 2: from the fused learned-logit draw `sm`;
                          // 3: from the fused prioritized draw `per`
  union {                 // one draw per launch: the kernel argument stays small
    UniformDraw draw;
    SoftmaxDraw sm;
    PerSampleArgs per;
  };
  // Batch record: block (rb 0, z 0) of sample b also copies action / reward /
  // discount of its slot into rec[b] = {a as int bits, r, d, 0}, so the head
  // reads one record per sample instead of the slot -> record chain.
  const int32_t* action = nullptr;
  const float* reward = nullptr;
  const float* discount = nullptr;
  float4* rec = nullptr;
  // Stack copy (the MGSC theta' pass): the conv1 blocks of sample 0, stack 0,
  // copy the bytes they stage (zero padding applied) to xout [4][84][84], so
  // the HVP launches read the online transition's input without the slot ->
  // frame-index -> frame chain.
  uint8_t* xout = nullptr;
};

struct Conv1FwdArgs {
  Conv1Src src;
  NetZ nz;
  int64_t w_off, b_off;
  int B, Z;
  int linear;  // 1: write the pre-activation (no ReLU)
  float* out;  // y1 [Z][B][400][32]
  Handoff pub;  // PUB: y1 rows handed to conv2 in the same launch (fwd_conv_kernel)
  TangentDot dot = {nullptr, nullptr, 0};  // MGSC tangent: dot products instead of stores (part != null)
};

// bf16 operand fragments of v_mfma_f32_32x32x16_bf16
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// w == hi + mid + lo exactly, each piece a bf16 (8 significant bits): hi is w
// truncated to bf16, mid the truncated remainder, lo the rest (at most 8
// significant bits left of w's 24).  Both subtractions are exact.  Valid for
// every w whose lo piece is a normal number (|w| > 2^-110), i.e. all weights.
__device__ __forceinline__ void split3_bf16(float w, unsigned& hi, unsigned& mid, unsigned& lo) {
  const unsigned hb = __float_as_uint(w) & 0xFFFF0000u;
  const float r1 = w - __uint_as_float(hb);
  const unsigned mb = __float_as_uint(r1) & 0xFFFF0000u;
  const float r2 = r1 - __uint_as_float(mb);
  hi = hb >> 16;
  mid = mb >> 16;
  lo = __float_as_uint(r2) >> 16;
}

// grid (4 row blocks, B, Z); 256 threads.  The pixels are integers 0..255,
// exact in bf16, and every weight is the exact sum of three bf16 pieces, so
// conv1 runs on v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate) with every
// product x * piece exact in f32 and f32 accumulation: y1 = (sum x w) / 255
// + b, the pixel normalisation of networks.py:192 applied once to the f32
// sum instead of to each pixel (the two differ by f32 rounding only).
// Wave w owns K slab kh in {2w, 2w + 1} (64 of the 256 k) for all 100
// positions (4 tiles of 32, the last 4/32 live) and keeps its 64 x 32 weight
// slab in registers as 3 x 4 fragments; the 4 slab partials are summed through
// LDS in a fixed order.  MFMA A = weights (row = co), B = patches (col =
// position), so a lane's accumulators are 4 groups of 4 consecutive co.
// LDS: the [ci][24][84] bf16 input window (16 KB), then, aliased, the
// [wave][100][C1_RLD] f32 partials (56 KB).  PUB: y1 stores are 16-byte
// write-through and the block arrives on its sample's counter.
constexpr int C1_RLD = 36;  // partial row stride (floats): 16-byte lane stores spread over the banks
constexpr size_t kConv1FwdSmem = 4 * C1_POS * C1_RLD * sizeof(float);

__device__ __forceinline__ unsigned bf16_pair_u8(unsigned lo, unsigned hi) {
  // float(v) of v in 0..255 has at most 8 significant bits: its top half is its bf16
  return (__float_as_uint((float)hi) & 0xFFFF0000u) | (__float_as_uint((float)lo) >> 16);
}

// 16 pixels (16 bytes) -> 16 bf16 at dst (32 bytes, 16-byte aligned)
__device__ __forceinline__ void store_bytes_as_bf16(uint16_t* dst, uint4 v) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
  uint4 o[2];
  unsigned* ov = reinterpret_cast<unsigned*>(o);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ov[2 * i] = bf16_pair_u8(w[i] & 0xFF, (w[i] >> 8) & 0xFF);
    ov[2 * i + 1] = bf16_pair_u8((w[i] >> 16) & 0xFF, w[i] >> 24);
  }
  reinterpret_cast<uint4*>(dst)[0] = o[0];
  reinterpret_cast<uint4*>(dst)[1] = o[1];
}

// Stages input rows [20*rb, 20*rb + 24) of sample b, stack `which`, as
// s_in[ci][row][col] = pixel (bf16).
// F: the fused draw mode (src.fused), a template parameter so a launch only
// carries the draw code it runs.
template <int F>
__device__ __forceinline__ void stage_conv1_input(uint16_t* s_in, const Conv1Src& src, int b, int which, int rb,
                                                       int z = 0, int sk = -1) {
  const int row0 = rb * C1S * C1_ROWS;
  constexpr int QPC = C1_PLANE / 16;  // 126 16-byte pieces per channel
  if (src.states) {
    const uint4* g = reinterpret_cast<const uint4*>(src.states + ((int64_t)b * FH + row0) * FW * FC);
    // both 16-byte pieces of a thread in flight before the first LDS store (a
    // guarded loop loaded, waited and stored them one at a time)
    constexpr int NS = C1_PLANE * FC / 16, RS = (NS + 255) / 256;  // 504, 2
    uint4 vs[RS];
#pragma unroll
    for (int r = 0; r < RS; ++r) vs[r] = g[min((int)threadIdx.x + 256 * r, NS - 1)];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const int i = threadIdx.x + 256 * r;
      if (i >= NS) break;
      const uint4 v = vs[r];  // 4 pixels x 4 channels
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
      const int p = 4 * i;
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) {
        const int sh = 8 * ci;
        uint2 o;
        o.x = bf16_pair_u8((w[0] >> sh) & 0xFF, (w[1] >> sh) & 0xFF);
        o.y = bf16_pair_u8((w[2] >> sh) & 0xFF, (w[3] >> sh) & 0xFF);
        *reinterpret_cast<uint2*>(s_in + ci * C1_PLANE + p) = o;
      }
    }
  } else {
    // slot -> 4 frame ids -> 504 16-byte pieces (2 per thread), all loads in
    // flight before the first LDS store.
    int slot;
    double per_prob = 0.0;  // F == 3: the draw's probability (thread 0)
    if constexpr (F == 1) {  // fused sampler: draw b of this step; block (0, b, 0) publishes it
      slot = uniform_slot(*src.draw.counter, b, src.draw);
      if (threadIdx.x == 0 && rb == 0 && z == 0) src.draw.slots_out[b] = slot;
    } else if constexpr (F == 2) {  // fused learned-logit draw (every block of b runs the search)
      slot = softmax_draw_slot(src.sm, b);
      if (threadIdx.x == 0 && rb == 0 && z == 0) src.sm.slots_out[b] = slot;
    } else if constexpr (F == 3) {  // fused prioritized draw (the tree top staged in s_in first)
      const PerDrawOut d = per_draw_slot(src.per, b, reinterpret_cast<double*>(s_in), rb == 0 && z == 0);
      slot = d.slot;
      per_prob = d.prob;
    } else {
      slot = src.slots[b];
    }
    if (sk >= 0) DQZ_STAMP(sk, 0);
    const int32_t* fr = src.fidx + (int64_t)slot * 8 + which * 4;
    const int f0 = fr[0], f1 = fr[1], f2 = fr[2], f3 = fr[3];
    const bool wrec = src.rec != nullptr && threadIdx.x == 0 && rb == 0 && z == 0;
    float4 recv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (wrec) recv = make_float4(__int_as_float(src.action[slot]), src.reward[slot], src.discount[slot], 0.f);
    constexpr int NP = FC * QPC;  // 504
    uint4 v[2];
    int fq[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = min((int)threadIdx.x + 256 * q, NP - 1);
      const int ci = i / QPC, j = i % QPC;
      const int f = ci == 0 ? f0 : ci == 1 ? f1 : ci == 2 ? f2 : f3;
      fq[q] = f;
      const uint4* g = reinterpret_cast<const uint4*>(src.frames + (int64_t)max(f, 0) * FB + row0 * FW);
      v[q] = g[j];
    }
    // the fused PER draw's IS weight, while the frame loads are in flight
    if constexpr (F == 3)
      if (threadIdx.x == 0 && rb == 0 && z == 0) per_publish_weight(src.per, b, per_prob);
    if (sk >= 0) DQZ_STAMP(sk, 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = (int)threadIdx.x + 256 * q;
      if (i < NP) {
        const int ci = i / QPC, j = i % QPC;
        if (fq[q] < 0) v[q] = make_uint4(0u, 0u, 0u, 0u);  // trailing zero padding
        store_bytes_as_bf16(s_in + ci * C1_PLANE + j * 16, v[q]);
        if (src.xout && b == 0 && which == 0 && z == 0)
          reinterpret_cast<uint4*>(src.xout + (int64_t)ci * FB + row0 * FW)[j] = v[q];
      }
    }
    if (wrec) src.rec[b] = recv;
    if (sk >= 0) DQZ_STAMP(sk, 2);
  }
}

// s / 255: reciprocal product plus one FMA residual correction (within an
// ulp of the IEEE quotient; the IEEE division sequence costs ~10 VALU)
__device__ __forceinline__ float div255(float s) {
  constexpr float r = 1.0f / 255.0f;
  const float q = s * r;
  return __builtin_fmaf(__builtin_fmaf(-q, 255.0f, s), r, q);
}

template <bool PUB, int F>
__device__ __forceinline__ void conv1_fwd_body(const Conv1FwdArgs& a, float* smem, const SampleJob sj) {
  DQZ_STAMP(0, 0);
  uint16_t* s_in = reinterpret_cast<uint16_t*>(smem);  // [4][24][84] bf16
  const int rb = sj.job, b = sj.s % a.B, z = sj.s / a.B;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, r = lane & 31;
  const int c4 = threadIdx.x & 7;  // epilogue channel quad (fixed per thread: 256 % 8 == 0)
  const float4 bias = reinterpret_cast<const float4*>(a.nz.p[z] + a.b_off)[c4];  // loaded early
  // weight slab: step s covers kh = 2 wave + (s >> 1), ci = 2 (s & 1) + h, kw = j (element j)
  const float* W = a.nz.p[z] + a.w_off;  // HWIO [8][8][4][32]
  float wv[4][8];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) wv[s][j] = W[(((2 * wave + (s >> 1)) * C1K + j) * FC + 2 * (s & 1) + h) * C1CO + r];
  stage_conv1_input<F>(s_in, a.src, b, a.nz.which[z], rb, z, 14);
  bf16x8 wf[4][3];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    unsigned pk[3][4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      unsigned h0, m0, l0, h1, m1, l1;
      split3_bf16(wv[s][j], h0, m0, l0);
      split3_bf16(wv[s][j + 1], h1, m1, l1);
      pk[0][j / 2] = h0 | (h1 << 16);
      pk[1][j / 2] = m0 | (m1 << 16);
      pk[2][j / 2] = l0 | (l1 << 16);
    }
#pragma unroll
    for (int q = 0; q < 3; ++q) wf[s][q] = __builtin_bit_cast(bf16x8, make_uint4(pk[q][0], pk[q][1], pk[q][2], pk[q][3]));
  }
  DQZ_STAMP(0, 1);
  __syncthreads();

  f32x16 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = f32x16{};
    const int p = min(32 * t + r, C1_POS - 1);
    const uint16_t* pa = s_in + h * C1_PLANE + (C1S * (p / C1O) + 2 * wave) * FW + C1S * (p % C1O);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // 8 consecutive pixels of one input row (8-byte aligned)
      const uint2* q2 = reinterpret_cast<const uint2*>(pa + 2 * (s & 1) * C1_PLANE + (s >> 1) * FW);
      const uint2 x0 = q2[0], x1 = q2[1];
      const bf16x8 xb = __builtin_bit_cast(bf16x8, make_uint4(x0.x, x0.y, x1.x, x1.y));
#pragma unroll
      for (int q = 0; q < 3; ++q) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[s][q], xb, acc[t], 0, 0, 0);
    }
  }
  DQZ_STAMP(0, 2);
  __syncthreads();  // every wave is past its s_in reads: the partials alias it
  float* red = smem + wave * C1_POS * C1_RLD;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int pos = 32 * t + r;  // C/D: col = lane & 31 = position, rows co = (g & 3) + 8 (g >> 2) + 4 h
    if (pos < C1_POS)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(red + pos * C1_RLD + 8 * g + 4 * h) =
            f32x4{acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]};
  }
  __syncthreads();
  // (fields read once: inside the store loop they could alias `out`)
  float* out = a.out + (((int64_t)z * a.B + b) * C1M + rb * C1_POS) * C1CO;
  const bool linear = a.linear;
  const bool dot = a.dot.part != nullptr;
  const float* dyp = a.dot.dy + (((int64_t)z * a.B + b) * C1M + rb * C1_POS) * C1CO;
  float dacc = 0.f;
  constexpr int PL = C1_POS * C1_RLD;
  for (int i = threadIdx.x; i < C1_POS * C1CO / 4; i += 256) {
    const int o = (i >> 3) * C1_RLD + 4 * c4;
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(smem + o);
    const f32x4 s1 = *reinterpret_cast<const f32x4*>(smem + PL + o);
    const f32x4 s2 = *reinterpret_cast<const f32x4*>(smem + 2 * PL + o);
    const f32x4 s3 = *reinterpret_cast<const f32x4*>(smem + 3 * PL + o);
    const f32x4 sum = ((s0 + s1) + s2) + s3;
    const float bb[4] = {bias.x, bias.y, bias.z, bias.w};
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float y = div255(sum[e]) + bb[e];
      v[e] = linear ? y : relu(y);
    }
    if constexpr (PUB) {
      store_sc1_f4(out, C1_POS * C1CO * 4, 16 * i, v);
    } else if (dot) {
      const f32x4 d = *reinterpret_cast<const f32x4*>(dyp + 4 * i);
      dacc += ((v[0] * d[0] + v[1] * d[1]) + (v[2] * d[2] + v[3] * d[3]));
    } else {
      *reinterpret_cast<f32x4*>(out + 4 * i) = v;
    }
  }
  if constexpr (PUB) a.pub.arrive(sj.s);
  if (!PUB && dot) {
    __syncthreads();  // every thread is past its partial-row reads: smem is free
    const float r = block_sum256(dacc, smem);
    if (threadIdx.x == 0) a.dot.part[(int64_t)b * META_DOT_SLOTS + a.dot.slot0 + rb] = r;
  }
  DQZ_STAMP(0, 3);
}

struct Conv1DwArgs {
  Conv1Src src;
  int which, B;
  const float* dy1;  // [B][400][32] (online copy)
  float* part;       // [B*4][257][32]: dW rows 0..255 (HWIO order), db row 256
  Handoff sync1;     // dy1 arrival counters (conv1_dw_half in bwd_bc_kernel)
};

// Half-channel job of conv1 dW for the merged backward launch (bwd_bc_kernel):
// rows block rb of sample b, input channels {2 ch, 2 ch + 1}.  Its 128 dW rows
// (kh 8 x kw 8 x ci 2) are four 32-row tiles, one per wave (wave w: kh 2w,
// 2w + 1; tile row m = 16 (kh - 2w) + 2 kw + ci'), each summed over the 100
// positions.  As in conv1 forward the pixels are exact in bf16, and dy1 is
// split into three exact bf16 pieces (split3_bf16), so the sums run on
// v_mfma_f32_32x32x16_bf16 with exact products and f32 accumulation.  K order:
// 16 chunks of 8 positions (output row oh = c / 3, columns 8 (c % 3) + j; the
// columns past 19 and chunk 15 are zero on the dy1 side), instruction s takes
// chunks 2s (lane half 0) and 2s + 1.  dy1 comes from this launch's conv2 dX
// jobs: the block waits for its sample's counter, loads dy1 with sc1 loads
// (thread: 8 positions of one channel, for two chunks) and writes the pieces
// as a [piece][co][k] bf16 image, k contiguous, so the A fragment is one
// 16-byte LDS read; the B fragment gathers 8 pixels of the patch.
constexpr int C1H_TLD = 136;  // bf16 per co row of the dy1 image (272 B: 16-byte lane reads spread over the banks)
constexpr int C1H_SMEM = (2 * C1_PLANE * 2 + 3 * C1CO * C1H_TLD * 2) / 4 + 16 * C1CO;  // floats

__device__ __forceinline__ void conv1_dw_half(const Conv1DwArgs& a, float* smem, int rb, int ch, int b) {
  DQZ_STAMP(8, 0);
  uint16_t* s_in = reinterpret_cast<uint16_t*>(smem);  // 2 planes x 2016 bf16
  uint16_t* s_dt = s_in + 2 * C1_PLANE;                 // [3][32][C1H_TLD] bf16
  float* s_bp = smem + (2 * C1_PLANE + 3 * C1CO * C1H_TLD) / 2;  // [16][32] per-chunk dy1 sums (db)
  // frames of the two channels: slot -> fidx -> 2 x 126 16-byte pieces
  const int row0 = rb * C1S * C1_ROWS;
  constexpr int QPC = C1_PLANE / 16;  // 126
  const int slot = a.src.slots[b];
  const int32_t* fr = a.src.fidx + (int64_t)slot * 8 + a.which * 4 + 2 * ch;
  const int fa = fr[0], fb = fr[1];
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  const int tid = threadIdx.x;
  const int cl = tid / QPC, pj = tid % QPC;  // threads 0..251: channel cl, piece pj
  const int f = cl == 0 ? fa : fb;
  if (tid < 2 * QPC && f >= 0)
    v = reinterpret_cast<const uint4*>(a.src.frames + (int64_t)f * FB + row0 * FW)[pj];
  a.sync1.wait(b);
  const float* dyb = a.dy1 + ((int64_t)b * C1M + rb * C1_POS) * C1CO;
  const int co = tid & 31, c0 = tid >> 5;  // this thread: chunks c0 and c0 + 8 of channel co
  float dv[2][8];
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = c0 + 8 * it, oh = c / 3, ow0 = 8 * (c % 3);
#pragma unroll
    for (int j = 0; j < 8; ++j)
      dv[it][j] = (c < 15 && ow0 + j < C1O)
                      ? load_sc1_f1(dyb, C1_POS * C1CO * 4, (oh * C1O + ow0 + j) * C1CO + co) : 0.f;
  }
  if (tid < 2 * QPC) store_bytes_as_bf16(s_in + cl * C1_PLANE + pj * 16, v);
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int c = c0 + 8 * it;
    unsigned pk[3][4];
    float sb = 0.f;
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      unsigned h0, m0, l0, h1, m1, l1;
      split3_bf16(dv[it][j], h0, m0, l0);
      split3_bf16(dv[it][j + 1], h1, m1, l1);
      pk[0][j / 2] = h0 | (h1 << 16);
      pk[1][j / 2] = m0 | (m1 << 16);
      pk[2][j / 2] = l0 | (l1 << 16);
      sb += dv[it][j];
      sb += dv[it][j + 1];
    }
#pragma unroll
    for (int q = 0; q < 3; ++q)
      *reinterpret_cast<uint4*>(s_dt + (q * C1CO + co) * C1H_TLD + 8 * c) =
          make_uint4(pk[q][0], pk[q][1], pk[q][2], pk[q][3]);
    s_bp[c * C1CO + co] = sb;
  }
  __syncthreads();
  DQZ_STAMP(8, 1);
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, i = lane & 31;
  float* part = a.part + ((int64_t)b * C1_BLOCKS + rb) * (C1KK + 1) * C1CO;
  if (ch == 0 && tid < C1CO) {  // bias row
    float sb = 0.f;
    for (int c = 0; c < 15; ++c) sb += s_bp[c * C1CO + tid];
    part[C1KK * C1CO + tid] = sb;
  }
  const int kh = 2 * wave + (i >> 4), kw = (i >> 1) & 7, cp = i & 1;
  const uint16_t* pb = s_in + cp * C1_PLANE + kh * FW + kw;
  const uint16_t* pa = s_dt + i * C1H_TLD + 8 * h;
  f32x16 acc = {};
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    // chunk c = 2s + h: patch pixels at output row c / 3, columns 8 (c % 3) + j
    // (chunk 15 reads chunk 0's pixels: its dy1 side is zero)
    constexpr int R = 4 * FW;
    const int o0 = (2 * s) / 3 * R + 32 * ((2 * s) % 3);
    const int o1 = 2 * s + 1 < 15 ? (2 * s + 1) / 3 * R + 32 * ((2 * s + 1) % 3) : 0;
    const uint16_t* px = pb + (h ? o1 : o0);
    unsigned xp[4];
#pragma unroll
    for (int j = 0; j < 8; j += 2) xp[j / 2] = (unsigned)px[4 * j] | ((unsigned)px[4 * j + 4] << 16);
    const bf16x8 xb = __builtin_bit_cast(bf16x8, make_uint4(xp[0], xp[1], xp[2], xp[3]));
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const bf16x8 dq = __builtin_bit_cast(bf16x8, *reinterpret_cast<const uint4*>(pa + q * C1CO * C1H_TLD + 16 * s));
      // A = dy1 pieces (rows: co), B = the patch (columns: dW row m)
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(dq, xb, acc, 0, 0, 0);
    }
  }
  // C col = lane & 31 = m -> kh = 2 wave + (m >> 4), kw = (m >> 1) & 7, ci = 2 ch + (m & 1);
  // rows co = (r & 3) + 8 (r >> 2) + 4 h: one float4 store per r >> 2.  The
  // sums are over raw pixels: dW = (sum x dy) / 255 (networks.py:192)
  {
    const int row = (2 * wave + (i >> 4)) * 32 + ((i >> 1) & 7) * 4 + 2 * ch + (i & 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<f32x4*>(part + row * C1CO + 8 * q + 4 * h) =
          f32x4{div255(acc[4 * q]), div255(acc[4 * q + 1]), div255(acc[4 * q + 2]), div255(acc[4 * q + 3])};
  }
  DQZ_STAMP(8, 3);
}

}  // namespace dqz
