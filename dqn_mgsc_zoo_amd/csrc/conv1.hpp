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

namespace dqz {

struct Conv1Src {
  const uint8_t* frames;  // frame pool (null when `states` is used)
  const int32_t* fidx;    // [capacity][8]
  const int32_t* slots;   // [B]
  const uint8_t* states;  // direct uint8 [B][84][84][4] input, or null
  int fused;              // 1: slots come from the fused uniform sampler `draw`
  UniformDraw draw;
  // Batch record: block (rb 0, z 0) of sample b also copies action / reward /
  // discount of its slot into rec[b] = {a as int bits, r, d, 0}, so the head
  // reads one record per sample instead of the slot -> record chain.
  const int32_t* action = nullptr;
  const float* reward = nullptr;
  const float* discount = nullptr;
  float4* rec = nullptr;
};

__device__ __forceinline__ void store_bytes_as_f32(float* dst, uint4 v) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float4 f;
    f.x = u8n(w[i] & 0xFF);
    f.y = u8n((w[i] >> 8) & 0xFF);
    f.z = u8n((w[i] >> 16) & 0xFF);
    f.w = u8n(w[i] >> 24);
    *reinterpret_cast<float4*>(dst + 4 * i) = f;
  }
}

// Stages input rows [20*rb, 20*rb + 24) of sample b, stack `which`, as
// s_in[ci][row][col] = pixel / 255.
__device__ __forceinline__ void stage_conv1_input(float* s_in, const Conv1Src& src, int b, int which, int rb,
                                                  int z = 0, int sk = -1) {
  const int row0 = rb * C1S * C1_ROWS;
  constexpr int QPC = C1_PLANE / 16;  // 126 16-byte pieces per channel
  if (src.states) {
    const uint4* g = reinterpret_cast<const uint4*>(src.states + ((int64_t)b * FH + row0) * FW * FC);
    for (int i = threadIdx.x; i < C1_PLANE * FC / 16; i += blockDim.x) {
      const uint4 v = g[i];  // 4 pixels x 4 channels
      const unsigned w[4] = {v.x, v.y, v.z, v.w};
      const int p = 4 * i;
#pragma unroll
      for (int ci = 0; ci < 4; ++ci) {
        float4 f;
        f.x = u8n((w[0] >> (8 * ci)) & 0xFF);
        f.y = u8n((w[1] >> (8 * ci)) & 0xFF);
        f.z = u8n((w[2] >> (8 * ci)) & 0xFF);
        f.w = u8n((w[3] >> (8 * ci)) & 0xFF);
        *reinterpret_cast<float4*>(s_in + ci * C1_PLANE + p) = f;
      }
    }
  } else {
    // slot -> 4 frame ids -> 504 16-byte pieces (2 per thread), all loads in
    // flight before the first LDS store.
    int slot;
    if (src.fused) {  // fused sampler: draw b of this step; block (0, b, 0) publishes it
      slot = uniform_slot(*src.draw.counter, b, src.draw);
      if (threadIdx.x == 0 && rb == 0 && z == 0) src.draw.slots_out[b] = slot;
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
    if (sk >= 0) DQZ_STAMP(sk, 1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int i = (int)threadIdx.x + 256 * q;
      if (i < NP) {
        const int ci = i / QPC, j = i % QPC;
        float* dst = s_in + ci * C1_PLANE + j * 16;
        if (fq[q] < 0) v[q] = make_uint4(0u, 0u, 0u, 0u);  // trailing zero padding
        store_bytes_as_f32(dst, v[q]);
      }
    }
    if (wrec) src.rec[b] = recv;
    if (sk >= 0) DQZ_STAMP(sk, 2);
  }
}

struct Conv1FwdArgs {
  Conv1Src src;
  NetZ nz;
  int64_t w_off, b_off;
  int B, Z;
  int linear;  // 1: write the pre-activation (no ReLU)
  float* out;  // y1 [Z][B][400][32]
  Handoff pub;  // PUB: y1 rows handed to conv2 in the same launch (fwd_conv_kernel)
};

// grid (4 row blocks, B, Z); 256 threads; each wave owns 32 positions x 32
// channels (the 4th wave's tile is 4/32 live).  PUB: y1 stores are sc1 and
// the block arrives on its sample's counter (common.hpp Handoff).
template <bool PUB>
__device__ __forceinline__ void conv1_fwd_body(const Conv1FwdArgs& a, float* smem, const SampleJob sj) {
  DQZ_STAMP(0, 0);
  float* s_in = smem;                  // 8064
  float* s_w = smem + C1_IN_FLOATS;    // 256 x 32
  const int rb = sj.job, b = sj.s % a.B, z = sj.s / a.B;
  const float bias = a.nz.p[z][a.b_off + (threadIdx.x & 31)];  // epilogue operand, loaded early
  const float4* w4 = reinterpret_cast<const float4*>(a.nz.p[z] + a.w_off);
  // 256 x 32 weights = 8 float4 per thread, staged first: they arrive with
  // the sampler's counter load, and (left to the compiler) their loads would
  // sink below the frame gather and add a round trip at the end.
  float4 wv[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) wv[q] = w4[threadIdx.x + 256 * q];
#pragma unroll
  for (int q = 0; q < 8; ++q) reinterpret_cast<float4*>(s_w)[threadIdx.x + 256 * q] = wv[q];
  stage_conv1_input(s_in, a.src, b, a.nz.which[z], rb, z, 14);
  DQZ_STAMP(0, 1);
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, i = lane & 31;
  const int p = min(32 * wave + i, C1_POS - 1);
  const int oh = p / C1O, ow = p % C1O;
  const float* pa = s_in + h * C1_PLANE + (C1S * oh) * FW + C1S * ow;
  const float* pb = s_w + h * C1CO + i;
  f32x16 acc = {};
#pragma unroll
  for (int j = 0; j < 128; ++j) {
    // k = 2j + h  ->  kh = j >> 4, kw = (j >> 1) & 7, ci = 2 (j & 1) + h
    const float av = pa[2 * (j & 1) * C1_PLANE + (j >> 4) * FW + ((j >> 1) & 7)];
    const float bv = pb[64 * j];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
  }
  DQZ_STAMP(0, 2);
  // C/D map of 32x32x2: col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 h
  // (fields read once: inside the store loop they could alias `out`, and the
  // compiler would re-read them behind a vmcnt(0) per store)
  float* out = a.out + (((int64_t)z * a.B + b) * C1M + rb * C1_POS) * C1CO;
  const bool linear = a.linear;
  // Materialise the bias before the store loop: otherwise its (long landed)
  // load is waited for with a vmcnt(0) inside every exec-masked store group,
  // and vmcnt counts the stores issued so far too.
  float bias_r = bias;
  asm volatile("" : "+v"(bias_r));
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int pos = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (pos < C1_POS) {
      const float v = acc[r] + bias_r;
      if constexpr (PUB)
        __hip_atomic_store(out + pos * C1CO + i, linear ? v : relu(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        out[pos * C1CO + i] = linear ? v : relu(v);
    }
  }
  if constexpr (PUB) a.pub.arrive(sj.s);
  DQZ_STAMP(0, 3);
}

__global__ __launch_bounds__(256) void conv1_fwd_kernel(Conv1FwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const SampleJob sj = xcd_sample_job(C1_BLOCKS, a.Z * a.B);
  if (!sj.valid) return;
  conv1_fwd_body<false>(a, smem, sj);
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
// (kh 8 x kw 8 x ci 2) are four 32-row MFMA tiles, one per wave (wave w: kh
// 2w, 2w + 1; tile row m = 16 (kh - 2w) + 2 kw + ci'), each accumulated over
// the 100 positions in a fixed order.  LDS: two input planes + the 100 x 32 dy1 block (29 KB).  dy1
// comes from this launch's conv2 dX jobs: the block waits for its sample's
// counter and loads dy1 with sc1 loads.
constexpr int C1H_SMEM = 2 * C1_PLANE + C1_POS * C1CO;  // 7232 floats

__device__ __forceinline__ void conv1_dw_half(const Conv1DwArgs& a, float* smem, int rb, int ch, int b) {
  DQZ_STAMP(8, 0);
  float* s_in = smem;                 // 2 planes x 2016
  float* s_dy = smem + 2 * C1_PLANE;  // 100 x 32
  // frames of the two channels: slot -> fidx -> 2 x 126 16-byte pieces
  const int row0 = rb * C1S * C1_ROWS;
  constexpr int QPC = C1_PLANE / 16;  // 126
  const int slot = a.src.slots[b];
  const int32_t* fr = a.src.fidx + (int64_t)slot * 8 + a.which * 4 + 2 * ch;
  const int fa = fr[0], fb = fr[1];
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  const int tid = threadIdx.x;
  const int cl = tid / QPC, j = tid % QPC;  // threads 0..251: channel cl, piece j
  const int f = cl == 0 ? fa : fb;
  if (tid < 2 * QPC && f >= 0)
    v = reinterpret_cast<const uint4*>(a.src.frames + (int64_t)f * FB + row0 * FW)[j];
  a.sync1.wait(b);
  const float4* dy4 = reinterpret_cast<const float4*>(a.dy1 + ((int64_t)b * C1M + rb * C1_POS) * C1CO);
  constexpr int ND4 = C1_POS * C1CO / 4;  // 800
  float4 dv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) dv[q] = load_sc1_f4(dy4, ND4 * 16, min(tid + 256 * q, ND4 - 1));
  if (tid < 2 * QPC) store_bytes_as_f32(s_in + cl * C1_PLANE + j * 16, v);
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (tid + 256 * q < ND4) reinterpret_cast<float4*>(s_dy)[tid + 256 * q] = dv[q];
  __syncthreads();
  DQZ_STAMP(8, 1);
  const int lane = tid & 63, wave = tid >> 6;
  const int h = lane >> 5, i = lane & 31;
  const int kh = 2 * wave + (i >> 4), kw = (i >> 1) & 7, cp = i & 1;
  float* part = a.part + ((int64_t)b * C1_BLOCKS + rb) * (C1KK + 1) * C1CO;
  if (ch == 0 && tid < C1CO) {  // bias row
    float sb = 0.f;
    for (int p = 0; p < C1_POS; ++p) sb += s_dy[p * C1CO + tid];
    part[C1KK * C1CO + tid] = sb;
  }
  const float* pa = s_in + cp * C1_PLANE + kh * FW + kw + 4 * h;
  const float* pb = s_dy + h * C1CO + i;
  f32x16 acc = {};
#pragma unroll
  for (int jj = 0; jj < C1_POS / 2; ++jj) {
    const int p0 = 2 * jj;  // positions p0 + h share an output row
    const float av = pa[(C1S * (p0 / C1O)) * FW + C1S * (p0 % C1O)];
    const float bv = pb[64 * jj];
    // A = dy1 (rows: co), B = the frame patch (columns: dW row m): four
    // consecutive co per accumulator group, same bits as the transposed form
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(bv, av, acc, 0, 0, 0);
  }
  // C col = lane & 31 = m -> kh = 2 wave + (m >> 4), kw = (m >> 1) & 7, ci = 2 ch + (m & 1);
  // rows co = (r & 3) + 8 (r >> 2) + 4 h: one float4 store per r >> 2
  {
    const int row = (2 * wave + (i >> 4)) * 32 + ((i >> 1) & 7) * 4 + 2 * ch + (i & 1);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<f32x4*>(part + row * C1CO + 8 * q + 4 * h) =
          f32x4{acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
  }
  DQZ_STAMP(8, 3);
}

constexpr size_t kConv1FwdSmem = (C1_IN_FLOATS + C1KK * C1CO) * sizeof(float);

}  // namespace dqz
