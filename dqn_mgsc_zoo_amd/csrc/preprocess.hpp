// preprocess.hpp — the Atari observation step of processors.atari on device
// (processors.py:488-497): max-pool of the last RGB frames, rgb2y, PIL
// BILINEAR resize to 84x84, in one launch.
//
// rgb2y (processors.py:367-371) is numpy's tensordot with
// [0.299, 0.587, 1 - (0.299 + 0.587)] followed by astype(uint8); numpy's
// BLAS evaluates it as fma(b, w2, fma(r, w0, g * w1)) in float64 (equal for
// every one of the 2^24 RGB triples on this image), so the kernel does
// exactly that and truncates.
//
// The resize is Pillow's 8-bit two-pass resampler (libImaging/Resample.c):
// per output coordinate a triangle filter whose support scales with the
// reduction factor, weights normalised in double and rounded to int32 with
// 22 fractional bits (round half away from zero) on the host
// (dqz_frame_plan_create), integer accumulation from 2^21, >> 22 and a clip
// to [0, 255] after each pass, horizontal pass first over the source rows
// the vertical pass uses.  A workgroup owns FR_ROWS output rows: it converts
// the band of source rows they need into LDS, runs the horizontal pass on
// that band, then the vertical pass.
#pragma once
#include "common.hpp"

namespace dqz {

constexpr int FR_PREC = 22;  // Pillow PRECISION_BITS = 32 - 8 - 2
constexpr int FR_ROWS = 4;   // output rows per workgroup

struct FramePlan {
  int in_h, in_w, out_h, out_w;
  int kh, kv;         // coefficients per output column / row
  int max_band;       // most source rows any workgroup needs
  const int32_t* hb;  // [out_w][2] first source column, count
  const int32_t* hk;  // [out_w][kh]
  const int32_t* vb;  // [out_h][2] first source row, count
  const int32_t* vk;  // [out_h][kv]
};

__device__ __forceinline__ uint8_t clip8(int acc) {
  const int v = acc >> FR_PREC;
  return (uint8_t)(v < 0 ? 0 : v > 255 ? 255 : v);
}

__device__ __forceinline__ uint32_t max_u8x4(uint32_t a, uint32_t b) {
  uint32_t r = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) r |= max((a >> (8 * k)) & 0xFFu, (b >> (8 * k)) & 0xFFu) << (8 * k);
  return r;
}

__device__ __forceinline__ uint8_t rgb2y_u8(unsigned r, unsigned g, unsigned b) {
  const double w0 = 0.299, w1 = 0.587, w2 = 1.0 - (0.299 + 0.587);
  const double y = __builtin_fma((double)b, w2, __builtin_fma((double)r, w0, (double)g * w1));
  return (uint8_t)(unsigned)y;  // astype(np.uint8) of a value in [0, 256): truncation
}

// rgb: n frames of [in_h][in_w][3] uint8, frame_stride bytes apart; the
// pixel is the element-wise max over the frames (np.max(..., axis=0)).
__global__ __launch_bounds__(256) void atari_frame_kernel(FramePlan p, const uint8_t* __restrict__ rgb, int n,
                                                          int64_t frame_stride, uint8_t* __restrict__ out) {
  extern __shared__ uint8_t fr_smem[];
  const int yy0 = blockIdx.x * FR_ROWS, yy1 = min(yy0 + FR_ROWS, p.out_h);
  const int r0 = p.vb[2 * yy0];
  const int r1 = p.vb[2 * (yy1 - 1)] + p.vb[2 * (yy1 - 1) + 1];
  const int band = r1 - r0;
  uint8_t* sy = fr_smem;                       // [band][in_w] luma
  uint8_t* st = fr_smem + p.max_band * p.in_w;  // [band][out_w] after the horizontal pass
  // 1. max-pool + rgb2y of the band; four pixels (three 32-bit words) per item
  //    when the row is word-aligned (the Atari 160-pixel rows are)
  if (p.in_w % 4 == 0) {
    const int groups = p.in_w / 4;
    for (int i = threadIdx.x; i < band * groups; i += blockDim.x) {
      const int r = i / groups, c4 = i % groups;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(rgb + ((int64_t)(r0 + r) * p.in_w + 4 * c4) * 3);
      uint32_t w[3] = {src[0], src[1], src[2]};
      for (int f = 1; f < n; ++f) {
        const uint32_t* q = reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(src) + f * frame_stride);
#pragma unroll
        for (int k = 0; k < 3; ++k) w[k] = max_u8x4(w[k], q[k]);
      }
      uint8_t* dst = sy + r * p.in_w + 4 * c4;
#pragma unroll
      for (int px = 0; px < 4; ++px) {
        const int b0 = 3 * px;
        const unsigned R = (w[b0 >> 2] >> (8 * (b0 & 3))) & 0xFF;
        const unsigned G = (w[(b0 + 1) >> 2] >> (8 * ((b0 + 1) & 3))) & 0xFF;
        const unsigned B = (w[(b0 + 2) >> 2] >> (8 * ((b0 + 2) & 3))) & 0xFF;
        dst[px] = rgb2y_u8(R, G, B);
      }
    }
  } else {
    for (int i = threadIdx.x; i < band * p.in_w; i += blockDim.x) {
      const int r = i / p.in_w, c = i % p.in_w;
      const uint8_t* px = rgb + ((int64_t)(r0 + r) * p.in_w + c) * 3;
      unsigned R = px[0], G = px[1], B = px[2];
      for (int f = 1; f < n; ++f) {
        const uint8_t* q = px + f * frame_stride;
        R = max(R, (unsigned)q[0]);
        G = max(G, (unsigned)q[1]);
        B = max(B, (unsigned)q[2]);
      }
      sy[i] = rgb2y_u8(R, G, B);
    }
  }
  __syncthreads();
  // 2. horizontal pass over the band
  for (int i = threadIdx.x; i < band * p.out_w; i += blockDim.x) {
    const int r = i / p.out_w, xx = i % p.out_w;
    const int x0 = p.hb[2 * xx], cnt = p.hb[2 * xx + 1];
    const uint8_t* row = sy + r * p.in_w + x0;
    const int32_t* k = p.hk + xx * p.kh;
    int acc = 1 << (FR_PREC - 1);
    for (int x = 0; x < cnt; ++x) acc += (int)row[x] * k[x];
    st[i] = clip8(acc);
  }
  __syncthreads();
  // 3. vertical pass for this workgroup's output rows
  for (int i = threadIdx.x; i < (yy1 - yy0) * p.out_w; i += blockDim.x) {
    const int yy = yy0 + i / p.out_w, xx = i % p.out_w;
    const int y0 = p.vb[2 * yy] - r0, cnt = p.vb[2 * yy + 1];
    const int32_t* k = p.vk + yy * p.kv;
    int acc = 1 << (FR_PREC - 1);
    for (int y = 0; y < cnt; ++y) acc += (int)st[(y0 + y) * p.out_w + xx] * k[y];
    out[yy * p.out_w + xx] = clip8(acc);
  }
}

}  // namespace dqz
