// Microbenchmark: per-kernel cost inside a hipGraph on gfx950.
//   empty       : kernel that does nothing (256 WGs)
//   one_load    : each WG loads one value written by the previous kernel, writes one
//   chain3      : three dependent loads (index -> index -> value), like slot->fidx->frame
//   stream_4mb  : 256 WGs each read 16 KB (4 MB total), write 1 value
// Prints microseconds per kernel from graph replay of 200 kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_empty(float*) {}
__global__ void k_one_load(float* buf) {
  float v = buf[blockIdx.x * 64];
  if (threadIdx.x == 0) buf[blockIdx.x * 64 + 1] = v + 1.f;
}
__global__ void k_chain3(const int* idx, float* buf) {
  int a = idx[blockIdx.x];
  int b = idx[a];
  float v = buf[b * 64];
  if (threadIdx.x == 0) buf[blockIdx.x * 64 + 1] = v + 1.f;
}
__global__ void k_stream(const float4* src, float* out) {
  const float4* p = src + (size_t)blockIdx.x * 1024;
  float4 r[4];
  for (int q = 0; q < 4; ++q) r[q] = p[threadIdx.x + 256 * q];
  float s = 0.f;
  for (int q = 0; q < 4; ++q) s += r[q].x + r[q].y + r[q].z + r[q].w;
  if (s == 12345.f) out[blockIdx.x] = s;
}

template <class F>
float time_graph(hipStream_t st, F launch, int n) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeGlobal);
  for (int i = 0; i < n; ++i) launch();
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 3; ++w) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0, st);
  const int reps = 10;
  for (int r = 0; r < reps; ++r) hipGraphLaunch(ge, st);
  hipEventRecord(e1, st);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1000.f / (reps * n);
}

int main() {
  hipStream_t st;
  hipStreamCreate(&st);
  float* buf;
  int* idx;
  float4* big;
  hipMalloc(&buf, 256 * 64 * 4 * 4);
  hipMalloc(&idx, 4096 * 4);
  hipMalloc(&big, (size_t)256 * 1024 * 16);
  hipMemset(buf, 0, 256 * 64 * 16);
  std::vector<int> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = (i * 7 + 3) % 256;
  hipMemcpy(idx, h.data(), 4096 * 4, hipMemcpyHostToDevice);
  hipMemset(big, 0, (size_t)256 * 1024 * 16);
  const int n = 200;
  for (int wgs : {1, 256, 1024}) {
    printf("WGs=%d\n", wgs);
    printf("  empty      %.2f us\n", time_graph(st, [&] { hipLaunchKernelGGL(k_empty, dim3(wgs), dim3(256), 0, st, buf); }, n));
    printf("  one_load   %.2f us\n", time_graph(st, [&] { hipLaunchKernelGGL(k_one_load, dim3(wgs < 256 ? wgs : 256), dim3(256), 0, st, buf); }, n));
    printf("  chain3     %.2f us\n", time_graph(st, [&] { hipLaunchKernelGGL(k_chain3, dim3(wgs < 256 ? wgs : 256), dim3(256), 0, st, idx, buf); }, n));
    printf("  stream_4mb %.2f us\n", time_graph(st, [&] { hipLaunchKernelGGL(k_stream, dim3(256), dim3(256), 0, st, big, buf); }, n));
  }
  return 0;
}
