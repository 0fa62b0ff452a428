// Microbenchmark of the learned-logit sampler pieces at 1M logits (gfx950).
// Graph-replayed launch times (us per launch, 200 launches per graph):
//   empty_245       an empty launch of 245 blocks (launch floor)
//   stream_245      loads of 4 MB by 245 x 256 lanes (float4), sum in f32
//   chunk_sums_all  chunk_sums_kernel over every chunk (a re-seed's pass)
//   chunk_sums_none the same launch with no dirty chunk (the per-write pass floor)
//   sample32        softmax_sample_kernel: 32 queries (chunk sums + one chunk each)
//   sample1         one query
//   add_running     logits_add_running_kernel (one add + its chunk sum)
//   put1            logits_put1_kernel
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I dqn_mgsc_zoo_amd/csrc -I include
//        tools/softmax_micro.hip -o tools/softmax_micro.bin
#include <vector>
#include <cmath>
#include <random>
#include "sampling.hpp"

using namespace dqz;

__global__ void k_empty() {}

__global__ __launch_bounds__(256) void k_stream(const float* __restrict__ x, int64_t n, double* out) {
  const int64_t base = (int64_t)blockIdx.x * SM_CHUNK;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t j = base + 4 * (threadIdx.x + 256 * q);
    if (j + 3 < n) {
      const float4 f = *reinterpret_cast<const float4*>(x + j);
      s += f.x + f.y + f.z + f.w;
    }
  }
  if (s == 12345.f) out[blockIdx.x] = s;
}


template <class F>
float time_graph(hipStream_t st, F launch, int n = 200) {
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
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1000.f / (reps * n);
}

int main() {
  const int64_t n = 1000000;
  const int nb = (int)((n + SM_CHUNK - 1) / SM_CHUNK);
  const int nq = 32;
  hipStream_t st;
  hipStreamCreate(&st);
  std::vector<float> h(n);
  std::mt19937 rng(0);
  std::normal_distribution<float> nd;
  for (auto& v : h) v = nd(rng);
  double S = 0.0;
  float c = h[0];
  for (float v : h) c = std::max(c, v);
  for (float v : h) S += std::exp((double)v - (double)c);
  float* x;
  float* p;
  double *bsum, *u, *scratch;
  int64_t* out;
  int* words;
  LogitRun* run;
  float* lse;
  hipMalloc(&x, n * 4);
  hipMalloc(&p, n * 4);
  hipMalloc(&bsum, nb * 8);
  hipMalloc(&scratch, nb * 8);
  hipMalloc(&u, nq * 8);
  hipMalloc(&out, nq * 8);
  hipMalloc(&words, 3 * 64 * 4);
  hipMalloc(&run, sizeof(LogitRun));
  hipMalloc(&lse, 4);
  hipMemset(words, 0, 3 * 64 * 4);
  hipMemcpy(x, h.data(), n * 4, hipMemcpyHostToDevice);
  LogitRun r{S, c, 1};
  hipMemcpy(run, &r, sizeof r, hipMemcpyHostToDevice);
  std::vector<double> hu(nq);
  for (int i = 0; i < nq; ++i) hu[i] = (i + 0.5) / nq;
  hipMemcpy(u, hu.data(), nq * 8, hipMemcpyHostToDevice);
  int* dirty;
  hipMalloc(&dirty, nb * 4);
  hipMemset(dirty, 0, nb * 4);
  hipLaunchKernelGGL(chunk_sums_kernel, dim3(nb), dim3(SM_THREADS), 0, st, x, n, run, bsum, (int*)nullptr);
  hipStreamSynchronize(st);
  printf("{\"empty_245\": %.2f", time_graph(st, [&] { hipLaunchKernelGGL(k_empty, dim3(nb), dim3(256), 0, st); }));
  printf(", \"stream_245\": %.2f",
         time_graph(st, [&] { hipLaunchKernelGGL(k_stream, dim3(nb), dim3(256), 0, st, x, n, scratch); }));
  printf(", \"chunk_sums_all\": %.2f", time_graph(st, [&] {
           hipLaunchKernelGGL(chunk_sums_kernel, dim3(nb), dim3(SM_THREADS), 0, st, x, n, run, bsum, (int*)nullptr);
         }));
  printf(", \"chunk_sums_none\": %.2f", time_graph(st, [&] {
           hipLaunchKernelGGL(chunk_sums_kernel, dim3(nb), dim3(SM_THREADS), 0, st, x, n, run, bsum, dirty);
         }));
  printf(", \"sample32\": %.2f", time_graph(st, [&] {
           hipLaunchKernelGGL(softmax_sample_kernel, dim3(nq), dim3(SM_THREADS), 0, st, x, n, run, bsum, nb,
                              SampleSync{words}, 0ull, (uint64_t*)nullptr, u, nq, (int32_t*)nullptr, out);
         }));
  printf(", \"sample1\": %.2f", time_graph(st, [&] {
           hipLaunchKernelGGL(softmax_sample_kernel, dim3(1), dim3(SM_THREADS), 0, st, x, n, run, bsum, nb,
                              SampleSync{words}, 0ull, (uint64_t*)nullptr, u, 1, (int32_t*)nullptr, out);
         }));
  int64_t pos = 0;
  printf(", \"add_running\": %.2f", time_graph(st, [&] {
           pos = (pos + 4099) % n;
           hipLaunchKernelGGL(logits_add_running_kernel, dim3(1), dim3(SM_THREADS), 0, st, x, n, run, bsum, pos, pos,
                              n, lse);
         }));
  printf(", \"put1\": %.2f", time_graph(st, [&] {
           pos = (pos + 4099) % n;
           hipLaunchKernelGGL(logits_put1_kernel, dim3(1), dim3(SM_THREADS), 0, st, x, n, run, bsum, pos, 0.5f);
         }));
  printf("}\n");
  return 0;
}
