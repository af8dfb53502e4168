// Dependent-launch floor on one stream: N trivial kernels back to back, eager and as a
// replayed HIP graph, timed with events (per-kernel cost of a small build's level chain).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

__global__ void k_touch(unsigned* p, int i) {
  if (threadIdx.x == 0 && blockIdx.x == 0) p[i & 255] += 1;
}

int main() {
  unsigned* d = nullptr;
  (void)hipMalloc(&d, 4096);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int blocks : {1, 64, 512}) {
    for (int n : {8, 32}) {
      auto chain = [&]() {
        for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_touch, dim3(blocks), dim3(256), 0, s, d, i);
      };
      for (int w = 0; w < 3; ++w) chain();
      (void)hipStreamSynchronize(s);
      float best = 1e9f;
      for (int r = 0; r < 20; ++r) {
        (void)hipEventRecord(a, s);
        chain();
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        best = ms < best ? ms : best;
      }
      hipGraph_t g;
      hipGraphExec_t ge;
      (void)hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
      chain();
      (void)hipStreamEndCapture(s, &g);
      (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
      for (int w = 0; w < 3; ++w) (void)hipGraphLaunch(ge, s);
      (void)hipStreamSynchronize(s);
      float bestg = 1e9f;
      for (int r = 0; r < 20; ++r) {
        (void)hipEventRecord(a, s);
        (void)hipGraphLaunch(ge, s);
        (void)hipEventRecord(b, s);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        bestg = ms < bestg ? ms : bestg;
      }
      std::printf("{\"blocks\": %d, \"kernels\": %d, \"eager_us_per_kernel\": %.2f, \"graph_us_per_kernel\": %.2f}\n",
                  blocks, n, best * 1e3 / n, bestg * 1e3 / n);
      (void)hipGraphExecDestroy(ge);
      (void)hipGraphDestroy(g);
    }
  }
  return 0;
}
