// Microbenchmark: cost of one same-address atomicAdd per workgroup (look-back tickets,
// shared statistics counters) against padded shards, for 5K..160K workgroups.
#include <hip/hip_runtime.h>
#include <cstdio>

using u32 = unsigned int;
using u64 = unsigned long long;

template <int MODE>
__global__ __launch_bounds__(256) void k(u32* __restrict__ ctr, u32* __restrict__ sink) {
  __shared__ u32 s;
  if (threadIdx.x == 0) {
    if (MODE == 0) s = atomicAdd(ctr, 1u);                                  // one address
    if (MODE == 1) s = atomicAdd(&ctr[(blockIdx.x & 63) * 2], 1u);          // 64 shards, 8 B apart
    if (MODE == 2) s = atomicAdd(&ctr[(blockIdx.x & 1023) * 16], 1u);       // 1024 shards, 64 B apart
    if (MODE == 3) s = blockIdx.x;                                          // none
  }
  __syncthreads();
  if (s == 0xffffffffu) sink[0] = s;
}

int main() {
  u32 *ctr, *sink;
  hipMalloc(&ctr, 1024 * 64 * 4);
  hipMalloc(&sink, 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"one_address", "shards64_8B", "shards1024_64B", "none"};
  for (u32 nb : {5000u, 20000u, 80000u, 160000u})
    for (int mode = 0; mode < 4; ++mode) {
      float best = 1e9;
      for (int rep = 0; rep < 5; ++rep) {
        hipMemset(ctr, 0, 1024 * 64 * 4);
        hipEventRecord(a);
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, dim3(nb), dim3(256), 0, 0, ctr, sink); break;
          case 1: hipLaunchKernelGGL(k<1>, dim3(nb), dim3(256), 0, 0, ctr, sink); break;
          case 2: hipLaunchKernelGGL(k<2>, dim3(nb), dim3(256), 0, 0, ctr, sink); break;
          case 3: hipLaunchKernelGGL(k<3>, dim3(nb), dim3(256), 0, 0, ctr, sink); break;
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("{\"blocks\": %u, \"mode\": \"%s\", \"ms\": %.4f}\n", nb, names[mode], best);
    }
  return 0;
}
