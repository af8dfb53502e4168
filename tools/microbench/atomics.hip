// Microbenchmark: random-access primitive rates on MI355X (tables >> L2/MALL or MALL-sized).
// load / store / CAS (agent, workgroup scope) / atomicMin no-return / LDS-style.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

using u64 = unsigned long long;
using u32 = unsigned int;

__device__ __forceinline__ u64 mix(u64 x) {
  x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33; return x;
}

template <int MODE>
__global__ void k(u64* __restrict__ tab, u64 mask, u64 n, u64 salt, u64* __restrict__ sink) {
  const u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const u64 h = mix(i ^ salt);
  const u64 s = h & mask;
  u64 r = 0;
  if (MODE == 0) r = tab[s];                                                   // load
  if (MODE == 1) tab[s] = h;                                                   // store
  if (MODE == 2) r = atomicCAS(&tab[s], ~0ull, h);                             // CAS agent
  if (MODE == 3) atomicMin(&tab[s], h);                                        // min no-return
  if (MODE == 4) { u64 e = ~0ull; __hip_atomic_compare_exchange_strong(&tab[s], &e, h, __ATOMIC_RELAXED,
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); r = e; }  // CAS workgroup scope
  if (MODE == 5) r = atomicMin(&tab[s], h);                                    // min returning
  if (MODE == 6) { u64 v = tab[s]; if (v == ~0ull) v = atomicCAS(&tab[s], ~0ull, h); r = v; }  // load then CAS
  if (MODE == 7) { reinterpret_cast<u32*>(tab)[s] = u32(h); }                 // 4-B store
  if (r == 0x12345) sink[0] = r;
}

int main(int argc, char** argv) {
  const u64 n = 41666667;
  std::vector<u64> caps = {1ull << 23, 1ull << 27};   // 64 MB (MALL) and 1 GB (HBM)
  u64* tab; u64* sink;
  hipMalloc(&tab, (1ull << 27) * 8);
  hipMalloc(&sink, 8);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  const char* names[] = {"load8", "store8", "cas_agent", "min_noret", "cas_wg", "min_ret", "load_then_cas", "store4"};
  for (u64 cap : caps) {
    for (int mode = 0; mode < 8; ++mode) {
      float best = 1e9;
      for (int rep = 0; rep < 4; ++rep) {
        hipMemset(tab, 0xff, cap * 8);
        hipEventRecord(a);
        dim3 g((n + 255) / 256);
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 1: hipLaunchKernelGGL(k<1>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 2: hipLaunchKernelGGL(k<2>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 3: hipLaunchKernelGGL(k<3>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 4: hipLaunchKernelGGL(k<4>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 5: hipLaunchKernelGGL(k<5>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 6: hipLaunchKernelGGL(k<6>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
          case 7: hipLaunchKernelGGL(k<7>, g, 256, 0, 0, tab, cap - 1, n, u64(rep), sink); break;
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (ms < best) best = ms;
      }
      printf("{\"cap_mb\": %llu, \"op\": \"%s\", \"ms\": %.4f, \"Gops\": %.2f}\n", cap * 8 >> 20, names[mode], best,
             n / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
