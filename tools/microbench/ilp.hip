// Microbenchmark: random-access throughput vs independent accesses in flight per thread
// (U loads / load-then-CAS per thread) for MALL-sized and HBM-sized tables on MI355X.
// Question: are the leaf probe (128 MB table) and the node insert (1 GB table) bound by
// the memory system or by the accesses one wave keeps in flight?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

using u64 = unsigned long long;

__device__ __forceinline__ u64 mix(u64 x) {
  x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33; return x;
}

// MODE 0: 8-B loads; 1: 4-B loads; 2: load-then-CAS (8 B)
template <int MODE, int U>
__global__ __launch_bounds__(256) void k(u64* __restrict__ tab, u64 mask, u64 n, u64 salt, u64* __restrict__ sink) {
  const u64 base = (u64(blockIdx.x) * 256 + threadIdx.x) * U;
  u64 r = 0;
  u64 s[U], h[U];
#pragma unroll
  for (int u = 0; u < U; ++u) { h[u] = mix((base + u) ^ salt); s[u] = h[u] & mask; }
  if (MODE == 0) {
    u64 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + u < n ? tab[s[u]] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) r ^= v[u];
  } else if (MODE == 1) {
    unsigned v[U];
    const unsigned* t4 = reinterpret_cast<const unsigned*>(tab);
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + u < n ? t4[s[u]] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u) r ^= v[u];
  } else {
    u64 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = base + u < n ? tab[s[u]] : 0;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (base + u < n && v[u] == ~0ull) r ^= atomicCAS(&tab[s[u]], ~0ull, h[u]);
  }
  if (r == 0x12345) sink[0] = r;
}

template <int MODE, int U>
float run(u64* tab, u64 cap, u64 n, u64* sink, int rep) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  if (MODE == 2) hipMemset(tab, 0xff, cap * 8);
  hipEventRecord(a);
  const u64 threads = (n + U - 1) / U;
  hipLaunchKernelGGL((k<MODE, U>), dim3((threads + 255) / 256), dim3(256), 0, 0, tab, cap - 1, n, u64(rep), sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipEventDestroy(a);
  hipEventDestroy(b);
  return ms;
}

template <int MODE, int U>
void sweep(u64* tab, u64 cap, u64 n, u64* sink, const char* name) {
  float best = 1e9;
  for (int rep = 0; rep < 4; ++rep) {
    const float ms = run<MODE, U>(tab, cap, n, sink, rep);
    if (ms < best) best = ms;
  }
  printf("{\"cap_mb\": %llu, \"op\": \"%s\", \"per_thread\": %d, \"ms\": %.4f, \"Gops\": %.2f}\n", cap * 8 >> 20, name,
         U, best, n / (best * 1e-3) / 1e9);
  fflush(stdout);
}

int main() {
  const u64 n = 83333333;
  u64* tab;
  u64* sink;
  hipMalloc(&tab, (1ull << 27) * 8);
  hipMalloc(&sink, 8);
  hipMemset(tab, 0x11, (1ull << 27) * 8);
  for (u64 cap : {1ull << 22, 1ull << 24, 1ull << 27}) {   // 32 MB, 128 MB, 1 GB
    sweep<0, 1>(tab, cap, n, sink, "load8");
    sweep<0, 2>(tab, cap, n, sink, "load8");
    sweep<0, 4>(tab, cap, n, sink, "load8");
    sweep<0, 8>(tab, cap, n, sink, "load8");
    sweep<1, 1>(tab, cap, n, sink, "load4");
    sweep<1, 4>(tab, cap, n, sink, "load4");
    sweep<2, 1>(tab, cap, n / 2, sink, "load_then_cas");
    sweep<2, 2>(tab, cap, n / 2, sink, "load_then_cas");
    sweep<2, 4>(tab, cap, n / 2, sink, "load_then_cas");
    hipMemset(tab, 0x11, (1ull << 27) * 8);
  }
  return 0;
}
