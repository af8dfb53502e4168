// Microbenchmark: load-then-CAS of n random keys into a 2^27-slot (1 GB) table, in one
// pass or in 2^r passes over table regions (each pass re-reads the key array and
// inserts only the keys homed in its region), block-per-chunk or grid-stride.
#include <hip/hip_runtime.h>
#include <cstdio>

using u64 = unsigned long long;
using u32 = unsigned int;

__device__ __forceinline__ u64 mix(u64 x) {
  x ^= x >> 31; x *= 0x7fb5d329728ea185ull; x ^= x >> 27; x *= 0x81dadef4bc2dd44dull; x ^= x >> 33; return x;
}

__global__ void k_keys(u64* keys, u64 n, u64 salt) {
  const u64 i = u64(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < n) keys[i] = mix(i ^ salt);
}

// ITEMS sub-blocks per block; pass = blockIdx / bpp
template <int ITEMS>
__global__ __launch_bounds__(256) void k_ins(const u64* __restrict__ keys, u64 n, u64* __restrict__ tab, u32 cbits,
                                             u32 rbits, u32 bpp, u32* __restrict__ sink) {
  const u32 pass = blockIdx.x / bpp;
  const u64 blk = blockIdx.x - u64(pass) * bpp;
  const u64 mask = (1ull << cbits) - 1;
  u32 acc = 0;
#pragma unroll
  for (int it = 0; it < ITEMS; ++it) {
    const u64 i = (blk * ITEMS + it) * 256 + threadIdx.x;
    if (i >= n) break;
    const u64 key = keys[i];
    u64 s = mix(key) & mask;
    if (rbits && (s >> (cbits - rbits)) != pass) continue;
    for (;;) {
      u64 cur = tab[s];
      if (cur == ~0ull) cur = atomicCAS(&tab[s], ~0ull, key);
      if (cur == ~0ull || cur == key) break;
      s = (s + 1) & mask;
    }
    acc += u32(s);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <int ITEMS>
float run(const u64* keys, u64 n, u64* tab, u32 cbits, u32 rbits, u32* sink) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e9;
  const u32 bpp = u32((n + 256 * ITEMS - 1) / (256 * ITEMS));
  for (int rep = 0; rep < 4; ++rep) {
    hipMemset(tab, 0xff, (1ull << cbits) * 8);
    hipEventRecord(a);
    hipLaunchKernelGGL(k_ins<ITEMS>, dim3(bpp << rbits), dim3(256), 0, 0, keys, n, tab, cbits, rbits, bpp, sink);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const u64 n = 41666667;
  u64 *keys, *tab;
  u32* sink;
  hipMalloc(&keys, n * 8);
  hipMalloc(&tab, (1ull << 27) * 8);
  hipMalloc(&sink, 4);
  hipLaunchKernelGGL(k_keys, dim3((n + 255) / 256), dim3(256), 0, 0, keys, n, 7ull);
  for (u32 cbits : {26u, 27u})
    for (u32 rbits = 0; rbits <= 4; ++rbits) {
      const float m1 = run<1>(keys, n, tab, cbits, rbits, sink);
      const float m8 = run<8>(keys, n, tab, cbits, rbits, sink);
      printf("{\"table_mb\": %llu, \"passes\": %u, \"ms_items1\": %.4f, \"ms_items8\": %.4f}\n",
             ((1ull << cbits) * 8) >> 20, 1u << rbits, m1, m8);
    }
  return 0;
}
