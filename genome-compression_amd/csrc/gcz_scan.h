// Single-pass exclusive prefix sum of u32 values (decoupled look-back), the
// scan every bucketed pass of the build and of the ratio path uses (bucket-major
// count matrices, popcount prefixes of first-occurrence bitmaps, .dag byte
// offsets).  Replaces the rocPRIM scan.  Out = u32, or u64 when the total may
// pass 2^32 (a tile's own sum, kScanTile values, must fit 32 bits).
//
// One launch: a tile of kScanItems x 256 elements per workgroup, tiles taken
// in ticket order (so every predecessor is resident and the look-back cannot
// deadlock), one 64-bit status|value descriptor per tile, relaxed agent-scope
// atomics (the value travels in the descriptor, so no payload fence is needed).
// desc[ntiles] and *ticket must be zero before the launch.
#pragma once

#include <hip/hip_runtime.h>

#include "gcz_device.h"

namespace gcz_dev {

constexpr int kScanThreads = 1024;
constexpr int kScanItems = 16;
constexpr u64 kScanTile = u64(kScanThreads) * kScanItems;   // 16 Ki elements (a short look-back chain)

__host__ __device__ inline u64 scan_tiles(u64 n) { return (n + kScanTile - 1) / kScanTile; }

// Look-back of tile `tile` (taken in ticket order) whose own sum is agg, run by one whole
// wave: publishes the aggregate, adds up the predecessors' values until an inclusive
// prefix, publishes its own and returns the exclusive prefix (the same in every lane).
__device__ __forceinline__ u64 tile_lookback(u64* __restrict__ desc, u64 tile, u64 agg) {
  const int lane = threadIdx.x & 63;
  if (tile == 0) {
    if (lane == 0) __hip_atomic_store(&desc[0], kStP | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return 0;
  }
  if (lane == 0) __hip_atomic_store(&desc[tile], kStA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u64 prefix = 0;
  long long look = (long long)tile - 1;
  for (;;) {
    const long long idx = look - lane;
    const u64 d = idx >= 0 ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
    const u64 st = d >> 62;
    const u64 pm = __ballot(st == 2);
    const u64 zm = __ballot(st == 0 && idx >= 0);
    const int firstP = pm ? __ffsll((long long)pm) - 1 : 64;
    const u64 need = firstP >= 63 ? ~0ull : ((1ull << (firstP + 1)) - 1);
    if (zm & need) {
      __builtin_amdgcn_s_sleep(1);
      continue;
    }
    prefix += wave_sum(lane <= firstP && idx >= 0 ? (d & kValMask) : 0ull);
    if (firstP < 64 || look - 64 < 0) break;
    look -= 64;
  }
  if (lane == 0) __hip_atomic_store(&desc[tile], kStP | (prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return prefix;
}

// In: u32 operator()(u64 i) const for i < n.
template <class In, class Out = u32>
__global__ __launch_bounds__(kScanThreads) void k_scan_excl(In in, u64 n, Out* __restrict__ out,
                                                           u64* __restrict__ desc, u32* __restrict__ ticket,
                                                           u64* __restrict__ total) {
  __shared__ u32 s_tile;
  __shared__ u32 s_wave[kScanThreads / 64];
  __shared__ u64 s_prefix;
  __shared__ u32 s_tr[kScanTile + kScanTile / 16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  __syncthreads();
  const u64 tile = s_tile;
  const u64 t0 = tile * kScanTile;
  // coalesced loads (element e * 256 + tid), transposed through LDS so that each
  // thread scans kScanItems consecutive elements
  // LDS index of tile element j padded by j / 16: the blocked reads are conflict-free
#pragma unroll
  for (int e = 0; e < kScanItems; ++e) {
    const u32 j = u32(e) * kScanThreads + tid;
    const u64 i = t0 + j;
    s_tr[j + (j >> 4)] = i < n ? in(i) : 0u;
  }
  __syncthreads();
  u32 v[kScanItems];
  u32 sum = 0;
#pragma unroll
  for (int e = 0; e < kScanItems; ++e) {
    v[e] = s_tr[tid * (kScanItems + 1) + e];
    sum += v[e];
  }
  u32 incl = sum;   // inclusive scan over the wave
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  if (wave == 0) {
    u32 agg = 0;
    for (int w = 0; w < kScanThreads / 64; ++w) agg += s_wave[w];
    const u64 prefix = tile_lookback(desc, tile, agg);
    if (lane == 0) {
      s_prefix = prefix;
      if (total && (tile + 1) * kScanTile >= n) *total = prefix + agg;
    }
  }
  __syncthreads();
  u32 run = incl - sum;   // tile-local; the tile prefix is added at the store
  for (int w = 0; w < wave; ++w) run += s_wave[w];
  const Out tprefix = Out(s_prefix);
  __syncthreads();   // (every thread has read its items)
#pragma unroll
  for (int e = 0; e < kScanItems; ++e) {   // exclusive prefixes back through LDS, stored coalesced
    s_tr[tid * (kScanItems + 1) + e] = run;
    run += v[e];
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kScanItems; ++e) {
    const u32 j = u32(e) * kScanThreads + tid;
    const u64 i = t0 + j;
    if (i < n) out[i] = tprefix + Out(s_tr[j + (j >> 4)]);
  }
}

struct ScanU32 {   // array input, zero past its end (scan n + 1 elements: out[n] = total)
  const u32* a;
  u64 n;
  __device__ __forceinline__ u32 operator()(u64 i) const { return i < n ? a[i] : 0u; }
};

}  // namespace gcz_dev
