// k_tail alone on a synthetic level of n0 words (ids with repeats): per-level wall-clock
// stamps (GCZ_TAIL_PROBE) and the launch time from events.  Build:
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I genome-compression_amd/csrc -I include \
//         tools/microbench/tail.hip -o tools/microbench/tail
#define GCZ_TAIL_PROBE 1
#include "gcz_device.h"

#include <cstdio>
#include <random>
#include <vector>

using namespace gcz_dev;

int main(int argc, char** argv) {
  const u32 n0 = argc > 1 ? u32(std::atoi(argv[1])) : 6662u;
  const u32 idmax = argc > 2 ? u32(std::atoi(argv[2])) : n0 / 2;   // repeats: ids < idmax
  std::mt19937 rng(7);
  std::vector<u32> w(n0);
  for (auto& x : w) x = (rng() % idmax) | ((rng() & 3u) << 29);
  int D = 0;
  for (u32 n = n0; ; ) { ++D; if (n <= 1) break; n = (n + 1) / 2; }
  D -= 1;   // levels from n0 words down to 1
  u32* d_in;
  uint2* d_nodes;
  Header* d_hdr;
  (void)hipMalloc(&d_in, n0 * 4);
  (void)hipMalloc(&d_nodes, size_t(2) * n0 * 8);
  (void)hipMalloc(&d_hdr, sizeof(Header));
  (void)hipMemcpy(d_in, w.data(), n0 * 4, hipMemcpyHostToDevice);
  (void)hipMemset(d_hdr, 0, sizeof(Header));
  TailOut to{};
  u64 o = 0;
  for (int k = 0, n = int(n0); k < D; ++k) { to.layer_off[k] = o; o += (n + 1) / 2; n = (n + 1) / 2; }
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(k_tail), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(kTailLds));
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  float best = 1e9f;
  for (int r = 0; r < 50; ++r) {
    (void)hipEventRecord(a, nullptr);
    hipLaunchKernelGGL(k_tail, dim3(1), dim3(kTailThreads), kTailLds, nullptr, d_in, u64(n0), nullptr, 0, D, d_nodes,
                       to, d_hdr, nullptr, TailSettle{});
    (void)hipEventRecord(b, nullptr);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  unsigned long long st[64];
  (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(gcz_tail_probe), sizeof(st));
  std::printf("{\"n0\": %u, \"levels\": %d, \"event_us\": %.2f, \"stamps_us\": [", n0, D, best * 1e3);
  for (int i = 1; i <= D; ++i) std::printf("%s%.2f", i > 1 ? ", " : "", double(st[i] - st[0]) / 100.0);
  std::printf("], \"end_us\": %.2f}\n", double(st[63] - st[0]) / 100.0);
  return 0;
}
