// Where the drop-in's first-tree latency goes on a fresh process: HIP runtime init, the
// libgcz context, and the first / second build + sort + .dag of a small genome.
// usage: init_probe <fasta> [L]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <vector>

#include "gcz.h"

static double ms_since(std::chrono::steady_clock::time_point& t) {
  const auto n = std::chrono::steady_clock::now();
  const double d = std::chrono::duration<double, std::milli>(n - t).count();
  t = n;
  return d;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const int L = argc > 2 ? std::atoi(argv[2]) : 12;
  std::ifstream f(argv[1], std::ios::binary);
  std::vector<char> data((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
  auto t = std::chrono::steady_clock::now();
  int n = 0;
  (void)hipGetDeviceCount(&n);
  std::printf("hipGetDeviceCount %.2f ms\n", ms_since(t));
  (void)hipSetDevice(0);
  std::printf("hipSetDevice %.2f ms\n", ms_since(t));
  (void)hipFree(nullptr);
  std::printf("hipFree(0) %.2f ms\n", ms_since(t));
  gcz_ctx* c = nullptr;
  if (gcz_ctx_create(0, &c) != GCZ_OK) return 1;
  std::printf("gcz_ctx_create %.2f ms\n", ms_since(t));
  for (int rep = 0; rep < 3; ++rep) {
    if (gcz_build_host_fasta(c, data.data(), data.size(), L) != GCZ_OK) return 1;
    std::printf("build %d %.2f ms\n", rep, ms_since(t));
    if (gcz_sort_device(c) != GCZ_OK) return 1;
    std::printf("sort %d %.2f ms\n", rep, ms_since(t));
    uint64_t nb = 0;
    if (!gcz_device_dag(c, &nb)) return 1;
    std::printf("dag %d %.2f ms (%llu bytes)\n", rep, ms_since(t), (unsigned long long)nb);
  }
  gcz_ctx_destroy(c);
  return 0;
}
