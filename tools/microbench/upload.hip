// Host -> device upload of a 1 GB memory-mapped file: the runtime's pageable copy,
// pinned staging rings (W worker threads x 2 slots, own streams), and registering
// the mapping itself.  GB/s per variant (json lines).
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "/tmp/up.bin";
  const size_t n = size_t(1) << 30;
  {
    int fd = open(path, O_CREAT | O_TRUNC | O_WRONLY, 0644);
    std::vector<char> buf(size_t(64) << 20, 'A');
    for (size_t o = 0; o < n; o += buf.size()) (void)!write(fd, buf.data(), buf.size());
    close(fd);
  }
  int fd = open(path, O_RDONLY);
  const char* m = static_cast<const char*>(mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0));
  void* d = nullptr;
  (void)hipMalloc(&d, n);
  hipStream_t s;
  (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  for (int rep = 0; rep < 2; ++rep) {
    double t0 = now();
    (void)hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    std::printf("{\"variant\": \"pageable\", \"GBs\": %.1f}\n", n / (now() - t0) / 1e9);
  }
  for (unsigned flags : {0u, unsigned(hipHostMallocNumaUser)}) {
    for (int W : {1, 2, 4, 8}) {
      for (size_t slot : {size_t(4) << 20, size_t(16) << 20}) {
        std::vector<void*> sl(2 * W);
        std::vector<hipEvent_t> ev(2 * W);
        std::vector<hipStream_t> st(W);
        double ta = now();
        for (int i = 0; i < 2 * W; ++i) {
          (void)hipHostMalloc(&sl[i], slot, flags);
          (void)hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
        }
        const double talloc = now() - ta;
        for (int w = 0; w < W; ++w) (void)hipStreamCreateWithFlags(&st[w], hipStreamNonBlocking);
        double best = 0;
        for (int rep = 0; rep < 2; ++rep) {
          const size_t pieces = n / slot;
          double t0 = now();
          std::vector<std::thread> th;
          for (int w = 0; w < W; ++w)
            th.emplace_back([&, w] {
              (void)hipSetDevice(0);
              int k = 0;
              for (size_t i = w; i < pieces; i += W, ++k) {
                const int q = 2 * w + (k & 1);
                if (k >= 2) (void)hipEventSynchronize(ev[q]);
                std::memcpy(sl[q], m + i * slot, slot);
                (void)hipMemcpyAsync(static_cast<char*>(d) + i * slot, sl[q], slot, hipMemcpyHostToDevice, st[w]);
                (void)hipEventRecord(ev[q], st[w]);
              }
            });
          for (auto& x : th) x.join();
          for (int w = 0; w < W; ++w) (void)hipStreamSynchronize(st[w]);
          const double g = n / (now() - t0) / 1e9;
          best = g > best ? g : best;
        }
        std::printf("{\"variant\": \"pinned_ring\", \"flags\": %u, \"workers\": %d, \"slot_MB\": %zu, \"GBs\": %.1f, "
                    "\"alloc_ms\": %.1f}\n", flags, W, slot >> 20, best, talloc * 1e3);
        for (int i = 0; i < 2 * W; ++i) {
          (void)hipHostFree(sl[i]);
          (void)hipEventDestroy(ev[i]);
        }
        for (int w = 0; w < W; ++w) (void)hipStreamDestroy(st[w]);
      }
    }
  }
  {   // pin the mapping itself
    double t0 = now();
    hipError_t e = hipHostRegister(const_cast<char*>(m), n, hipHostRegisterReadOnly);
    const double treg = now() - t0;
    if (e == hipSuccess) {
      double t1 = now();
      (void)hipMemcpyAsync(d, m, n, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      std::printf("{\"variant\": \"register_mapping\", \"GBs\": %.1f, \"register_ms\": %.1f}\n", n / (now() - t1) / 1e9,
                  treg * 1e3);
      (void)hipHostUnregister(const_cast<char*>(m));
    } else {
      std::printf("{\"variant\": \"register_mapping\", \"error\": \"%s\"}\n", hipGetErrorString(e));
    }
  }
  {   // a plain pinned buffer, DMA only (the link's ceiling)
    void* p = nullptr;
    (void)hipHostMalloc(&p, n, 0);
    std::memcpy(p, m, n);
    double t0 = now();
    (void)hipMemcpyAsync(d, p, n, hipMemcpyHostToDevice, s);
    (void)hipStreamSynchronize(s);
    std::printf("{\"variant\": \"pinned_dma_only\", \"GBs\": %.1f}\n", n / (now() - t0) / 1e9);
    t0 = now();
    std::memcpy(p, m, n);
    std::printf("{\"variant\": \"host_memcpy_1thread\", \"GBs\": %.1f}\n", n / (now() - t0) / 1e9);
    (void)hipHostFree(p);
  }
  {   // destination first touch: a fresh allocation per copy, and a fresh one touched by a memset first
    for (int rep = 0; rep < 2; ++rep) {
      void* f = nullptr;
      (void)hipMalloc(&f, n);
      double t0 = now();
      (void)hipMemcpyAsync(f, m, n, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      std::printf("{\"variant\": \"pageable_fresh_dst\", \"GBs\": %.1f}\n", n / (now() - t0) / 1e9);
      (void)hipFree(f);
      (void)hipMalloc(&f, n);
      t0 = now();
      (void)hipMemsetAsync(f, 0, n, s);
      (void)hipStreamSynchronize(s);
      const double tm = now() - t0;
      t0 = now();
      (void)hipMemcpyAsync(f, m, n, hipMemcpyHostToDevice, s);
      (void)hipStreamSynchronize(s);
      std::printf("{\"variant\": \"pageable_touched_dst\", \"GBs\": %.1f, \"touch_ms\": %.1f}\n",
                  n / (now() - t0) / 1e9, tm * 1e3);
      (void)hipFree(f);
    }
  }
  unlink(path);
  return 0;
}
