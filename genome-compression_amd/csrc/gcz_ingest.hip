// FASTA ingest on the device: the fasta_reader line
// contract (src/fasta_reader.cpp:40-68) over a file already in
// HBM, producing the concatenated bases the build consumes.
//
// At a line start the reader peeks once: '>' or '\n' skips that line, and the
// line after a skipped one is data without a second peek.  So in a run of
// consecutive marker lines (header or empty) the 1st, 3rd, ... are skipped and
// the 2nd, 4th, ... are data; every other line is data.  On the device:
//   1. newline positions (stream compaction),
//   2. per line: marker flag, the last non-marker line before it (max-scan),
//      hence skip / data and the data length; an exclusive sum gives each
//      data line's output offset,
//   3. reader buffers: the reference fills cap = B*L data bytes per buffer
//      (src/fasta_reader.cpp:22-31,47-64) and a line that crosses a buffer
//      boundary resumes with a fresh peek (:48-51): a '>' there drops the rest of
//      the line and makes the next line data.  One thread per boundary checks
//      the byte at it; the first such boundary becomes a per-line override
//      (cut length, forced-data next line) and steps 2-3 repeat from it.  Any
//      '>' inside a data line is otherwise an unknown symbol, so valid FASTA
//      never loops,
//   4. a byte-parallel copy: each block stages the line boundaries of its
//      2 KiB input window in LDS and every byte finds its line there.
// The compaction and the scans are one reduce-then-scan scheme (k_rts_*): tile
// reductions, one workgroup scanning the tile values, and a pass that rescans
// every tile from its carry and hands each element its prefix.
#include "gcz_ctx.h"

using namespace gcz_dev;
using namespace gcz_host;

struct gcz_ingest_state {
  DevBuf nlpos, nsel, lastnm, len, off, tmp, bases, cut, forced, ev;   // tmp: tile values + carries
};

void gcz_ingest_state_free(gcz_ctx* c) {
  gcz_ingest_state* s = c->ingest;
  if (!s) return;
  for (DevBuf* b : {&s->nlpos, &s->nsel, &s->lastnm, &s->len, &s->off, &s->tmp, &s->bases, &s->cut, &s->forced,
                    &s->ev})
    if (b->ptr) (void)hipFree(b->ptr);
  delete s;
  c->ingest = nullptr;
}

namespace {

constexpr int kWin = 2048;   // input bytes per copy block (LDS: 2 x 16 KiB line tables)

// ---- reduce-then-scan over u64 values (Op: Sum or Max) ----
constexpr int kRtsThreads = 1024;
constexpr int kRtsItems = 16;
constexpr u64 kRtsTile = u64(kRtsThreads) * kRtsItems;

struct OpSum {
  static __device__ __forceinline__ long long id() { return 0; }
  static __device__ __forceinline__ long long op(long long a, long long b) { return a + b; }
};
struct OpMax {
  static __device__ __forceinline__ long long id() { return -1; }
  static __device__ __forceinline__ long long op(long long a, long long b) { return a > b ? a : b; }
};

// exclusive block scan of one value per thread; *total = the block's reduction
template <class Op>
__device__ __forceinline__ long long block_excl(long long v, long long* s_w, long long* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  long long inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const long long y = __shfl_up(inc, o, 64);
    if (lane >= o) inc = Op::op(inc, y);
  }
  if (lane == 63) s_w[wave] = inc;
  __syncthreads();
  long long pre = Op::id();
  for (int w = 0; w < wave; ++w) pre = Op::op(pre, s_w[w]);
  long long tot = Op::id();
  for (int w = 0; w < kRtsThreads / 64; ++w) tot = Op::op(tot, s_w[w]);
  __syncthreads();
  *total = tot;
  long long ex = __shfl_up(inc, 1, 64);
  if (lane == 0) ex = Op::id();
  return Op::op(pre, ex);
}

// thread t of a tile holds kRtsItems consecutive elements
template <class In, class Op>
__global__ __launch_bounds__(kRtsThreads) void k_rts_reduce(In in, u64 n, long long* __restrict__ part) {
  __shared__ long long s_w[kRtsThreads / 64];
  const u64 i0 = u64(blockIdx.x) * kRtsTile + u64(threadIdx.x) * kRtsItems;
  long long v = Op::id();
  for (int e = 0; e < kRtsItems; ++e)
    if (i0 + e < n) v = Op::op(v, in(i0 + e));
  long long tot;
  (void)block_excl<Op>(v, s_w, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// one workgroup: part[t] -> exclusive carry[t], carry[nt] = the total
template <class Op>
__global__ __launch_bounds__(kRtsThreads) void k_rts_carry(const long long* __restrict__ part, u64 nt,
                                                           long long* __restrict__ carry) {
  __shared__ long long s_w[kRtsThreads / 64];
  long long run = Op::id();
  for (u64 b = 0; b < nt; b += kRtsThreads) {
    const u64 t = b + threadIdx.x;
    long long tot;
    const long long ex = block_excl<Op>(t < nt ? part[t] : Op::id(), s_w, &tot);
    if (t < nt) carry[t] = Op::op(run, ex);
    run = Op::op(run, tot);
  }
  if (threadIdx.x == 0) carry[nt] = run;
}

// sink(i, exclusive prefix, value) for every element
template <class In, class Op, class Sink>
__global__ __launch_bounds__(kRtsThreads) void k_rts_apply(In in, u64 n, const long long* __restrict__ carry,
                                                           Sink sink) {
  __shared__ long long s_w[kRtsThreads / 64];
  const u64 i0 = u64(blockIdx.x) * kRtsTile + u64(threadIdx.x) * kRtsItems;
  long long v[kRtsItems];
  long long agg = Op::id();
  for (int e = 0; e < kRtsItems; ++e) {
    v[e] = i0 + e < n ? in(i0 + e) : Op::id();
    agg = Op::op(agg, v[e]);
  }
  long long tot;
  long long run = Op::op(carry[blockIdx.x], block_excl<Op>(agg, s_w, &tot));
  for (int e = 0; e < kRtsItems; ++e) {
    if (i0 + e >= n) break;
    sink(i0 + e, run, v[e]);
    run = Op::op(run, v[e]);
  }
}

struct NewlineFlag {
  const unsigned char* f;
  __device__ __forceinline__ long long operator()(u64 i) const { return f[i] == '\n' ? 1 : 0; }
};
struct NewlineSink {   // compaction: newline number -> byte position
  u64* nl;
  __device__ __forceinline__ void operator()(u64 i, long long pre, long long v) const {
    if (v) nl[pre] = i;
  }
};
struct U64In {
  const u64* a;
  __device__ __forceinline__ long long operator()(u64 i) const { return (long long)a[i]; }
};
struct ExclSink {
  u64* out;
  __device__ __forceinline__ void operator()(u64 i, long long pre, long long) const { out[i] = u64(pre); }
};
struct InclMaxSink {
  long long* out;
  __device__ __forceinline__ void operator()(u64 i, long long pre, long long v) const { out[i] = pre > v ? pre : v; }
};

// Line i spans [st, en): st = 0 or one past newline i-1, en = newline i or n.
// Overrides from reader-buffer boundaries (null until the first one): forced[i]
// = line i is read as data without a peek; cut[i] = data bytes kept of line i.
struct Lines {
  const unsigned char* f;
  const u64* nl;   // newline positions
  u64 nnl, n, nlines;
  const unsigned char* forced;
  const u64* cut;
  __device__ __forceinline__ u64 st(u64 i) const { return i == 0 ? 0 : nl[i - 1] + 1; }
  __device__ __forceinline__ u64 en(u64 i) const { return i < nnl ? nl[i] : n; }
  __device__ __forceinline__ bool marker(u64 i) const {
    if (forced && forced[i]) return false;
    const unsigned char c = f[st(i)];
    return c == '>' || c == '\n';
  }
};

// value for the max-scan: own index for a data-by-content line, -1 for a marker line
struct NonMarkerIndex {
  Lines ln;
  __device__ __forceinline__ long long operator()(u64 i) const { return ln.marker(i) ? -1ll : (long long)i; }
};

__device__ __forceinline__ bool skipped(const Lines& ln, const long long* lastnm, u64 i) {
  if (!ln.marker(i)) return false;
  const long long run0 = lastnm[i] + 1;            // first line of this run of marker lines
  return ((long long)i - run0) % 2 == 0;
}

__global__ __launch_bounds__(kBlock) void k_line_len(Lines ln, const long long* __restrict__ lastnm,
                                                     u64* __restrict__ len) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= ln.nlines) return;
  u64 l = skipped(ln, lastnm, i) ? 0 : ln.en(i) - ln.st(i);
  if (ln.cut && ln.cut[i] < l) l = ln.cut[i];
  len[i] = l;
}

// last line whose output offset is < b (off is non-decreasing)
__device__ __forceinline__ u64 line_before(const u64* off, u64 nlines, u64 b) {
  u64 lo = 0, hi = nlines;   // first line with off >= b
  while (lo < hi) {
    const u64 mid = (lo + hi) / 2;
    if (off[mid] < b) lo = mid + 1;
    else hi = mid;
  }
  return lo - 1;   // off[0] = 0 < b
}

// Boundaries k*cap, k0 <= k <= k1 (all strictly inside the data): the smallest k
// whose boundary splits a line at a '>' (src/fasta_reader.cpp:48-51).
__global__ __launch_bounds__(kBlock) void k_boundary_check(Lines ln, const u64* __restrict__ off,
                                                           const u64* __restrict__ len, u64 cap, u64 k0, u64 k1,
                                                           u64* __restrict__ ev) {
  const u64 k = k0 + u64(blockIdx.x) * kBlock + threadIdx.x;
  if (k > k1) return;
  const u64 b = k * cap;
  const u64 i = line_before(off, ln.nlines, b);
  if (off[i] + len[i] > b && ln.f[ln.st(i) + (b - off[i])] == '>') atomicMin(reinterpret_cast<unsigned long long*>(ev), k);
}

// The first event found by k_boundary_check becomes line overrides.
__global__ void k_boundary_apply(Lines ln, const u64* __restrict__ off, u64 cap, const u64* __restrict__ ev,
                                 u64* __restrict__ cut, unsigned char* __restrict__ forced) {
  const u64 k = *ev;
  if (k == ~0ull) return;
  const u64 b = k * cap;
  const u64 i = line_before(off, ln.nlines, b);
  cut[i] = b - off[i];
  if (i + 1 < ln.nlines) forced[i + 1] = 1;
}

// first line whose end is >= pos (the line containing pos, or starting at it)
__device__ __forceinline__ u64 line_at(const Lines& ln, u64 pos) {
  u64 lo = 0, hi = ln.nnl;   // newlines nl[0..nnl): line i ends at nl[i]
  while (lo < hi) {
    const u64 mid = (lo + hi) / 2;
    if (ln.nl[mid] < pos) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kBlock) void k_copy_lines(Lines ln, const u64* __restrict__ len,
                                                       const u64* __restrict__ off, unsigned char* __restrict__ out) {
  __shared__ u64 s_st[kWin + 1];
  __shared__ u64 s_off[kWin + 1];
  __shared__ u64 s_lim[kWin + 1];   // end of the kept bytes of the line (st when skipped)
  __shared__ u64 s_l0;
  __shared__ u32 s_cnt;
  const u64 b0 = u64(blockIdx.x) * kWin;
  const u64 b1 = b0 + kWin < ln.n ? b0 + kWin : ln.n;
  if (threadIdx.x == 0) {
    const u64 l0 = line_at(ln, b0);
    const u64 l1 = line_at(ln, b1 == 0 ? 0 : b1 - 1);
    s_l0 = l0;
    s_cnt = u32(l1 - l0 + 1);
  }
  __syncthreads();
  const u64 l0 = s_l0;
  const u32 cnt = s_cnt;
  for (u32 k = threadIdx.x; k < cnt; k += kBlock) {
    const u64 i = l0 + k;
    s_st[k] = ln.st(i);
    s_off[k] = off[i];
    s_lim[k] = s_st[k] + len[i];
  }
  __syncthreads();
  for (u64 p = b0 + threadIdx.x; p < b1; p += kBlock) {
    const unsigned char c = ln.f[p];
    if (c == '\n') continue;
    u32 lo = 0, hi = cnt - 1;   // last local line with st <= p
    while (lo < hi) {
      const u32 mid = (lo + hi + 1) / 2;
      if (s_st[mid] <= p) lo = mid;
      else hi = mid - 1;
    }
    if (p < s_lim[lo]) out[s_off[lo] + (p - s_st[lo])] = c;
  }
}

dim3 grid_of(u64 n) { return dim3(unsigned(std::max<u64>(1, (n + kBlock - 1) / kBlock))); }

}  // namespace

#define I_HIP(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return c->fail(GCZ_ERR_DEVICE, #x, hipGetErrorString(e_));     \
  } while (0)

// Bases of a FASTA file in device memory -> ctx-owned device buffer; returns the count.
// Reader buffers of buffer_strands strands (0 = the reference default 1 << 22).
int gcz_fasta_extract_on_device(gcz_ctx* c, const unsigned char* d_file, u64 n, int Lleaf, u64 buffer_strands,
                                const unsigned char** d_bases, u64* nbases) {
  if (!c->ingest) c->ingest = new gcz_ingest_state();
  gcz_ingest_state& s = *c->ingest;
  *nbases = 0;
  *d_bases = nullptr;
  if (Lleaf < 1 || Lleaf > 16) return GCZ_ERR_ARG;
  int rc;
  if ((rc = c->ensure(s.nsel, 16)) || (rc = c->ensure(s.bases, n + 16)) || (rc = c->ensure(s.ev, 16))) return rc;
  *d_bases = s.bases.as<unsigned char>();
  if (n == 0) return GCZ_OK;
  const u64 cap = gcz::reader_buffer_bytes(n, Lleaf, buffer_strands);
  // reduce-then-scan of m elements: tile values and carries in s.tmp
  auto rts_tiles = [](u64 m) { return std::max<u64>(1, (m + kRtsTile - 1) / kRtsTile); };
  const u64 ntmax = rts_tiles(n + 1);   // bytes, or lines (<= n + 1)
  if ((rc = c->ensure(s.tmp, (2 * ntmax + 2) * 8 + 16))) return rc;
  long long* part = s.tmp.as<long long>();
  long long* carry = part + ntmax;
  // 1. newline positions (counted first, so the position array is exact)
  {
    const u64 nt = rts_tiles(n);
    hipLaunchKernelGGL((k_rts_reduce<NewlineFlag, OpSum>), dim3(unsigned(nt)), dim3(kRtsThreads), 0, c->stream,
                       NewlineFlag{d_file}, n, part);
    hipLaunchKernelGGL((k_rts_carry<OpSum>), dim3(1), dim3(kRtsThreads), 0, c->stream, part, nt, carry);
    I_HIP(hipGetLastError());
  }
  u64 nnl = 0;
  unsigned char last = 0;
  I_HIP(hipMemcpyAsync(&nnl, carry + rts_tiles(n), 8, hipMemcpyDeviceToHost, c->stream));
  I_HIP(hipMemcpyAsync(&last, d_file + n - 1, 1, hipMemcpyDeviceToHost, c->stream));
  I_HIP(hipStreamSynchronize(c->stream));
  if ((rc = c->ensure(s.nlpos, nnl * 8 + 16))) return rc;
  hipLaunchKernelGGL((k_rts_apply<NewlineFlag, OpSum, NewlineSink>), dim3(unsigned(rts_tiles(n))),
                     dim3(kRtsThreads), 0, c->stream, NewlineFlag{d_file}, n, carry, NewlineSink{s.nlpos.as<u64>()});
  I_HIP(hipGetLastError());
  Lines ln{d_file, s.nlpos.as<u64>(), nnl, n, nnl + (last != '\n' ? 1 : 0), nullptr, nullptr};
  const u64 L = ln.nlines;
  if ((rc = c->ensure(s.lastnm, L * 8 + 16)) || (rc = c->ensure(s.len, L * 8 + 16)) ||
      (rc = c->ensure(s.off, L * 8 + 16)))
    return rc;
  const u64 ntl = rts_tiles(L);
  u64 total = 0;
  for (u64 k0 = 1;;) {
    // 2. skip / data per line (the last non-marker line: an inclusive max-scan), output offsets
    hipLaunchKernelGGL((k_rts_reduce<NonMarkerIndex, OpMax>), dim3(unsigned(ntl)), dim3(kRtsThreads), 0, c->stream,
                       NonMarkerIndex{ln}, L, part);
    hipLaunchKernelGGL((k_rts_carry<OpMax>), dim3(1), dim3(kRtsThreads), 0, c->stream, part, ntl, carry);
    hipLaunchKernelGGL((k_rts_apply<NonMarkerIndex, OpMax, InclMaxSink>), dim3(unsigned(ntl)), dim3(kRtsThreads), 0,
                       c->stream, NonMarkerIndex{ln}, L, carry, InclMaxSink{s.lastnm.as<long long>()});
    I_HIP(hipGetLastError());
    hipLaunchKernelGGL(k_line_len, grid_of(L), dim3(kBlock), 0, c->stream, ln, s.lastnm.as<long long>(),
                       s.len.as<u64>());
    hipLaunchKernelGGL((k_rts_reduce<U64In, OpSum>), dim3(unsigned(ntl)), dim3(kRtsThreads), 0, c->stream,
                       U64In{s.len.as<u64>()}, L, part);
    hipLaunchKernelGGL((k_rts_carry<OpSum>), dim3(1), dim3(kRtsThreads), 0, c->stream, part, ntl, carry);
    hipLaunchKernelGGL((k_rts_apply<U64In, OpSum, ExclSink>), dim3(unsigned(ntl)), dim3(kRtsThreads), 0, c->stream,
                       U64In{s.len.as<u64>()}, L, carry, ExclSink{s.off.as<u64>()});
    I_HIP(hipGetLastError());
    u64 tail[2] = {0, 0};
    I_HIP(hipMemcpyAsync(&tail[0], s.off.as<u64>() + L - 1, 8, hipMemcpyDeviceToHost, c->stream));
    I_HIP(hipMemcpyAsync(&tail[1], s.len.as<u64>() + L - 1, 8, hipMemcpyDeviceToHost, c->stream));
    I_HIP(hipStreamSynchronize(c->stream));
    total = tail[0] + tail[1];
    // 3. reader-buffer boundaries strictly inside the data, from k0 on
    const u64 k1 = total ? (total - 1) / cap : 0;
    if (k0 > k1) break;
    I_HIP(hipMemsetAsync(s.ev.ptr, 0xff, 8, c->stream));
    hipLaunchKernelGGL(k_boundary_check, grid_of(k1 - k0 + 1), dim3(kBlock), 0, c->stream, ln, s.off.as<u64>(),
                       s.len.as<u64>(), cap, k0, k1, s.ev.as<u64>());
    u64 ev = ~0ull;
    I_HIP(hipMemcpyAsync(&ev, s.ev.ptr, 8, hipMemcpyDeviceToHost, c->stream));
    I_HIP(hipStreamSynchronize(c->stream));
    if (ev == ~0ull) break;
    if (!ln.cut) {   // first event: the override arrays
      if ((rc = c->ensure(s.cut, L * 8 + 16)) || (rc = c->ensure(s.forced, L + 16))) return rc;
      I_HIP(hipMemsetAsync(s.cut.ptr, 0xff, L * 8, c->stream));
      I_HIP(hipMemsetAsync(s.forced.ptr, 0, L, c->stream));
      ln.cut = s.cut.as<u64>();
      ln.forced = s.forced.as<unsigned char>();
    }
    hipLaunchKernelGGL(k_boundary_apply, dim3(1), dim3(1), 0, c->stream, ln, s.off.as<u64>(), cap,
                       s.ev.as<u64>(), s.cut.as<u64>(), s.forced.as<unsigned char>());
    I_HIP(hipGetLastError());
    k0 = ev + 1;
  }
  // one line without a break, read whole (no header, no reader-buffer override): the
  // file itself is the genome, no copy
  if (nnl == 0 && !ln.cut && total == n) {
    *d_bases = d_file;
    *nbases = total;
    return GCZ_OK;
  }
  // 4. copy
  hipLaunchKernelGGL(k_copy_lines, dim3(unsigned((n + kWin - 1) / kWin)), dim3(kBlock), 0, c->stream, ln,
                     s.len.as<u64>(), s.off.as<u64>(), s.bases.as<unsigned char>());
  I_HIP(hipGetLastError());
  I_HIP(hipStreamSynchronize(c->stream));
  *nbases = total;
  return GCZ_OK;
}

extern "C" {

int gcz_build_device_fasta(gcz_ctx* c, const void* d_file, uint64_t n, int L) {
  if (!c || (!d_file && n)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  const unsigned char* b = nullptr;
  u64 nb = 0;
  if (int rc = gcz_fasta_extract_on_device(c, static_cast<const unsigned char*>(d_file), n, L, 0, &b, &nb))
    return rc;
  return c->build(b, nullptr, nb, 0, L);
}

int gcz_build_device_fasta_buffered(gcz_ctx* c, const void* d_file, uint64_t n, int L, uint64_t buffer_strands,
                                    uint64_t first_strand) {
  if (!c || (!d_file && n) || L < 1 || L > 16) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  // fasta_reader{path, buffer_strands}: buffers of B strands (src/fasta_reader.cpp:21-31)
  const u64 B = gcz::reader_buffer_bytes(n, L, buffer_strands) / u64(L);
  const unsigned char* b = nullptr;
  u64 nb = 0;
  if (int rc = gcz_fasta_extract_on_device(c, static_cast<const unsigned char*>(d_file), n, L, buffer_strands, &b, &nb))
    return rc;
  // buffers already handed out by read_into are not part of the tree (src/shared_tree.cpp:722);
  // none left is an empty root list there (reduce_roots' roots.front(): undefined), an error here
  if (first_strand > 0 && first_strand >= nb / u64(L))
    return c->fail(GCZ_ERR_ARG, "gcz_build_device_fasta_buffered", "every reader buffer was already read");
  if (first_strand % B) return c->fail(GCZ_ERR_ARG, "gcz_build_device_fasta_buffered", "first_strand is not a buffer start");
  const u64 skip = std::min<u64>(nb / u64(L), first_strand) * u64(L);
  b += skip;
  nb -= skip;
  if (skip & 3) {   // the leaf kernels stage with 4-B loads
    if (int rc = c->ensure(c->seg_in, nb + 16)) return rc;
    I_HIP(hipMemcpyAsync(c->seg_in.ptr, b, nb, hipMemcpyDeviceToDevice, c->stream));
    b = c->seg_in.as<unsigned char>();
  }
  c->segment_strands = B;
  return c->build(b, nullptr, nb, 0, L);
}

int gcz_build_host_fasta_buffered(gcz_ctx* c, const void* fasta, uint64_t nbytes, int L, uint64_t buffer_strands,
                                  uint64_t first_strand) {
  if (!c || (!fasta && nbytes)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (int rc = c->ensure(c->input, nbytes + 16)) return rc;
  if (nbytes && c->upload(c->input.ptr, fasta, nbytes))
    return c->fail(GCZ_ERR_DEVICE, "gcz_build_host_fasta_buffered", "H2D copy failed");
  return gcz_build_device_fasta_buffered(c, c->input.ptr, nbytes, L, buffer_strands, first_strand);
}

int gcz_fasta_extract_device(gcz_ctx* c, const void* d_file, uint64_t n, int L, uint64_t buffer_strands, void* d_out,
                             uint64_t cap, uint64_t* nbases) {
  if (!c || (!d_file && n) || !nbases) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  const unsigned char* b = nullptr;
  u64 nb = 0;
  if (int rc = gcz_fasta_extract_on_device(c, static_cast<const unsigned char*>(d_file), n, L, buffer_strands, &b,
                                           &nb))
    return rc;
  *nbases = nb;
  if (!d_out) return GCZ_OK;
  if (cap < nb) return GCZ_ERR_ARG;
  I_HIP(hipMemcpyAsync(d_out, b, nb, hipMemcpyDeviceToDevice, c->stream));
  I_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

}  // extern "C"
