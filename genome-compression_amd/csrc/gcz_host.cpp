// Host-side operations of libgcz: the shared_tree container operations that sit
// after the build (frequency sort, bytes(), serialize(), width()), the FASTA
// line contract, and the synthetic genome generator.  No HIP calls here, so
// these entry points work on machines without a GPU.
#include <algorithm>
#include <cstring>
#include <mutex>
#include <new>
#include <numeric>
#include <thread>
#include <vector>

#include <sys/mman.h>

#include "gcz_internal.h"
#include "synth.h"

using gcz::kIndexMask;
using gcz::kNullIndex;
using gcz::ul;

namespace {

// Stable permutation of `n` children by descending reference count, ties by old
// index (std::stable_sort in sort_leaves/sort_nodes, src/shared_tree.cpp:409-436).
// Returns newpos[old] (invert_indices, :360-365).  Counting sort when the count
// range is small, which it is for every real tree.
std::vector<uint32_t> frequency_order(const uint32_t* parent, size_t nwords, size_t n) {
  std::vector<uint32_t> cnt(n, 0);
  for (size_t i = 0; i < nwords; ++i)                        // histogram, :316-326
    if (ul(parent[i]) != kNullIndex) ++cnt[parent[i] & kIndexMask];
  uint32_t maxc = 0;
  for (uint32_t c : cnt) maxc = std::max(maxc, c);
  std::vector<uint32_t> newpos(n);
  if (maxc <= (1u << 22)) {
    std::vector<uint64_t> start(size_t(maxc) + 2, 0);
    for (uint32_t c : cnt) ++start[maxc - c + 1];            // bucket 0 = largest count
    for (size_t b = 1; b < start.size(); ++b) start[b] += start[b - 1];
    for (size_t i = 0; i < n; ++i) newpos[i] = uint32_t(start[maxc - cnt[i]]++);
  } else {
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return cnt[a] > cnt[b]; });
    for (size_t i = 0; i < n; ++i) newpos[idx[i]] = uint32_t(i);
  }
  return newpos;
}

// rewire_nodes (src/shared_tree.cpp:383-403): new index, m/t/v bits kept, null untouched.
void rewire(uint32_t* parent, size_t nwords, const std::vector<uint32_t>& newpos) {
  for (size_t i = 0; i < nwords; ++i)
    if (ul(parent[i]) != kNullIndex) parent[i] = (parent[i] & gcz::kFlagMask) | newpos[parent[i] & kIndexMask];
}

// Pointer compression (src/shared_tree.cpp:25-67,122-142).
int segment(uint32_t idx) {
  if (idx == kNullIndex) return 3;
  if (idx < 16u) return 0;
  if (idx < 16u + 4096u) return 1;
  if (idx < 16u + 4096u + 1048576u) return 2;
  return 3;
}
constexpr uint32_t kSegBits[4] = {4, 12, 20, 28};
constexpr uint32_t kSegStart[4] = {0, 16, 16 + 4096, 16 + 4096 + 1048576};

inline uint64_t ptr_bytes(uint32_t w) { return (4 + kSegBits[segment(w & kIndexMask)]) / 8; }

uint8_t* put_be(uint8_t* o, uint64_t v, int nbytes) {       // binary_write, utility.h:178-184
  for (int i = nbytes - 1; i >= 0; --i) *o++ = uint8_t(v >> (8 * i));
  return o;
}

uint8_t* put_ptr(uint8_t* o, uint32_t w) {                   // pointer::serialize, :133-142
  const uint32_t idx = w & kIndexMask;
  const int seg = segment(idx);
  const uint32_t off = idx == kNullIndex ? 0xfffffffu : idx - kSegStart[seg];
  int sh = int(kSegBits[seg]) - 4;
  *o++ = uint8_t((off >> sh) | (((w >> 29) & 1) << 4) | (((w >> 30) & 1) << 5) | (seg << 6));
  for (sh -= 8; sh >= 0; sh -= 8) *o++ = uint8_t(off >> sh);
  return o;
}


}  // namespace

namespace gcz {

TreeView view_of(gcz_tree* t) {
  TreeView v;
  v.L = t->L;
  v.leaves = t->leaves.data();
  v.n_leaves = t->leaves.size();
  for (auto& layer : t->layers) {
    v.layer.push_back(layer.data());
    v.layer_n.push_back(layer.size() / 2);
  }
  v.root = t->root;
  return v;
}

// shared_tree::sort_tree (src/shared_tree.cpp:443-483).  The reference's two
// std::async batches touch disjoint layers and a parent's reordering does not
// change its children's counts, so the net effect is: leaves and node layers
// 0..D-2 each permuted independently by their parent's histogram (the top
// layer and the root are unchanged).  Layers are processed in parallel.
void view_sort(TreeView& t) {
  const size_t D = t.layer.size();
  if (D == 0) return;
  auto parent_words = [&](size_t c) { return std::vector<uint32_t>(t.layer[c], t.layer[c] + 2 * t.layer_n[c]); };
  std::vector<std::vector<uint32_t>> perm(D);
  {
    std::vector<std::thread> th;
    for (size_t c = 0; c < D; ++c) {
      const size_t n = c == 0 ? t.n_leaves : t.layer_n[c - 1];
      th.emplace_back([&, c, n] { perm[c] = frequency_order(t.layer[c], 2 * t.layer_n[c], n); });
    }
    for (auto& x : th) x.join();
  }
  (void)parent_words;
  std::vector<std::thread> th;
  th.emplace_back([&] {
    std::vector<uint64_t> nl(t.leaves, t.leaves + t.n_leaves);
    for (size_t i = 0; i < nl.size(); ++i) t.leaves[perm[0][i]] = nl[i];   // reorder_layer :371-377
  });
  for (size_t l = 0; l + 1 < D; ++l) {
    th.emplace_back([&, l] {
      const auto& np = perm[l + 1];
      std::vector<uint32_t> w(t.layer[l], t.layer[l] + 2 * t.layer_n[l]);
      for (size_t i = 0; i < np.size(); ++i) {
        t.layer[l][2 * size_t(np[i])] = w[2 * i];
        t.layer[l][2 * size_t(np[i]) + 1] = w[2 * i + 1];
      }
    });
  }
  for (auto& x : th) x.join();
  th.clear();
  for (size_t c = 0; c < D; ++c) th.emplace_back([&, c] { rewire(t.layer[c], 2 * t.layer_n[c], perm[c]); });
  for (auto& x : th) x.join();
}

// shared_tree::bytes (src/shared_tree.cpp:488-496).
uint64_t view_bytes(const TreeView& t) {
  uint64_t b = ptr_bytes(t.root) + 8 + t.n_leaves * uint64_t((t.L + 1) / 2);
  for (size_t l = 0; l < t.layer.size(); ++l) {
    b += 8;
    for (size_t i = 0; i < 2 * t.layer_n[l]; ++i) b += ptr_bytes(t.layer[l][i]);
  }
  return b;
}

// shared_tree::serialize (src/shared_tree.cpp:504-513).  0 when cap is too small.
uint64_t view_serialize(const TreeView& t, uint8_t* buf, uint64_t cap) {
  const uint64_t need = view_bytes(t);
  if (cap < need) return 0;
  uint8_t* o = put_ptr(buf, t.root);
  o = put_be(o, t.n_leaves, 8);
  const int lb = (t.L + 1) / 2;
  for (size_t i = 0; i < t.n_leaves; ++i) o = put_be(o, t.leaves[i], lb);
  for (size_t l = 0; l < t.layer.size(); ++l) {
    o = put_be(o, t.layer_n[l], 8);
    for (size_t i = 0; i < 2 * t.layer_n[l]; ++i) o = put_ptr(o, t.layer[l][i]);
  }
  return uint64_t(o - buf);
}

// shared_tree::width via children() (include/shared_tree.h:165,
// src/shared_tree.cpp:252-259), bottom-up.
uint64_t view_width(const TreeView& t) {
  if (t.layer.empty()) return 0;
  std::vector<uint64_t> below;
  for (size_t l = 0; l < t.layer.size(); ++l) {
    std::vector<uint64_t> cur(t.layer_n[l]);
    for (size_t i = 0; i < cur.size(); ++i) {
      uint64_t s = 0;
      for (int c = 0; c < 2; ++c) {
        const uint32_t w = t.layer[l][2 * i + c];
        if (ul(w) == kNullIndex) continue;
        s += l == 0 ? 1 : below[w & kIndexMask];
      }
      cur[i] = s;
    }
    below.swap(cur);
  }
  return ul(t.root) == kNullIndex ? 0 : below[t.root & kIndexMask];
}

}  // namespace gcz

namespace {
}  // namespace

extern "C" {

gcz_tree* gcz_tree_new(void) { return new gcz_tree(); }
void gcz_tree_free(gcz_tree* t) { delete t; }
int gcz_tree_n_layers(const gcz_tree* t) { return int(t->layers.size()); }
uint64_t gcz_tree_n_leaves(const gcz_tree* t) { return t->leaves.size(); }
uint64_t gcz_tree_layer_size(const gcz_tree* t, int k) {
  return (k >= 0 && size_t(k) < t->layers.size()) ? t->layers[k].size() / 2 : 0;
}
uint32_t gcz_tree_root(const gcz_tree* t) { return t->root; }
int gcz_tree_L(const gcz_tree* t) { return t->L; }
const uint64_t* gcz_tree_leaves(const gcz_tree* t) { return t->leaves.data(); }
const uint32_t* gcz_tree_layer(const gcz_tree* t, int k) {
  return (k >= 0 && size_t(k) < t->layers.size()) ? t->layers[k].data() : nullptr;
}

void gcz_tree_sort(gcz_tree* t) {
  gcz::TreeView v = gcz::view_of(t);
  gcz::view_sort(v);
}

uint64_t gcz_tree_bytes(const gcz_tree* t) { return gcz::view_bytes(gcz::view_of(const_cast<gcz_tree*>(t))); }

uint64_t gcz_tree_serialize(const gcz_tree* t, uint8_t* buf, uint64_t cap) {
  return gcz::view_serialize(gcz::view_of(const_cast<gcz_tree*>(t)), buf, cap);
}

uint64_t gcz_tree_width(const gcz_tree* t) { return gcz::view_width(gcz::view_of(const_cast<gcz_tree*>(t))); }

void gcz_tree_set_leaves(gcz_tree* t, int L, const uint64_t* leaves, uint64_t n) {
  t->L = L;
  t->leaves.assign(leaves, leaves + n);
  t->layers.clear();
}

void gcz_tree_push_layer(gcz_tree* t, const uint32_t* words, uint64_t n_nodes) {
  t->layers.emplace_back(words, words + 2 * n_nodes);
}

void gcz_tree_set_root(gcz_tree* t, uint32_t root) { t->root = root; }

// pointer::deserialize (src/shared_tree.cpp:147-163) + shared_tree::deserialize
// (:520-538): root, u64 leaf count, leaves of ceil(L/2) bytes, then layers
// (u64 count + pointer pairs) until the input ends.  invariant = false.
int gcz_tree_deserialize(gcz_tree* t, int L, const uint8_t* buf, uint64_t n) {
  uint64_t pos = 0;
  bool ok = true;
  auto get_be = [&](int nbytes) -> uint64_t {
    uint64_t v = 0;
    if (pos + uint64_t(nbytes) > n) { ok = false; return 0; }
    for (int i = 0; i < nbytes; ++i) v = (v << 8) | buf[pos++];
    return v;
  };
  auto get_ptr = [&]() -> uint32_t {
    const uint32_t first = uint32_t(get_be(1));
    const int seg = (first >> 6) & 3;
    const uint32_t t_bit = (first >> 5) & 1, m_bit = (first >> 4) & 1;
    uint64_t off = uint64_t(first & 0xf) << (kSegBits[seg] - 4);
    for (int sh = int(kSegBits[seg]) - 12; sh >= 0; sh -= 8) off |= get_be(1) << sh;
    const uint32_t idx = (seg == 3 && off == 0xfffffffu) ? kNullIndex : uint32_t(kSegStart[seg] + off);
    return idx | (m_bit << 29) | (t_bit << 30);   // pointer{data, m, t, false}
  };
  gcz_tree nt;
  nt.L = L;
  nt.root = get_ptr();
  const uint64_t nl = get_be(8);
  if (!ok || nl > n) return GCZ_ERR_ARG;
  nt.leaves.resize(nl);
  for (uint64_t i = 0; i < nl && ok; ++i) nt.leaves[i] = get_be((L + 1) / 2);
  while (ok && pos < n) {
    const uint64_t cnt = get_be(8);
    if (!ok || cnt > n) return GCZ_ERR_ARG;
    std::vector<uint32_t> w(2 * cnt);
    for (uint64_t i = 0; i < 2 * cnt && ok; ++i) w[i] = get_ptr();
    nt.layers.push_back(std::move(w));
  }
  if (!ok) return GCZ_ERR_ARG;
  *t = std::move(nt);
  return GCZ_OK;
}

// fasta_reader::load_buffer line contract (src/fasta_reader.cpp:40-68): at each
// line start a '>' or '\n' skips ONE line, the next line is data without a
// second peek; data line bodies are concatenated.  Reader buffers hold
// cap = min(n/L + 1, buffer_strands) * L data bytes (:22-31); a data line that
// crosses a buffer boundary resumes with a fresh peek there (:48-51), so a '>'
// at the boundary drops the rest of that line and makes the next line data.
uint64_t gcz_fasta_extract(const uint8_t* f, uint64_t n, int L, uint64_t buffer_strands, uint8_t* out) {
  if (L < 1) return 0;
  const uint64_t cap = gcz::reader_buffer_bytes(n, L, buffer_strands);
  uint64_t pos = 0, j = 0;
  bool forced = false;
  while (pos < n) {
    if (!forced && (f[pos] == '>' || f[pos] == '\n')) {
      const void* nl = std::memchr(f + pos, '\n', n - pos);
      pos = nl ? uint64_t(static_cast<const uint8_t*>(nl) - f) + 1 : n;
      forced = true;
      continue;
    }
    forced = false;
    const void* nl = std::memchr(f + pos, '\n', n - pos);
    uint64_t end = nl ? uint64_t(static_cast<const uint8_t*>(nl) - f) : n;
    for (uint64_t k = j / cap + 1; k * cap < j + (end - pos); ++k)
      if (f[pos + (k * cap - j)] == '>') {
        end = pos + (k * cap - j);
        forced = true;
        break;
      }
    if (out + j != f + pos) std::memmove(out + j, f + pos, end - pos);
    j += end - pos;
    pos = nl ? uint64_t(static_cast<const uint8_t*>(nl) - f) + 1 : n;
  }
  return j;
}

void gcz_synth_fill(char* out, int kind, uint64_t seed, uint64_t begin, uint64_t end) {
  const uint64_t n = end > begin ? end - begin : 0;
  unsigned T = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (n < (1u << 22)) T = 1;
  std::vector<std::thread> th;
  for (unsigned t = 0; t < T; ++t) {
    const uint64_t a = begin + n * t / T, b = begin + n * (t + 1) / T;
    th.emplace_back([=] { gcz_synth_fill_range(out + (a - begin), kind, seed, a, b); });
  }
  for (auto& x : th) x.join();
}

uint64_t gcz_synth_default_seed(void) { return GCZ_SYNTH_SEED; }

// Host storage of the tree containers (include/shared_tree.h, gcz_uninit_allocator): large
// arrays are 2 MB-aligned anonymous mappings advised as transparent huge pages, carved from a
// pre-faulted pool when one is there (gcz_host_prefault: the drop-in faults the pool in while
// the HIP runtime starts, so the fetch's copies find their pages present), else mapped fresh.
// Pieces are whole 2 MB units, so gcz_host_free unmaps exactly its piece, pool or not.
namespace {
constexpr uint64_t kHuge = uint64_t(2) << 20;
constexpr uint64_t kBig = uint64_t(4) << 20;
std::mutex g_pool_mu;
uintptr_t g_pool_cur = 0, g_pool_end = 0;

uint64_t huge_round(uint64_t b) { return (b + kHuge - 1) & ~(kHuge - 1); }

void* map_huge(uint64_t sz) {   // sz: a multiple of kHuge
  void* m = ::mmap(nullptr, sz + kHuge, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (m == MAP_FAILED) return nullptr;
  const uintptr_t base = reinterpret_cast<uintptr_t>(m), a = (base + kHuge - 1) & ~uintptr_t(kHuge - 1);
  if (a > base) ::munmap(m, a - base);   // trim to [a, a + sz)
  if (base + sz + kHuge > a + sz) ::munmap(reinterpret_cast<void*>(a + sz), base + sz + kHuge - (a + sz));
  (void)::madvise(reinterpret_cast<void*>(a), sz, MADV_HUGEPAGE);
  return reinterpret_cast<void*>(a);
}
}  // namespace

// A C entry point: nullptr when the memory is not there (nothing may throw through the C ABI;
// gcz_uninit_allocator turns nullptr into std::bad_alloc on the C++ side).
void* gcz_host_alloc(uint64_t bytes) {
  if (bytes < kBig) return ::operator new(bytes ? bytes : 1, std::nothrow);
  const uint64_t sz = huge_round(bytes);
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    if (g_pool_end - g_pool_cur >= sz) {
      void* p = reinterpret_cast<void*>(g_pool_cur);
      g_pool_cur += sz;
      return p;
    }
  }
  return map_huge(sz);
}

void gcz_host_free(void* p, uint64_t bytes) {
  if (!p) return;
  if (bytes < kBig) {
    ::operator delete(p);
    return;
  }
  ::munmap(p, huge_round(bytes));
}

int gcz_host_prefault(uint64_t bytes, int threads) {
  gcz_host_pool_release(0);
  if (bytes < kBig) return GCZ_OK;
  const uint64_t sz = huge_round(bytes);
  void* p = map_huge(sz);
  if (!p) return GCZ_ERR_DEVICE;
  unsigned char* b = static_cast<unsigned char*>(p);
  const int T = std::max(1, std::min(threads, 16));
  auto touch = [&](int t) {   // one write per 4 KB page: the fault maps it (a huge page where THP allows)
    const uint64_t lo = sz * uint64_t(t) / uint64_t(T) & ~uint64_t(4095), hi = sz * uint64_t(t + 1) / uint64_t(T);
    for (uint64_t o = lo; o < hi; o += 4096) b[o] = 0;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(touch, t);
  touch(0);
  for (auto& x : th) x.join();
  std::lock_guard<std::mutex> g(g_pool_mu);
  g_pool_cur = reinterpret_cast<uintptr_t>(p);
  g_pool_end = g_pool_cur + sz;
  return GCZ_OK;
}

void gcz_host_pool_release(int async) {
  uintptr_t a, b;
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    a = g_pool_cur;
    b = g_pool_end;
    g_pool_cur = g_pool_end = 0;
  }
  if (b <= a) return;
  if (async)   // (the range is no longer the pool's: a later prefault cannot be unmapped by this)
    std::thread([a, b] { ::munmap(reinterpret_cast<void*>(a), b - a); }).detach();
  else
    ::munmap(reinterpret_cast<void*>(a), b - a);
}

}  // extern "C"
