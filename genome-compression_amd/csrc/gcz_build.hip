// MI355X (gfx950) shared_tree construction: leaf packing, per-level
// canonicalise + hash-cons, first-occurrence ID assignment, unique emission.
//
// Replaces tree_constructor (reference include/shared_tree.h:245-316,
// src/shared_tree.cpp:621-763).  One global level-by-level build; the
// reference's 2^22/2^25-strand segmentation is output-invisible.
//
// Per level (n input words -> p = ceil(n/2) pairs; the leaf level has p = S):
//   insert    canonical key of each pair/leaf -> open-addressing table in HBM:
//             CAS on the 64-bit key, atomicMin of the position.  Writes the
//             provisional word rec[j] = slot | m<<29 | t<<30 | v<<31.
//   flagscan  first occurrence <=> slot.pos == j.  Wave ballot -> 64-element
//             group masks; in-tile scan + decoupled look-back across tiles ->
//             group prefixes; first occurrences get id = first-occurrence rank,
//             emit the unique node/leaf at out[id] and their final word.
//             Others keep minpos in place of the slot index.
//   resolve   non-first occurrences: id = rank of minpos from its group's
//             {mask, prefix} (one 16-B read into a p/4-byte array).
// The next level reads the final words directly (coalesced); no per-element
// id table lookups remain.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "gcz_internal.h"

namespace {

using u32 = uint32_t;
using u64 = unsigned long long;

constexpr u32 kNullWord = 0x9fffffffu;
constexpr u32 kIdx = 0x1fffffffu;
constexpr u32 kBits = 0xe0000000u;
constexpr u64 kEmpty = ~0ull;              // stored key; stored = key ^ 1 (see kEmpty note below)
constexpr int kBlock = 256;
constexpr int kItems = 8;                  // flagscan elements per thread
constexpr int kTile = kBlock * kItems;     // 2048 elements per look-back tile
constexpr int kGroupsPerTile = kTile / 64; // 32
constexpr u32 kMaxProbe = 1u << 16;

// kEmpty note: table keys are stored as key ^ 1, so a stored ~0 means key
// 0xffff_ffff_ffff_fffe.  That value is never a key: as a leaf its transpose
// (..fff7) is smaller so it is never canonical (dna.cpp:135-143); as a node
// its left word would carry both the mirror and invariant bits, which the
// pointer ctor forbids (shared_tree.cpp:85-86).  memset(0xff) clears a table.

struct __align__(16) Slot {
  u64 key;
  u32 pos;
  u32 pad;
};
struct __align__(16) Group {
  u64 mask;    // first-occurrence flags of 64 consecutive elements
  u32 prefix;  // first occurrences before this group (global, this level)
  u32 pad;
};

struct Header {
  u64 count[GCZ_MAX_LAYERS + 1];  // [0] unique leaves, [1+k] unique nodes of layer k
  u64 err_offset;                 // first unknown symbol (min), ~0 if none
  u32 overflow;
  u32 inserts;                    // new keys in an adaptively sized leaf table
  u32 ticket[GCZ_MAX_LAYERS + 1]; // look-back tile tickets per level
  u32 root;
  u32 pad;
};

__device__ __forceinline__ u32 slot_hash(u64 k) {
  k ^= k >> 31;
  k *= 0x7fb5d329728ea185ull;
  k ^= k >> 27;
  k *= 0x81dadef4bc2dd44dull;
  k ^= k >> 33;
  return u32(k);
}

// ---- word algebra: reference src/shared_tree.cpp:76-107 -------------------
__device__ __forceinline__ u32 ulw(u32 w) { return w & 0x7fffffffu; }
// transform ctor (shared_tree.cpp:76-80): m' = (M != m) && !v ; t' = (T != t) && !null
__device__ __forceinline__ u32 xf(u32 w, u32 M, u32 T) {
  const u32 v = w >> 31, m = (w >> 29) & 1u, t = (w >> 30) & 1u;
  const u32 nm = (M ^ m) & (v ^ 1u);
  const u32 nt = (T ^ t) & u32(ulw(w) != kIdx);
  return (w & 0x9fffffffu) | (nm << 29) | (nt << 30);
}
__device__ __forceinline__ u32 make_word(u32 idx, u32 m, u32 t, u32 v) {
  return idx | ((m & (v ^ 1u)) << 29) | (t << 30) | (v << 31);
}

// node::canonical (include/shared_tree.h:115-126): min over (key, m, t).
// Candidates id=(l,r) mir=(M(r),M(l)) tra=(T(l),T(r)) inv=(I(r),I(l)).
__device__ __forceinline__ void node_canonical(u32 l, u32 r, u32& cl, u32& cr, u32& cm, u32& ct) {
  const u32 ml = xf(l, 1, 0), mr = xf(r, 1, 0);
  const u32 tl = xf(l, 0, 1), tr = xf(r, 0, 1);
  const u32 il = xf(l, 1, 1), ir = xf(r, 1, 1);
  // key with (m,t) appended below it: lexicographic (key, m, t) in one 66-bit compare.
  // key fits in 62 bits, so (key << 2 | m << 1 | t) is exact in 64 bits.
  auto k = [](u32 a, u32 b, u32 m, u32 t) -> u64 {
    return ((u64(ulw(a)) << 31 | ulw(b)) << 2) | (m << 1) | t;
  };
  u64 best = k(l, r, 0, 0);
  cl = l; cr = r; cm = 0; ct = 0;
  u64 c = k(mr, ml, 1, 0);
  if (c < best) { best = c; cl = mr; cr = ml; cm = 1; ct = 0; }
  c = k(tl, tr, 0, 1);
  if (c < best) { best = c; cl = tl; cr = tr; cm = 0; ct = 1; }
  c = k(ir, il, 1, 1);
  if (c < best) { best = c; cl = ir; cr = il; cm = 1; ct = 1; }
}

// ---- leaf codec: reference src/dna.cpp:104-143 -----------------------------
__device__ __forceinline__ u64 leaf_transposed(u64 v) {
  v = ((v >> 1) & 0x5555555555555555ull) | ((v & 0x5555555555555555ull) << 1);
  v = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
  return v;
}
// reverse the low L nibbles (higher nibbles dropped), dna::mirrored :116-121
__device__ __forceinline__ u64 leaf_mirrored(u64 v, int L) {
  u64 y = __builtin_bswap64(v);
  y = ((y >> 4) & 0x0f0f0f0f0f0f0f0full) | ((y & 0x0f0f0f0f0f0f0f0full) << 4);
  return L == 16 ? y : (y >> (64 - 4 * L));
}
__device__ __forceinline__ u64 leaf_canonical(u64 x, int L, u32& m, u32& t, u32& v) {
  const u64 tx = leaf_transposed(x);
  const u64 mx = leaf_mirrored(x, L);
  const u64 ix = leaf_mirrored(tx, L);
  v = x == mx;
  u64 best = x; m = 0; t = 0;
  if (tx < best) { best = tx; m = 0; t = 1; }
  if (mx < best) { best = mx; m = 1; t = 0; }
  if (ix < best) { best = ix; m = 1; t = 1; }
  return best;
}

// ---- hash tables -------------------------------------------------------------
// Both tables map a canonical key to (slot, minimum position).  The slot index
// is what the insert pass records per element; flagscan reads the slot back.
//
// PackedTab (default): one 8-B word per slot,
//     word = quotient(h) << (D+P) | displacement << P | pos
// where h = mix(key) is a bijection on K key bits, the home slot is h's low c
// bits and the quotient its high K-c bits.  The CAS that claims a slot also
// stores the position, so a new key costs ONE memory-side atomic; repeats of a
// key carry identical high bits and lower pos with a 64-bit atomicMin.  The
// key is recovered exactly from (slot, word) by inverting the mix.
// Used when quotient + displacement + position bits fit in 64.
//
// WideTab (fallback, e.g. L = 16 leaves): 16-B slots {key ^ 1, pos}; CAS on
// the key then atomicMin on pos.
//
// Both probe linearly with a plain load first.  The load may be stale (this
// CU's L1 / this XCD's L2), but slots only go EMPTY -> claimed and positions
// only decrease, so staleness costs at most an extra CAS/atomicMin.

__device__ __forceinline__ u32 enc_child(u32 w, u32 B) {      // pointer word -> B+3 bits
  const u32 idx = w & kIdx;
  const u32 code = idx == kIdx ? ((1u << B) - 1u) : idx;      // null index -> all-ones code
  return (code << 3) | (((w >> 29) & 1u) << 2) | (((w >> 30) & 1u) << 1) | (w >> 31);
}
__device__ __forceinline__ u32 dec_child(u32 e, u32 B) {
  const u32 code = e >> 3;
  if (code == (1u << B) - 1u) return kNullWord;
  return code | (((e >> 2) & 1u) << 29) | (((e >> 1) & 1u) << 30) | ((e & 1u) << 31);
}

struct WideTab {
  Slot* tab;
  u32 mask;
  u32 limit;
  u32 B;   // unused

  __device__ __forceinline__ u64 node_key(u32 cl, u32 cr) const { return (u64(cl) << 32) | cr; }
  __device__ __forceinline__ void node_words(u64 key, u32& cl, u32& cr) const {
    cl = u32(key >> 32); cr = u32(key);
  }
  __device__ __forceinline__ u32 insert(u64 key, u32 pos, Header* __restrict__ hdr) const {
    const u64 skey = key ^ 1ull;
    u32 s = slot_hash(skey) & mask;
    for (u32 probe = 0; probe < limit; ++probe) {
      const Slot cur = tab[s];
      u64 k = cur.key;
      if (k == kEmpty) k = atomicCAS(&tab[s].key, kEmpty, skey);
      if (k == kEmpty || k == skey) {
        if (cur.pos > pos) atomicMin(&tab[s].pos, pos);
        return s;
      }
      s = (s + 1) & mask;
    }
    atomicOr(&hdr->overflow, 1u);
    return 0;
  }
  __device__ __forceinline__ void read(u32 s, u64& key, u32& pos) const {
    const Slot sl = tab[s];
    key = sl.key ^ 1ull;
    pos = sl.pos;
  }
};

struct PackedTab {
  u64* tab;
  u32 mask;
  u32 limit;   // <= 2^D - 2 probes
  u32 B;       // child index bits (node levels)
  u32 c, P, D, sh;
  u64 kmask, c1, c2, c1i, c2i;

  __device__ __forceinline__ u64 node_key(u32 cl, u32 cr) const {
    return (u64(enc_child(cl, B)) << (B + 3)) | enc_child(cr, B);
  }
  __device__ __forceinline__ void node_words(u64 key, u32& cl, u32& cr) const {
    cl = dec_child(u32(key >> (B + 3)), B);
    cr = dec_child(u32(key & ((1ull << (B + 3)) - 1)), B);
  }
  __device__ __forceinline__ u64 mix(u64 x) const {
    x ^= x >> sh; x = (x * c1) & kmask;
    x ^= x >> sh; x = (x * c2) & kmask;
    x ^= x >> sh;
    return x;
  }
  __device__ __forceinline__ u64 unmix(u64 h) const {
    h ^= h >> sh; h = (h * c2i) & kmask;
    h ^= h >> sh; h = (h * c1i) & kmask;
    h ^= h >> sh;
    return h;
  }
  __device__ __forceinline__ u32 insert(u64 key, u32 pos, Header* __restrict__ hdr) const {
    const u64 h = mix(key);
    u32 s = u32(h) & mask;
    const u64 qd = (h >> c) << D;             // quotient, displacement bits free
    const u64 pmask = (1ull << P) - 1;
    for (u32 d = 0; d < limit; ++d) {
      const u64 mine = ((qd | d) << P) | pos;
      u64 cur = tab[s];
      if (cur == kEmpty) {
        cur = atomicCAS(&tab[s], kEmpty, mine);
        if (cur == kEmpty) return s;
      }
      if ((cur >> P) == (mine >> P)) {
        if ((cur & pmask) > pos) atomicMin(&tab[s], mine);
        return s;
      }
      s = (s + 1) & mask;
    }
    atomicOr(&hdr->overflow, 1u);
    return 0;
  }
  __device__ __forceinline__ void read(u32 s, u64& key, u32& pos) const {
    const u64 w = tab[s];
    pos = u32(w & ((1ull << P) - 1));
    const u32 d = u32((w >> P) & ((1ull << D) - 1));
    const u64 q = w >> (P + D);
    const u64 home = (s - d) & mask;
    key = unmix((q << c) | home);
  }
};

// ---- kernels -----------------------------------------------------------------

// nac codes of an ASCII byte, include/dna.h:20-32 (to_nac, src/dna.cpp:25-49); -1 unknown
__device__ __forceinline__ int nac_code(int c) {
  const int u = (c >= 'a' && c <= 'z') ? c - 32 : c;
  switch (u) {
    case 'A': return 1;  case 'C': return 2;  case 'G': return 4;  case 'T': return 8;
    case 'R': return 3;  case 'Y': return 12; case 'K': return 7;  case 'M': return 14;
    case 'B': return 5;  case 'V': return 10; case 'D': return 11; case 'H': return 13;
    case 'S': return 0;  case 'W': return 9;  case 'N': return 6;  case '-': return 15;
    default: return -1;
  }
}

// Leaf level from raw bases: pack L symbols (dna::dna(string_view) +
// dna::set, dna.cpp:79-84,187-197), canonicalise (dna.cpp:135-143), insert.
// Bases for the block are staged through LDS with coalesced 4-B loads.
template <int L, class Tab>
__global__ __launch_bounds__(kBlock) void k_leaf_bases(const unsigned char* __restrict__ bases, u64 S, Tab T,
                                                      u32* __restrict__ rec, Header* __restrict__ hdr) {
  __shared__ signed char lut[256];
  __shared__ __align__(16) unsigned char buf[kBlock * L + 16];
  const int tid = threadIdx.x;
  lut[tid] = (signed char)nac_code(tid);
  const u64 first = u64(blockIdx.x) * kBlock;
  const u64 nstr = (S - first) < u64(kBlock) ? (S - first) : u64(kBlock);
  const u64 byte0 = first * L;                 // multiple of 4 (kBlock = 256)
  const u64 nbytes = nstr * L;
  const u32* src = reinterpret_cast<const u32*>(bases + byte0);
  u32* dst = reinterpret_cast<u32*>(buf);
  const u32 nwords = u32(nbytes / 4);
  for (u32 w = tid; w < nwords; w += kBlock) dst[w] = src[w];
  for (u32 b = nwords * 4 + tid; b < nbytes; b += kBlock) buf[b] = bases[byte0 + b];
  __syncthreads();
  if (u64(tid) >= nstr) return;
  u64 x = 0;
  int bad = -1;
#pragma unroll
  for (int c = 0; c < L; ++c) {
    const int code = lut[buf[tid * L + c]];
    if (code < 0 && bad < 0) bad = c;
    x |= u64(code & 15) << (4 * c);
  }
  const u64 i = first + tid;
  if (bad >= 0) atomicMin(&hdr->err_offset, i * L + u64(bad));
  u32 m, t, v;
  const u64 key = leaf_canonical(x, L, m, t, v);
  const u32 s = T.insert(key, u32(i), hdr);
  rec[i] = make_word(s, m, t, v);
}

// Leaf level from packed strands (shared_tree(std::vector<dna>&)).
template <class Tab>
__global__ __launch_bounds__(kBlock) void k_leaf_packed(const u64* __restrict__ leaves, u64 S, int L, Tab T,
                                                       u32* __restrict__ rec, Header* __restrict__ hdr) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= S) return;
  u32 m, t, v;
  const u64 key = leaf_canonical(leaves[i], L, m, t, v);
  const u32 s = T.insert(key, u32(i), hdr);
  rec[i] = make_word(s, m, t, v);
}

// Node level: pair (2j, 2j+1) of the previous level's final words; the odd
// tail pairs with the null pointer (foreach_pair, include/utility.h:17-29).
// tree_constructor::emplace_node, src/shared_tree.cpp:662-672.
template <class Tab>
__global__ __launch_bounds__(kBlock) void k_node_insert(const u32* __restrict__ in, u64 n, u64 p, Tab T,
                                                       u32* __restrict__ rec, Header* __restrict__ hdr) {
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= p) return;
  u32 l, r;
  if (2 * j + 1 < n) {
    const uint2 w = reinterpret_cast<const uint2*>(in)[j];
    l = w.x; r = w.y;
  } else {
    l = in[2 * j]; r = kNullWord;
  }
  u32 cl, cr, m, t;
  node_canonical(l, r, cl, cr, m, t);
  const u32 v = ulw(l) == ulw(xf(r, 1, 0));      // left == right.mirrored() (:670)
  const u32 s = T.insert(T.node_key(cl, cr), u32(j), hdr);
  rec[j] = make_word(s, m, t, v);
}

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr u64 kStA = 1ull << 62;   // tile aggregate published
constexpr u64 kStP = 2ull << 62;   // tile inclusive prefix published
constexpr u64 kValMask = (1ull << 62) - 1;

// First-occurrence flags + device-wide scan (decoupled look-back) + emission.
// kLeaf: unique output is u64 leaves, else uint2 {left,right} node words.
template <bool kLeaf, class Tab>
__global__ __launch_bounds__(kBlock) void k_flagscan(u32* __restrict__ words, u64 p, Tab T,
                                                    Group* __restrict__ grp, u64* __restrict__ desc,
                                                    u32* __restrict__ ticket, void* __restrict__ out,
                                                    u64* __restrict__ count_out) {
  __shared__ u32 s_tile;
  __shared__ u32 s_cnt[kGroupsPerTile];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(ticket, 1u);
  __syncthreads();
  const u64 tile = s_tile;
  const u64 base = tile * kTile;

  u32 rec[kItems], pos[kItems];
  u64 key[kItems], mask[kItems];
#pragma unroll
  for (int e = 0; e < kItems; ++e) {
    const u64 j = base + u64(e) * kBlock + tid;
    rec[e] = j < p ? words[j] : 0u;
  }
#pragma unroll
  for (int e = 0; e < kItems; ++e) {
    const u64 j = base + u64(e) * kBlock + tid;
    if (j < p) {
      T.read(rec[e] & kIdx, key[e], pos[e]);
    } else {
      key[e] = 0; pos[e] = ~0u;
    }
  }
#pragma unroll
  for (int e = 0; e < kItems; ++e) {
    const u64 j = base + u64(e) * kBlock + tid;
    mask[e] = __ballot(j < p && u64(pos[e]) == j);
    if (lane == 0) s_cnt[e * 4 + wave] = u32(__popcll(mask[e]));
  }
  __syncthreads();
  if (wave == 0) {
    const u32 c = lane < kGroupsPerTile ? s_cnt[lane] : 0u;
    u32 incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const u64 agg = __shfl(incl, 63, 64);
    u64 prefix = 0;
    if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&desc[0], kStP | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&desc[tile], kStA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      long long look = (long long)tile - 1;
      for (;;) {
        const long long idx = look - lane;
        const u64 d = idx >= 0 ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        const u64 st = d >> 62;
        const u64 pm = __ballot(st == 2);
        const u64 zm = __ballot(st == 0);
        const int firstP = pm ? __ffsll((long long)pm) - 1 : 64;
        const u64 need = firstP >= 63 ? ~0ull : ((1ull << (firstP + 1)) - 1);
        if (zm & need) {
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        prefix += wave_sum(lane <= firstP ? (d & kValMask) : 0ull);
        if (firstP < 64) break;
        look -= 64;
      }
      if (lane == 0) __hip_atomic_store(&desc[tile], kStP | (prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane < kGroupsPerTile) s_cnt[lane] = u32(prefix + incl - c);
    if (lane == 0 && (tile + 1) * kTile >= p) *count_out = prefix + agg;
  }
  __syncthreads();
  const u64 lt = (1ull << lane) - 1;
#pragma unroll
  for (int e = 0; e < kItems; ++e) {
    const u64 j = base + u64(e) * kBlock + tid;
    const u32 gpre = s_cnt[e * 4 + wave];
    if (lane == 0) {
      Group g;
      g.mask = mask[e]; g.prefix = gpre; g.pad = 0;
      grp[(base >> 6) + e * 4 + wave] = g;
    }
    if (j >= p) continue;
    if ((mask[e] >> lane) & 1ull) {
      const u32 id = gpre + u32(__popcll(mask[e] & lt));
      if (kLeaf) {
        reinterpret_cast<u64*>(out)[id] = key[e];
      } else {
        uint2 w;
        T.node_words(key[e], w.x, w.y);
        reinterpret_cast<uint2*>(out)[id] = w;
      }
      words[j] = id | (rec[e] & kBits);
    } else {
      words[j] = pos[e] | (rec[e] & kBits);
    }
  }
}

// Non-first occurrences: id = rank of the first occurrence (minpos).
__global__ __launch_bounds__(kBlock) void k_resolve(u32* __restrict__ words, u64 p,
                                                   const Group* __restrict__ grp) {
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= p) return;
  const Group g = grp[j >> 6];
  if ((g.mask >> (j & 63)) & 1ull) return;
  const u32 w = words[j];
  const u32 q = w & kIdx;
  const Group h = grp[q >> 6];
  const u32 id = h.prefix + u32(__popcll(h.mask & ((1ull << (q & 63)) - 1)));
  words[j] = id | (w & kBits);
}

__global__ void k_root(const u32* __restrict__ words, Header* __restrict__ hdr) { hdr->root = words[0]; }

// ---- host side -----------------------------------------------------------------

#define HIP_TRY(x)                                                          \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) return fail(GCZ_ERR_DEVICE, #x, hipGetErrorString(e_)); \
  } while (0)

u64 next_pow2(u64 x) {
  u64 p = 1;
  while (p < x) p <<= 1;
  return p;
}

struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};

u64 inv64(u64 a) {                 // inverse of an odd number mod 2^64 (Newton)
  u64 x = a;
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}

u32 bit_width(u64 x) {
  u32 b = 0;
  while (x) { ++b; x >>= 1; }
  return b;
}

u32 log2_exact(u64 x) { return bit_width(x) - 1; }

constexpr u32 kAdaptiveProbeLimit = 256;
constexpr u64 kMixC1 = 0x9E3779B97F4A7C15ull;
constexpr u64 kMixC2 = 0xD6E8FEB86659FD93ull;

// A level's table: packed 8-B words when quotient+displacement+position fit
// in 64 bits, else 16-B wide slots.
struct LevelTab {
  bool packed = false;
  PackedTab pt{};
  WideTab wt{};
  u64 cap = 0;
  u64 bytes() const { return cap * (packed ? 8 : 16); }
};

LevelTab plan_table(void* buf, u64 cap, u32 K, u64 npos, u32 B, bool allow_packed, u32 wide_limit) {
  LevelTab lt;
  lt.cap = cap;
  const u32 c = log2_exact(cap);
  const u32 Q = K > c ? K - c : 0;
  const u32 P = std::max<u32>(1, bit_width(npos - 1));
  const int room = 64 - int(Q) - int(P);
  if (allow_packed && K <= 64 && room >= 6) {
    lt.packed = true;
    PackedTab& t = lt.pt;
    t.tab = static_cast<u64*>(buf);
    t.mask = u32(cap - 1);
    t.D = u32(std::min(room, 8));
    t.limit = (1u << t.D) - 2;
    t.B = B;
    t.c = c;
    t.P = P;
    t.sh = (K + 1) / 2;
    t.kmask = K >= 64 ? ~0ull : ((1ull << K) - 1);
    t.c1 = kMixC1; t.c2 = kMixC2;
    t.c1i = inv64(kMixC1); t.c2i = inv64(kMixC2);
  } else {
    lt.wt.tab = static_cast<Slot*>(buf);
    lt.wt.mask = u32(cap - 1);
    lt.wt.limit = wide_limit;
    lt.wt.B = B;
  }
  return lt;
}

enum KernelId { KID_LEAF, KID_NODE, KID_FLAGSCAN_LEAF, KID_FLAGSCAN_NODE, KID_RESOLVE, KID_MEMSET, KID_COUNT };
const char* kKernelNames[KID_COUNT] = {"leaf_insert", "node_insert", "flagscan_leaf", "flagscan_node",
                                       "resolve", "table_clear"};

}  // namespace

struct gcz_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  std::string last_error;
  DevBuf wa, wb, grp, desc, tab, leaves_out, nodes_out, hdr, input;
  Header* h_hdr = nullptr;   // pinned
  // last build
  gcz_info info{};
  std::vector<u64> layer_off;  // node offsets (in nodes) per layer within nodes_out
  u64 leaf_cap_hint = 0;
  // profiling
  bool profile = false;
  bool force_wide = false;   // GCZ_TABLE=wide: always use 16-B slots (testing)
  std::vector<std::pair<int, std::pair<hipEvent_t, hipEvent_t>>> pending;
  std::vector<hipEvent_t> event_pool;
  size_t event_used = 0;
  u64 prof_launches[KID_COUNT] = {};
  double prof_ms[KID_COUNT] = {};
  hipEvent_t ev_start = nullptr, ev_stop = nullptr;

  int fail(int code, const char* what, const char* detail) {
    last_error = std::string(what) + ": " + detail;
    info.status = code;
    return code;
  }

  int ensure(DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.ptr) return GCZ_OK;
    if (b.ptr) {
      HIP_TRY(hipStreamSynchronize(stream));
      HIP_TRY(hipFree(b.ptr));
      b.ptr = nullptr; b.bytes = 0;
    }
    HIP_TRY(hipMalloc(&b.ptr, bytes));
    b.bytes = bytes;
    return GCZ_OK;
  }

  hipEvent_t next_event() {
    if (event_used == event_pool.size()) {
      hipEvent_t e;
      (void)hipEventCreate(&e);
      event_pool.push_back(e);
    }
    return event_pool[event_used++];
  }

  void prof_begin(int kid, hipEvent_t& a) {
    if (!profile) return;
    a = next_event();
    (void)hipEventRecord(a, stream);
    (void)kid;
  }
  void prof_end(int kid, hipEvent_t a) {
    if (!profile) return;
    hipEvent_t b = next_event();
    (void)hipEventRecord(b, stream);
    pending.push_back({kid, {a, b}});
  }
  void prof_collect() {
    for (auto& pe : pending) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, pe.second.first, pe.second.second);
      prof_ms[pe.first] += ms;
      prof_launches[pe.first] += 1;
    }
    pending.clear();
    event_used = 0;
  }

  int build(const void* d_bases, const u64* d_leaves, u64 nbases, u64 S, int L);
};

namespace {

template <class Tab>
void launch_leaf_bases(int L, dim3 g, hipStream_t st, const unsigned char* b, u64 S, const Tab& T, u32* rec,
                       Header* hdr) {
  switch (L) {
#define GCZ_CASE(X) \
  case X: hipLaunchKernelGGL((k_leaf_bases<X, Tab>), g, dim3(kBlock), 0, st, b, S, T, rec, hdr); break;
    GCZ_CASE(1) GCZ_CASE(2) GCZ_CASE(3) GCZ_CASE(4) GCZ_CASE(5) GCZ_CASE(6) GCZ_CASE(7) GCZ_CASE(8)
    GCZ_CASE(9) GCZ_CASE(10) GCZ_CASE(11) GCZ_CASE(12) GCZ_CASE(13) GCZ_CASE(14) GCZ_CASE(15) GCZ_CASE(16)
#undef GCZ_CASE
    default: break;
  }
}

}  // namespace

int gcz_ctx::build(const void* d_bases, const u64* d_leaves, u64 nbases, u64 S, int L) {
  info = gcz_info{};
  info.L = L;
  info.status = GCZ_OK;
  if (L < 1 || L > 16) return fail(GCZ_ERR_ARG, "build", "leaf length L must be in 1..16");
  if (d_bases) S = nbases / u64(L);
  if (S == 0) return fail(GCZ_ERR_EMPTY, "build", "fewer than L bases: nothing to build");
  if (S > u64(kIdx)) return fail(GCZ_ERR_CAPACITY, "build", "more than 2^29-1 strands");
  info.n_strands = S;

  // level plan
  std::vector<u64> pk;                     // pairs per node layer
  for (u64 n = S;;) {
    const u64 p = (n + 1) / 2;
    pk.push_back(p);
    if (p == 1) break;
    n = p;
  }
  if (pk.size() > GCZ_MAX_LAYERS) return fail(GCZ_ERR_CAPACITY, "build", "too many layers");
  const int D = int(pk.size());
  layer_off.assign(D + 1, 0);
  for (int k = 0; k < D; ++k) layer_off[k + 1] = layer_off[k] + pk[k];
  u64 ntiles_total = (S + kTile - 1) / kTile;
  std::vector<u64> desc_off(D + 1);
  desc_off[0] = 0;
  for (int k = 0; k < D; ++k) {
    desc_off[k + 1] = ntiles_total;
    ntiles_total += (pk[k] + kTile - 1) / kTile;
  }

  // leaf table: big enough for S when S is small; otherwise start at 2^23 slots
  // (every ACGT 12-mer class fits) and grow if the probe bound overflows.
  const u64 full_cap = std::max<u64>(256, next_pow2(2 * S));
  u64 leaf_cap = full_cap;
  if (S > (1ull << 22)) leaf_cap = std::min(full_cap, std::max<u64>(1ull << 23, leaf_cap_hint));
  const u64 node_cap0 = std::max<u64>(256, next_pow2(2 * pk[0]));

  u32* in = nullptr;
  int rc;
  if ((rc = ensure(wa, S * 4 + 16))) return rc;
  if ((rc = ensure(wb, ((S + 1) / 2) * 4 + 16))) return rc;
  if ((rc = ensure(grp, ((S + 63) / 64 + kGroupsPerTile) * sizeof(Group)))) return rc;
  if ((rc = ensure(desc, ntiles_total * 8 + 64))) return rc;
  if ((rc = ensure(leaves_out, S * 8 + 16))) return rc;
  if ((rc = ensure(nodes_out, layer_off[D] * 8 + 16))) return rc;
  if ((rc = ensure(hdr, sizeof(Header)))) return rc;
  if (!h_hdr) HIP_TRY(hipHostMalloc((void**)&h_hdr, sizeof(Header), hipHostMallocDefault));

  Header* d_hdr = static_cast<Header*>(hdr.ptr);
  u32* A = static_cast<u32*>(wa.ptr);
  u32* Bw = static_cast<u32*>(wb.ptr);
  Group* d_grp = static_cast<Group*>(grp.ptr);
  u64* d_desc = static_cast<u64*>(desc.ptr);

  if (!ev_start) {
    HIP_TRY(hipEventCreate(&ev_start));
    HIP_TRY(hipEventCreate(&ev_stop));
  }

  for (bool allow_packed : {!force_wide, false}) {
    HIP_TRY(hipEventRecord(ev_start, stream));
    HIP_TRY(hipMemsetAsync(d_hdr, 0, sizeof(Header), stream));
    HIP_TRY(hipMemsetAsync(&d_hdr->err_offset, 0xff, 8, stream));
    HIP_TRY(hipMemsetAsync(d_desc, 0, ntiles_total * 8, stream));
    if ((rc = ensure(tab, std::max(leaf_cap, node_cap0) * 16))) return rc;

    // ---- leaf level ----
    LevelTab lt;
    for (;;) {
      const bool adaptive = leaf_cap < 2 * S;
      const u32 limit = adaptive ? kAdaptiveProbeLimit : kMaxProbe;
      // packed leaves only from bases (< 2^4L by construction); user leaves may carry any bits
      lt = plan_table(tab.ptr, leaf_cap, d_bases ? 4 * u32(L) : 64, S, 0, allow_packed && d_bases, limit);
      if (lt.packed && lt.pt.limit > limit) lt.pt.limit = limit;
      hipEvent_t e0{};
      prof_begin(KID_MEMSET, e0);
      HIP_TRY(hipMemsetAsync(tab.ptr, 0xff, lt.bytes(), stream));
      prof_end(KID_MEMSET, e0);
      const dim3 g(unsigned((S + kBlock - 1) / kBlock));
      prof_begin(KID_LEAF, e0);
      if (d_bases) {
        if (lt.packed) launch_leaf_bases(L, g, stream, static_cast<const unsigned char*>(d_bases), S, lt.pt, A, d_hdr);
        else launch_leaf_bases(L, g, stream, static_cast<const unsigned char*>(d_bases), S, lt.wt, A, d_hdr);
      } else {
        hipLaunchKernelGGL((k_leaf_packed<WideTab>), g, dim3(kBlock), 0, stream, d_leaves, S, L, lt.wt, A, d_hdr);
      }
      HIP_TRY(hipGetLastError());
      prof_end(KID_LEAF, e0);
      if (!adaptive) break;
      HIP_TRY(hipMemcpyAsync(h_hdr, d_hdr, sizeof(Header), hipMemcpyDeviceToHost, stream));
      HIP_TRY(hipStreamSynchronize(stream));
      if (!h_hdr->overflow) break;
      leaf_cap = std::min(full_cap, leaf_cap * 8);
      if ((rc = ensure(tab, std::max(leaf_cap, node_cap0) * 16))) return rc;
      HIP_TRY(hipMemsetAsync(d_hdr, 0, sizeof(Header), stream));
      HIP_TRY(hipMemsetAsync(&d_hdr->err_offset, 0xff, 8, stream));
    }
    leaf_cap_hint = leaf_cap;
    {
      const dim3 gs(unsigned((S + kTile - 1) / kTile));
      hipEvent_t e0{};
      prof_begin(KID_FLAGSCAN_LEAF, e0);
      if (lt.packed)
        hipLaunchKernelGGL((k_flagscan<true, PackedTab>), gs, dim3(kBlock), 0, stream, A, S, lt.pt, d_grp,
                           d_desc + desc_off[0], &d_hdr->ticket[0], leaves_out.ptr, &d_hdr->count[0]);
      else
        hipLaunchKernelGGL((k_flagscan<true, WideTab>), gs, dim3(kBlock), 0, stream, A, S, lt.wt, d_grp,
                           d_desc + desc_off[0], &d_hdr->ticket[0], leaves_out.ptr, &d_hdr->count[0]);
      HIP_TRY(hipGetLastError());
      prof_end(KID_FLAGSCAN_LEAF, e0);
      prof_begin(KID_RESOLVE, e0);
      hipLaunchKernelGGL(k_resolve, dim3(unsigned((S + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, A, S,
                         d_grp);
      HIP_TRY(hipGetLastError());
      prof_end(KID_RESOLVE, e0);
    }

    // ---- node layers ----
    in = A;
    u32* outw = Bw;
    u64 n = S;
    u64 bound = std::min(S, leaf_cap);        // child ids of layer 0 are leaf ids < #slots
    for (int k = 0; k < D; ++k) {
      const u64 p = pk[k];
      const u64 cap = std::max<u64>(256, next_pow2(2 * p));
      const u32 Bk = std::max<u32>(1, bit_width(bound));
      const LevelTab nt = plan_table(tab.ptr, cap, 2 * (Bk + 3), p, Bk, allow_packed, kMaxProbe);
      hipEvent_t e0{};
      prof_begin(KID_MEMSET, e0);
      HIP_TRY(hipMemsetAsync(tab.ptr, 0xff, nt.bytes(), stream));
      prof_end(KID_MEMSET, e0);
      prof_begin(KID_NODE, e0);
      const dim3 gi(unsigned((p + kBlock - 1) / kBlock));
      if (nt.packed)
        hipLaunchKernelGGL((k_node_insert<PackedTab>), gi, dim3(kBlock), 0, stream, in, n, p, nt.pt, outw, d_hdr);
      else
        hipLaunchKernelGGL((k_node_insert<WideTab>), gi, dim3(kBlock), 0, stream, in, n, p, nt.wt, outw, d_hdr);
      HIP_TRY(hipGetLastError());
      prof_end(KID_NODE, e0);
      prof_begin(KID_FLAGSCAN_NODE, e0);
      const dim3 gs(unsigned((p + kTile - 1) / kTile));
      uint2* out_k = static_cast<uint2*>(nodes_out.ptr) + layer_off[k];
      if (nt.packed)
        hipLaunchKernelGGL((k_flagscan<false, PackedTab>), gs, dim3(kBlock), 0, stream, outw, p, nt.pt, d_grp,
                           d_desc + desc_off[k + 1], &d_hdr->ticket[k + 1], out_k, &d_hdr->count[k + 1]);
      else
        hipLaunchKernelGGL((k_flagscan<false, WideTab>), gs, dim3(kBlock), 0, stream, outw, p, nt.wt, d_grp,
                           d_desc + desc_off[k + 1], &d_hdr->ticket[k + 1], out_k, &d_hdr->count[k + 1]);
      HIP_TRY(hipGetLastError());
      prof_end(KID_FLAGSCAN_NODE, e0);
      prof_begin(KID_RESOLVE, e0);
      hipLaunchKernelGGL(k_resolve, gi, dim3(kBlock), 0, stream, outw, p, d_grp);
      HIP_TRY(hipGetLastError());
      prof_end(KID_RESOLVE, e0);
      std::swap(in, outw);
      n = p;
      bound = p;
    }
    hipLaunchKernelGGL(k_root, dim3(1), dim3(1), 0, stream, in, d_hdr);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ev_stop, stream));
    HIP_TRY(hipMemcpyAsync(h_hdr, d_hdr, sizeof(Header), hipMemcpyDeviceToHost, stream));
    HIP_TRY(hipStreamSynchronize(stream));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, ev_start, ev_stop));
    info.build_ms = ms;
    if (profile) prof_collect();
    // a packed table whose displacement field overflowed: rebuild with wide slots
    if (!(h_hdr->overflow && allow_packed)) break;
  }

  if (h_hdr->err_offset != ~0ull) {
    info.error_offset = h_hdr->err_offset;
    unsigned char sym = 0;
    if (d_bases) HIP_TRY(hipMemcpy(&sym, static_cast<const unsigned char*>(d_bases) + h_hdr->err_offset, 1,
                                   hipMemcpyDeviceToHost));
    info.error_symbol = sym;
    return fail(GCZ_ERR_SYMBOL, "build", "unknown nucleotide symbol");
  }
  if (h_hdr->overflow) return fail(GCZ_ERR_CAPACITY, "build", "hash table probe limit exceeded");
  info.n_layers = D;
  info.n_leaves = h_hdr->count[0];
  // keep the next build's adaptive leaf table at load <= 1/2 (speed only)
  leaf_cap_hint = std::max(leaf_cap_hint, next_pow2(2 * info.n_leaves));
  for (int k = 0; k < D; ++k) info.layer_size[k] = h_hdr->count[k + 1];
  info.root = h_hdr->root;
  return GCZ_OK;
}

extern "C" {

int gcz_ctx_create(int device, gcz_ctx** out) {
  if (!out) return GCZ_ERR_ARG;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return GCZ_ERR_DEVICE;
  if (device < 0 || device >= ndev) return GCZ_ERR_ARG;
  if (hipSetDevice(device) != hipSuccess) return GCZ_ERR_DEVICE;
  auto* c = new gcz_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return GCZ_ERR_DEVICE;
  }
  c->stream = c->own_stream;
  if (const char* t = std::getenv("GCZ_TABLE")) c->force_wide = std::strcmp(t, "wide") == 0;
  *out = c;
  return GCZ_OK;
}

void gcz_ctx_destroy(gcz_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->stream);
  for (DevBuf* b : {&c->wa, &c->wb, &c->grp, &c->desc, &c->tab, &c->leaves_out, &c->nodes_out, &c->hdr, &c->input})
    if (b->ptr) (void)hipFree(b->ptr);
  if (c->h_hdr) (void)hipHostFree(c->h_hdr);
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  if (c->ev_start) (void)hipEventDestroy(c->ev_start);
  if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
  if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
  delete c;
}

int gcz_ctx_set_stream(gcz_ctx* c, void* s) {
  if (!c) return GCZ_ERR_ARG;
  c->stream = s ? static_cast<hipStream_t>(s) : c->own_stream;
  return GCZ_OK;
}
void* gcz_ctx_stream(gcz_ctx* c) { return c ? c->stream : nullptr; }
const char* gcz_ctx_last_error(gcz_ctx* c) { return c ? c->last_error.c_str() : "null context"; }

void* gcz_dev_alloc(gcz_ctx* c, uint64_t bytes) {
  if (!c || hipSetDevice(c->device) != hipSuccess) return nullptr;
  void* p = nullptr;
  return hipMalloc(&p, bytes ? bytes : 1) == hipSuccess ? p : nullptr;
}

int gcz_dev_free(gcz_ctx* c, void* p) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  (void)hipStreamSynchronize(c->stream);
  return hipFree(p) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_memcpy_h2d(gcz_ctx* c, void* dst, const void* src, uint64_t bytes) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->stream) != hipSuccess) return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_memcpy_d2h(gcz_ctx* c, void* dst, const void* src, uint64_t bytes) {
  if (!c) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->stream) != hipSuccess) return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_ctx_sync(gcz_ctx* c) {
  if (!c) return GCZ_ERR_ARG;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_build_device_bases(gcz_ctx* c, const void* d_bases, uint64_t nbases, int L) {
  if (!c || (!d_bases && nbases)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (reinterpret_cast<uintptr_t>(d_bases) & 3) {   // the leaf kernel stages with 4-B loads
    if (int rc = c->ensure(c->input, nbases + 16)) return rc;
    if (hipMemcpyAsync(c->input.ptr, d_bases, nbases, hipMemcpyDeviceToDevice, c->stream) != hipSuccess)
      return c->fail(GCZ_ERR_DEVICE, "gcz_build_device_bases", "realign copy failed");
    d_bases = c->input.ptr;
  }
  return c->build(d_bases, nullptr, nbases, 0, L);
}

int gcz_build_device_leaves(gcz_ctx* c, const uint64_t* d_leaves, uint64_t S, int L) {
  if (!c || (!d_leaves && S)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  return c->build(nullptr, reinterpret_cast<const u64*>(d_leaves), 0, S, L);
}

int gcz_build_host_leaves(gcz_ctx* c, const uint64_t* leaves, uint64_t S, int L) {
  if (!c || (!leaves && S)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (int rc = c->ensure(c->input, S * 8 + 16)) return rc;
  if (S && hipMemcpyAsync(c->input.ptr, leaves, S * 8, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return c->fail(GCZ_ERR_DEVICE, "gcz_build_host_leaves", "H2D copy failed");
  return c->build(nullptr, static_cast<const u64*>(c->input.ptr), 0, S, L);
}

int gcz_build_host_fasta(gcz_ctx* c, const void* fasta, uint64_t nbytes, int L) {
  if (!c || (!fasta && nbytes)) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  const auto* f = static_cast<const uint8_t*>(fasta);
  const bool plain = nbytes == 0 || (f[0] != '>' && f[0] != '\n' && !std::memchr(f, '\n', nbytes));
  std::vector<uint8_t> tmp;
  const uint8_t* bases = f;
  uint64_t nb = nbytes;
  if (!plain) {
    tmp.resize(nbytes);
    nb = gcz_fasta_extract(f, nbytes, tmp.data());
    bases = tmp.data();
  }
  if (int rc = c->ensure(c->input, nb + 16)) return rc;
  if (nb && hipMemcpyAsync(c->input.ptr, bases, nb, hipMemcpyHostToDevice, c->stream) != hipSuccess)
    return c->fail(GCZ_ERR_DEVICE, "gcz_build_host_fasta", "H2D copy failed");
  if (hipStreamSynchronize(c->stream) != hipSuccess)
    return c->fail(GCZ_ERR_DEVICE, "gcz_build_host_fasta", "sync failed");
  return c->build(c->input.ptr, nullptr, nb, 0, L);
}

int gcz_info_get(gcz_ctx* c, gcz_info* out) {
  if (!c || !out) return GCZ_ERR_ARG;
  *out = c->info;
  return GCZ_OK;
}

int gcz_copy_leaves(gcz_ctx* c, uint64_t* host_out) {
  if (!c || !host_out || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  if (c->info.n_leaves &&
      hipMemcpyAsync(host_out, c->leaves_out.ptr, c->info.n_leaves * 8, hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

int gcz_copy_layer(gcz_ctx* c, int k, uint32_t* host_out) {
  if (!c || !host_out || c->info.status != GCZ_OK || k < 0 || k >= c->info.n_layers) return GCZ_ERR_ARG;
  if (hipSetDevice(c->device) != hipSuccess) return GCZ_ERR_DEVICE;
  const u64 n = c->info.layer_size[k];
  if (n && hipMemcpyAsync(host_out, static_cast<uint2*>(c->nodes_out.ptr) + c->layer_off[k], n * 8,
                          hipMemcpyDeviceToHost, c->stream) != hipSuccess)
    return GCZ_ERR_DEVICE;
  return hipStreamSynchronize(c->stream) == hipSuccess ? GCZ_OK : GCZ_ERR_DEVICE;
}

const uint64_t* gcz_device_leaves(gcz_ctx* c) {
  return c && c->info.status == GCZ_OK ? static_cast<const uint64_t*>(c->leaves_out.ptr) : nullptr;
}
const uint32_t* gcz_device_layer(gcz_ctx* c, int k) {
  if (!c || c->info.status != GCZ_OK || k < 0 || k >= c->info.n_layers) return nullptr;
  return reinterpret_cast<const uint32_t*>(static_cast<uint2*>(c->nodes_out.ptr) + c->layer_off[k]);
}

int gcz_tree_fetch(gcz_ctx* c, gcz_tree* t) {
  if (!c || !t || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  t->L = c->info.L;
  t->root = c->info.root;
  t->leaves.resize(c->info.n_leaves);
  if (int rc = gcz_copy_leaves(c, t->leaves.data())) return rc;
  t->layers.assign(c->info.n_layers, {});
  for (int k = 0; k < c->info.n_layers; ++k) {
    t->layers[k].resize(2 * c->info.layer_size[k]);
    if (int rc = gcz_copy_layer(c, k, t->layers[k].data())) return rc;
  }
  return GCZ_OK;
}

int gcz_profile_enable(gcz_ctx* c, int on) {
  if (!c) return GCZ_ERR_ARG;
  c->profile = on != 0;
  return GCZ_OK;
}
int gcz_profile_entry(gcz_ctx* c, int k, const char** name, uint64_t* launches, double* total_ms) {
  if (!c || k < 0 || k >= KID_COUNT) return -1;
  if (name) *name = kKernelNames[k];
  if (launches) *launches = c->prof_launches[k];
  if (total_ms) *total_ms = c->prof_ms[k];
  return 0;
}
void gcz_profile_reset(gcz_ctx* c) {
  if (!c) return;
  for (int k = 0; k < KID_COUNT; ++k) { c->prof_launches[k] = 0; c->prof_ms[k] = 0; }
}

}  // extern "C"
