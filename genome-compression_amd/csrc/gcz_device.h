// Device code of the MI355X (gfx950) shared_tree construction.
// Included by gcz_build.hip only.
//
// Replaces tree_constructor (reference include/shared_tree.h:245-316,
// src/shared_tree.cpp:621-763) with one global level-by-level build; the
// reference's 2^22 / 2^25-strand segmentation is output-invisible.
//
// Per level (n input words -> p = ceil(n/2) pairs; the leaf level has p = S):
//
//   insert    canonical key of each leaf/pair -> open-addressing table in HBM
//             (hash-consing, tree_constructor::emplace_leaf/emplace_node).
//             Records the provisional word rec[j] = slot | m<<29 | t<<30 | v<<31
//             and marks nf[j] = 1 ("not first") for every element that is
//             provably not its key's first occurrence (see Tables below).
//   flagscan  first occurrence <=> nf[j] == 0.  Wave ballot -> 64-element group
//             masks, in-tile scan, decoupled look-back across tiles -> ids are
//             the dense first-occurrence ranks (the reference's parent.node_count
//             at emplace time, shared_tree.cpp:632,666).  First occurrences emit
//             the unique leaf/node at out[id] and write their final word.
//   resolve   non-first occurrences get the id of their key's first occurrence:
//             leaves through the slot, which flagscan settled with the id; nodes
//             through the slot's minimum position -> its group's {mask, prefix}.
//
// The leaf level runs in chunks of strands (insert, flagscan, resolve per
// chunk): a strand whose key was settled by an earlier chunk gets its final
// word straight from the insert probe, so only keys new to a chunk pay for the
// scan and the resolve read.
//
// The next level reads the final words directly (coalesced 8-B pairs).
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

#include <cstdint>
#include <cstdlib>

#include "gcz_internal.h"

namespace gcz_dev {

using u32 = uint32_t;
using u64 = unsigned long long;

constexpr u32 kNullWord = 0x9fffffffu;
constexpr u32 kIdx = 0x1fffffffu;
constexpr u32 kBits = 0xe0000000u;
constexpr u64 kEmpty = ~0ull;
constexpr int kBlock = 256;
constexpr int kItems = 32;                 // flagscan elements per thread on large levels
constexpr int kTile = kBlock * kItems;     // 8192 elements per look-back tile
constexpr int kGroupsPerTile = kTile / 64; // 128
constexpr int kItemsSmall = 8;             // ... on levels below 2^20 elements: more tiles, shorter ones
constexpr int kTileSmall = kBlock * kItemsSmall;
constexpr int kLeafItems = kItems;         // leaf flagscan: most strands are already settled
constexpr int kLeafTile = kBlock * kLeafItems;
// Look-back tile of a scan over n elements: long tiles keep the look-back chain short
// on big levels, short ones keep enough tiles in flight on small ones.
constexpr int kItemsTiny = 1;              // ... and one per thread up to 2^17 (direct prefix, no look-back)
constexpr int kTileTiny = kBlock * kItemsTiny;
inline u64 tiny_tile_max() {   // (GCZ_TINY_MAX overrides, process-wide: every caller sizes alike)
  static const u64 v = [] {
    const char* e = std::getenv("GCZ_TINY_MAX");
    return e ? u64(std::strtoull(e, nullptr, 10)) : u64(1) << 17;
  }();
  return v;
}
inline u64 scan_tile(u64 n) {
  return n >= (1ull << 20) ? u64(kTile) : n > tiny_tile_max() ? u64(kTileSmall) : u64(kTileTiny);
}
constexpr u32 kMaxProbe = 1u << 16;

struct __align__(16) Slot {   // WideTab slot; key stored as key ^ 1 (see WideTab)
  u64 key;
  u32 pos;
  u32 pad;
};

struct __align__(16) Group {
  u64 mask;    // first-occurrence flags of 64 consecutive elements
  u32 prefix;  // first occurrences before this group (global, this level)
  u32 pad;
};

// Scan slots: leaf chunk c uses slot c, node layer k uses slot kLayerSlot + k.
constexpr int kMaxChunks = 64;
constexpr int kLayerSlot = kMaxChunks;
constexpr int kScanSlots = kMaxChunks + GCZ_MAX_LAYERS;

struct Header {
  u64 count[kScanSlots];   // leaf chunk c: unique leaves after chunk c (cumulative); layer k: its uniques
  u32 ticket[kScanSlots];  // look-back tile tickets
  u64 err_offset;          // first unknown symbol (min), ~0 if none
  u64 hashed[64];          // node pairs that went through the table (statistics, sharded)
  u64 gate[GCZ_MAX_LAYERS];  // gate[k] == size of layer k  =>  layer k+1 is direct (see k_resolve_node)
  u32 hashed_next[GCZ_MAX_LAYERS];  // some pair of layer k (k >= 1) has two repeated children
  u64 dupstat[64];         // in-block repeats among the first leaf chunk's strands (sharded)
  u32 predup;              // node inserts pre-dedupe each block in LDS (repetitive data)
  u32 overflow;            // a node-level probe bound was exceeded
  u32 leaf_overflow;       // the (adaptively sized) leaf table was too small
  u32 root;
  u32 bkt_overflow;         // a node-level bucket exceeded the LDS dedupe (k_bkt_dedupe)
  u32 dense_fail;           // a strand is not pure ACGT: the dense leaf level does not apply (gcz_dense.h)
  u32 nnf;                  // two-pass level: its not-first positions (k_bkt_dedupe2), listed up to kNfListCap
  u32 redo[GCZ_MAX_LAYERS]; // level k: buckets the bitmap dedupe handed to k_bkt_dedupe2 (k_bkt_dedupe_bm)
};

// A two-pass level with at most this many repeats (e.g. 13 of 41.7 M pairs on layer 0 of
// 1 Gbase uniform) is ranked without the look-back chain: id = position - repeats before it,
// counted from the dedupe's list (k_flagscan_node's sparse path).
constexpr u32 kNfListCap = 2048;

// ---- word algebra: reference src/shared_tree.cpp:76-107 --------------------
__device__ __forceinline__ u32 ulw(u32 w) { return w & 0x7fffffffu; }   // to_ulong
// transform ctor (shared_tree.cpp:76-80): m' = (M != m) && !v ; t' = (T != t) && !null
__device__ __forceinline__ u32 xf(u32 w, u32 M, u32 T) {
  const u32 v = w >> 31, m = (w >> 29) & 1u, t = (w >> 30) & 1u;
  const u32 nm = (M ^ m) & (v ^ 1u);
  const u32 nt = (T ^ t) & u32(ulw(w) != kIdx);
  return (w & 0x9fffffffu) | (nm << 29) | (nt << 30);
}
__device__ __forceinline__ u32 make_word(u32 idx, u32 m, u32 t, u32 v) {   // ctor :85-86
  return idx | ((m & (v ^ 1u)) << 29) | (t << 30) | (v << 31);
}

// node::canonical (include/shared_tree.h:115-126): min over (key, m, t) of
// id=(l,r) mir=(M(r),M(l)) tra=(T(l),T(r)) inv=(I(r),I(l)); key = to_ulong pair.
__device__ __forceinline__ void node_canonical(u32 l, u32 r, u32& cl, u32& cr, u32& cm, u32& ct) {
  const u32 ml = xf(l, 1, 0), mr = xf(r, 1, 0);
  const u32 tl = xf(l, 0, 1), tr = xf(r, 0, 1);
  const u32 il = xf(l, 1, 1), ir = xf(r, 1, 1);
  // (key << 2 | m << 1 | t): the 62-bit key with (m,t) appended is one compare
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
  if (c < best) { cl = ir; cr = il; cm = 1; ct = 1; }
}

// ---- leaf codec: reference src/dna.cpp:104-143 ------------------------------
__device__ __forceinline__ u64 leaf_transposed(u64 v) {
  v = ((v >> 1) & 0x5555555555555555ull) | ((v & 0x5555555555555555ull) << 1);
  v = ((v >> 2) & 0x3333333333333333ull) | ((v & 0x3333333333333333ull) << 2);
  return v;
}
// reverse the low L nibbles, higher nibbles dropped (dna::mirrored :116-121)
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

// nac code of an ASCII byte, include/dna.h:20-32 (to_nac, src/dna.cpp:25-49); -1 unknown
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

// ---- hash tables ---------------------------------------------------------------
// Both tables map a canonical key to (slot, minimum position) and, as a side
// effect of the insert, mark every element that is provably NOT the first
// occurrence of its key:
//   * an element that sees its key already holding a smaller position marks
//     itself;
//   * an element that lowers the slot's position marks the element it
//     displaced (the returning atomicMin tells which);
// the slot's position sequence is decreasing, so exactly the final minimum
// (the first occurrence) stays unmarked.  Unique keys cost one CAS.
//
// PackedTab (default): one 8-B word per slot,
//     word = quotient(h) << (D+P) | displacement << P | pos
// h = mix(key) is a bijection on the K key bits; the home slot is h's low c
// bits, the quotient its high K-c bits.  The claiming CAS also stores the
// position; repeats share the high bits, so a 64-bit atomicMin lowers pos.
// The key is recovered exactly from (slot, word) by inverting the mix.
//
// WideTab (fallback: keys that do not pack, e.g. L = 16 leaves): 16-B slots
// {key ^ 1, pos}; CAS on the key then atomicMin on pos.  key ^ 1 == ~0 would
// need key 0xffff_ffff_ffff_fffe, which is never canonical (its transpose
// ..fff7 is smaller, dna.cpp:135-143) and never a node key (left word with
// both mirror and invariant bits, which the pointer ctor forbids).
//
// Probes read the slot with a plain load first; it may be stale (this CU's L1
// or this XCD's L2), but slots only go EMPTY -> claimed and positions only
// decrease, so staleness costs at most an extra CAS / atomicMin.

__device__ __forceinline__ u32 slot_hash(u64 k) {
  k ^= k >> 31;
  k *= 0x7fb5d329728ea185ull;
  k ^= k >> 27;
  k *= 0x81dadef4bc2dd44dull;
  k ^= k >> 33;
  return u32(k);
}

// pointer word -> B+2 bits: index code, mirror, transpose.  The invariant bit is left out:
// it is a property of the child's id (src/shared_tree.cpp:670 gives every occurrence of a key
// the same value), so keys stay distinct -- the same to_ulong key as node::operator==.
__device__ __forceinline__ u32 enc_child(u32 w, u32 B) {
  const u32 idx = w & kIdx;
  const u32 code = idx == kIdx ? ((1u << B) - 1u) : idx;      // null index -> all-ones code
  return (code << 2) | (((w >> 29) & 1u) << 1) | ((w >> 30) & 1u);
}

// not-first marks: 0 = maybe first, 1 = not first (resolve through the slot),
// 2 = key settled by an earlier leaf chunk (final word already written)
// 3 = multi-rank leaf level: the key was seeded with its GLOBAL id (rank 0's dictionary,
// gcz_dist.hip), the word already holds the final id
constexpr unsigned char kNfMaybe = 0, kNfNot = 1, kNfDone = 2, kNfGlobal = 3;
// 4 = a node pair collapsed onto an earlier repeat of its key in the same 4096-pair block of
// the bucketed partition (k_bkt_part on repetitive data); its word holds that position until
// the flag scan points it at the key's first occurrence
constexpr unsigned char kNfDup = 4;
__device__ __forceinline__ void mark(unsigned char* nf, u32 pos) { nf[pos] = kNfNot; }

// Marks of one level: nf (not first) and, on node levels, multi (the key has
// more than one occurrence).  When an insert learns of another occurrence
// `other` of its key, the later of the two positions is not first and the
// earlier one is multi.  The final minimum is always marked multi when its
// key repeats: either it lowered the slot from another position (and marks
// itself), or it claimed the slot and every later occurrence finds it there.
struct Marks {
  unsigned char* nf;
  unsigned char* multi;   // null on the leaf level (not tracked)
};
__device__ __forceinline__ void mark_dup(const Marks& mk, u32 self, u32 other) {
  if (other < self) {
    mk.nf[self] = kNfNot;
    if (mk.multi) mk.multi[other] = 1;
  } else {
    mk.nf[other] = kNfNot;
    if (mk.multi) mk.multi[self] = 1;
  }
}

// Result of a leaf-chunk insert: the slot, or the settled id of the key.
struct Ins {
  u32 slot;
  u32 id;      // valid when settled
  bool settled;
  bool global = false;   // settled with a global id (seeded)
};

struct WideTab {
  Slot* tab;
  u32 mask;
  u32 limit;
  u32 B;   // unused

  __device__ __forceinline__ u64 node_key(u32 cl, u32 cr) const { return (u64(cl) << 32) | cr; }
  __device__ __forceinline__ u32 insert(u64 key, u32 pos, const Marks& mk, u32* __restrict__ ovf) const {
    const u64 skey = key ^ 1ull;
    u32 s = slot_hash(skey) & mask;
    for (u32 probe = 0; probe < limit; ++probe) {
      const Slot cur = tab[s];
      u64 k = cur.key;
      if (k == kEmpty) {
        k = atomicCAS(&tab[s].key, kEmpty, skey);
        if (k == kEmpty) {                       // claimed: now lower pos from EMPTY
          const u32 old = atomicMin(&tab[s].pos, pos);
          if (old != ~0u) mark_dup(mk, pos, old);
          return s;
        }
      }
      if (k == skey) {
        if (cur.pos < pos) { mark_dup(mk, pos, cur.pos); return s; }
        const u32 old = atomicMin(&tab[s].pos, pos);
        if (old != ~0u) mark_dup(mk, pos, old);
        return s;
      }
      s = (s + 1) & mask;
    }
    atomicOr(ovf, 1u);
    return 0;
  }
  __device__ __forceinline__ void read(u32 s, u64& key, u32& pos) const {
    const Slot sl = tab[s];
    key = sl.key ^ 1ull;
    pos = sl.pos;
  }
  // Leaf chunks: a slot whose key's first occurrence lies in an earlier chunk
  // carries its final id in pad (0xffffffff until settled).
  __device__ __forceinline__ Ins insert_chunk(u64 key, u32 pos, const Marks& mk,
                                              u32* __restrict__ ovf) const {
    const u64 skey = key ^ 1ull;
    u32 s = slot_hash(skey) & mask;
    for (u32 probe = 0; probe < limit; ++probe) {
      const Slot cur = tab[s];
      if (cur.key == skey && cur.pad != ~0u) return {s, cur.pad, true};
      if (cur.key == kEmpty || cur.key == skey) return {insert(key, pos, mk, ovf), 0, false};
      s = (s + 1) & mask;
    }
    atomicOr(ovf, 1u);
    return {0, 0, false};
  }
  __device__ __forceinline__ void settle(u32 s, u32 id) const { tab[s].pad = id; }
  __device__ __forceinline__ u32 settled_id(u32 s) const { return tab[s].pad; }
};

struct PackedTab {
  u64* tab;
  u32 mask;
  u32 limit;   // <= 2^D - 2 probes
  u32 B;       // child index bits (node levels)
  u32 c, P, D, sh;
  u32 cas_first;   // probe the home slot with the CAS itself (sparse small-build tables: one round trip)
  u64 kmask, c1, c2, c1i, c2i;

  __device__ __forceinline__ u64 node_key(u32 cl, u32 cr) const {
    return (u64(enc_child(cl, B)) << (B + 2)) | enc_child(cr, B);
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
  __device__ __forceinline__ u32 insert(u64 key, u32 pos, const Marks& mk, u32* __restrict__ ovf) const {
    const u64 h = mix(key);
    u32 s = u32(h) & mask;
    const u64 qd = (h >> c) << D;             // quotient; displacement bits below
    const u64 pmask = (1ull << P) - 1;
    for (u32 d = 0; d < limit; ++d) {
      const u64 mine = ((qd | d) << P) | pos;
      u64 cur = d == 0 && cas_first ? kEmpty : tab[s];
      if (cur == kEmpty) {
        cur = atomicCAS(&tab[s], kEmpty, mine);
        if (cur == kEmpty) return s;            // new key: one atomic, nothing to mark
      }
      if ((cur >> P) == (mine >> P)) {
        if (u32(cur & pmask) < pos) { mark_dup(mk, pos, u32(cur & pmask)); return s; }
        const u64 old = atomicMin(&tab[s], mine);
        mark_dup(mk, pos, u32(old & pmask));
        return s;
      }
      s = (s + 1) & mask;
    }
    atomicOr(ovf, 1u);
    return 0;
  }
  __device__ __forceinline__ void read(u32 s, u64& key, u32& pos) const {
    const u64 w = tab[s] & ~(kSettled | kGlobal);
    pos = u32(w & ((1ull << P) - 1));
    const u32 d = u32((w >> P) & ((1ull << D) - 1));
    const u64 q = w >> (P + D);
    const u64 home = (s - d) & mask;
    key = unmix((q << c) | home);
  }
  // Leaf chunks (needs Q + D + P <= 63): a settled slot keeps its key bits and
  // holds the final id in the position field, with bit 63 set.
  static constexpr u64 kSettled = 1ull << 63;
  static constexpr u64 kGlobal = 1ull << 62;   // settled by seed(): the id is global (needs K + 2)
  __device__ __forceinline__ Ins insert_chunk(u64 key, u32 pos, const Marks& mk,
                                              u32* __restrict__ ovf) const {
    const u64 h = mix(key);
    u32 s = u32(h) & mask;
    const u64 qd = (h >> c) << D;
    const u64 pmask = (1ull << P) - 1;
    for (u32 d = 0; d < limit; ++d) {
      const u64 mine = ((qd | d) << P) | pos;
      u64 cur = d == 0 && cas_first ? kEmpty : tab[s];
      if (cur == kEmpty) {
        cur = atomicCAS(&tab[s], kEmpty, mine);
        if (cur == kEmpty) return {s, 0, false};
      }
      if (((cur & ~(kSettled | kGlobal)) >> P) == (mine >> P)) {
        if (cur & kSettled) return {s, u32(cur & pmask), true, (cur & kGlobal) != 0};
        if (u32(cur & pmask) < pos) { mark_dup(mk, pos, u32(cur & pmask)); return {s, 0, false}; }
        const u64 old = atomicMin(&tab[s], mine);
        mark_dup(mk, pos, u32(old & pmask));
        return {s, 0, false};
      }
      s = (s + 1) & mask;
    }
    atomicOr(ovf, 1u);
    return {0, 0, false};
  }
  __device__ __forceinline__ void settle(u32 s, u32 id) const {
    tab[s] = kSettled | (tab[s] & ~((1ull << P) - 1)) | id;
  }
  // Multi-rank leaf level: a key of rank 0's dictionary enters a fresh table settled with
  // its global id, so this rank's strands of that key take the final word from the probe.
  __device__ __forceinline__ void seed(u64 key, u32 id, u32* __restrict__ ovf) const {
    const u64 h = mix(key);
    u32 s = u32(h) & mask;
    const u64 qd = (h >> c) << D;
    for (u32 d = 0; d < limit; ++d) {
      const u64 mine = kSettled | kGlobal | ((qd | d) << P) | id;
      const u64 cur = atomicCAS(&tab[s], kEmpty, mine);
      if (cur == kEmpty) return;   // dictionary keys are distinct: never found, only placed
      s = (s + 1) & mask;
    }
    atomicOr(ovf, 1u);
  }
  __device__ __forceinline__ u32 settled_id(u32 s) const { return u32(tab[s] & ((1ull << P) - 1)); }
};

// ---- insert kernels -----------------------------------------------------------

// Leaf level from raw bases: pack L symbols (dna::dna(string_view) + dna::set,
// dna.cpp:79-84,187-197), canonicalise (:135-143), hash-cons (emplace_leaf,
// shared_tree.cpp:630-637).  The block's bases are staged through LDS with
// coalesced 4-B loads.
// Strands [i0, i1) of the current leaf chunk; i0 is a multiple of kBlock.
template <int L, class Tab>
__global__ __launch_bounds__(kBlock) void k_leaf_bases(const unsigned char* __restrict__ bases, u64 i0, u64 i1,
                                                      Tab T, u32* __restrict__ rec, unsigned char* __restrict__ nf,
                                                      Header* __restrict__ hdr, u64* __restrict__ lkey) {
  __shared__ signed char lut[256];
  __shared__ __align__(16) unsigned char buf[L % 4 == 0 ? 16 : kBlock * L + 16];
  const int tid = threadIdx.x;
  lut[tid] = (signed char)nac_code(tid);
  const u64 first = i0 + u64(blockIdx.x) * kBlock;
  const u64 nstr = (i1 - first) < u64(kBlock) ? (i1 - first) : u64(kBlock);
  u64 x = 0;
  int bad = -1;
  if constexpr (L % 4 == 0) {   // a strand is L / 4 aligned words: the wave's loads are contiguous
    u32 wv[L / 4];
    if (u64(tid) < nstr) {
      const u32* src = reinterpret_cast<const u32*>(bases + (first + tid) * L);
#pragma unroll
      for (int q = 0; q < L / 4; ++q) wv[q] = src[q];
    }
    __syncthreads();   // (the table; the loads are in flight)
    if (u64(tid) >= nstr) return;
#pragma unroll
    for (int c = 0; c < L; ++c) {
      const int code = lut[(wv[c / 4] >> (8 * (c % 4))) & 0xffu];
      if (code < 0 && bad < 0) bad = c;
      x |= u64(code & 15) << (4 * c);
    }
  } else {   // staged through LDS (coalesced 4-B loads of the block's bytes)
    const u64 byte0 = first * L;                 // multiple of 4 (kBlock = 256)
    const u64 nbytes = nstr * L;
    const u32* src = reinterpret_cast<const u32*>(bases + byte0);
    u32* dst = reinterpret_cast<u32*>(buf);
    const u32 nwords = u32(nbytes / 4);
    if (nstr == u64(kBlock)) {   // full block: L / 4 words per thread, all loads in flight at once
      constexpr int kW = (L + 3) / 4;
      u32 v[kW];
#pragma unroll
      for (int q = 0; q < kW; ++q) {
        const u32 w = u32(q) * kBlock + tid;
        v[q] = w < nwords ? src[w] : 0u;
      }
#pragma unroll
      for (int q = 0; q < kW; ++q) {
        const u32 w = u32(q) * kBlock + tid;
        if (w < nwords) dst[w] = v[q];
      }
    } else {
      for (u32 w = tid; w < nwords; w += kBlock) dst[w] = src[w];
      for (u32 b = nwords * 4 + tid; b < nbytes; b += kBlock) buf[b] = bases[byte0 + b];
    }
    __syncthreads();
    if (u64(tid) >= nstr) return;
#pragma unroll
    for (int c = 0; c < L; ++c) {
      const int code = lut[buf[tid * L + c]];
      if (code < 0 && bad < 0) bad = c;
      x |= u64(code & 15) << (4 * c);
    }
  }
  const u64 i = first + tid;
  if (bad >= 0) atomicMin(&hdr->err_offset, i * L + u64(bad));
  u32 m, t, v;
  const u64 key = leaf_canonical(x, L, m, t, v);
  if (lkey) lkey[i] = key;   // (fused small build: the flag scan emits first occurrences from it)
  const Ins r = T.insert_chunk(key, u32(i), Marks{nf, nullptr}, &hdr->leaf_overflow);
  if (r.settled) nf[i] = r.global ? kNfGlobal : kNfDone;
  rec[i] = make_word(r.settled ? r.id : r.slot, m, t, v);
}

[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_leaf_seed(const u64* __restrict__ dict, u64 n, PackedTab T,
                                                             u32* __restrict__ ovf) {
  const u64 d = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (d < n) T.seed(dict[d], u32(d), ovf);
}

// In-block repeats of the first leaf chunk (equal provisional slot words mean equal
// keys): the statistic that switches the node inserts' LDS pre-dedupe on.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_dup_probe(const u32* __restrict__ rec, u64 i0,
                                                                              u64 i1, Header* __restrict__ hdr) {
  __shared__ u32 s_k[2 * kBlock];
  __shared__ u32 s_n;
  for (int q = threadIdx.x; q < 2 * kBlock; q += kBlock) s_k[q] = ~0u;
  if (threadIdx.x == 0) s_n = 0;
  __syncthreads();
  const u64 i = i0 + u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i < i1) {
    const u32 w = rec[i] & kIdx;
    u32 h = (w * 2654435761u) >> 23;   // 9 bits
    for (;;) {
      u32 c = s_k[h];
      if (c == ~0u) c = atomicCAS(&s_k[h], ~0u, w);
      if (c == w && c != ~0u) { atomicAdd(&s_n, 1u); break; }
      if (c == ~0u) break;
      h = (h + 1) & (2 * kBlock - 1);
    }
  }
  __syncthreads();
  if (threadIdx.x == 0 && s_n) atomicAdd(&hdr->dupstat[blockIdx.x & 63], u64(s_n));
}

[[maybe_unused]] static __global__ void k_dup_decide(Header* __restrict__ hdr, u64 sampled, u32 force) {
  u64 d = 0;
  for (int q = 0; q < 64; ++q) d += hdr->dupstat[q];
  hdr->predup = force == 1 ? 1u : force == 2 ? 0u : u32(d * 20 > sampled);   // > 5 % in-block repeats
}

// Leaf level from packed strands (shared_tree(std::vector<dna>&), :212-215).
template <class Tab>
__global__ __launch_bounds__(kBlock) void k_leaf_packed(const u64* __restrict__ leaves, u64 i0, u64 i1, int L,
                                                       Tab T, u32* __restrict__ rec, unsigned char* __restrict__ nf,
                                                       Header* __restrict__ hdr, u64* __restrict__ lkey) {
  const u64 i = i0 + u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= i1) return;
  u32 m, t, v;
  const u64 key = leaf_canonical(leaves[i], L, m, t, v);
  if (lkey) lkey[i] = key;
  const Ins r = T.insert_chunk(key, u32(i), Marks{nf, nullptr}, &hdr->leaf_overflow);
  if (r.settled) nf[i] = r.global ? kNfGlobal : kNfDone;
  rec[i] = make_word(r.settled ? r.id : r.slot, m, t, v);
}

// Pair (2j, 2j+1) of the previous level's final words; the odd tail pairs with
// the null pointer (foreach_pair, include/utility.h:17-29).
__device__ __forceinline__ void load_pair(const u32* __restrict__ in, u64 n, u64 j, u32& l, u32& r) {
  if (2 * j + 1 < n) {
    const uint2 w = reinterpret_cast<const uint2*>(in)[j];
    l = w.x; r = w.y;
  } else {
    l = in[2 * j]; r = kNullWord;
  }
}

// Reader-buffer segments (gcz_build_*_fasta_buffered): the reference reduces every
// fasta_reader buffer of B strands to its own subtree, pairing inside the buffer only and an
// odd buffer's last element with null, before it combines the roots
// (src/shared_tree.cpp:719-736, reduce_segment include/shared_tree.h:305-316).  At a node
// level whose full segments hold an odd number Bk of input elements, this copies the level's
// input with a null element after every segment but the last, so that the ordinary (2j, 2j+1)
// pairing of the copy pairs exactly like the reference.  The null slots are marked as repeated
// (not singletons), so a pair (x, null) is hash-consed unless x itself is a singleton.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_seg_expand(const u32* __restrict__ in, const unsigned char* __restrict__ nf,
                                                       const unsigned char* __restrict__ mu, u64 Bk, u64 nout,
                                                       u32* __restrict__ out, unsigned char* __restrict__ onf,
                                                       unsigned char* __restrict__ omu) {
  const u64 o = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (o >= nout) return;
  const u64 s = o / (Bk + 1), q = o - s * (Bk + 1);
  if (q == Bk) {
    out[o] = kNullWord;
    if (onf) {
      onf[o] = kNfNot;
      omu[o] = 1;
    }
  } else {
    const u64 i = s * Bk + q;
    out[o] = in[i];
    if (onf) {
      onf[o] = nf[i];
      omu[o] = mu[i];
    }
  }
}

// Node level, tree_constructor::emplace_node (src/shared_tree.cpp:662-672).
//
// Singleton propagation: a previous-level element that is the only occurrence
// of its key (first, not multi) is referenced by exactly one input word, so
// every symmetry variant of a pair containing it contains that one word: the
// pair's key cannot occur anywhere else.  Such pairs skip the table entirely
// (first occurrence, only occurrence); only pairs of two repeated children
// are hash-consed.  prev_nf/prev_multi are null when the children are leaves
// (not tracked).
//
// Direct levels: when every element of the previous level is the only
// occurrence of its key (its unique count equals its size), every pair of
// this level is too, so ids are positions: the insert writes the final word
// and the unique node itself, and flagscan/resolve/clear of the level exit.
__device__ __forceinline__ bool level_direct(const u64* prev_count, u64 prev_n) {
  return prev_count && *prev_count == prev_n;
}

// Hashed-pair statistics: one atomic per block into 1024 shards, one 64-B line each
// (a handful of shared counters serialises ~10^5 block atomics: +0.3 ms on layer 0).
constexpr int kStatShards = 1024, kStatStride = 8;
constexpr size_t kStatBytes = size_t(kStatShards) * kStatStride * 8;

[[maybe_unused]] static __global__ __launch_bounds__(1024) void k_stats_sum(const u64* __restrict__ shards, u64* __restrict__ out) {
  __shared__ u64 s_sum[1024 / 64];
  u64 v = shards[threadIdx.x * kStatStride];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) s_sum[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 t = 0;
    for (int w = 0; w < 1024 / 64; ++w) t += s_sum[w];
    *out = t;
  }
}

// Build start in one launch (instead of a memset per buffer): the header (zero, the
// error offset ~0), the look-back descriptors, the statistics shards and, when the
// hash-table leaf level runs, its table (0xff) and not-first marks.
struct InitPlan {
  Header* hdr;
  uint4* desc;  u64 ndesc16;
  uint4* stats; u64 nstats16;
  uint4* tab;   u64 ntab16;     // 0xff
  uint4* nf;    u64 nnf16;
  // fused small-build levels: the first node level's table (ones) and marks (zero)
  uint4* ftab;  u64 nftab16;
  uint4* fnf;   uint4* fmulti; u64 nfm16;
  // further zeroed regions (the fused multi-rank schedule's header, look-back words and C / D
  // slots: no memset launch each)
  uint4* zero[4]; u64 nzero16[4];
};

[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_build_init(InitPlan ip) {
  const u64 t = u64(blockIdx.x) * kBlock + threadIdx.x, st = u64(gridDim.x) * kBlock;
  if (blockIdx.x == 0) {
    u32* h = reinterpret_cast<u32*>(ip.hdr);
    constexpr u32 nw = sizeof(Header) / 4, e0 = offsetof(Header, err_offset) / 4;
    for (u32 i = threadIdx.x; i < nw; i += kBlock) h[i] = (i == e0 || i == e0 + 1) ? ~0u : 0u;
  }
  const uint4 z = make_uint4(0, 0, 0, 0), f = make_uint4(~0u, ~0u, ~0u, ~0u);
  for (u64 i = t; i < ip.ndesc16; i += st) ip.desc[i] = z;
  for (u64 i = t; i < ip.nstats16; i += st) ip.stats[i] = z;
  for (u64 i = t; i < ip.ntab16; i += st) ip.tab[i] = f;
  for (u64 i = t; i < ip.nnf16; i += st) ip.nf[i] = z;
  for (u64 i = t; i < ip.nftab16; i += st) ip.ftab[i] = f;
  for (u64 i = t; i < ip.nfm16; i += st) {
    ip.fnf[i] = z;
    ip.fmulti[i] = z;
  }
#pragma unroll
  for (int k = 0; k < 4; ++k)
    for (u64 i = t; i < ip.nzero16[k]; i += st) ip.zero[k][i] = z;
}

// Build end in one launch: the root word (when the level loop, not k_tail, ended the
// build) and the two hashed-pair statistics.
// The build's statistics shards summed into hdr->hashed by a 1024-thread block (k_build_finish,
// or k_tail when it ends the build); v0/v1 are this thread's shard pair, loaded early.
__device__ __forceinline__ void stats_sum(u64 v0, u64 v1, Header* __restrict__ hdr) {
  __shared__ u64 s_sum[2][1024 / 64];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    v0 += __shfl_xor(v0, o, 64);
    v1 += __shfl_xor(v1, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    s_sum[0][threadIdx.x >> 6] = v0;
    s_sum[1][threadIdx.x >> 6] = v1;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    u64 a = 0, b = 0;
    for (int w = 0; w < 1024 / 64; ++w) {
      a += s_sum[0][w];
      b += s_sum[1][w];
    }
    hdr->hashed[0] = a;
    hdr->hashed[1] = b;
  }
}

[[maybe_unused]] static __global__ __launch_bounds__(1024) void k_build_finish(const u32* __restrict__ root_word,
                                                                               const u64* __restrict__ shards,
                                                                               Header* __restrict__ hdr) {
  stats_sum(shards[threadIdx.x * kStatStride], shards[threadIdx.x * kStatStride + 1], hdr);
  if (threadIdx.x == 0 && root_word) hdr->root = root_word[0];
}

// ---- fused small-build levels --------------------------------------------------------
// Small builds (no bucketed level, no host look at the gates) run each node level as two
// launches instead of four: the insert of level k settles level k-1's repeats itself (the
// resolve: a not-first child word takes its key's first id, which level k-1's flag scan
// left by table slot) and writes the final words back into its input; the insert of
// level k clears level k+1's table (three rotating regions: level k-1's is still read)
// and the flag scan of level k clears level k+1's marks (the parity set level k's insert
// read last).  The previous level's gate is decided by the insert from its count and
// look-ahead flag (block 0 stores it for the launches behind).
struct NoRes {
  static constexpr bool kOn = false;
  const unsigned char* nf = nullptr;
  __device__ __forceinline__ u32 operator()(unsigned char, u32 w) const { return w; }
};
// k_resolve_leaf's / k_resolve_node's rule with the ids by slot (k_flagscan_leaf's lsid,
// k_flagscan_node's sid): a not-first word holds its key's slot
struct SlotRes {
  static constexpr bool kOn = true;
  const unsigned char* nf;   // the previous level's not-first marks
  const u32* sid;
  __device__ __forceinline__ u32 operator()(unsigned char f, u32 w) const {   // f = the word's mark
    return f == kNfNot ? sid[w & kIdx] | (w & kBits) : w;
  }
};
struct FuseIn {
  const u64* pcount = nullptr;     // previous level's unique count (null: not fused, use prev_count)
  const u32* phashed = nullptr;    // ... and its look-ahead flag
  u64* gate_out = nullptr;         // where the previous level's gate goes
  uint4* clear = nullptr;          // the table of the level after this one: filled with ones
  u64 clear16 = 0;
};

template <class Tab, class Res>
__global__ __launch_bounds__(kBlock) void k_node_insert(u32* __restrict__ in, u64 n, u64 p, Tab T,
                                                       const unsigned char* __restrict__ prev_nf,
                                                       const unsigned char* __restrict__ prev_multi,
                                                       u32* __restrict__ rec, Marks mk,
                                                       Header* __restrict__ hdr, const u64* prev_count,
                                                       uint2* __restrict__ out, u64* __restrict__ count_out,
                                                       u32 id_off, u64* __restrict__ stats, u32 bkt, Res res,
                                                       FuseIn fz) {
  if (fz.clear) {
    const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u);
    for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < fz.clear16; i += u64(gridDim.x) * kBlock)
      fz.clear[i] = ones;
  }
  // k_bkt_* insert this level (bkt 2: the two-pass partition, on any data; 1: the single pass,
  // on non-repetitive data only)
  if (bkt && !level_direct(prev_count, n) && (bkt == 2 || hdr->predup == 0)) return;
  // every load that depends on nothing goes out first: the pair, the previous level's
  // marks of its two children, the gate inputs
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  const bool two = 2 * j + 1 < n;
  u32 l = kNullWord, r = kNullWord;
  uchar2 f = make_uchar2(0, 0), g = make_uchar2(0, 0);   // (nf, multi) of 2j in .x, of 2j + 1 in .y
  const unsigned char* fnf = Res::kOn ? res.nf : prev_nf;
  if (j < p) {
    load_pair(in, n, j, l, r);
    if (fnf) f = two ? reinterpret_cast<const uchar2*>(fnf)[j] : make_uchar2(fnf[2 * j], 0);
    if (prev_nf) g = two ? reinterpret_cast<const uchar2*>(prev_multi)[j] : make_uchar2(prev_multi[2 * j], 0);
  }
  bool direct;
  if (fz.pcount) {
    direct = *fz.pcount == n || *fz.phashed == 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) *fz.gate_out = direct ? n : ~0ull;
  } else {
    direct = level_direct(prev_count, n);
  }
  if constexpr (Res::kOn) {   // settle the previous level's repeats; the final words go back
    if (j < p) {
      const u32 l2 = res(f.x, l), r2 = two ? res(f.y, r) : r;
      if (l2 != l || r2 != r) {
        if (two) reinterpret_cast<uint2*>(in)[j] = make_uint2(l2, r2);
        else in[2 * j] = l2;
      }
      l = l2;
      r = r2;
    }
  }
  if (direct) {
    if (j == 0) *count_out = p;
    if (j >= p) return;
    u32 cl, cr, m, t;
    node_canonical(l, r, cl, cr, m, t);
    const u32 v = ulw(l) == ulw(xf(r, 1, 0));
    uint2 w;
    w.x = cl; w.y = cr;
    out[j] = w;
    rec[j] = make_word(u32(j) + id_off, m, t, v);   // id_off: first pair of this rank (multi-rank build)
    return;
  }
  // Repetitive data (hdr->predup, decided from the first leaf chunk): repeats of a
  // key inside the block collapse onto its earliest position first, in an LDS
  // table; only that representative touches the HBM table, the others are not
  // first (an earlier position holds their key) and take its slot, and the
  // representative is marked multi.  Output-invisible: the same marks and slots
  // the global inserts would have produced.
  __shared__ u32 s_hashed;
  __shared__ unsigned long long s_key[2 * kBlock];
  __shared__ u32 s_pos[2 * kBlock];
  __shared__ u32 s_slot[2 * kBlock];
  __shared__ u32 s_dup[2 * kBlock];
  const bool pre = hdr->predup != 0;
  if (threadIdx.x == 0) s_hashed = 0;
  if (pre)
    for (int q = threadIdx.x; q < 2 * kBlock; q += kBlock) {
      s_key[q] = kEmpty;
      s_pos[q] = ~0u;
      s_dup[q] = 0;
    }
  __syncthreads();
  bool single = true;
  u32 m = 0, t = 0, v = 0, ls = 0;
  u64 key = 0;
  if (j < p) {
    u32 cl, cr;
    node_canonical(l, r, cl, cr, m, t);
    v = ulw(l) == ulw(xf(r, 1, 0));      // left == right.mirrored() (:670)
    single = false;
    if (prev_nf) single = (f.x == 0 && g.x == 0) || (two && f.y == 0 && g.y == 0);
    key = T.node_key(cl, cr);
    if (pre && !single) {
      u32 h = slot_hash(key) & (2 * kBlock - 1);
      for (;;) {
        unsigned long long c = s_key[h];
        if (c == kEmpty) c = atomicCAS(&s_key[h], kEmpty, (unsigned long long)key);
        if (c == key) s_dup[h] = 1;                 // another position of the block holds it
        if (c == kEmpty || c == key) break;
        h = (h + 1) & (2 * kBlock - 1);
      }
      atomicMin(&s_pos[h], u32(j));
      ls = h;
    }
  }
  if (pre) __syncthreads();
  const bool rep = !pre || single || s_pos[ls] == u32(j);
  u32 s = 0;
  if (j < p && !single && rep) {
    s = T.insert(key, u32(j), mk, &hdr->overflow);
    if (pre) {
      s_slot[ls] = s;
      if (s_dup[ls]) mk.multi[j] = 1;
    }
  }
  if (pre) __syncthreads();
  if (j < p && !single && !rep) {
    s = s_slot[ls];
    mk.nf[j] = kNfNot;
  }
  if (j < p) rec[j] = make_word(s, m, t, v);
  // statistics: pairs hashed, one LDS add per wave, one sharded global add per block
  const u64 hb = __ballot(j < p && !single && rep);
  if ((threadIdx.x & 63) == 0 && hb) atomicAdd(&s_hashed, u32(__popcll(hb)));
  __syncthreads();
  if (threadIdx.x == 0 && s_hashed) atomicAdd(&stats[(blockIdx.x & (kStatShards - 1)) * kStatStride], u64(s_hashed));
}

// ---- flag scan ------------------------------------------------------------------

// Workgroup barrier that waits for LDS operations only (__syncthreads also drains the wave's
// outstanding global loads and stores: vmcnt(0)), for loops that exchange data through LDS
// while their global loads for the next step are in flight.
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ u64 wave_sum(u64 v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

constexpr u64 kStA = 1ull << 62;   // tile aggregate published
constexpr u64 kStP = 2ull << 62;   // tile inclusive prefix published
constexpr u64 kValMask = (1ull << 62) - 1;

// Shared part of both flagscan kernels: takes a tile ticket (tiles are
// processed in ticket order, so every predecessor is resident), reads the
// not-first marks, ballots 64-element groups, scans them within the tile and
// across tiles by decoupled look-back.  On return s_pre[g] holds the number
// of first occurrences before group g of the tile (global), mask[e] the
// group masks of this thread's wave, and the level total is in *count_out.
// The look-back descriptor is one 64-bit word (status | value), so it needs
// no separate payload and no fences (relaxed agent-scope atomics).
template <int ITEMS>
struct TileScan {
  u64 base;
  u64 mask[ITEMS];
};

// Elements are positions [j0, p) of the level (j0 > 0 for later leaf chunks);
// ids start at id0.  ts.base is the first position of the tile.
//
// desc == null (small levels, p <= kSmallScanMax): no look-back chain; every tile
// counts the first occurrences before it directly from the marks (16-B loads of
// [j0, base), zero bytes counted by a SWAR test), so no tile waits for another.
// The reads total p^2 / (2 * tile) bytes: a few MB at most.
constexpr unsigned long long kSmallScanMax = 1ull << 17;

__device__ __forceinline__ u32 zero_bytes(u32 x) {   // bytes of x equal to 0 (= kNfMaybe)
  const u32 t = ((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x;
  return u32(__popc(~t & 0x80808080u));
}

struct NoPrefetch {
  __device__ __forceinline__ void operator()() const {}
};

// Tile prefixes ahead of a scan (the alternative to the look-back chain on large levels):
// block t counts the first occurrences (zero marks) of tile t of T = kBlock * ITEMS positions,
// and the last block to finish turns the counts into exclusive prefixes tpre[t] (and resets
// the done counter for the next level).
// (nfl / nnf / dup_flag: the flag scan's sparse path will run instead -- nothing to count)
template <int ITEMS>
__global__ __launch_bounds__(kBlock) void k_tile_count(const unsigned char* __restrict__ nf, u64 p,
                                                       const u64* prev_count, u64 n, u32* __restrict__ tpre,
                                                       u32* __restrict__ done, const u32* __restrict__ nfl,
                                                       const u32* __restrict__ nnf, const u32* __restrict__ dup_flag) {
  if (prev_count && level_direct(prev_count, n)) return;
  if (nfl && !(dup_flag && *dup_flag != 0) && *nnf <= kNfListCap) return;
  constexpr u32 T = u32(kBlock) * ITEMS;
  __shared__ u32 s_red[kBlock / 64];
  __shared__ u32 s_last;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u64 base = u64(blockIdx.x) * T;
  u32 c = 0;
  if (base + T <= p) {
    const uint4* q = reinterpret_cast<const uint4*>(nf + base);
    for (u32 i = u32(tid); i < T / 16; i += kBlock) {
      const uint4 v = q[i];
      c += zero_bytes(v.x) + zero_bytes(v.y) + zero_bytes(v.z) + zero_bytes(v.w);
    }
  } else {
    for (u64 j = base + u64(tid); j < p; j += kBlock) c += nf[j] == kNfMaybe ? 1u : 0u;
  }
  c = u32(wave_sum(u64(c)));
  if (lane == 0) s_red[wave] = c;
  __syncthreads();
  if (tid == 0) {
    u32 t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += s_red[w];
    tpre[blockIdx.x] = t;
    __threadfence();
    s_last = atomicAdd(done, 1u) == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();
  // the last block: exclusive scan of the gridDim.x tile counts, in place
  const u32 nt = gridDim.x, per = (nt + kBlock - 1) / kBlock, t0 = u32(tid) * per;
  u32 loc = 0;
  for (u32 t = t0; t < t0 + per && t < nt; ++t) loc += __hip_atomic_load(&tpre[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  u32 inc = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();
  if (lane == 63) s_red[wave] = inc;
  __syncthreads();
  u32 run = inc - loc;
  for (int w = 0; w < wave; ++w) run += s_red[w];
  for (u32 t = t0; t < t0 + per && t < nt; ++t) {
    const u32 v = __hip_atomic_load(&tpre[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    tpre[t] = run;
    run += v;
  }
  if (tid == 0) *done = 0;
}

// after_marks() runs once the tile's marks are read and before the scan waits: loads
// issued there (e.g. the first occurrences' input pairs) overlap the look-back.
// tpre (optional, with desc): the tiles' prefixes, counted ahead (k_tile_count): tiles in
// block order, no look-back chain.
template <int ITEMS, class AfterMarks = NoPrefetch>
__device__ __forceinline__ void tile_scan(TileScan<ITEMS>& ts, u32* s_tile, u32* s_pre,
                                          const unsigned char* __restrict__ nf, u64 j0, u64 p, u64 id0,
                                          u64* __restrict__ desc, u32* __restrict__ ticket,
                                          u64* __restrict__ count_out, AfterMarks after_marks = {},
                                          const u32* __restrict__ tpre = nullptr) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool direct = desc == nullptr;
  const bool counted = tpre != nullptr;
  if (tid == 0) *s_tile = direct || counted ? 0u : atomicAdd(ticket, 1u);
  __syncthreads();
  const u64 tile = direct || counted ? u64(blockIdx.x) : u64(*s_tile);
  ts.base = j0 + tile * (kBlock * ITEMS);
  // short tiles: the marks' loads go out before the prefix count's (long tiles read them
  // one ballot at a time: registers)
  constexpr bool kEarlyMarks = ITEMS <= kItemsSmall;
  unsigned char mv[kEarlyMarks ? ITEMS : 1];
  if constexpr (kEarlyMarks) {
#pragma unroll
    for (int e = 0; e < ITEMS; ++e) {
      const u64 j = ts.base + u64(e) * kBlock + tid;
      mv[e] = j < p ? nf[j] : kNfNot;
    }
  }
  if (direct) {   // firsts in [j0, base): j0 and base are multiples of 256
    const uint4* q = reinterpret_cast<const uint4*>(nf + j0);
    const u64 nq = (ts.base - j0) / 16;
    u32 c = 0;
    for (u64 i0 = tid; i0 < nq; i0 += 16 * kBlock) {   // sixteen predicated loads in flight per pass
      uint4 v[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const u64 i = i0 + u64(e) * kBlock;
        v[e] = i < nq ? q[i] : make_uint4(~0u, ~0u, ~0u, ~0u);   // (no zero byte)
      }
#pragma unroll
      for (int e = 0; e < 16; ++e) c += zero_bytes(v[e].x) + zero_bytes(v[e].y) + zero_bytes(v[e].z) + zero_bytes(v[e].w);
    }
    c = u32(wave_sum(u64(c)));
    __syncthreads();   // (every thread has read *s_tile)
    if (lane == 0 && c) atomicAdd(s_tile, c);
  }
#pragma unroll
  for (int e = 0; e < ITEMS; ++e) {
    bool first;
    if constexpr (kEarlyMarks) {
      first = mv[e] == kNfMaybe;
    } else {
      const u64 j = ts.base + u64(e) * kBlock + tid;
      first = j < p && nf[j] == kNfMaybe;
    }
    ts.mask[e] = __ballot(first);
    if (lane == 0) s_pre[e * 4 + wave] = u32(__popcll(ts.mask[e]));
  }
  after_marks();
  __syncthreads();
  constexpr int NG = 4 * ITEMS;             // 64-element groups per tile
  constexpr int PER = (NG + 63) / 64;        // groups per lane of the scanning wave
  if (wave == 0) {
    u32 cs[PER];
    u32 c = 0;
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int g = lane * PER + q;
      cs[q] = g < NG ? s_pre[g] : 0u;
      c += cs[q];
    }
    u32 incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    const u64 agg = __shfl(incl, 63, 64);
    u64 prefix = tile == 0 ? id0 : 0;   // descriptors' P values already include id0
    if (direct) {
      prefix = id0 + *s_tile;
    } else if (counted) {
      prefix = id0 + tpre[tile];
    } else if (tile == 0) {
      if (lane == 0) __hip_atomic_store(&desc[0], kStP | (id0 + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      if (lane == 0) __hip_atomic_store(&desc[tile], kStA | agg, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      long long look = (long long)tile - 1;
      for (;;) {
        const long long idx = look - lane;
        const u64 d =
            idx >= 0 ? __hip_atomic_load(&desc[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
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
      if (lane == 0)
        __hip_atomic_store(&desc[tile], kStP | (prefix + agg), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    u32 run = u32(prefix + incl - c);
#pragma unroll
    for (int q = 0; q < PER; ++q) {
      const int g = lane * PER + q;
      if (g < NG) s_pre[g] = run;
      run += cs[q];
    }
    if (lane == 0 && ts.base + kBlock * ITEMS >= p) *count_out = prefix + agg;
  }
  __syncthreads();
}

// Leaves (one launch per leaf chunk, positions [j0, p), ids from id0 =
// uniques of earlier chunks): first occurrences read their slot to recover the
// canonical leaf, emit it, and settle the slot with their id, which both the
// chunk's resolve and later chunks' inserts read.
template <class Tab, int ITEMS>
__global__ __launch_bounds__(kBlock) void k_flagscan_leaf(u32* __restrict__ words, u64 j0, u64 p, Tab T,
                                                         const unsigned char* __restrict__ nf,
                                                         u64* __restrict__ desc, u32* __restrict__ ticket,
                                                         u64* __restrict__ out, const u64* __restrict__ id0_p,
                                                         u64* __restrict__ count_out, const u64* __restrict__ lkey,
                                                         u32* __restrict__ lsid) {
  __shared__ u32 s_tile;
  __shared__ u32 s_pre[4 * ITEMS];
  TileScan<ITEMS> ts;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // fused small build (lkey, lsid given; one chunk, direct tiles): the slot words and keys
  // are read up front, first occurrences emit the key the insert stored and leave their
  // id by slot for level 0's insert -- no table read, no settle
  constexpr bool kShort = ITEMS <= kItemsSmall;
  const bool early = kShort && lsid != nullptr && desc == nullptr;
  u32 rw[kShort ? ITEMS : 1];
  u64 kw[kShort ? ITEMS : 1];
  if constexpr (kShort) {
#pragma unroll
    for (int e = 0; e < ITEMS; ++e) {
      rw[e] = 0;
      kw[e] = 0;
      const u64 j = j0 + u64(blockIdx.x) * (kBlock * ITEMS) + u64(e) * kBlock + tid;
      if (early && j < p) {
        rw[e] = words[j];
        kw[e] = lkey[j];
      }
    }
  }
  const u64 id0 = id0_p ? *id0_p : 0;
  tile_scan(ts, &s_tile, s_pre, nf, j0, p, id0, desc, ticket, count_out);
  const u64 lt = (1ull << lane) - 1;
#pragma unroll
  for (int e = 0; e < ITEMS; ++e) {
    const u64 j = ts.base + u64(e) * kBlock + tid;
    if (j < p && ((ts.mask[e] >> lane) & 1ull)) {
      const u32 id = s_pre[e * 4 + wave] + u32(__popcll(ts.mask[e] & lt));
      bool done = false;
      if constexpr (kShort) {
        if (early) {
          out[id] = kw[e];
          lsid[rw[e] & kIdx] = id;
          words[j] = id | (rw[e] & kBits);
          done = true;
        }
      }
      if (!done) {
        const u32 rec = words[j];
        u64 key;
        u32 pos;
        T.read(rec & kIdx, key, pos);
        out[id] = key;
        T.settle(rec & kIdx, id);
        if (lsid) lsid[rec & kIdx] = id;
        words[j] = id | (rec & kBits);
      }
    }
  }
}

// Nodes: first occurrences recompute their canonical pair from the input
// (coalesced) instead of reading the table, emit it, and publish the group
// records that resolve_node uses.
//
// With `multi` and `hashed_next` given it also looks one level ahead: a pair of
// the next level goes through the table only if both its children repeat
// (singleton propagation); if no such pair exists, every pair of the next level
// is a first occurrence and that level is direct (k_resolve_node opens its gate).
// Sparse ranking of one tile of T = kBlock * ITEMS positions [base, base + T) when the
// level's not-first positions are few and listed (any order, c <= kNfListCap): a position's
// rank among the first ones is itself minus the listed positions before it -- no look-back
// chain.  LDS: the tile's listed positions as bits, their exclusive popcount per 32-bit word,
// and the count of listed positions before the tile.
template <int ITEMS>
struct SparseTile {
  static constexpr u32 T = u32(kBlock) * ITEMS, NWB = T / 32;
  u32* bits;
  u32* bpre;
  u64 base, before;
  __device__ __forceinline__ bool listed(u32 k) const { return (bits[k >> 5] >> (k & 31)) & 1u; }
  __device__ __forceinline__ u64 nb(u32 k) const {   // listed positions before base + k
    return before + bpre[k >> 5] + u32(__popc(bits[k >> 5] & ((1u << (k & 31)) - 1u)));
  }
};
template <int ITEMS>
__device__ __forceinline__ SparseTile<ITEMS> sparse_tile(const u32* __restrict__ list, u32 c, u64 base) {
  using ST = SparseTile<ITEMS>;
  __shared__ u32 s_bits[ST::NWB], s_bpre[ST::NWB], s_red[kBlock / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (u32 w = u32(tid); w < ST::NWB; w += kBlock) s_bits[w] = 0;
  __syncthreads();
  u32 before = 0;
  for (u32 k = u32(tid); k < c; k += kBlock) {
    const u64 q = list[k];
    if (q < base) ++before;
    else if (q < base + ST::T) atomicOr(&s_bits[u32(q - base) >> 5], 1u << (u32(q - base) & 31));
  }
  before = u32(wave_sum(u64(before)));
  if (lane == 0) s_red[wave] = before;
  __syncthreads();
  before = 0;
  for (int w = 0; w < kBlock / 64; ++w) before += s_red[w];
  const u32 v = u32(tid) < ST::NWB ? u32(__popc(s_bits[tid])) : 0u;   // (NWB <= kBlock)
  u32 inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(inc, o, 64);
    if (lane >= o) inc += y;
  }
  __syncthreads();   // (s_red read by every thread above)
  if (lane == 63) s_red[wave] = inc;
  __syncthreads();
  u32 pre = inc - v;
  for (int w = 0; w < wave; ++w) pre += s_red[w];
  if (u32(tid) < ST::NWB) s_bpre[tid] = pre;
  __syncthreads();
  return ST{s_bits, s_bpre, base, before};
}

template <int ITEMS>
__global__ __launch_bounds__(kBlock) void k_flagscan_node(u32* __restrict__ words, u64 p,
                                                         const u32* __restrict__ in, u64 n,
                                                         const unsigned char* __restrict__ nf,
                                                         Group* __restrict__ grp, u64* __restrict__ desc,
                                                         u32* __restrict__ ticket, uint2* __restrict__ out,
                                                         u64* __restrict__ count_out, const u64* prev_count,
                                                         const unsigned char* __restrict__ multi,
                                                         u32* __restrict__ hashed_next, uint4* __restrict__ clr_nf,
                                                         uint4* __restrict__ clr_multi, u64 clr16,
                                                         u32* __restrict__ sid, const u32* __restrict__ dup_flag,
                                                         const u32* __restrict__ nfl = nullptr,
                                                         const u32* __restrict__ nnf = nullptr,
                                                         const u32* __restrict__ tpre = nullptr) {
  // fused small-build levels: clear the marks of the level after this one (its parity
  // set held the previous level's marks, last read by this level's insert)
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < clr16; i += u64(gridDim.x) * kBlock) {
    clr_nf[i] = make_uint4(0, 0, 0, 0);
    clr_multi[i] = make_uint4(0, 0, 0, 0);
  }
  __shared__ u32 s_tile;
  __shared__ u32 s_pre[4 * ITEMS];
  __shared__ u32 s_hashed;
  TileScan<ITEMS> ts;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // Short tiles read their whole input up front (pairs, multi marks, the insert's slot
  // words), before the gate and the prefix count: one round trip for all of it.  Long
  // tiles (registers) and look-back tiles (tile known late) read the pairs of their
  // first occurrences while the scan waits.
  constexpr bool kPre = ITEMS <= kItemsSmall;
  const bool early = kPre && desc == nullptr;
  u32 pl[ITEMS], pr[ITEMS], sw[ITEMS];
  unsigned char mu[ITEMS];
  if (kPre) {
#pragma unroll
    for (int e = 0; e < ITEMS; ++e) {
      pl[e] = pr[e] = sw[e] = 0;
      mu[e] = 0;
    }
  }
  if (early) {
#pragma unroll
    for (int e = 0; e < ITEMS; ++e) {
      const u64 j = u64(blockIdx.x) * (kBlock * ITEMS) + u64(e) * kBlock + tid;
      if (j < p) {
        load_pair(in, n, j, pl[e], pr[e]);
        if (hashed_next || sid) mu[e] = multi[j];
        if (sid) sw[e] = words[j];
      }
    }
  }
  if (level_direct(prev_count, n)) return;
  if (threadIdx.x == 0) s_hashed = 0;
  if (nfl && !(dup_flag && *dup_flag != 0) && *nnf <= kNfListCap) {
    // Sparse repeats (two-pass level, the dedupe listed every not-first position): tiles in
    // block order, no look-back chain -- a position's id is itself minus the repeats before it.
    const u32 c = *nnf;
    const SparseTile<ITEMS> st = sparse_tile<ITEMS>(nfl, c, u64(blockIdx.x) * (u32(kBlock) * ITEMS));
    const u64 base = st.base;
    if (blockIdx.x == 0 && tid == 0) *count_out = p - c;
    bool hashed = false;
    // EB items' pairs and marks loaded before any is used (the ranks need no scan here)
    constexpr int EB = ITEMS < 8 ? ITEMS : 8;
#pragma unroll
    for (int e0 = 0; e0 < ITEMS; e0 += EB) {
      u32 bl[EB], br[EB];
      unsigned char bm[EB];
#pragma unroll
      for (int q = 0; q < EB; ++q) {
        const u64 j = base + u64(e0 + q) * kBlock + tid;
        bl[q] = br[q] = 0;
        bm[q] = 0;
        if (j < p) {
          load_pair(in, n, j, bl[q], br[q]);
          if (hashed_next) bm[q] = multi[j];
        }
      }
#pragma unroll
      for (int q = 0; q < EB; ++q) {
        const u32 k = u32(e0 + q) * kBlock + u32(tid);
        const u64 j = base + k;
        const bool listed = j < p && st.listed(k);
        const bool is_first = j < p && !listed;
        const u64 mask = __ballot(is_first);
        const u64 nb = st.nb(k);
        if (lane == 0) {
          Group g;
          g.mask = mask; g.prefix = u32(j - nb); g.pad = 0;
          grp[(base >> 6) + u64(e0 + q) * 4 + wave] = g;
        }
        if (hashed_next) {
          const bool rep = j < p && (!is_first || bm[q] != 0);
          const bool partner = __shfl_xor(int(rep), 1, 64) != 0;
          if ((lane & 1) == 0 && rep && (j + 1 < p ? partner : true)) hashed = true;
        }
        if (is_first) {
          const u32 id = u32(j - nb);
          u32 cl, cr, m, t;
          node_canonical(bl[q], br[q], cl, cr, m, t);
          out[id] = make_uint2(cl, cr);
          words[j] = make_word(id, m, t, ulw(bl[q]) == ulw(xf(br[q], 1, 0)));
        } else if (listed) {
          // a repeat (the resolve's work, done here: k_resolve_node skips sparse levels): its
          // word holds its key's first position f, whose id is f minus the repeats before it
          const u32 w = words[j];
          const u32 f = w & kIdx;
          u32 before = 0;
          for (u32 i = 0; i < c; ++i) before += nfl[i] < f ? 1u : 0u;
          words[j] = (f - before) | (w & kBits);
        }
      }
    }
    if (hashed_next) {
      if (__ballot(hashed) && lane == 0) s_hashed = 1;
      __syncthreads();
      if (threadIdx.x == 0 && s_hashed) *hashed_next = 1;
    }
    return;
  }
  auto fetch = [&]() {
    if constexpr (kPre) {
      if (!early) {
#pragma unroll
        for (int e = 0; e < ITEMS; ++e) {
          const u64 j = ts.base + u64(e) * kBlock + tid;
          if (j < p && ((ts.mask[e] >> lane) & 1ull)) load_pair(in, n, j, pl[e], pr[e]);
        }
      }
    }
  };
  tile_scan(ts, &s_tile, s_pre, nf, 0, p, 0, desc, ticket, count_out, fetch, tpre);
  const u64 lt = (1ull << lane) - 1;
  bool hashed = false;
  const bool dups = dup_flag && *dup_flag != 0;   // block-collapsed repeats (k_bkt_part) exist
  u32 nfirst = 0;   // this thread's items that are not first occurrences (the dups pass below)
#pragma unroll
  for (int e = 0; e < ITEMS; ++e) {
    const u64 j = ts.base + u64(e) * kBlock + tid;
    const bool is_first = j < p && ((ts.mask[e] >> lane) & 1ull);
    if (!is_first) nfirst |= 1u << e;
    unsigned char me = 0;   // multi mark: needed for first occurrences only
    if ((hashed_next || sid) && is_first) me = early ? mu[e] : multi[j];
    if (hashed_next) {   // next-level pair (j, j+1): both children repeat?  (first <=> mask bit)
      const bool rep = j < p && (!is_first || me != 0);
      const bool partner = __shfl_xor(int(rep), 1, 64) != 0;
      if ((lane & 1) == 0 && rep && (j + 1 < p ? partner : true)) hashed = true;
    }
    const u32 gpre = s_pre[e * 4 + wave];
    if (lane == 0) {
      Group g;
      g.mask = ts.mask[e]; g.prefix = gpre; g.pad = 0;
      grp[(ts.base >> 6) + e * 4 + wave] = g;
    }
    if (is_first) {
      const u32 id = gpre + u32(__popcll(ts.mask[e] & lt));
      u32 l, r, cl, cr, m, t;
      if constexpr (kPre) {
        l = pl[e];
        r = pr[e];
      } else {
        load_pair(in, n, j, l, r);
      }
      // fused small builds: a repeated key's id by its slot, for the next insert's resolver
      // (only repeated keys are ever looked up, and their first occurrence is multi)
      if (sid && me) sid[(early ? sw[e] : words[j]) & kIdx] = id;
      node_canonical(l, r, cl, cr, m, t);
      uint2 w;
      w.x = cl; w.y = cr;
      out[id] = w;
      words[j] = make_word(id, m, t, ulw(l) == ulw(xf(r, 1, 0)));   // the insert's bits, recomputed
    }
  }
  if (dups) {
    // collapsed repeats (nf = kNfDup, k_bkt_part): their word holds the block representative,
    // the key's first occurrence itself or a repeat whose word the bucket dedupe pointed at the
    // first occurrence (only first occurrences' words change in this kernel, so that word is
    // stable); the latter's first position is copied here.  Eight items at a time, each step's
    // loads issued together (a dependent chain of four per repeat otherwise).
    constexpr int DB = ITEMS < 8 ? ITEMS : 8;
#pragma unroll
    for (int e0 = 0; e0 < ITEMS; e0 += DB) {
      unsigned char f[DB];
      u32 w[DB], g[DB];
#pragma unroll
      for (int q = 0; q < DB; ++q) {
        const u64 j = ts.base + u64(e0 + q) * kBlock + tid;
        f[q] = j < p && ((nfirst >> (e0 + q)) & 1u) ? nf[j] : kNfMaybe;
      }
#pragma unroll
      for (int q = 0; q < DB; ++q) w[q] = f[q] == kNfDup ? words[ts.base + u64(e0 + q) * kBlock + tid] : 0u;
#pragma unroll
      for (int q = 0; q < DB; ++q) g[q] = f[q] == kNfDup ? u32(nf[w[q] & kIdx]) : 0u;
#pragma unroll
      for (int q = 0; q < DB; ++q)
        if (f[q] == kNfDup && g[q] != kNfMaybe)
          words[ts.base + u64(e0 + q) * kBlock + tid] = (words[w[q] & kIdx] & kIdx) | (w[q] & kBits);
    }
  }
  if (hashed_next) {
    if (__ballot(hashed) && lane == 0) s_hashed = 1;
    __syncthreads();
    if (threadIdx.x == 0 && s_hashed) *hashed_next = 1;
  }
}

// ---- resolve ----------------------------------------------------------------------

// Non-first leaves of a chunk: their key's first occurrence is in this chunk
// and has settled the slot.
template <class Tab>
__global__ __launch_bounds__(kBlock) void k_resolve_leaf(u32* __restrict__ words, u64 j0, u64 p, Tab T,
                                                        const unsigned char* __restrict__ nf) {
  const u64 j = j0 + u64(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= p || nf[j] != kNfNot) return;
  const u32 w = words[j];
  words[j] = T.settled_id(w & kIdx) | (w & kBits);
}

// Block 0 also opens the next level's gate: gate = p (the next level is direct)
// when this level is all unique or none of the next level's pairs hashes.  One mark per
// thread: 16 per thread (one 16-B load) was 34 us faster on uniform data but 0.15-0.4 ms
// slower on tandem data (its repeats' dependent loads serialised per thread), not kept.
template <class Tab>
__global__ __launch_bounds__(kBlock) void k_resolve_node(u32* __restrict__ words, u64 p, Tab T,
                                                        const unsigned char* __restrict__ nf,
                                                        const Group* __restrict__ grp, const u64* prev_count,
                                                        u64 n, const u64* __restrict__ count,
                                                        const u32* __restrict__ hashed_next, u64* __restrict__ gate,
                                                        const Header* __restrict__ hdr, u32 bkt,
                                                        u32 sparse = 0) {
  if (gate && blockIdx.x == 0 && threadIdx.x == 0)
    *gate = (*count == p || (hashed_next && *hashed_next == 0)) ? p : ~0ull;
  if (level_direct(prev_count, n)) return;
  // the flag scan's sparse path resolved the level's few repeats itself
  if (sparse && bkt == 2 && hdr->predup == 0 && hdr->nnf <= kNfListCap) return;
  // (a grid smaller than p / kBlock strides: fewer empty workgroups on levels without repeats;
  // four elements per step, each step's loads issued together: mark, word, group record)
  const bool bucketed = bkt && (bkt == 2 || hdr->predup == 0);   // the word holds the first position
  const u64 S = u64(gridDim.x) * kBlock;
  constexpr int RB = 4;
  for (u64 j0 = u64(blockIdx.x) * kBlock + threadIdx.x; j0 < p; j0 += RB * S) {
    bool rep[RB];
    u32 w[RB], q[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      const u64 j = j0 + u64(k) * S;
      const unsigned char f = j < p ? nf[j] : kNfMaybe;
      rep[k] = f == kNfNot || f == kNfDup;
    }
#pragma unroll
    for (int k = 0; k < RB; ++k) w[k] = rep[k] ? words[j0 + u64(k) * S] : 0u;
#pragma unroll
    for (int k = 0; k < RB; ++k) {
      q[k] = 0;
      if (!rep[k]) continue;
      u64 key;
      if (bucketed) q[k] = w[k] & kIdx;
      else T.read(w[k] & kIdx, key, q[k]);   // q = the key's first position
    }
    Group h[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if (rep[k]) h[k] = grp[q[k] >> 6];
#pragma unroll
    for (int k = 0; k < RB; ++k)
      if (rep[k])
        words[j0 + u64(k) * S] =
            (h[k].prefix + u32(__popcll(h[k].mask & ((1ull << (q[k] & 63)) - 1)))) | (w[k] & kBits);
  }
}

// ---- bucketed node insert (non-repetitive data) ---------------------------------------
// Same marks and ids as k_node_insert's table, with no HBM-resident table: the hashed
// pairs of a level are partitioned by the top bits of a hash of their canonical key into
// nb = 2^bb buckets (count -> column-major count matrix -> exclusive scan -> scatter), and
// each bucket (all occurrences of its keys) is deduplicated by one workgroup in LDS.
// Repeats get nf = not-first and their key's first position in the word (k_resolve_node
// reads it instead of a table slot); a key's first occurrence is marked multi.  Runs only
// when hdr->predup == 0 (a hot key would overflow its bucket: hdr->bkt_overflow, and the
// host rebuilds with the table).  One 8-B record per hashed pair: the packed table's
// K-bit key mix h (a bijection, so equal h <=> equal key) without its top bb bits (the
// bucket), above the pair's 16-bit offset in its count chunk (chunk g of a record at
// index i of bucket b: the last g with off[b * G + g] <= i); the host takes this path
// only when K - bb + 16 <= 64.
constexpr int kBktThreads = 1024;
constexpr int kBktItems = 64;                        // pairs per thread of count / scatter
constexpr u64 kBktChunk = u64(kBktThreads) * kBktItems;   // pairs per count-matrix column (2^16)
constexpr u32 kBktRP = 16;                          // record offset bits
constexpr int kBktMaxG = 8192;                      // count chunks (p < 2^29; dedupe LDS <= 32 KB)
constexpr int kBktMaxLog = 14;                       // nb <= 16384 (LDS counters, 64 KB)
constexpr u32 kBktSlots = 6144;                      // LDS table of the dedupe (72 KB: 2 workgroups per CU)
constexpr int kBktCapItems = 5;
constexpr int kBktCap = 4608;                        // ... holding a bucket of <= 4608 pairs (load <= 3/4)

__device__ __forceinline__ u64 bkt_hash(u64 k) {     // murmur3 fmix64
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

struct BktPlan {
  PackedTab T;   // key encoding and mix of this level
  u32 K, bb;     // key bits, bucket bits
  __device__ __forceinline__ u32 bucket(u64 h) const { return bb ? u32(h >> (K - bb)) : 0u; }
};

// Pair j of a level: canonical key, word bits, and whether it goes through the dedupe
// (a pair with a child that occurs once in the previous level is itself unique).
__device__ __forceinline__ bool bkt_pair(const u32* __restrict__ in, u64 n, u64 j,
                                         const unsigned char* __restrict__ prev_nf,
                                         const unsigned char* __restrict__ prev_multi, const BktPlan& bp,
                                         u64& key, u32& bits) {
  u32 l, r, cl, cr, m, t;
  load_pair(in, n, j, l, r);
  node_canonical(l, r, cl, cr, m, t);
  const u32 v = ulw(l) == ulw(xf(r, 1, 0));   // left == right.mirrored() (shared_tree.cpp:670)
  bits = make_word(0, m, t, v);
  key = bp.T.mix(bp.T.node_key(cl, cr));   // K bits
  if (!prev_nf) return true;
  if (2 * j + 1 < n) {
    const uchar2 f = reinterpret_cast<const uchar2*>(prev_nf)[j];
    const uchar2 g = reinterpret_cast<const uchar2*>(prev_multi)[j];
    return !((f.x == 0 && g.x == 0) || (f.y == 0 && g.y == 0));
  }
  return !(prev_nf[2 * j] == 0 && prev_multi[2 * j] == 0);
}

// Count chunk of a workgroup: the 8 XCDs (workgroups dealt round-robin) each take a
// contiguous run of chunks, so the neighbouring count-matrix entries and the neighbouring
// record runs of a bucket (chunk g, then g + 1, ...) are written and read through one
// XCD's L2 and merge there into whole lines.
__device__ __forceinline__ u64 bkt_chunk(u64 G) {
  const u64 b = blockIdx.x, per = G / 8;
  return b < 8 * per ? (b % 8) * per + b / 8 : b;
}

__device__ __forceinline__ bool bkt_skip(const Header* hdr, const u64* prev_count, u64 n) {
  return hdr && (level_direct(prev_count, n) || hdr->predup != 0);   // (null: the multi-rank owner)
}
// the two-pass partition also takes repetitive data (k_bkt_part collapses block repeats)
__device__ __forceinline__ bool bkt2_skip(const Header* hdr, const u64* prev_count, u64 n) {
  return hdr && level_direct(prev_count, n);
}

// Column g of the count matrix: cnt[b * G + g] = hashed pairs of chunk g in bucket b.
[[maybe_unused]] static __global__ __launch_bounds__(kBktThreads) void k_bkt_count(const u32* __restrict__ in, u64 n, u64 p,
                                                          const unsigned char* __restrict__ prev_nf,
                                                          const unsigned char* __restrict__ prev_multi, BktPlan bp,
                                                          u32* __restrict__ cnt, u64 G, const Header* __restrict__ hdr,
                                                          const u64* prev_count, u64* __restrict__ stats) {
  if (bkt_skip(hdr, prev_count, n)) return;
  __shared__ u32 hist[1 << kBktMaxLog];
  __shared__ u32 s_hashed;
  const u32 nb = 1u << bp.bb;
  for (u32 q = threadIdx.x; q < nb; q += kBktThreads) hist[q] = 0;
  if (threadIdx.x == 0) s_hashed = 0;
  __syncthreads();
  const u64 g = bkt_chunk(G), j0 = g * kBktChunk;
  u32 hashed = 0;
#pragma unroll 4
  for (int e = 0; e < kBktItems; ++e) {
    const u64 j = j0 + u64(e) * kBktThreads + threadIdx.x;
    if (j >= p) break;
    u64 key;
    u32 bits;
    if (bkt_pair(in, n, j, prev_nf, prev_multi, bp, key, bits)) {
      atomicAdd(&hist[bp.bucket(key)], 1u);
      ++hashed;
    }
  }
  const u64 wsum = wave_sum(u64(hashed));
  if ((threadIdx.x & 63) == 0 && wsum) atomicAdd(&s_hashed, u32(wsum));
  __syncthreads();
  for (u32 q = threadIdx.x; q < nb; q += kBktThreads) cnt[u64(q) * G + g] = hist[q];
  if (g == 0 && threadIdx.x == 0) cnt[u64(nb) * G] = 0;   // the scan's total lands here
  if (threadIdx.x == 0 && s_hashed)   // second word of each shard line: bucketed pairs
    atomicAdd(&stats[(blockIdx.x & (kStatShards - 1)) * kStatStride + 1], u64(s_hashed));
}

// Same chunks as k_bkt_count; off = exclusive scan of cnt.  Writes every pair's
// provisional word (position field 0) and the hashed pairs' (key, position) records.
[[maybe_unused]] static __global__ __launch_bounds__(kBktThreads) void k_bkt_scatter(const u32* __restrict__ in, u64 n, u64 p,
                                                            const unsigned char* __restrict__ prev_nf,
                                                            const unsigned char* __restrict__ prev_multi, BktPlan bp,
                                                            const u32* __restrict__ off, u64 G, u64* __restrict__ rrec,
                                                            u32* __restrict__ rec, const Header* __restrict__ hdr,
                                                            const u64* prev_count) {
  if (bkt_skip(hdr, prev_count, n)) return;
  __shared__ u32 cur[1 << kBktMaxLog];
  const u32 nb = 1u << bp.bb;
  const u64 g = bkt_chunk(G), j0 = g * kBktChunk;
  const u64 lowmask = bp.K - bp.bb >= 64 ? ~0ull : (1ull << (bp.K - bp.bb)) - 1;
  for (u32 q = threadIdx.x; q < nb; q += kBktThreads) cur[q] = off[u64(q) * G + g];
  __syncthreads();
#pragma unroll 4
  for (int e = 0; e < kBktItems; ++e) {
    const u64 j = j0 + u64(e) * kBktThreads + threadIdx.x;
    if (j >= p) break;
    u64 key;
    u32 bits;
    if (bkt_pair(in, n, j, prev_nf, prev_multi, bp, key, bits)) {
      const u32 d = atomicAdd(&cur[bp.bucket(key)], 1u);
      rrec[d] = ((key & lowmask) << kBktRP) | (j - j0);
    }
    rec[j] = bits;
  }
}

// One workgroup per bucket (at most kBktCap records, else hdr->bkt_overflow and the host
// rebuilds with the table): an LDS hash-cons of its records, then marks and first
// positions for the keys that occur more than once.
__device__ __forceinline__ u32 bkt_pos(const u32* s_off, u64 G, u32 i, u64 r) {
  u32 lo = 0, hi = u32(G) - 1;   // chunk of record i: the last g with s_off[g] <= i
  while (lo < hi) {
    const u32 mid = (lo + hi + 1) >> 1;
    if (s_off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return (lo << kBktRP) | u32(r & ((1u << kBktRP) - 1));
}

[[maybe_unused]] static __global__ __launch_bounds__(kBktThreads) void k_bkt_dedupe(const u32* __restrict__ off, u64 G,
                                                           const u64* __restrict__ rrec,
                                                           u32* __restrict__ rec, Marks mk, Header* __restrict__ hdr,
                                                           const u64* prev_count, u64 n) {
  if (bkt_skip(hdr, prev_count, n)) return;
  constexpr u32 TS = kBktSlots;
  __shared__ u64 s_key[TS];
  __shared__ u32 s_pos[TS];
  __shared__ u32 s_dup[TS / 32];
  extern __shared__ u32 s_off[];   // G entries (dynamic)
  const u64 b = blockIdx.x;
  const u32 start = off[b * G], end = off[(b + 1) * G];
  if (end - start > u32(kBktCap)) {   // a hot key: the table path handles this data
    if (threadIdx.x == 0) hdr->bkt_overflow = 1;
    return;
  }
  for (u32 q = threadIdx.x; q < G; q += kBktThreads) s_off[q] = off[b * G + q];
  for (u32 q = threadIdx.x; q < TS; q += kBktThreads) {
    s_key[q] = kEmpty;
    s_pos[q] = ~0u;
  }
  for (u32 q = threadIdx.x; q < TS / 32; q += kBktThreads) s_dup[q] = 0;
  u64 key[kBktCapItems], raw[kBktCapItems];
  u32 pos[kBktCapItems], slot[kBktCapItems];
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    const u32 i = start + u32(e) * kBktThreads + threadIdx.x;
    raw[e] = i < end ? rrec[i] : 0ull;
    key[e] = i < end ? raw[e] >> kBktRP : kEmpty;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    if (key[e] == kEmpty) continue;
    u32 h = u32((u64(u32(bkt_hash(key[e]))) * TS) >> 32);
    for (;;) {
      unsigned long long c = s_key[h];
      if (c == kEmpty) c = atomicCAS(&s_key[h], kEmpty, (unsigned long long)key[e]);
      if (c == key[e]) atomicOr(&s_dup[h >> 5], 1u << (h & 31));   // another position holds it
      if (c == kEmpty || c == key[e]) break;
      h = h + 1 == TS ? 0u : h + 1;
    }
    slot[e] = h;
  }
  __syncthreads();
  // only keys with several records need positions (most buckets have none)
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    if (key[e] == kEmpty || !((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u)) continue;
    pos[e] = bkt_pos(s_off, G, start + u32(e) * kBktThreads + threadIdx.x, raw[e]);
    atomicMin(&s_pos[slot[e]], pos[e]);
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    if (key[e] == kEmpty || !((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u)) continue;
    const u32 first = s_pos[slot[e]];
    if (pos[e] != first) {
      mk.nf[pos[e]] = kNfNot;
      rec[pos[e]] = first | (rec[pos[e]] & kBits);
    } else {
      mk.multi[pos[e]] = 1;
    }
  }
}

// ---- two-pass partition (levels where a record can carry its full position) ----------
// The single-pass scatter above writes ~2.5 records per bucket per chunk, so its 8-B
// stores never fill a line.  Here the records are partitioned twice, each pass writing
// whole runs:
//   part: per chunk of kPartChunk pairs, the records sorted in LDS by 2^b1 coarse
//         buckets (h's top bits; ~64 records per bucket at b1 = 8) and written back
//         contiguously at the chunk's slot, with the chunk's run table rt[chunk][0..2^b1]
//         (no count matrix, no scan, no capacity to overflow); record = h's low K - b1
//         bits above the 14-bit offset in the chunk;
//   fine: per slice of SC (a power of two) consecutive chunks of one coarse bucket
//         (<= kFineCap records in LDS), its runs gathered and counting-sorted in LDS by
//         the next b2 bits; records become h's low K - b1 - b2 bits above the
//         P = log2(SC) + 14-bit position within the slice, written back contiguously
//         with the slice's fine offsets;
//   dedupe: one workgroup per fine bucket, reading its run in each slice of its coarse
//         bucket; position = slice start + the record's field (no search).
constexpr int kFineCap = 8192;          // records per fine-pass slice (64 KB of LDS: two workgroups per CU)
constexpr int kFineItems = kFineCap / kBktThreads;
constexpr int kFineMaxB2 = 8;           // fine buckets per coarse bucket <= 256
constexpr u32 kPartMaxB1 = 8;           // coarse buckets <= 256
constexpr u32 kPartLog = 14;
constexpr u64 kPartChunk = u64(1) << kPartLog;   // pairs per part chunk (its records fill 128 KB of LDS)
constexpr int kPartItems = int(kPartChunk / kBktThreads);

struct Bkt2Plan {
  PackedTab T;
  u32 K, b1, b2, P;    // key bits, coarse / fine bucket bits, position-in-slice bits (log2(SC) + 14)
  u32 SC, nslice;      // chunks per fine slice, slices per coarse bucket
  u64 G;               // part chunks
  u32* olist;          // owner dedupe (kOwner): the not-first records' indices, appended ...
  u32* ocnt;           // ... at this cursor (the D records, k_own_getid_list); null: none
  u32 wmarks;          // k_bkt_part writes every pair's not-first / multi mark (no k_clear pass)
  u32* nfl;            // k_bkt_dedupe2: the not-first positions (hdr->nnf counts them); null: none
  u32 wave1;           // k_bkt_part collapse: a wave of one key touches the table once (GCZ_PART_WAVE)
  u32* redo;           // k_bkt_dedupe_bm: buckets over its capacity, for k_bkt_dedupe2_redo (null: the
  u32* redo_cnt;       // overflow flag instead), appended at this cursor
  // single device (not the owners): the level's input words.  Without the block collapse
  // (hdr->predup == 0) k_bkt_part writes no provisional word; the dedupes take a repeat's
  // m / t / v bits from its pair instead (first occurrences get theirs from the flag scan)
  const u32* in;
  u64 n;
  u32 xcd;             // XCD-contiguous workgroup order: bit 1 k_bkt_dedupe_bm, bit 2 k_bkt_fine (GCZ_BKT_XCD)
};

// m / t / v bits of repeat `pos` of a two-pass level, for its word (first position | bits)
__device__ __forceinline__ u32 repeat_bits(const Bkt2Plan& bp, const u32* rec, u32 pos, bool collapse) {
  if (!bp.in || collapse) return rec[pos] & kBits;
  u32 l, r, cl, cr, m, t;
  load_pair(bp.in, bp.n, pos, l, r);
  node_canonical(l, r, cl, cr, m, t);
  return make_word(0, m, t, ulw(l) == ulw(xf(r, 1, 0)));
}

// Append the not-first positions of a wave to bp.nfl (one atomic per wave; none once the
// list is over its cap -- the count then only tells the flag scan to take the look-back path).
__device__ __forceinline__ void nf_list_add(const Bkt2Plan& bp, Header* hdr, bool nf, u32 pos) {
  if (!bp.nfl) return;
  const u64 m = __ballot(nf);
  if (!m) return;
  const int lane = int(threadIdx.x & 63), lead = __ffsll((long long)m) - 1;
  u32 base = 0;
  if (lane == lead)
    base = *reinterpret_cast<volatile u32*>(&hdr->nnf) > kNfListCap ? ~0u : atomicAdd(&hdr->nnf, u32(__popcll(m)));
  base = __shfl(base, lead, 64);
  if (!nf || base == ~0u) return;
  const u32 k = base + u32(__popcll(m & ((1ull << lane) - 1ull)));
  if (k < kNfListCap) bp.nfl[k] = pos;
}

// Exclusive prefix of n <= 256 LDS counters in place (one wave, 4 per lane); c[n] = the total.
__device__ __forceinline__ void lds_excl256(u32* c, u32 n) {
  if (threadIdx.x < 64) {
    const u32 lane = threadIdx.x;
    u32 v[4], sum = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32 i = lane * 4 + k;
      v[k] = i < n ? c[i] : 0u;
      sum += v[k];
    }
    u32 inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(inc, o, 64);
      if (int(lane) >= o) inc += y;
    }
    u32 run = inc - sum;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const u32 i = lane * 4 + k;
      if (i < n) c[i] = run;
      run += v[k];
    }
    if (lane == 63) c[n] = inc;
  }
}

// Repetitive data (hdr->predup): before partitioning, the repeats of a key inside each
// block of 4096 consecutive pairs collapse onto the block's earliest occurrence of it (an LDS
// table per block): only that representative is partitioned (marked multi), the others are
// marked kNfDup with the representative's position in their word (k_flagscan_node then
// points them at the key's first occurrence).  Hot keys -- tandem repeats -- thus reach the
// buckets once per block instead of once per occurrence.
constexpr u32 kColBlock = 4096;   // pairs per collapse block (4 of them per part chunk)
constexpr u32 kColSlots = 8192;   // its LDS table (load <= 1/2), in the part's staging area

[[maybe_unused]] static __global__ __launch_bounds__(kBktThreads) void k_bkt_part(
    const u32* __restrict__ in, u64 n, u64 p, const unsigned char* __restrict__ prev_nf,
    const unsigned char* __restrict__ prev_multi, Bkt2Plan bp, u64* __restrict__ seg, u32* __restrict__ rt,
    u32* __restrict__ rec, Marks mk, Header* __restrict__ hdr, const u64* prev_count, u64* __restrict__ stats,
    uint2* __restrict__ nodes, u64* __restrict__ count_out, u32 id_off) {
  if (bkt2_skip(hdr, prev_count, n)) {
    // the level turned out direct (every child unique): ids are positions; this launch writes
    // the words and nodes k_node_insert's direct path would (the host launches no insert on
    // two-pass levels, so its ~p/256 empty workgroups are not paid)
    const u64 j0 = u64(blockIdx.x) * kPartChunk;
    if (blockIdx.x == 0 && threadIdx.x == 0) *count_out = p;
    for (u64 j = j0 + threadIdx.x; j < p && j < j0 + kPartChunk; j += kBktThreads) {
      u32 l, r, cl, cr, m, t;
      load_pair(in, n, j, l, r);
      node_canonical(l, r, cl, cr, m, t);
      nodes[j] = make_uint2(cl, cr);
      rec[j] = make_word(u32(j) + id_off, m, t, ulw(l) == ulw(xf(r, 1, 0)));
    }
    return;
  }
  extern __shared__ u64 stage[];   // kPartChunk records (dynamic)
  __shared__ u32 cur[(1u << kPartMaxB1) + 1];
  if (bp.nfl && blockIdx.x == 0 && threadIdx.x == 0) hdr->nnf = 0;   // (the dedupe counts after this launch)
  const bool collapse = hdr && hdr->predup != 0;
  const u32 nb1 = 1u << bp.b1;
  for (u32 q = threadIdx.x; q <= nb1; q += kBktThreads) cur[q] = 0;
  // the block table lives in the staging area until the records are staged: block q's
  // entries carry the tag q + 1 (a slot of another tag is free: no clearing): key | tag << 58
  // (K <= 58 on this path), the earliest offset as tag << 16 | 0xffff - offset (atomicMax),
  // the repeat flag as the tag
  unsigned long long* s_ck = reinterpret_cast<unsigned long long*>(stage);
  u32* s_cp = reinterpret_cast<u32*>(stage + kColSlots);
  unsigned char* s_cd = reinterpret_cast<unsigned char*>(stage + kColSlots + kColSlots / 2);
  if (collapse)
    for (u32 q = threadIdx.x; q < kColSlots + kColSlots / 2 + kColSlots / 8; q += kBktThreads) stage[q] = 0;
  __syncthreads();
  const u64 g = bkt_chunk(bp.G), j0 = g * kPartChunk;
  const u32 sh1 = bp.K - bp.b1;
  const u64 lowmask = sh1 >= 64 ? ~0ull : (1ull << sh1) - 1;
  BktPlan kp{bp.T, bp.K, bp.b1};
  u64 r[kPartItems];
  u32 slot[kPartItems];   // coarse bucket << 16 | rank in it; ~0: not hashed
  u32 hashed = 0;
  auto place = [&](int e, u64 j, u64 key) {   // the record of a hashed pair into its coarse run
    const u32 c = bp.b1 ? u32(key >> sh1) : 0u;
    r[e] = ((key & lowmask) << kPartLog) | (j - j0);
    slot[e] = (c << 16) | atomicAdd(&cur[c], 1u);
    ++hashed;
  };
  // bp.wmarks: every pair's marks written here (0, or the collapse's), whole lines per wave --
  // the level needs no clearing pass; the bytes up to the next 16 are zeroed too (vector reads)
  const u64 p16 = (p + 15) & ~u64(15);
  auto marks = [&](u64 j, unsigned char nfv, unsigned char muv) {
    if (bp.wmarks && j < p16) {
      mk.nf[j] = nfv;
      mk.multi[j] = muv;
    }
  };
  if (!collapse) {
#pragma unroll
    for (int e = 0; e < kPartItems; ++e) {
      const u64 j = j0 + u64(e) * kBktThreads + threadIdx.x;
      slot[e] = ~0u;
      marks(j, 0, 0);
      if (j >= p) continue;
      u64 key;
      u32 bits;
      if (bkt_pair(in, n, j, prev_nf, prev_multi, kp, key, bits)) place(e, j, key);
      if (!bp.in) rec[j] = bits;
    }
  } else {
    // each block's repeats onto its earliest occurrence of the key; the next block's pairs
    // are loaded while this block hashes in LDS
    constexpr int BI = kColBlock / kBktThreads;   // items per block
    u64 kn[BI];
    u32 bn[BI];
    bool hn[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
      const u64 j = j0 + u64(i) * kBktThreads + threadIdx.x;
      kn[i] = 0;
      bn[i] = 0;
      hn[i] = j < p && bkt_pair(in, n, j, prev_nf, prev_multi, kp, kn[i], bn[i]);
    }
#pragma unroll
    for (int q = 0; q < kPartItems / BI; ++q) {
      u64 key[BI];
      u32 bits[BI], cs[BI];
      bool h[BI];
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        key[i] = kn[i];
        bits[i] = bn[i];
        h[i] = hn[i];
      }
      if (q + 1 < kPartItems / BI)
#pragma unroll
        for (int i = 0; i < BI; ++i) {
          const u64 j = j0 + u64((q + 1) * BI + i) * kBktThreads + threadIdx.x;
          kn[i] = 0;
          bn[i] = 0;
          hn[i] = j < p && bkt_pair(in, n, j, prev_nf, prev_multi, kp, kn[i], bn[i]);
        }
      const u64 tag = u64(q + 1);
      const int lane = int(threadIdx.x & 63);
#pragma unroll
      for (int i = 0; i < BI; ++i) {   // claim (or find) the key's slot, the earliest offset, the flag
        cs[i] = 0;
        // a wave whose hashed pairs all carry one key (a tandem repeat whose period divides the
        // pair's span): only its first such lane -- the earliest offset -- touches the table
        const u64 hm = bp.wave1 ? __ballot(h[i]) : 0ull;
        if (hm) {
          const int lead = __ffsll((long long)hm) - 1;
          const u64 k0 = __shfl(key[i], lead, 64);
          if (__ballot(h[i] && key[i] == k0) == hm && __popcll(hm) > 1) {
            u32 s0 = 0;
            if (lane == lead) {
              const u64 mk2 = (tag << 58) | key[i];
              const u32 off = u32(i) * kBktThreads + threadIdx.x;
              u32 s2 = u32((u64(u32(bkt_hash(key[i]))) * kColSlots) >> 32);
              for (;;) {
                unsigned long long cv = s_ck[s2];
                if ((cv >> 58) != tag) {
                  const unsigned long long old = atomicCAS(&s_ck[s2], cv, (unsigned long long)mk2);
                  if (old == cv) break;
                  cv = old;
                  if ((cv >> 58) != tag) continue;
                }
                if (cv == mk2) break;
                s2 = s2 + 1 == kColSlots ? 0u : s2 + 1;
              }
              s_cd[s2] = (unsigned char)tag;   // several: the other lanes
              atomicMax(&s_cp[s2], (u32(tag) << 16) | (0xffffu - off));
              s0 = s2;
            }
            cs[i] = __shfl(s0, lead, 64);
            continue;
          }
        }
        if (!h[i]) continue;
        const u64 mk2 = (tag << 58) | key[i];
        const u32 off = u32(i) * kBktThreads + threadIdx.x;
        u32 s2 = u32((u64(u32(bkt_hash(key[i]))) * kColSlots) >> 32);
        bool several = false;
        for (;;) {
          unsigned long long cv = s_ck[s2];
          if ((cv >> 58) != tag) {   // free in this block: claim it
            const unsigned long long old = atomicCAS(&s_ck[s2], cv, (unsigned long long)mk2);
            if (old == cv) break;
            cv = old;
            if ((cv >> 58) != tag) continue;
          }
          if (cv == mk2) {
            several = true;
            break;
          }
          s2 = s2 + 1 == kColSlots ? 0u : s2 + 1;
        }
        if (several) s_cd[s2] = (unsigned char)tag;
        atomicMax(&s_cp[s2], (u32(tag) << 16) | (0xffffu - off));
        cs[i] = s2;
      }
      lds_sync();
#pragma unroll
      for (int i = 0; i < BI; ++i) {
        const int e = q * BI + i;
        const u64 j = j0 + u64(e) * kBktThreads + threadIdx.x;
        slot[e] = ~0u;
        bool dup = false;
        unsigned char nfv = 0, muv = 0;
        if (h[i] && s_cd[cs[i]] == (unsigned char)tag) {
          const u32 rep = u32(j0 + u64(q * BI) * kBktThreads) + (0xffffu - (s_cp[cs[i]] & 0xffffu));
          if (rep != u32(j)) {   // collapsed: not partitioned
            nfv = kNfDup;
            rec[j] = rep | bits[i];
            dup = true;
          } else {
            muv = 1;
          }
        }
        if (bp.wmarks) {
          marks(j, nfv, muv);
        } else {
          if (nfv) mk.nf[j] = nfv;
          if (muv) mk.multi[j] = muv;
        }
        if (h[i] && !dup) place(e, j, key[i]);
        if (j < p && !dup) rec[j] = bits[i];
      }
      lds_sync();   // (the next block's tag overwrites these slots; its pairs' loads stay in flight)
    }
  }
  __syncthreads();
  lds_excl256(cur, nb1);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kPartItems; ++e)
    if (slot[e] != ~0u) stage[cur[slot[e] >> 16] + (slot[e] & 0xffffu)] = r[e];
  __syncthreads();
  const u32 total = cur[nb1];
  u64* out = seg + g * kPartChunk;
  for (u32 i = threadIdx.x; i < total; i += kBktThreads) out[i] = stage[i];
  u32* rts = rt + g * (nb1 + 1);
  for (u32 q = threadIdx.x; q <= nb1; q += kBktThreads) rts[q] = cur[q];
  const u64 wsum = wave_sum(u64(hashed));
  if ((threadIdx.x & 63) == 0 && wsum)   // second word of each shard line: bucketed pairs
    atomicAdd(&stats[(blockIdx.x & (kStatShards - 1)) * kStatStride + 1], wsum);
}

// One workgroup per (coarse bucket, slice): out region (c * nslice + s) * kFineCap,
// fine offsets fo[(c * nslice + s) * (2^b2 + 1) + f].
[[maybe_unused]] static __global__ __launch_bounds__(kBktThreads) void k_bkt_fine(
    const u64* __restrict__ seg, const u32* __restrict__ rt, Bkt2Plan bp, u64* __restrict__ out,
    u32* __restrict__ fo, Header* __restrict__ hdr, const u64* prev_count, u64 n, u32* __restrict__ ovf) {
  if (bkt2_skip(hdr, prev_count, n)) return;
  extern __shared__ u64 stage[];   // kFineCap records (dynamic)
  __shared__ u32 s_pre[129], s_beg[128];   // runs of the slice's chunks (SC <= 128)
  __shared__ u32 s_w[2];
  __shared__ u32 hist[(1u << kFineMaxB2) + 1];
  const u32 nb1 = 1u << bp.b1, nb2 = 1u << bp.b2;
  // bp.xcd bit 2: workgroups taken slice-major in XCD-contiguous runs, so the coarse buckets c and
  // c + 1 of one slice -- adjacent runs of the same chunks, run-table entries on one line -- are
  // read through one L2 (the output stays at (c * nslice + slice))
  u32 c, sl;
  if (bp.xcd & 2u) {
    const u32 b = u32(bkt_chunk(gridDim.x));
    sl = b / nb1;
    c = b % nb1;
  } else {
    c = blockIdx.x / bp.nslice;
    sl = blockIdx.x % bp.nslice;
  }
  const u64 wg = u64(c) * bp.nslice + sl;
  const u64 g0 = u64(sl) * bp.SC;
  const u32 nsc = u32(g0 + bp.SC <= bp.G ? bp.SC : bp.G - g0);
  {   // run (chunk g0 + t, bucket c): one lane each, a two-wave scan of the lengths
    const u32 t = threadIdx.x, lane = t & 63, wave = t >> 6;
    u32 len = 0;
    if (t < nsc) {
      const u32* q = rt + (g0 + t) * (nb1 + 1) + c;
      s_beg[t] = q[0];
      len = q[1] - q[0];
    }
    u32 inc = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(inc, o, 64);
      if (int(lane) >= o) inc += y;
    }
    if (wave < 2 && lane == 63) s_w[wave] = inc;
    __syncthreads();
    const u32 pre = wave == 1 ? s_w[0] : 0u;
    if (t < nsc) s_pre[t] = pre + inc - len;
    if (t == nsc - 1) s_pre[nsc] = pre + inc;
  }
  for (u32 q = threadIdx.x; q < nb2; q += kBktThreads) hist[q] = 0;
  __syncthreads();
  const u32 total = s_pre[nsc];
  u32* fos = fo + wg * (nb2 + 1);
  if (total > u32(kFineCap)) {   // a hot key the probe missed: the table path handles this data
    if (threadIdx.x == 0) *ovf = 1;
    for (u32 q = threadIdx.x; q <= nb2; q += kBktThreads) fos[q] = 0;
    return;
  }
  const u32 sh2 = bp.K - bp.b1 - bp.b2;   // key bits kept in the final record
  const u64 keep = sh2 >= 64 ? ~0ull : (1ull << sh2) - 1;
  __shared__ u32 s_gs[kFineCap / 64];   // the run holding record 64 g
  for (u32 t = threadIdx.x; t < nsc; t += kBktThreads)
    for (u32 g = (s_pre[t] + 63) >> 6; (g << 6) < s_pre[t + 1]; ++g) s_gs[g] = t;
  __syncthreads();
  u64 r[kFineItems];
  u32 slot[kFineItems];
#pragma unroll
  for (int e = 0; e < kFineItems; ++e) {
    const u32 i = u32(e) * kBktThreads + threadIdx.x;
    slot[e] = ~0u;
    if (i >= total) continue;
    // run of record i: the last s with s_pre[s] <= i, between the runs of its group's first
    // record and the next group's (one or two steps unless the runs there are short)
    u32 s = s_gs[i >> 6], hi = (i >> 6) + 1 < ((total + 63) >> 6) ? s_gs[(i >> 6) + 1] : nsc - 1;
    while (s < hi) {
      const u32 mid = (s + hi + 1) >> 1;
      if (s_pre[mid] <= i) s = mid;
      else hi = mid - 1;
    }
    const u64 v = seg[(g0 + s) * kPartChunk + s_beg[s] + (i - s_pre[s])];
    const u64 key = v >> kPartLog;   // K - b1 bits
    const u64 pos = (u64(s) << kPartLog) | (v & (kPartChunk - 1));   // within the slice
    const u32 f = bp.b2 ? u32(key >> sh2) : 0u;
    r[e] = ((key & keep) << bp.P) | pos;
    slot[e] = (f << 16) | atomicAdd(&hist[f], 1u);
  }
  __syncthreads();
  lds_excl256(hist, nb2);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kFineItems; ++e)
    if (slot[e] != ~0u) stage[hist[slot[e] >> 16] + (slot[e] & 0xffffu)] = r[e];
  for (u32 q = threadIdx.x; q <= nb2; q += kBktThreads) fos[q] = hist[q];
  __syncthreads();
  u64* o = out + wg * kFineCap;
  for (u32 i = threadIdx.x; i < total; i += kBktThreads) o[i] = stage[i];
}

// One workgroup per fine bucket b = c * 2^b2 + f.  kOwner (the multi-rank owner dedupe,
// positions = receive indices): every record of a repeated key gets the key's first index
// in oslot (`rec`), instead of the not-first words pointing at it, and mk.nf is the reply
// itself (k_own_reply_marks' flags: 7 not first, 6 the first of a repeated key, 0 else).
// (dedupe2_bucket: the workgroup's bucket `bucket`; k_bkt_dedupe2 takes bucket = blockIdx.x,
// k_bkt_dedupe2_redo the buckets the bitmap dedupe handed back)
template <bool kOwner>
__device__ __forceinline__ void dedupe2_bucket(u32 bucket, const u64* __restrict__ recs, const u32* __restrict__ fo,
                                               Bkt2Plan bp, u32* __restrict__ rec, Marks mk, Header* __restrict__ hdr,
                                               u32* __restrict__ ovf) {
  constexpr u32 TS = kBktSlots;
  const bool collapse = !kOwner && hdr && hdr->predup != 0;   // (repeat_bits: the provisional words exist)
  __shared__ u64 s_key[TS];
  __shared__ u32 s_pos[TS];
  __shared__ u32 s_dup[TS / 32];
  __shared__ u32 s_pre[513], s_beg[512];   // slices per coarse bucket <= 512
  __shared__ u32 s_wt[kBktThreads / 64];
  const u32 nb2 = 1u << bp.b2;
  const u32 c = bucket >> bp.b2, f = bucket & (nb2 - 1);
  const u32 ns = bp.nslice;
  {   // this bucket's run in every slice: loaded in parallel, block exclusive scan of the lengths
    const u32 t = threadIdx.x, lane = t & 63, wave = t >> 6;
    u32 len = 0;
    if (t < ns) {
      const u32* fs = fo + u64(c * ns + t) * (nb2 + 1);
      const u32 a = fs[f];
      len = fs[f + 1] - a;
      s_beg[t] = a;
    }
    u32 inc = len;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(inc, o, 64);
      if (int(lane) >= o) inc += y;
    }
    if (lane == 63) s_wt[wave] = inc;
    __syncthreads();
    u32 pre = 0;
    for (u32 w = 0; w < wave; ++w) pre += s_wt[w];
    if (t < ns) s_pre[t] = pre + inc - len;
    if (t == ns - 1) s_pre[ns] = pre + inc;
  }
  for (u32 q = threadIdx.x; q < TS; q += kBktThreads) {
    s_key[q] = kEmpty;
    s_pos[q] = ~0u;
  }
  for (u32 q = threadIdx.x; q < TS / 32; q += kBktThreads) s_dup[q] = 0;
  __syncthreads();
  const u32 total = s_pre[ns];
  const u64 pmask = (1ull << bp.P) - 1;
  auto record = [&](u32 i, u64& key, u32& pos) {   // record i of the bucket: its key bits and position
    u32 lo = 0, hi = ns - 1;   // slice of record i: the last s with s_pre[s] <= i
    while (lo < hi) {
      const u32 mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const u64 v = recs[u64(c * ns + lo) * kFineCap + s_beg[lo] + (i - s_pre[lo])];
    key = v >> bp.P;
    pos = u32(u64(lo) * bp.SC * kPartChunk + (v & pmask));
  };
  if (total > u32(kBktCap)) {
    // More records than registers hold (hot keys: repeats beyond the block collapse): the
    // same three steps in passes over the records, the LDS table kept across them.  Only
    // more distinct keys than the table holds overflow (the host rebuilds with the table).
    __shared__ u32 s_full;
    if (threadIdx.x == 0) s_full = 0;
    __syncthreads();
    auto find = [&](u64 key, bool insert) -> u32 {   // slot of key (inserting), ~0 when full
      u32 h = u32((u64(u32(bkt_hash(key))) * TS) >> 32);
      for (u32 probe = 0; probe < TS; ++probe) {
        unsigned long long cv = s_key[h];
        if (cv == kEmpty && insert) cv = atomicCAS(&s_key[h], kEmpty, (unsigned long long)key);
        if (cv == key) {
          if (insert) atomicOr(&s_dup[h >> 5], 1u << (h & 31));
          return h;
        }
        if (cv == kEmpty) return h;
        h = h + 1 == TS ? 0u : h + 1;
      }
      return ~0u;
    };
    const u32 wlane = threadIdx.x & 63u;   // (every lane of a wave runs the same passes)
    for (u32 i = threadIdx.x; i - wlane < total; i += kBktThreads) {
      const bool act = i < total;
      u64 key = kEmpty;
      u32 pos = 0, sl = 0;
      if (act) record(i, key, pos);
      if (act) sl = find(key, true);
      if (act && sl == ~0u) s_full = 1;
    }
    __syncthreads();
    if (s_full) {
      if (threadIdx.x == 0) *ovf = 1;
      return;
    }
    for (int pass = 0; pass < 2; ++pass) {   // 0: first positions of repeated keys, 1: the marks
      for (u32 i = threadIdx.x; i - wlane < total; i += kBktThreads) {
        const bool act = i < total;
        u64 key = kEmpty;
        u32 pos = 0, sl = 0;
        if (act) {
          record(i, key, pos);
          sl = find(key, false);
        }
        const bool dup = act && ((s_dup[sl >> 5] >> (sl & 31)) & 1u);
        if (pass == 0) {
          if (dup) atomicMin(&s_pos[sl], pos);
          continue;
        }
        if constexpr (!kOwner) nf_list_add(bp, hdr, dup && pos != s_pos[sl], pos);
        if (!dup) continue;
        const u32 first = s_pos[sl];
        if constexpr (kOwner) {
          rec[pos] = first;
          mk.nf[pos] = pos != first ? 7 : 6;
          if (bp.olist && pos != first) bp.olist[atomicAdd(bp.ocnt, 1u)] = pos;
        } else if (pos != first) {
          mk.nf[pos] = kNfNot;
          rec[pos] = first | repeat_bits(bp, rec, pos, collapse);
        } else {
          mk.multi[pos] = 1;
        }
      }
      __syncthreads();
    }
    return;
  }
  __shared__ u32 s_gs[(kBktCap + 63) / 64];   // the slice holding record 64 g
  for (u32 t = threadIdx.x; t < ns; t += kBktThreads)
    for (u32 g = (s_pre[t] + 63) >> 6; (g << 6) < s_pre[t + 1]; ++g) s_gs[g] = t;
  __syncthreads();
  u64 key[kBktCapItems];
  u32 pos[kBktCapItems], slot[kBktCapItems];
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    const u32 i = u32(e) * kBktThreads + threadIdx.x;
    key[e] = kEmpty;
    if (i >= total) continue;
    // slice of record i: the last s with s_pre[s] <= i, between the slices of its group's
    // first record and the next group's
    u32 lo = s_gs[i >> 6], hi = (i >> 6) + 1 < ((total + 63) >> 6) ? s_gs[(i >> 6) + 1] : ns - 1;
    while (lo < hi) {
      const u32 mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const u64 v = recs[u64(c * ns + lo) * kFineCap + s_beg[lo] + (i - s_pre[lo])];
    key[e] = v >> bp.P;
    pos[e] = u32(u64(lo) * bp.SC * kPartChunk + (v & pmask));
  }
  auto insert = [&](u64 k, bool several) -> u32 {   // slot of k; a second holder sets its repeat bit
    u32 h = u32((u64(u32(bkt_hash(k))) * TS) >> 32);
    for (;;) {
      unsigned long long cv = s_key[h];
      if (cv == kEmpty) cv = atomicCAS(&s_key[h], kEmpty, (unsigned long long)k);
      if (cv == k) several = true;   // another position holds it
      if (cv == kEmpty || cv == k) break;
      h = h + 1 == TS ? 0u : h + 1;
    }
    if (several) atomicOr(&s_dup[h >> 5], 1u << (h & 31));
    return h;
  };
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    slot[e] = 0;
    if (key[e] != kEmpty) slot[e] = insert(key[e], false);
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e)
    if (key[e] != kEmpty && ((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u)) atomicMin(&s_pos[slot[e]], pos[e]);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kBktCapItems; ++e) {
    const bool dup = key[e] != kEmpty && ((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u);
    if constexpr (!kOwner) nf_list_add(bp, hdr, dup && pos[e] != s_pos[slot[e]], pos[e]);
    if (!dup) continue;
    const u32 first = s_pos[slot[e]];
    if constexpr (kOwner) {
      rec[pos[e]] = first;
      mk.nf[pos[e]] = pos[e] != first ? 7 : 6;
      if (bp.olist && pos[e] != first) bp.olist[atomicAdd(bp.ocnt, 1u)] = pos[e];
    } else if (pos[e] != first) {
      mk.nf[pos[e]] = kNfNot;
      rec[pos[e]] = first | repeat_bits(bp, rec, pos[e], collapse);
    } else {
      mk.multi[pos[e]] = 1;
    }
  }
}

template <bool kOwner>
__global__ __launch_bounds__(kBktThreads) void k_bkt_dedupe2(
    const u64* __restrict__ recs, const u32* __restrict__ fo, Bkt2Plan bp, u32* __restrict__ rec, Marks mk,
    Header* __restrict__ hdr, const u64* prev_count, u64 n, u32* __restrict__ ovf) {
  if (bkt2_skip(hdr, prev_count, n)) return;
  if (!kOwner && hdr->predup) bp.nfl = nullptr;   // (collapsed levels: the flag scan takes the look-back path)
  dedupe2_bucket<kOwner>(blockIdx.x, recs, fo, bp, rec, mk, hdr, ovf);
}

// The buckets k_bkt_dedupe_bm handed back (more records or repeated keys than it holds: hot keys
// of repetitive data), each workgroup taking list entries in turn; an empty list exits at once.
[[maybe_unused]] static __global__ __launch_bounds__(kBktThreads) void k_bkt_dedupe2_redo(
    const u64* __restrict__ recs, const u32* __restrict__ fo, Bkt2Plan bp, u32* __restrict__ rec, Marks mk,
    Header* __restrict__ hdr, const u64* prev_count, u64 n, u32* __restrict__ ovf) {
  if (bkt2_skip(hdr, prev_count, n)) return;
  const u32 cnt = *reinterpret_cast<volatile u32*>(bp.redo_cnt);
  if (blockIdx.x >= cnt) return;
  if (hdr->predup) bp.nfl = nullptr;
  for (u32 i = blockIdx.x; i < cnt; i += gridDim.x) {
    dedupe2_bucket<false>(bp.redo[i], recs, fo, bp, rec, mk, hdr, ovf);
    __syncthreads();   // (the LDS table is the next bucket's)
  }
}

// The two-pass levels' dedupe in a quarter of k_bkt_dedupe2's workgroup and a third of its LDS,
// so a CU holds six buckets in flight instead of two (each bucket is a chain of dependent round
// trips: run offsets, records).  Equal keys share their low kBmLog bits (the record keys are bits
// of the level's key mix), so only records whose bits another record of the bucket also set --
// the "twice" bitmap, ~2 % of them on non-repetitive data -- are hash-consed exactly, in a table
// of kBmSlots keys.  A bucket of more than kBmItems * kBmThreads records or with more such keys
// than the table holds (hot keys of repetitive data) is handed back untouched: to
// k_bkt_dedupe2_redo through bp.redo (single device), else through the overflow flag (the fused
// multi-rank schedule's owners: every rank falls back to the general schedule).
constexpr int kBmThreads = 256;
constexpr int kBmLog = 15;                   // seen / twice bitmaps of 2^15 bits (4 KB each)
constexpr u32 kBmSlots = 1024;               // the candidates' keys (12 KB)
constexpr int kBmItems = kBktCap / kBmThreads;   // records per thread (a bucket <= kBktCap)
static_assert(kBmItems * kBmThreads == kBktCap, "the bucket capacity of the table path");

// kOwner: the fused multi-rank schedule's owner dedupe (k_bkt_dedupe2<true>'s outputs; its records
// are non-repetitive data by construction: that schedule declines repetitive genomes).
template <bool kOwner>
__global__ __launch_bounds__(kBmThreads) void k_bkt_dedupe_bm(const u64* __restrict__ recs, const u32* __restrict__ fo,
                                                             Bkt2Plan bp, u32* __restrict__ rec, Marks mk,
                                                             Header* __restrict__ hdr, const u64* prev_count, u64 n,
                                                             u32* __restrict__ ovf) {
  if (bkt2_skip(hdr, prev_count, n)) return;
  if (!kOwner && hdr->predup) bp.nfl = nullptr;   // (as k_bkt_dedupe2: collapsed levels take the look-back path)
  const bool collapse = !kOwner && hdr->predup != 0;   // (repeat_bits: the provisional words exist)
  __shared__ u32 s_seen[(1u << kBmLog) / 32], s_twice[(1u << kBmLog) / 32];
  __shared__ u64 s_key[kBmSlots];
  __shared__ u32 s_pos[kBmSlots];
  __shared__ u32 s_dup[kBmSlots / 32];
  __shared__ u32 s_pre[513], s_beg[512];   // slices per coarse bucket <= 512
  __shared__ u32 s_gs[(kBktCap + 63) / 64];
  __shared__ u32 s_wt[kBmThreads / 64];
  __shared__ u32 s_full;
  const u32 nb2 = 1u << bp.b2;
  // bp.xcd: the 8 XCDs (workgroups dealt round-robin) each take a contiguous run of buckets, so
  // neighbouring buckets -- whose fine offsets share lines and whose runs meet in every slice --
  // are read through one L2
  const u32 bucket = (bp.xcd & 1u) ? u32(bkt_chunk(gridDim.x)) : u32(blockIdx.x);
  const u32 c = bucket >> bp.b2, f = bucket & (nb2 - 1);
  const u32 ns = bp.nslice;
  const u32 t = threadIdx.x, lane = t & 63, wave = t >> 6;
  {   // this bucket's run in every slice (two slices a thread), block exclusive scan of the lengths
    u32 len[2] = {0, 0};
#pragma unroll
    for (u32 k = 0; k < 2; ++k) {
      const u32 s2 = 2 * t + k;
      if (s2 < ns) {
        const u32* fs = fo + u64(c * ns + s2) * (nb2 + 1);
        const u32 a = fs[f];
        len[k] = fs[f + 1] - a;
        s_beg[s2] = a;
      }
    }
    const u32 sum = len[0] + len[1];
    u32 inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(inc, o, 64);
      if (int(lane) >= o) inc += y;
    }
    if (lane == 63) s_wt[wave] = inc;
    for (u32 q = t; q < (1u << kBmLog) / 32; q += kBmThreads) {
      s_seen[q] = 0;
      s_twice[q] = 0;
    }
    for (u32 q = t; q < kBmSlots; q += kBmThreads) {
      s_key[q] = kEmpty;
      s_pos[q] = ~0u;
    }
    for (u32 q = t; q < kBmSlots / 32; q += kBmThreads) s_dup[q] = 0;
    if (t == 0) s_full = 0;
    __syncthreads();
    u32 pre = 0;
    for (u32 w = 0; w < wave; ++w) pre += s_wt[w];
    pre += inc - sum;
    if (2 * t < ns) s_pre[2 * t] = pre;
    if (2 * t + 1 < ns) s_pre[2 * t + 1] = pre + len[0];
    if (t == kBmThreads - 1) s_pre[ns] = pre + sum;
  }
  __syncthreads();
  const u32 total = s_pre[ns];
  auto hand_back = [&] {   // (nothing of this bucket written yet)
    if (t == 0) {
      if (!kOwner && bp.redo) bp.redo[atomicAdd(bp.redo_cnt, 1u)] = bucket;
      else *ovf = 1;
    }
  };
  if (total > u32(kBktCap)) {
    hand_back();
    return;
  }
  for (u32 s2 = t; s2 < ns; s2 += kBmThreads)
    for (u32 g = (s_pre[s2] + 63) >> 6; (g << 6) < s_pre[s2 + 1]; ++g) s_gs[g] = s2;
  __syncthreads();
  const u64 pmask = (1ull << bp.P) - 1;
  u64 key[kBmItems];
  u32 pos[kBmItems];
#pragma unroll
  for (int e = 0; e < kBmItems; ++e) {
    const u32 i = u32(e) * kBmThreads + t;
    key[e] = kEmpty;
    pos[e] = 0;
    if (i >= total) continue;
    u32 lo = s_gs[i >> 6], hi = (i >> 6) + 1 < ((total + 63) >> 6) ? s_gs[(i >> 6) + 1] : ns - 1;
    while (lo < hi) {
      const u32 mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    const u64 v = recs[u64(c * ns + lo) * kFineCap + s_beg[lo] + (i - s_pre[lo])];
    key[e] = v >> bp.P;
    pos[e] = u32(u64(lo) * bp.SC * kPartChunk + (v & pmask));
  }
  constexpr u32 bmask = (1u << kBmLog) - 1u;
#pragma unroll
  for (int e = 0; e < kBmItems; ++e) {   // seen once / twice by the key's low bits
    if (key[e] == kEmpty) continue;
    const u32 b = u32(key[e]) & bmask, m = 1u << (b & 31);
    if (atomicOr(&s_seen[b >> 5], m) & m) atomicOr(&s_twice[b >> 5], m);
  }
  __syncthreads();
  auto cand = [&](u64 k) { return k != kEmpty && ((s_twice[(u32(k) & bmask) >> 5] >> (u32(k) & 31)) & 1u); };
  u32 slot[kBmItems];
#pragma unroll
  for (int e = 0; e < kBmItems; ++e) {   // the candidates into the table; a second holder marks its key
    slot[e] = ~0u;
    if (!cand(key[e])) continue;
    const u64 k = key[e];
    u32 h = u32((u64(u32(bkt_hash(k))) * kBmSlots) >> 32);
    bool several = false;
    for (u32 probe = 0;; ++probe) {
      if (probe == kBmSlots) {
        s_full = 1;
        h = ~0u;
        break;
      }
      unsigned long long cv = s_key[h];
      if (cv == kEmpty) cv = atomicCAS(&s_key[h], kEmpty, (unsigned long long)k);
      if (cv == k) several = true;
      if (cv == kEmpty || cv == k) break;
      h = h + 1 == kBmSlots ? 0u : h + 1;
    }
    slot[e] = h;
    if (several && h != ~0u) atomicOr(&s_dup[h >> 5], 1u << (h & 31));
  }
  __syncthreads();
  if (s_full) {
    hand_back();
    return;
  }
#pragma unroll
  for (int e = 0; e < kBmItems; ++e)
    if (slot[e] != ~0u && ((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u)) atomicMin(&s_pos[slot[e]], pos[e]);
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kBmItems; ++e) {
    const bool dup = slot[e] != ~0u && ((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u);
    const u32 first = dup ? s_pos[slot[e]] : 0u;
    if constexpr (!kOwner) nf_list_add(bp, hdr, dup && pos[e] != first, pos[e]);
    if (!dup) continue;
    if constexpr (kOwner) {
      rec[pos[e]] = first;
      mk.nf[pos[e]] = pos[e] != first ? 7 : 6;
      if (bp.olist && pos[e] != first) bp.olist[atomicAdd(bp.ocnt, 1u)] = pos[e];
    } else if (pos[e] != first) {
      mk.nf[pos[e]] = kNfNot;
      rec[pos[e]] = first | repeat_bits(bp, rec, pos[e], collapse);
    } else {
      mk.multi[pos[e]] = 1;
    }
  }
}

// ---- direct subtrees ----------------------------------------------------------------
// Once level k0 is known to be direct (every element of level k0-1 unique), every
// later level is too and ids are positions.  Each workgroup takes an aligned chunk
// of kDirectChunk input words and computes up to kDirectLog levels of its subtree in
// LDS -- one launch instead of 4 per level.  Only the chunk holding the global tail
// is partial, so an odd local count there is the global odd tail (null right child).
constexpr int kDirectLog = 12;
constexpr int kDirectChunk = 1 << kDirectLog;

struct DirectPlan {
  u64 layer_off[GCZ_MAX_LAYERS];   // node offset of each layer's (rank-local) slice
  u64 n[GCZ_MAX_LAYERS + 1];       // n[i]: input words of level k0 + i (rank-local)
  u32 id_off[GCZ_MAX_LAYERS];      // id of local pair 0 of each level (multi-rank: the rank's first position)
};

// Multi-rank (gcz_dist.hip): the input words of the first level may still hold the previous
// exchanged level's LOCAL ids -- gid[local id] = the global id, or the local rank tagged
// kLocalIdBit to which the rank's offset is added (k_dist_remap's translation, done here
// on the load instead of in a pass of its own).
constexpr u32 kLocalIdBit = 1u << 31;
struct DirectRemap {
  const u32* gid;   // null: the words are global
  u32 off;
};
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_direct_levels(
    const u32* __restrict__ in, int k0, int nlev, uint2* __restrict__ nodes, DirectPlan dp, u32* __restrict__ words_out,
    Header* __restrict__ hdr, DirectRemap rm = {}, const u64* guard = nullptr, u64 expect = 0) {
  // guard: a speculative launch (gcz_build.hip, ahead of the host's look at the gate) runs only
  // when the gate says the level is direct
  if (guard && *guard != expect) return;
  __shared__ __align__(16) u32 buf[2][kDirectChunk];
  const u64 base0 = u64(blockIdx.x) * kDirectChunk;
  u32 c = u32(dp.n[0] - base0 < u64(kDirectChunk) ? dp.n[0] - base0 : u64(kDirectChunk));
  auto remap = [&](u32 w) {
    const u32 g = rm.gid[w & kIdx];
    return ((g & kLocalIdBit) ? (g & ~kLocalIdBit) + rm.off : g) | (w & kBits);
  };
  if (c == u32(kDirectChunk) && (reinterpret_cast<uintptr_t>(in) & 15u) == 0) {   // a whole chunk: every 16-B load in flight first
    constexpr int V = kDirectChunk / 4 / kBlock;
    uint4 v[V];
    const uint4* src = reinterpret_cast<const uint4*>(in + base0);
#pragma unroll
    for (int q = 0; q < V; ++q) v[q] = src[q * kBlock + threadIdx.x];
    if (rm.gid) {
#pragma unroll
      for (int q = 0; q < V; ++q) {
        v[q].x = remap(v[q].x);
        v[q].y = remap(v[q].y);
        v[q].z = remap(v[q].z);
        v[q].w = remap(v[q].w);
      }
    }
#pragma unroll
    for (int q = 0; q < V; ++q) reinterpret_cast<uint4*>(buf[0])[q * kBlock + threadIdx.x] = v[q];
  } else {
    for (u32 e = threadIdx.x; e < c; e += kBlock) buf[0][e] = rm.gid ? remap(in[base0 + e]) : in[base0 + e];
  }
  __syncthreads();
  int cur = 0;
  for (int i = 0; i < nlev; ++i) {
    const int k = k0 + i;
    const u32 p = (c + 1) / 2;
    const u64 base_out = base0 >> (i + 1);
    uint2* out = nodes + dp.layer_off[k];
    for (u32 j = threadIdx.x; j < p; j += kBlock) {
      const u32 l = buf[cur][2 * j];
      const u32 r = 2 * j + 1 < c ? buf[cur][2 * j + 1] : kNullWord;
      u32 cl, cr, m, t;
      node_canonical(l, r, cl, cr, m, t);
      const u32 v = ulw(l) == ulw(xf(r, 1, 0));
      out[base_out + j] = make_uint2(cl, cr);
      buf[cur ^ 1][j] = make_word(u32(base_out + j) + dp.id_off[k], m, t, v);
    }
    __syncthreads();
    cur ^= 1;
    c = p;
  }
  const u64 base_last = base0 >> nlev;
  for (u32 e = threadIdx.x; e < c; e += kBlock) words_out[base_last + e] = buf[cur][e];
  if (blockIdx.x == 0 && threadIdx.x == 0)
    for (int i = 0; i < nlev; ++i) hdr->count[kLayerSlot + k0 + i] = dp.n[i + 1];
}

// ---- fused top levels -------------------------------------------------------------
// Once a level's input fits one workgroup (n <= kTailMaxN), all remaining
// levels run in ONE launch: words ping-pong in LDS, each level is either
// direct (previous level all unique: ids are positions) or hash-consed in an
// LDS table (CAS claims, atomicMin keeps the first position, a block scan
// ranks the first occurrences) -- the same ids, nodes and words as the
// per-level kernels, without ~4 launches per level.
#ifndef GCZ_TAIL_MAXN
#define GCZ_TAIL_MAXN 8192   // (tools/microbench/tail.hip builds other sizes)
#endif
constexpr int kTailMaxN = GCZ_TAIL_MAXN;
constexpr unsigned long long kDirectCheckMin = 1ull << 16;   // levels below: no host look at the direct gate
constexpr unsigned long long kDupProbeMin = 1ull << 17;      // fewer strands: no repetitive-data probe
constexpr int kTailThreads = 1024;
constexpr int kTailItems = kTailMaxN / 2 / kTailThreads;   // pairs per thread
constexpr int kTailSlots = kTailMaxN;                       // LDS table: load <= 1/2
// dynamic LDS: the table (one 64-bit entry per slot) and the level's words (in place)
constexpr size_t kTailLds = size_t(kTailSlots) * 8 + size_t(kTailMaxN) * 4;

// A tail level's pair key in 32 bits: child words of the tail are ids < 8192 (14 bits, the
// null word's index field becomes 0x3fff) plus the mirror and transpose bits (ulw drops v).
__device__ __forceinline__ u32 tail_ck(u32 w) { return (w & 0x3fffu) | ((w >> 15) & 0xc000u); }

struct TailOut {
  u64 layer_off[GCZ_MAX_LAYERS];   // node offset of each layer within `nodes`
};

// Tail table entry: [level tag: 5 bits][pair key: 32 bits][position, then id: 16 bits].  An
// entry of another level's tag is a free slot, so the table is cleared once per launch, and
// the minimum position of a key is one 64-bit atomicMin (equal tag and key above it).
constexpr int kTailTagShift = 59, kTailKeyShift = 16;

// A workgroup barrier for LDS hand-offs only: __syncthreads() also drains every global
// store (s_waitcnt vmcnt(0)), a memory round trip per level for the tail's node writes,
// which nothing in the launch reads.
__device__ __forceinline__ void tail_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Fused small builds: the tail settles the last fused level's repeats itself (ids by slot,
// k_flagscan_node's sid) and decides that level's gate from its count and look-ahead flag.
struct TailSettle {
  const unsigned char* nf = nullptr;   // null: the input words are final, prev_count gates
  const u32* sid = nullptr;
  const u64* pcount = nullptr;
  const u32* phashed = nullptr;
  u64* gate_out = nullptr;
};

#ifdef GCZ_TAIL_PROBE   // (tools/microbench/tail.hip: wall-clock stamps of each tail level)
__device__ unsigned long long gcz_tail_probe[64];
#define GCZ_TAIL_STAMP(i) \
  if (threadIdx.x == 0) gcz_tail_probe[(i) & 63] = wall_clock64()
#else
#define GCZ_TAIL_STAMP(i)
#endif

[[maybe_unused]] static __global__ __launch_bounds__(kTailThreads) void k_tail(
    const u32* __restrict__ in, u64 n0, const u64* prev_count, int k0, int D, uint2* __restrict__ nodes, TailOut to,
    Header* __restrict__ hdr, const u64* __restrict__ shards, TailSettle st) {
  extern __shared__ __align__(16) unsigned char tail_lds[];
  unsigned long long* tab = reinterpret_cast<unsigned long long*>(tail_lds);
  u32* wbuf = reinterpret_cast<u32*>(tab + kTailSlots);
  __shared__ u32 wsum[kTailItems * (kTailThreads / 64)];
  __shared__ u64 s_off[GCZ_MAX_LAYERS];   // the layer offsets, read once (not per level from the arguments)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < GCZ_MAX_LAYERS) s_off[tid] = to.layer_off[tid];
  u64 sv0 = 0, sv1 = 0;   // shards != null: this launch ends the build (k_build_finish's sum)
  if (shards) {
    sv0 = shards[tid * kStatStride];
    sv1 = shards[tid * kStatStride + 1];
  }
  {   // the input words (and marks): every load in flight at once (n0 <= kTailMaxN)
    constexpr int kW = kTailMaxN / kTailThreads;
    u32 v[kW];
    unsigned char f[kW];
#pragma unroll
    for (int e = 0; e < kW; ++e) {
      const u64 i = u64(e) * kTailThreads + tid;
      v[e] = i < n0 ? in[i] : 0u;
      f[e] = st.nf && i < n0 ? st.nf[i] : kNfMaybe;
    }
#pragma unroll
    for (int e = 0; e < kW; ++e) {
      const u64 i = u64(e) * kTailThreads + tid;
      if (f[e] == kNfNot) v[e] = st.sid[v[e] & kIdx] | (v[e] & kBits);
      if (i < n0) wbuf[i] = v[e];
    }
  }
  for (int q = tid; q < kTailSlots; q += kTailThreads) tab[q] = 0;   // tag 0: no level
  u32 n = u32(n0);
  bool direct;
  if (st.nf) {
    direct = *st.pcount == n0 || *st.phashed == 0;
    if (tid == 0) *st.gate_out = direct ? n0 : ~0ull;
  } else {
    direct = prev_count && *prev_count == n0;
  }
  __syncthreads();
  int k = k0;
  GCZ_TAIL_STAMP(0);
  for (; k < D && n > 128; ++k) {   // the whole block while a level has more than 64 pairs
    GCZ_TAIL_STAMP(k - k0 + 1);
    const u32 p = (n + 1) / 2;
    uint2* out = nodes + s_off[k];
    const u64 tag = u64(k - k0 + 1) << kTailTagShift;   // (<= 14 levels: 8192 words down to 1)
    u32 cl[kTailItems], cr[kTailItems], mtv[kTailItems], slot[kTailItems];
#pragma unroll
    for (int e = 0; e < kTailItems; ++e) {   // pair j = e * kTailThreads + tid: position order is (e, tid)
      const u32 j = u32(e * kTailThreads + tid);
      cl[e] = cr[e] = mtv[e] = slot[e] = 0;
      if (j < p) {
        const u32 l = wbuf[2 * j], r = 2 * j + 1 < n ? wbuf[2 * j + 1] : kNullWord;
        u32 m, t;
        node_canonical(l, r, cl[e], cr[e], m, t);
        mtv[e] = make_word(0, m, t, ulw(l) == ulw(xf(r, 1, 0)));
      }
    }
    u32 count;
    if (direct) {
      tail_sync();   // (every read of the level's words is done: they are rewritten in place)
#pragma unroll
      for (int e = 0; e < kTailItems; ++e) {
        const u32 j = u32(e * kTailThreads + tid);
        if (j < p) {
          out[j] = make_uint2(cl[e], cr[e]);
          wbuf[j] = j | mtv[e];
        }
      }
      count = p;
    } else {
      u32 mask = 1;
      while (mask < 2 * p) mask <<= 1;
      mask -= 1;
#pragma unroll
      for (int e = 0; e < kTailItems; ++e) {
        const u32 j = u32(e * kTailThreads + tid);
        if (j < p) {
          const u32 key = (tail_ck(ulw(cl[e])) << 16) | tail_ck(ulw(cr[e]));
          const unsigned long long mine = tag | (u64(key) << kTailKeyShift) | j;
          u32 s = slot_hash(key) & mask;
          for (;;) {
            unsigned long long c = tab[s];
            if ((c >> kTailTagShift) != (tag >> kTailTagShift)) {   // free (an older level's entry)
              const unsigned long long o = atomicCAS(&tab[s], c, mine);
              if (o == c) break;
              c = o;
              if ((c >> kTailTagShift) != (tag >> kTailTagShift)) continue;
            }
            if (u32(c >> kTailKeyShift) == key) {
              atomicMin(&tab[s], mine);
              break;
            }
            s = (s + 1) & mask;
          }
          slot[e] = s;
        }
      }
      tail_sync();
      u64 bal[kTailItems];
#pragma unroll
      for (int e = 0; e < kTailItems; ++e) {
        const u32 j = u32(e * kTailThreads + tid);
        bal[e] = __ballot(j < p && u32(tab[slot[e]] & 0xffffu) == j);
        if (lane == 0) wsum[e * (kTailThreads / 64) + wave] = u32(__popcll(bal[e]));
      }
      tail_sync();   // (every position read is done: firsts now overwrite theirs with the id)
      // firsts before (item e, wave w): all of items < e, then waves < w -- every wave scans
      // the 64 (item, wave) counts itself
      constexpr int kNW = kTailThreads / 64;
      static_assert(kTailItems * kNW <= 64, "one wave-wide scan of the tail's (item, wave) counts");
      const u32 c = lane < kTailItems * kNW ? wsum[lane] : 0u;
      u32 incl = c;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
      }
      count = u32(__shfl(int(incl), 63, 64));
#pragma unroll
      for (int e = 0; e < kTailItems; ++e) {
        const u32 base = u32(__shfl(int(incl - c), e * kNW + wave, 64));
        if ((bal[e] >> lane) & 1ull) {
          const u32 id = base + u32(__popcll(bal[e] & ((1ull << lane) - 1)));
          tab[slot[e]] = (tab[slot[e]] & ~0xffffull) | id;
          out[id] = make_uint2(cl[e], cr[e]);
        }
      }
      tail_sync();
#pragma unroll
      for (int e = 0; e < kTailItems; ++e) {
        const u32 j = u32(e * kTailThreads + tid);
        if (j < p) wbuf[j] = u32(tab[slot[e]] & 0xffffu) | mtv[e];
      }
    }
    if (tid == 0) hdr->count[kLayerSlot + k] = count;
    direct = count == p;
    n = p;
    tail_sync();
  }
  if (shards) stats_sum(sv0, sv1, hdr);   // (its loads went out at the start)
  // the last levels (<= 64 pairs) in wave 0 alone, with no barriers: lane j holds pair j, a
  // key's first occurrence is the lowest lane holding it (a uniform sweep of readlanes),
  // ids are ranks among the first lanes
  if (wave != 0) return;
  for (; k < D; ++k) {
    GCZ_TAIL_STAMP(k - k0 + 1);
    const u32 p = (n + 1) / 2, j = u32(lane);
    u32 cl = 0, cr = 0, mtv = 0;
    if (j < p) {
      const u32 l = wbuf[2 * j], r = 2 * j + 1 < n ? wbuf[2 * j + 1] : kNullWord;
      u32 m, t;
      node_canonical(l, r, cl, cr, m, t);
      mtv = make_word(0, m, t, ulw(l) == ulw(xf(r, 1, 0)));
    }
    u32 id = j, count = p;
    if (!direct) {
      const u32 ka = ulw(cl), kb = ulw(cr);
      u32 f = 64;
      for (u32 q = 0; q < p; ++q) {
        const u32 qa = __builtin_amdgcn_readlane(ka, q), qb = __builtin_amdgcn_readlane(kb, q);
        if (f == 64 && qa == ka && qb == kb) f = q;
      }
      const u64 bal = __ballot(j < p && f == j);
      const u32 rank = u32(__popcll(bal & ((1ull << lane) - 1)));
      id = u32(__shfl(int(rank), int(f & 63), 64));
      count = u32(__popcll(bal));
      if (j < p && f == j) nodes[s_off[k] + rank] = make_uint2(cl, cr);
    } else if (j < p) {
      nodes[s_off[k] + j] = make_uint2(cl, cr);
    }
    if (j < p) wbuf[j] = id | mtv;   // (every lane has read the level: LDS is in order per wave)
    if (lane == 0) hdr->count[kLayerSlot + k] = count;
    direct = count == p;
    n = p;
  }
  if (lane == 0) hdr->root = wbuf[0];
  GCZ_TAIL_STAMP(63);
}

[[maybe_unused]] static __global__ void k_root(const u32* __restrict__ words, Header* __restrict__ hdr) { hdr->root = words[0]; }

// Clear a node level's table (all ones) and marks (zero) unless the level is direct.
[[maybe_unused]] static __global__ __launch_bounds__(kBlock) void k_clear(uint4* __restrict__ tab, u64 tab16, uint4* __restrict__ nf,
                                                 uint4* __restrict__ multi, u64 p16, const u64* prev_count,
                                                 u64 prev_n, const Header* __restrict__ hdr, u32 bkt) {
  if (level_direct(prev_count, prev_n)) return;
  if (bkt == 2 || (bkt && hdr->predup == 0)) tab16 = 0;   // bucketed insert: no table
  const uint4 ones = make_uint4(~0u, ~0u, ~0u, ~0u), zero = make_uint4(0, 0, 0, 0);
  const u64 stride = u64(gridDim.x) * kBlock;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < tab16; i += stride) tab[i] = ones;
  for (u64 i = u64(blockIdx.x) * kBlock + threadIdx.x; i < p16; i += stride) {
    nf[i] = zero;
    multi[i] = zero;
  }
}

}  // namespace gcz_dev
