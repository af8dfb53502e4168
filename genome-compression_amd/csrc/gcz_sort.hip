// Frequency sort, bytes() and the .dag writer on the device (SURVEY §8(f)
// rows 1-2).  Reference: shared_tree::histogram / sort_leaves / sort_nodes /
// sort_tree / rewire_nodes (src/shared_tree.cpp:316-483), bytes (:488-496),
// serialize (:504-513), pointer::serialize (:122-142); spec: SURVEY App. C.
//
// Net effect of sort_tree: every child layer (the leaves and node layers
// 0..D-2) is permuted independently by the reference counts its parent layer
// holds, descending, ties by the old index (std::stable_sort); parents are
// rewired with the m/t/v bits kept; the top layer and the root stay.  On the
// device:
//  * histogram per parent layer: a large layer that references each child many
//    times (the leaves) is partitioned by child-id range (2^15 ids per bucket: count
//    matrix, look-back scan, a scatter of 2-B records) and every bucket is counted by
//    one workgroup in LDS, which also reduces the layer's min / max count; other
//    layers count with global atomics (their references come in near id order);
//  * per child layer whose counts are not all equal (else the order is the
//    identity), a stable LSD counting sort of (hi - count) in passes of <= 8 bits:
//    per-tile digit counts, a scan, and a scatter whose in-tile ranks come from
//    wave ballots (a match mask per digit, so equal digits keep their order); the
//    last pass writes each element's new position directly;
//  * one pass over every node layer that rewires children and permutes the layer.
// The .dag is written by an exclusive scan of per-node byte sizes and one
// byte-scatter pass.
#include "gcz_ctx.h"
#include "gcz_scan.h"

using namespace gcz_dev;
using namespace gcz_host;

struct gcz_sort_state {
  bool warm = false;   // k_sort_warm launched (gcz_sort_reserve)
  DevBuf cnt, keys, keys2, vals, vals2, newpos, mm, acc, dag, nodes2, leaves2, dw1, dw2, text;
  DevBuf hmat, hoff, hrec, desc;   // partitioned histogram; scan descriptors
  DevBuf hslot, hval, hbs;         // its records' positions per word, new children, bucket starts
  DevBuf hpart;                    // per-block (min, max) counts
  u32* h_mm = nullptr;
  u64* h_tot = nullptr;
};

void gcz_sort_state_free(gcz_ctx* c) {
  gcz_sort_state* s = c->sortst;
  if (!s) return;
  for (DevBuf* b : {&s->cnt, &s->keys, &s->keys2, &s->vals, &s->vals2, &s->newpos, &s->mm, &s->acc, &s->dag,
                    &s->nodes2, &s->leaves2, &s->dw1, &s->dw2, &s->text, &s->hmat, &s->hoff, &s->hrec, &s->desc,
                    &s->hslot, &s->hval, &s->hbs, &s->hpart})
    if (b->ptr) (void)hipFree(b->ptr);
  if (s->h_mm) (void)hipHostFree(s->h_mm);
  if (s->h_tot) (void)hipHostFree(s->h_tot);
  delete s;
  c->sortst = nullptr;
}

namespace {

constexpr u32 kSegStart1 = 16, kSegStart2 = 16 + 4096, kSegStart3 = 16 + 4096 + 1048576;

__device__ __forceinline__ bool is_null(u32 w) { return ulw(w) == kIdx; }

__device__ __forceinline__ u32 ptr_bytes(u32 w) {   // pointer::bytes, src/shared_tree.cpp:122-125
  const u32 i = w & kIdx;
  if (i == kIdx) return 4;
  return i < kSegStart1 ? 1 : i < kSegStart2 ? 2 : i < kSegStart3 ? 3 : 4;
}

// pointer::serialize (src/shared_tree.cpp:133-142)
__device__ __forceinline__ void put_ptr(unsigned char* o, u32 w) {
  const u32 idx = w & kIdx;
  u32 seg, off;
  if (idx == kIdx) { seg = 3; off = 0xfffffffu; }
  else if (idx < kSegStart1) { seg = 0; off = idx; }
  else if (idx < kSegStart2) { seg = 1; off = idx - kSegStart1; }
  else if (idx < kSegStart3) { seg = 2; off = idx - kSegStart2; }
  else { seg = 3; off = idx - kSegStart3; }
  const int bits = 4 + 8 * int(seg);
  int sh = bits - 4;
  *o++ = (unsigned char)((off >> sh) | (((w >> 29) & 1u) << 4) | (((w >> 30) & 1u) << 5) | (seg << 6));
  for (sh -= 8; sh >= 0; sh -= 8) *o++ = (unsigned char)(off >> sh);
}

__device__ __forceinline__ void put_be(unsigned char* o, u64 v, int nbytes) {   // binary_write, utility.h:178-184
  for (int i = nbytes - 1; i >= 0; --i) *o++ = (unsigned char)(v >> (8 * i));
}

// ---- partitioned histogram (parent layers of >= 2^20 words) ----
// Buckets of 2^kHB child ids; chunks of kHChunk parent words (one count-matrix
// column each, dealt to XCDs in contiguous runs like the build's bucket chunks).
constexpr int kHThreads = 1024;
constexpr int kHItems = 64;
constexpr u64 kHChunk = u64(kHThreads) * kHItems;
constexpr int kHBatch = 16;
constexpr u32 kHB = 15;                 // ids per bucket: 2^15 (LDS counters, 128 KB)
constexpr u32 kHMaxBuckets = 4096;      // child layers of <= 2^27 nodes (LDS cursors, 16 KB)

__device__ __forceinline__ u64 h_chunk(u64 G) {
  const u64 b = blockIdx.x, per = G / 8;
  return b < 8 * per ? (b % 8) * per + b / 8 : b;
}

__global__ __launch_bounds__(kHThreads) void k_hcount(const u32* __restrict__ words, u64 nw, u32 nb, u64 G,
                                                      u32* __restrict__ mat) {
  __shared__ u32 hist[kHMaxBuckets];
  for (u32 q = threadIdx.x; q < nb; q += kHThreads) hist[q] = 0;
  __syncthreads();
  const u64 g = h_chunk(G), j0 = g * kHChunk;
  for (int e0 = 0; e0 < kHItems; e0 += kHBatch) {   // (a batch of loads in flight)
    u32 wv[kHBatch];
#pragma unroll
    for (int e = 0; e < kHBatch; ++e) {
      const u64 j = j0 + u64(e0 + e) * kHThreads + threadIdx.x;
      wv[e] = j < nw ? words[j] : kIdx;
    }
#pragma unroll
    for (int e = 0; e < kHBatch; ++e)
      if (!is_null(wv[e])) atomicAdd(&hist[(wv[e] & kIdx) >> kHB], 1u);
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < nb; q += kHThreads) mat[u64(q) * G + g] = hist[q];
}

// slot != null: also each word's record position (the rewire reads its new child back
// from there, k_hremap)
__global__ __launch_bounds__(kHThreads) void k_hscatter(const u32* __restrict__ words, u64 nw, u32 nb, u64 G,
                                                        const u32* __restrict__ off,
                                                        unsigned short* __restrict__ rec, u32* __restrict__ slot) {
  __shared__ u32 cur[kHMaxBuckets];
  const u64 g = h_chunk(G), j0 = g * kHChunk;
  for (u32 q = threadIdx.x; q < nb; q += kHThreads) cur[q] = off[u64(q) * G + g];
  __syncthreads();
#pragma unroll 8
  for (int e = 0; e < kHItems; ++e) {
    const u64 j = j0 + u64(e) * kHThreads + threadIdx.x;
    if (j >= nw) break;
    const u32 w = words[j];
    if (is_null(w)) continue;
    const u32 id = w & kIdx;
    const u32 d = atomicAdd(&cur[id >> kHB], 1u);
    rec[d] = (unsigned short)(id & ((1u << kHB) - 1));
    if (slot) slot[j] = d;
  }
}

// The same partition staged in LDS (buckets <= kHStagedMax): the chunk's records are
// placed at their in-chunk rank (LDS cursors from the chunk's count column), then stored
// as one contiguous run per bucket -- scattered 2-B stores become coalesced runs.
constexpr u32 kHStagedMax = 2048;

__global__ __launch_bounds__(kHThreads) void k_hscatter_lds(const u32* __restrict__ words, u64 nw, u32 nb, u64 G,
                                                            const u32* __restrict__ mat, const u32* __restrict__ off,
                                                            unsigned short* __restrict__ rec,
                                                            u32* __restrict__ slot) {
  __shared__ u32 s_cur[kHStagedMax];     // in-chunk starts, then cursors, then ends
  __shared__ u32 s_delta[kHStagedMax];   // global start - in-chunk start, per bucket
  __shared__ u32 s_wave[kHThreads / 64];
  __shared__ unsigned short s_rec[kHChunk];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u64 g = h_chunk(G), j0 = g * kHChunk;
  // exclusive scan of the chunk's bucket counts (two per thread: nb <= 2048)
  const u32 q0 = 2 * tid;
  const u32 c0 = q0 < nb ? mat[u64(q0) * G + g] : 0u, c1 = q0 + 1 < nb ? mat[u64(q0 + 1) * G + g] : 0u;
  const u32 o0 = q0 < nb ? off[u64(q0) * G + g] : 0u, o1 = q0 + 1 < nb ? off[u64(q0 + 1) * G + g] : 0u;
  u32 incl = c0 + c1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 y = __shfl_up(incl, o, 64);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wave[wave] = incl;
  __syncthreads();
  u32 base = 0;
  for (int w = 0; w < wave; ++w) base += s_wave[w];
  const u32 st0 = base + incl - (c0 + c1), st1 = st0 + c0;
  if (q0 < nb) { s_cur[q0] = st0; s_delta[q0] = o0 - st0; }
  if (q0 + 1 < nb) { s_cur[q0 + 1] = st1; s_delta[q0 + 1] = o1 - st1; }
  __syncthreads();
  for (int e0 = 0; e0 < kHItems; e0 += kHBatch) {   // (a batch of loads in flight)
    u32 wv[kHBatch];
#pragma unroll
    for (int e = 0; e < kHBatch; ++e) {
      const u64 j = j0 + u64(e0 + e) * kHThreads + tid;
      wv[e] = j < nw ? words[j] : kIdx;
    }
#pragma unroll
    for (int e = 0; e < kHBatch; ++e) {
      if (is_null(wv[e])) continue;
      const u64 j = j0 + u64(e0 + e) * kHThreads + tid;
      const u32 id = wv[e] & kIdx, q = id >> kHB;
      const u32 d = atomicAdd(&s_cur[q], 1u);
      s_rec[d] = (unsigned short)(id & ((1u << kHB) - 1));
      if (slot) slot[j] = s_delta[q] + d;
    }
  }
  __syncthreads();
  // s_cur[q] is now bucket q's in-chunk end: record i belongs to the first q with end > i
  const u32 nrec = s_cur[nb - 1];
  for (u32 i = tid; i < nrec; i += kHThreads) {
    u32 lo = 0, hi = nb - 1;
    while (lo < hi) {
      const u32 mid = (lo + hi) >> 1;
      if (s_cur[mid] > i) hi = mid;
      else lo = mid + 1;
    }
    rec[s_delta[lo] + i] = s_rec[i];
  }
}

// S workgroups per bucket, each counting a slice of its records in LDS counters for the
// bucket's 2^kHB ids.  S = 1: the counters are written coalesced and the block's min / max
// folded into mm[0..1]; S > 1: added into cnt (zeroed) with coalesced atomics (the layer's
// min / max taken afterwards).
__global__ __launch_bounds__(kHThreads) void k_hbucket(const unsigned short* __restrict__ rec,
                                                       const u32* __restrict__ off, u64 G, u64 nc, u32 S,
                                                       u32* __restrict__ cnt, u32* __restrict__ mm,
                                                       u32* __restrict__ bstart) {
  extern __shared__ u32 c32[];   // 2^kHB counters (dynamic: 128 KB)
  __shared__ u32 smin[kHThreads / 64], smax[kHThreads / 64];
  const u64 b = blockIdx.x / S;
  const u32 sub = blockIdx.x % S;
  for (u32 q = threadIdx.x; q < (1u << kHB); q += kHThreads) c32[q] = 0;
  __syncthreads();
  const u32 r0 = off[b * G], r1 = off[(b + 1) * G];
  if (bstart && sub == 0 && threadIdx.x == 0) {   // (the records' bucket boundaries, kept for k_hremap)
    bstart[b] = r0;
    if (b + 1 == gridDim.x / S) bstart[b + 1] = r1;
  }
  const u32 len = r1 - r0;
  const u32 s0 = r0 + u32(u64(len) * sub / S), s1 = r0 + u32(u64(len) * (sub + 1) / S);
  for (u32 i = s0 + threadIdx.x; i < s1; i += kHThreads) atomicAdd(&c32[rec[i]], 1u);
  __syncthreads();
  const u64 id0 = b << kHB;
  if (S > 1) {
    for (u32 q = threadIdx.x; q < (1u << kHB); q += kHThreads) {
      if (id0 + q >= nc) break;
      const u32 v = c32[q];
      if (v) atomicAdd(&cnt[id0 + q], v);
    }
    return;
  }
  u32 lo = ~0u, hi = 0;
  for (u32 q = threadIdx.x; q < (1u << kHB); q += kHThreads) {
    if (id0 + q >= nc) break;
    const u32 v = c32[q];
    cnt[id0 + q] = v;
    lo = min(lo, v);
    hi = max(hi, v);
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, u32(__shfl_xor(int(lo), o, 64)));
    hi = max(hi, u32(__shfl_xor(int(hi), o, 64)));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { smin[wave] = lo; smax[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kHThreads / 64; ++w) { lo = min(lo, smin[w]); hi = max(hi, smax[w]); }
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

// The partitioned layer's new child positions in record order: one workgroup per bucket
// with the bucket's 2^kHB new positions in LDS (a random gather into the whole newpos
// array becomes an LDS lookup; the rewire then reads val[slot[j]], whose records for a
// chunk of words sit in one short run per bucket).
__global__ __launch_bounds__(kHThreads) void k_hremap(const unsigned short* __restrict__ rec,
                                                      const u32* __restrict__ bstart, const u32* __restrict__ np,
                                                      u64 nc, u32 S, u32* __restrict__ val) {
  extern __shared__ u32 tab[];   // 2^kHB new positions (dynamic: 128 KB)
  const u64 b = blockIdx.x / S, id0 = b << kHB;
  const u32 sub = blockIdx.x % S;
  for (u32 q = threadIdx.x; q < (1u << kHB); q += kHThreads) tab[q] = id0 + q < nc ? np[id0 + q] : 0u;
  __syncthreads();
  const u32 r0 = bstart[b], len = bstart[b + 1] - r0;
  const u32 s0 = r0 + u32(u64(len) * sub / S), s1 = r0 + u32(u64(len) * (sub + 1) / S);
  for (u32 i = s0 + threadIdx.x; i < s1; i += kHThreads) val[i] = tab[rec[i]];
}

// ---- stable counting sort by count, descending (LSD passes of <= 8 bits) ----
// key = hi - count (ascending order <=> descending counts); a tile of kCsTile
// elements, each wave taking 1024 consecutive ones (item e of lane l: element
// e * 64 + l, in order), so ranks follow positions.
constexpr int kCsThreads = 256;
constexpr int kCsItems = 16;
constexpr u64 kCsWaveSpan = 64 * kCsItems;
constexpr u64 kCsTile = u64(kCsThreads) * kCsItems;

struct CsPass {
  const u32* cnt;      // first pass: counts (key = hi - cnt[i], value = i)
  const u32* keys;     // later passes: keys / values of the previous pass
  const u32* vals;
  u32 hi;
  u32 shift, bits;     // digit = (key >> shift) & (2^bits - 1)
  u64 n;
  __device__ __forceinline__ u32 key(u64 i) const { return cnt ? hi - cnt[i] : keys[i]; }
  __device__ __forceinline__ u32 val(u64 i) const { return cnt ? u32(i) : vals[i]; }
  __device__ __forceinline__ u32 digit(u32 k) const { return (k >> shift) & ((1u << bits) - 1u); }
};

// (equal digits of a wave counted once: the lowest lane of each match adds the match's size)
__global__ __launch_bounds__(kCsThreads) void k_cs_count(CsPass P, u64 ntiles, u32* __restrict__ mat) {
  __shared__ u32 hist[256];
  const u32 R = 1u << P.bits;
  for (u32 q = threadIdx.x; q < R; q += kCsThreads) hist[q] = 0;
  __syncthreads();
  const u64 t = blockIdx.x, i0 = t * kCsTile;
  const int lane = threadIdx.x & 63;
  const u64 lt = (1ull << lane) - 1;
  u32 key[kCsItems];
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = i0 + u64(e) * kCsThreads + threadIdx.x;
    key[e] = i < P.n ? P.key(i) : 0u;
  }
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = i0 + u64(e) * kCsThreads + threadIdx.x;
    const bool ok = i < P.n;
    const u32 d = P.digit(key[e]);
    u64 m = __ballot(ok);
    for (u32 b = 0; b < P.bits; ++b) {
      const u64 bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    if (ok && (m & lt) == 0) atomicAdd(&hist[d], u32(__popcll(m)));
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < R; q += kCsThreads) mat[u64(q) * ntiles + t] = hist[q];
}

// off = exclusive scan of the digit-major matrix.  last pass: newpos[value] = rank;
// else keys_out / vals_out at the rank.
__global__ __launch_bounds__(kCsThreads) void k_cs_scatter(CsPass P, u64 ntiles, const u32* __restrict__ off,
                                                           u32* __restrict__ keys_out, u32* __restrict__ vals_out,
                                                           u32* __restrict__ newpos) {
  __shared__ u32 wc[kCsThreads / 64][256];
  const u32 R = 1u << P.bits;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (u32 q = threadIdx.x; q < R * (kCsThreads / 64); q += kCsThreads) wc[q / R][q % R] = 0;
  __syncthreads();
  const u64 t = blockIdx.x;
  const u64 w0 = t * kCsTile + u64(wave) * kCsWaveSpan;
  const u64 lt = (1ull << lane) - 1;
  u32 key[kCsItems], rank[kCsItems];
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = w0 + u64(e) * 64 + lane;
    const bool ok = i < P.n;
    key[e] = ok ? P.key(i) : 0u;
    const u32 d = P.digit(key[e]);
    u64 m = __ballot(ok);
    for (u32 b = 0; b < P.bits; ++b) {
      const u64 bal = __ballot((d >> b) & 1u);
      m &= ((d >> b) & 1u) ? bal : ~bal;
    }
    const u32 base = ok ? wc[wave][d] : 0u;
    rank[e] = base + u32(__popcll(m & lt));
    if (ok && (m & lt) == 0) wc[wave][d] = base + u32(__popcll(m));   // the lowest lane of the match
  }
  __syncthreads();
  for (u32 q = threadIdx.x; q < R; q += kCsThreads) {   // exclusive prefix over the waves, per digit
    u32 run = off[u64(q) * ntiles + t];
    for (int w = 0; w < kCsThreads / 64; ++w) {
      const u32 v = wc[w][q];
      wc[w][q] = run;
      run += v;
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kCsItems; ++e) {
    const u64 i = w0 + u64(e) * 64 + lane;
    if (i >= P.n) continue;
    const u32 dst = wc[wave][P.digit(key[e])] + rank[e];
    if (newpos) newpos[P.val(i)] = dst;
    else {
      keys_out[dst] = key[e];
      vals_out[dst] = P.val(i);
    }
  }
}

__global__ void k_mm_init(u32* mm, int D) {
  for (int i = threadIdx.x; i < D; i += blockDim.x) { mm[2 * i] = ~0u; mm[2 * i + 1] = 0u; }
}

__global__ __launch_bounds__(kBlock) void k_perm_leaves(const u64* __restrict__ in, u64 n,
                                                        const u32* __restrict__ newpos, u64* __restrict__ out) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i < n) out[newpos[i]] = in[i];
}

// ---- multi-layer launches: entry e of a plan owns blocks [b0[e], b0[e + 1]) ----
struct RangePlan {
  u64 lo[GCZ_MAX_LAYERS];    // first element of the entry's range
  u64 n[GCZ_MAX_LAYERS];     // its elements
  u64 aux[GCZ_MAX_LAYERS];   // counters' offset (hist) / layer (min-max)
  u32 b0[GCZ_MAX_LAYERS + 1];
  int m;
};

constexpr int kRangeBatch = 8;   // loads in flight per thread

__device__ __forceinline__ int plan_entry(const RangePlan& p) {
  int e = 0;
  while (e + 1 < p.m && blockIdx.x >= p.b0[e + 1]) ++e;
  return e;
}

// counters of the listed child layers to zero: cnt[lo, lo + n)
__global__ __launch_bounds__(kBlock) void k_zero_ranges(RangePlan p, u32* __restrict__ cnt) {
  const int e = plan_entry(p);
  const u64 nb = p.b0[e + 1] - p.b0[e];
  for (u64 i = (blockIdx.x - p.b0[e]) * u64(kBlock) + threadIdx.x; i < p.n[e]; i += nb * kBlock) cnt[p.lo[e] + i] = 0;
}

// pointer::serialize of w as a word of its bytes in output order (the first byte lowest),
// and their count: the pointer's value (seg | t | m | offset) written big-endian
__device__ __forceinline__ u32 ptr_enc(u32 w, u32& nbytes) {
  const u32 idx = w & kIdx;   // (null: idx = kIdx, segment 3 with offset 0xfffffff)
  const u32 seg = u32(idx >= kSegStart1) + u32(idx >= kSegStart2) + u32(idx >= kSegStart3);
  const u32 base = seg == 0 ? 0u : seg == 1 ? kSegStart1 : seg == 2 ? kSegStart2 : kSegStart3;
  const u32 off = idx == kIdx ? 0xfffffffu : idx - base;
  const u32 top = 8 * seg;
  const u32 v = off | (((w >> 29) & 3u) << (top + 4)) | (seg << (top + 6));
  nbytes = seg + 1;
  return __builtin_bswap32(v) >> (24 - top);
}

// len <= 8 bytes (hi:lo, the first byte lowest) at byte o of a zeroed LDS buffer: ORed into
// their aligned words, so neighbours that share a word need no ordering
__device__ __forceinline__ void lds_emit(u32* __restrict__ buf, u32 o, u32 lo, u32 hi, u32 len) {
  const u32 r = o & 3, w0 = o >> 2, sh = 8 * r;
  atomicOr(&buf[w0], lo << sh);
  if (r + len > 4) atomicOr(&buf[w0 + 1], r ? __builtin_amdgcn_alignbit(hi, lo, 32 - sh) : hi);
  if (r + len > 8) atomicOr(&buf[w0 + 2], hi >> (32 - sh));
}

// histogram (src/shared_tree.cpp:316-326) of the listed parent layers: words [lo, lo + n)
// counted into cnt + aux (their references come in near id order: global atomics coalesce)
__global__ __launch_bounds__(kBlock) void k_hist_ranges(RangePlan p, const u32* __restrict__ words,
                                                        u32* __restrict__ cnt) {
  const int e = plan_entry(p);
  const u64 step = u64(p.b0[e + 1] - p.b0[e]) * kBlock, n = p.n[e];
  const u32* wv = words + p.lo[e];
  u32* c = cnt + p.aux[e];
  for (u64 i = (blockIdx.x - p.b0[e]) * u64(kBlock) + threadIdx.x; i < n; i += kRangeBatch * step) {
    u32 w[kRangeBatch];
#pragma unroll
    for (int q = 0; q < kRangeBatch; ++q) w[q] = i + q * step < n ? wv[i + q * step] : kIdx;
#pragma unroll
    for (int q = 0; q < kRangeBatch; ++q)
      if (!is_null(w[q])) atomicAdd(&c[w[q] & kIdx], 1u);
  }
}

// min / max count of the listed child layers: cnt[lo, lo + n), one (min, max) per block
// into part (device-scope atomics on two shared words would serialise thousands of blocks)
__global__ __launch_bounds__(kBlock) void k_minmax_ranges(RangePlan p, const u32* __restrict__ cnt,
                                                          u32* __restrict__ part) {
  __shared__ u32 smin[kBlock / 64], smax[kBlock / 64];
  const int e = plan_entry(p);
  const u64 nb = p.b0[e + 1] - p.b0[e];
  u32 lo = ~0u, hi = 0;
  const u64 step = nb * kBlock, n = p.n[e];
  const u32* cv = cnt + p.lo[e];
  for (u64 i = (blockIdx.x - p.b0[e]) * u64(kBlock) + threadIdx.x; i < n; i += kRangeBatch * step) {
    u32 v[kRangeBatch];
#pragma unroll
    for (int q = 0; q < kRangeBatch; ++q) v[q] = i + q * step < n ? cv[i + q * step] : ~0u;
#pragma unroll
    for (int q = 0; q < kRangeBatch; ++q) {
      lo = min(lo, v[q]);
      if (v[q] != ~0u) hi = max(hi, v[q]);
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    lo = min(lo, u32(__shfl_xor(int(lo), o, 64)));
    hi = max(hi, u32(__shfl_xor(int(hi), o, 64)));
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) { smin[wave] = lo; smax[wave] = hi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) { lo = min(lo, smin[w]); hi = max(hi, smax[w]); }
    part[2 * blockIdx.x] = lo;
    part[2 * blockIdx.x + 1] = hi;
  }
}

// the blocks' (min, max) of each entry into mm[2 aux, 2 aux + 1] (one workgroup)
__global__ __launch_bounds__(1024) void k_minmax_fold(RangePlan p, const u32* __restrict__ part,
                                                      u32* __restrict__ mm) {
  __shared__ u32 smin[16], smax[16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int e = 0; e < p.m; ++e) {
    u32 lo = ~0u, hi = 0;
    for (u32 b = p.b0[e] + threadIdx.x; b < p.b0[e + 1]; b += 1024) {
      lo = min(lo, part[2 * b]);
      hi = max(hi, part[2 * b + 1]);
    }
    for (int o = 32; o > 0; o >>= 1) {
      lo = min(lo, u32(__shfl_xor(int(lo), o, 64)));
      hi = max(hi, u32(__shfl_xor(int(hi), o, 64)));
    }
    if (lane == 0) { smin[wave] = lo; smax[wave] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int w = 1; w < 16; ++w) { lo = min(lo, smin[w]); hi = max(hi, smax[w]); }
      mm[2 * p.aux[e]] = lo;
      mm[2 * p.aux[e] + 1] = hi;
    }
    __syncthreads();
  }
}

// rewire_nodes (:383-403) with the child permutation and reorder_layer (:371-377) with
// the own one, for the listed node layers in one launch.  A layer whose own order
// stays is rewired in place (out == in); a permuted one goes to out at the same slots.
struct PermPlan {
  u64 node[GCZ_MAX_LAYERS];         // storage start of the entry's layer
  u64 count[GCZ_MAX_LAYERS];        // its nodes
  long long child[GCZ_MAX_LAYERS];  // offset of the child layer's newpos, -1: identity
  long long own[GCZ_MAX_LAYERS];    // offset of the layer's own newpos, -1: identity
  int via_slot[GCZ_MAX_LAYERS];     // children from val[slot[word]] (k_hremap) instead
  u32 b0[GCZ_MAX_LAYERS + 1];
  int m;
};
constexpr int kPermItems = 4;

__global__ __launch_bounds__(kBlock) void k_perm_nodes(const uint2* in, PermPlan pp, const u32* __restrict__ newpos,
                                                       const u32* __restrict__ slot, const u32* __restrict__ val,
                                                       uint2* inplace_or_out, uint2* out_perm) {
  int e = 0;
  while (e + 1 < pp.m && blockIdx.x >= pp.b0[e + 1]) ++e;
  // a layer's blocks dealt to the XCDs in contiguous runs (the val runs a chunk of words
  // reads stay in one L2)
  const u32 nbk = pp.b0[e + 1] - pp.b0[e], lb = blockIdx.x - pp.b0[e], per = nbk / 8;
  const u32 blk = lb < 8 * per ? (lb % 8) * per + lb / 8 : lb;
  const u64 i0 = u64(blk) * (kBlock * kPermItems) + threadIdx.x;
  const u64 node = pp.node[e], count = pp.count[e];
  const long long child = pp.child[e], own = pp.own[e];
  uint2 w[kPermItems];
#pragma unroll
  for (int q = 0; q < kPermItems; ++q) {
    const u64 i = i0 + u64(q) * kBlock;
    if (i < count) w[q] = in[node + i];
  }
  if (pp.via_slot[e]) {
    u32 nx[kPermItems], ny[kPermItems];
#pragma unroll
    for (int q = 0; q < kPermItems; ++q) {
      const u64 i = i0 + u64(q) * kBlock;
      uint2 sl = make_uint2(0u, 0u);
      if (i < count) sl = reinterpret_cast<const uint2*>(slot)[i];
      nx[q] = i < count && !is_null(w[q].x) ? val[sl.x] : 0u;
      ny[q] = i < count && !is_null(w[q].y) ? val[sl.y] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kPermItems; ++q) {
      if (!is_null(w[q].x)) w[q].x = (w[q].x & kBits) | nx[q];
      if (!is_null(w[q].y)) w[q].y = (w[q].y & kBits) | ny[q];
    }
  } else if (child >= 0) {
    const u32* cn = newpos + child;
    u32 nx[kPermItems], ny[kPermItems];
#pragma unroll
    for (int q = 0; q < kPermItems; ++q) {   // every gather in flight before the first use
      const u64 i = i0 + u64(q) * kBlock;
      const bool ok = i < count;
      nx[q] = ok && !is_null(w[q].x) ? cn[w[q].x & kIdx] : 0u;
      ny[q] = ok && !is_null(w[q].y) ? cn[w[q].y & kIdx] : 0u;
    }
#pragma unroll
    for (int q = 0; q < kPermItems; ++q) {
      if (!is_null(w[q].x)) w[q].x = (w[q].x & kBits) | nx[q];
      if (!is_null(w[q].y)) w[q].y = (w[q].y & kBits) | ny[q];
    }
  }
#pragma unroll
  for (int q = 0; q < kPermItems; ++q) {
    const u64 i = i0 + u64(q) * kBlock;
    if (i >= count) continue;
    if (own >= 0) out_perm[node + newpos[own + i]] = w[q];
    else inplace_or_out[node + i] = w[q];
  }
}

struct LayerStarts {
  u64 node[GCZ_MAX_LAYERS + 1];     // storage start of each layer within the node buffer (+ the end)
  u64 count[GCZ_MAX_LAYERS];        // nodes of each layer (storage holds ceil(n/2) slots, count <= that)
  u64 cstart[GCZ_MAX_LAYERS + 1];   // first node of each layer in the concatenation of the layers' nodes
};

// ---- bytes() and the .dag node section ----
// The nodes of all layers, concatenated (storage padding skipped), in tiles of kDagTile,
// element e * kDagThreads + tid of a tile per thread (coalesced 8-B loads).  A node's size
// is its two pointers' bytes, plus 8 for the layer count written right before the first
// node of each layer.  The layer is looked up once per wave on the scalar unit; only a
// wave that a layer start cuts walks per lane.
constexpr int kDagThreads = 256;
constexpr int kDagItems = 8;
constexpr u64 kDagTile = u64(kDagThreads) * kDagItems;       // 2 Ki nodes (several workgroups per CU)
constexpr int kDagGroups = kDagItems * (kDagThreads / 64);   // 64-node groups of a tile
constexpr int kDagPer = (kDagGroups + 63) / 64;              // groups per lane of the scanning wave
constexpr u32 kDagBuf = (u32(kDagTile) * 8 + 8 * GCZ_MAX_LAYERS + 32 + 15) / 16 * 16;

struct DagSlot {
  uint2 w;    // the node's words; after dag_encode, its bytes in output order (x: first four)
  u32 meta;   // layer | starts its layer << 8 | a node (not past the end) << 16 | bytes << 20
  __device__ __forceinline__ int k() const { return int(meta & 0xff); }
  __device__ __forceinline__ u32 nh() const { return (meta >> 8) & 0xff; }
  __device__ __forceinline__ bool valid() const { return (meta >> 16) & 1u; }
  __device__ __forceinline__ u32 len() const { return meta >> 20; }
};

// the node's serialized bytes (two pointers: 2..8 bytes) in place of its words
__device__ __forceinline__ void dag_encode(DagSlot& s) {
  u32 nx, ny;
  const u32 vx = ptr_enc(s.w.x, nx), vy = ptr_enc(s.w.y, ny);
  const u32 sx = 8 * nx;
  s.w.x = sx == 32 ? vx : vx | (vy << sx);
  s.w.y = sx == 32 ? vy : vy >> (32 - sx);
  s.meta |= (s.valid() ? nx + ny : 0u) << 20;
}

__device__ __forceinline__ u64 uniform64(u64 v) {   // (a wave-uniform value, into scalar registers)
  return (u64(u32(__builtin_amdgcn_readfirstlane(int(v >> 32)))) << 32) | u32(__builtin_amdgcn_readfirstlane(int(v)));
}

// a thread's kDagItems nodes of the tile starting at node c0 (of m)
__device__ __forceinline__ void dag_load(const uint2* __restrict__ nodes, u64 m, const LayerStarts& ls, int D, u64 c0,
                                         DagSlot (&sl)[kDagItems]) {
  int k = 0;
  while (k + 1 < D && c0 >= ls.cstart[k + 1]) ++k;
  u64 kcs = ls.cstart[k], kend = ls.cstart[k + 1], knd = ls.node[k];   // (scalar registers)
  u64 g[kDagItems];
#pragma unroll
  for (int e = 0; e < kDagItems; ++e) {
    const u64 cw = uniform64(c0 + u64(e) * kDagThreads + (threadIdx.x & ~63u));
    const u64 c = cw + (threadIdx.x & 63u);
    if (cw >= kend && cw < m) {   // (the wave starts in a later layer)
      while (k + 1 < D && cw >= ls.cstart[k + 1]) ++k;
      kcs = ls.cstart[k];
      kend = ls.cstart[k + 1];
      knd = ls.node[k];
    }
    int kk = k;
    u64 cs = kcs, nd = knd;
    if (c >= kend && c < m) {   // (a layer starts inside the wave: per lane)
      while (kk + 1 < D && c >= ls.cstart[kk + 1]) ++kk;
      cs = ls.cstart[kk];
      nd = ls.node[kk];
    }
    g[e] = nd + (c - cs);
    sl[e].meta = c < m ? u32(kk) | (u32(c == cs) << 8) | (1u << 16) : 0u;
  }
#pragma unroll
  for (int e = 0; e < kDagItems; ++e) sl[e].w = sl[e].valid() ? nodes[g[e]] : make_uint2(0u, 0u);
}

__device__ __forceinline__ u32 dag_size(const DagSlot& s) {
  return s.valid() ? 8 * s.nh() + ptr_bytes(s.w.x) + ptr_bytes(s.w.y) : 0u;
}

// Sum of the node section's pointer bytes (bytes(), src/shared_tree.cpp:488-496).
__global__ __launch_bounds__(kDagThreads) void k_node_bytes(const uint2* __restrict__ nodes, u64 n, LayerStarts ls,
                                                            int D, unsigned long long* __restrict__ acc) {
  __shared__ u32 part[kDagThreads / 64];
  DagSlot sl[kDagItems];
  dag_load(nodes, n, ls, D, u64(blockIdx.x) * kDagTile, sl);
  u32 b = 0;
#pragma unroll
  for (int e = 0; e < kDagItems; ++e)
    if (sl[e].valid()) b += ptr_bytes(sl[e].w.x) + ptr_bytes(sl[e].w.y);
  b = u32(wave_sum(u64(b)));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {   // line-padded shards (k_stats_sum): a few shared addresses would serialise
    u32 t = 0;
    for (int w = 0; w < kDagThreads / 64; ++w) t += part[w];
    if (t) atomicAdd(&acc[(blockIdx.x & (kStatShards - 1)) * kStatStride], (unsigned long long)t);
  }
}

// Per-tile byte counts of the node section (layer counts included): the tiles' prefixes
// come from a scan of these (a look-back chain over thousands of tiles waits on
// device-scope loads, which on this part cost more than a second read of the nodes).
__global__ __launch_bounds__(kDagThreads) void k_dag_sizes(const uint2* __restrict__ nodes, u64 n, LayerStarts ls,
                                                           int D, u32* __restrict__ tsum) {
  __shared__ u32 part[kDagThreads / 64];
  DagSlot sl[kDagItems];
  dag_load(nodes, n, ls, D, u64(blockIdx.x) * kDagTile, sl);
  u32 b = 0;
#pragma unroll
  for (int e = 0; e < kDagItems; ++e) b += dag_size(sl[e]);
  b = u32(wave_sum(u64(b)));
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = b;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 t = 0;
    for (int w = 0; w < kDagThreads / 64; ++w) t += part[w];
    tsum[blockIdx.x] = t;
  }
}

// The node section (serialize, src/shared_tree.cpp:504-513), one tile per workgroup at
// its prefix tpre[tile]: every slot's bytes (pointer::serialize, layer counts
// big-endian) staged in LDS at the tile's output alignment, then stored as aligned
// 16-B chunks (bytes at the two ends, which neighbouring tiles share).
__global__ __launch_bounds__(kDagThreads) void k_dag_nodes(const uint2* __restrict__ nodes, u64 n, LayerStarts ls,
                                                           int D, u64 hdr, const u64* __restrict__ tpre,
                                                           unsigned char* __restrict__ out) {
  __shared__ u32 s_grp[kDagGroups];
  __shared__ __attribute__((aligned(16))) unsigned char s_out[kDagBuf];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u64 tile = blockIdx.x;
  DagSlot sl[kDagItems];
  dag_load(nodes, n, ls, D, tile * kDagTile, sl);
  for (u32 q = tid; q < kDagBuf / 16; q += kDagThreads)   // (the slots' bytes are ORed in)
    reinterpret_cast<uint4*>(s_out)[q] = make_uint4(0u, 0u, 0u, 0u);
  u32 ex[kDagItems];
#pragma unroll
  for (int e = 0; e < kDagItems; ++e) {
    dag_encode(sl[e]);
    const u32 sz = 8 * sl[e].nh() + sl[e].len();
    u32 incl = sz;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    ex[e] = incl - sz;
    if (lane == 63) s_grp[e * (kDagThreads / 64) + wave] = incl;
  }
  __syncthreads();
  if (wave == 0) {
    u32 cs[kDagPer];
    u32 c = 0;
#pragma unroll
    for (int q = 0; q < kDagPer; ++q) {
      cs[q] = lane * kDagPer + q < kDagGroups ? s_grp[lane * kDagPer + q] : 0u;
      c += cs[q];
    }
    u32 incl = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const u32 y = __shfl_up(incl, o, 64);
      if (lane >= o) incl += y;
    }
    u32 run = incl - c;
#pragma unroll
    for (int q = 0; q < kDagPer; ++q) {
      if (lane * kDagPer + q < kDagGroups) s_grp[lane * kDagPer + q] = run;
      run += cs[q];
    }
  }
  __syncthreads();
  const u64 obase = hdr + tpre[tile];
  const u32 sh = u32(obase & 15);
  u32* buf = reinterpret_cast<u32*>(s_out);
#pragma unroll
  for (int e = 0; e < kDagItems; ++e) {
    u32 o = sh + s_grp[e * (kDagThreads / 64) + wave] + ex[e];
    const DagSlot& s = sl[e];
    const u32 nh = s.nh();
    if (nh) {   // (the layer's count, big-endian, before its first node)
      const u64 cnt = ls.count[s.k()];
      lds_emit(buf, o, __builtin_bswap32(u32(cnt >> 32)), __builtin_bswap32(u32(cnt)), 8);
      o += 8;
    }
    if (s.valid()) lds_emit(buf, o, s.w.x, s.w.y, s.len());
  }
  __syncthreads();
  const u32 end = sh + u32(tpre[tile + 1] - tpre[tile]);
  unsigned char* ob = out + (obase - sh);   // 16-B aligned (the buffer is)
  for (u32 c = tid; c * 16 < end; c += kDagThreads) {
    const u32 lo = c * 16, hi = lo + 16;
    if (lo >= sh && hi <= end) {
      *reinterpret_cast<uint4*>(ob + lo) = *reinterpret_cast<const uint4*>(s_out + lo);
    } else {
      for (u32 b = lo < sh ? sh : lo; b < hi && b < end; ++b) ob[b] = s_out[b];
    }
  }
}

// leaves (binary_write of each value, lb bytes); thread 0 also writes the root pointer
// and the leaf count before them
__global__ __launch_bounds__(kBlock) void k_write_leaves(const u64* __restrict__ leaves, u64 n, int lb, u32 root,
                                                         unsigned char* __restrict__ out) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  const u64 base = ptr_bytes(root) + 8;
  if (i == 0) {
    put_ptr(out, root);
    put_be(out + ptr_bytes(root), n, 8);
  }
  if (i < n) put_be(out + base + i * u64(lb), leaves[i], lb);
}

// ---- decompression ---------------------------------------------
// shared_tree::operator[] (src/shared_tree.cpp:268-291) for every index at once,
// top-down one layer per launch: a word w referencing node (l, r) of layer k
// stands for (M(r), M(l)) with w's transpose bit applied when w is mirrored,
// else (l, r) with it (the transform ctor, :76-80); access_leaf (:230-235)
// applies mirror / transpose to the canonical leaf.
__global__ __launch_bounds__(kBlock) void k_expand(const u32* __restrict__ w_in, u64 pw,
                                                   const uint2* __restrict__ layer, u32* __restrict__ w_out,
                                                   u64 nout) {
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= pw) return;
  const u32 w = w_in[j];
  const uint2 nd = layer[w & kIdx];
  const u32 m = (w >> 29) & 1u, t = (w >> 30) & 1u;
  const u32 a = m ? xf(nd.y, 1, t) : xf(nd.x, 0, t);
  const u32 b = m ? xf(nd.x, 1, t) : xf(nd.y, 0, t);
  w_out[2 * j] = a;
  if (2 * j + 1 < nout) w_out[2 * j + 1] = b;
}

__constant__ char kSym[16] = {'S', 'A', 'C', 'R', 'G', 'B', 'N', 'K', 'T', 'W', 'V', 'D', 'Y', 'H', 'M', '-'};

// One strand per thread, staged through LDS so the text is stored coalesced.
__global__ __launch_bounds__(kBlock) void k_leaves_text(const u32* __restrict__ words, u64 S,
                                                        const u64* __restrict__ leaves, int L,
                                                        unsigned char* __restrict__ out) {
  __shared__ unsigned char buf[kBlock * 16];
  const u64 s0 = u64(blockIdx.x) * kBlock;
  const u64 s = s0 + threadIdx.x;
  if (s < S) {
    const u32 w = words[s];
    u64 v = leaves[w & kIdx];
    if ((w >> 29) & 1u) v = leaf_mirrored(v, L);
    if ((w >> 30) & 1u) v = leaf_transposed(v);
    for (int i = 0; i < L; ++i) buf[threadIdx.x * L + i] = (unsigned char)kSym[(v >> (4 * i)) & 15];
  }
  __syncthreads();
  const u64 nstr = S - s0 < u64(kBlock) ? S - s0 : u64(kBlock);
  for (u64 b = threadIdx.x; b < nstr * u64(L); b += kBlock) out[s0 * L + b] = buf[b];
}

dim3 grid_of(u64 n) { return dim3(unsigned(std::max<u64>(1, (n + kBlock - 1) / kBlock))); }

LayerStarts layer_starts(const gcz_ctx* c) {
  LayerStarts ls{};
  const int D = c->info.n_layers;
  for (int k = 0; k <= D; ++k) ls.node[k] = c->layer_off[k];
  for (int k = 0; k < D; ++k) ls.count[k] = c->info.layer_size[k];
  for (int k = 0; k < D; ++k) ls.cstart[k + 1] = ls.cstart[k] + ls.count[k];
  return ls;
}

u32 host_ptr_bytes(u32 w) {
  const u32 i = w & kIdx;
  if (i == kIdx) return 4;
  return i < kSegStart1 ? 1 : i < kSegStart2 ? 2 : i < kSegStart3 ? 3 : 4;
}

}  // namespace

#define S_HIP(x)                                                                         \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess) return c->fail(GCZ_ERR_DEVICE, #x, hipGetErrorString(e_));     \
  } while (0)

static __global__ void k_sort_warm() {}

extern "C" {

// The sort's device buffers for the current tree, allocated ahead (the drop-in reserves them on
// a side thread while the tree is fetched: a first sort at 1 Gbase otherwise pays ~40 ms of
// allocation, profiles/r04/compress_e2e.txt); gcz_sort_device calls it too (then a no-op).
//
// It runs beside gcz_fetch_host on the same context, so it reads only the tree's shape and
// writes nothing the fetch reads: no last_error / info.status -- a failure comes back as a code
// (and *why), and gcz_sort_device, the only caller that goes on to use the buffers, reports it.
static int sort_reserve(gcz_ctx* c, const char** why) {
#define R_HIP(x)                       \
  do {                                 \
    if ((x) != hipSuccess) {           \
      *why = #x;                       \
      return GCZ_ERR_DEVICE;           \
    }                                  \
  } while (0)
  if (c->info.n_layers < 1) return GCZ_ERR_ARG;
  R_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  const int D = c->info.n_layers;
  const u64 nl = c->info.n_leaves;
  std::vector<u64> n_of(D), coff(D + 1, 0);
  for (int cl = 0; cl < D; ++cl) {
    n_of[cl] = cl == 0 ? nl : c->info.layer_size[cl - 1];
    coff[cl + 1] = coff[cl] + n_of[cl];
  }
  u64 nmax = 0, nwmax = 0, matmax = 0;
  std::vector<u32> hnb(D, 0);
  for (int cl = 0; cl < D; ++cl) {
    nmax = std::max(nmax, n_of[cl]);
    const u64 nw = 2 * c->info.layer_size[cl];
    const u64 nb = (n_of[cl] + (1ull << kHB) - 1) >> kHB;
    if (nw >= (1ull << 20) && nw >= 4 * n_of[cl] && nb >= 1 && nb <= kHMaxBuckets) {   // (as gcz_sort_device)
      hnb[cl] = u32(nb);
      nwmax = std::max(nwmax, nw);
      matmax = std::max(matmax, nb * ((nw + kHChunk - 1) / kHChunk) + 1);
    }
  }
  int scl = -1;
  for (int cl = 0; cl < D; ++cl)
    if (hnb[cl] && (scl < 0 || c->info.layer_size[cl] > c->info.layer_size[scl])) scl = cl;
  matmax = std::max(matmax, 256 * ((nmax + kCsTile - 1) / kCsTile) + 1);
  const u64 tilemax = scan_tiles(matmax);
  const u64 N = c->layer_off[D];
  R_HIP(c->ensure_quiet(s.cnt, coff[D] * 4 + 16));
  R_HIP(c->ensure_quiet(s.newpos, coff[D] * 4 + 16));
  R_HIP(c->ensure_quiet(s.keys, nmax * 4 + 16));
  R_HIP(c->ensure_quiet(s.keys2, nmax * 4 + 16));
  R_HIP(c->ensure_quiet(s.vals, nmax * 4 + 16));
  R_HIP(c->ensure_quiet(s.vals2, nmax * 4 + 16));
  R_HIP(c->ensure_quiet(s.mm, size_t(D) * 8 + 16));
  R_HIP(c->ensure_quiet(s.nodes2, N * 8 + 16));
  R_HIP(c->ensure_quiet(s.leaves2, nl * 8 + 16));
  R_HIP(c->ensure_quiet(s.hmat, matmax * 4 + 16));
  R_HIP(c->ensure_quiet(s.hoff, matmax * 4 + 16));
  R_HIP(c->ensure_quiet(s.hrec, nwmax * 2 + 16));
  R_HIP(c->ensure_quiet(s.desc, tilemax * 8 + 16));
  R_HIP(c->ensure_quiet(s.hpart, size_t(2048) * GCZ_MAX_LAYERS * 8 + 16));
  if (scl >= 0) {
    R_HIP(c->ensure_quiet(s.hslot, 2 * c->info.layer_size[scl] * 4 + 16));
    R_HIP(c->ensure_quiet(s.hval, 2 * c->info.layer_size[scl] * 4 + 16));
    R_HIP(c->ensure_quiet(s.hbs, (u64(hnb[scl]) + 1) * 4 + 16));
  }
  if (!s.h_mm) R_HIP(hipHostMalloc((void**)&s.h_mm, size_t(GCZ_MAX_LAYERS) * 8, hipHostMallocDefault));
  if (!s.warm) {   // this file's code object loaded now, not at the first sort's first launch
    hipLaunchKernelGGL(k_sort_warm, dim3(1), dim3(64), 0, c->stream);
    R_HIP(hipGetLastError());
    s.warm = true;
  }
  return GCZ_OK;
#undef R_HIP
}

int gcz_sort_reserve(gcz_ctx* c) {
  if (!c) return GCZ_ERR_ARG;
  const char* why = nullptr;
  return sort_reserve(c, &why);
}



int gcz_sort_device(gcz_ctx* c) {
  if (!c || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  {
    const char* why = "";
    if (int rc = sort_reserve(c, &why)) return rc == GCZ_ERR_DEVICE ? c->fail(rc, "sort buffers", why) : rc;
  }
  gcz_sort_state& s = *c->sortst;
  const int D = c->info.n_layers;
  const u64 nl = c->info.n_leaves;
  // child layer cl: 0 = leaves (parent: node layer 0), cl = k + 1 = node layer k (parent: layer k + 1)
  std::vector<u64> n_of(D), coff(D + 1, 0);
  for (int cl = 0; cl < D; ++cl) {
    n_of[cl] = cl == 0 ? nl : c->info.layer_size[cl - 1];
    coff[cl + 1] = coff[cl] + n_of[cl];
  }
  u64 nmax = 0, nwmax = 0, matmax = 0;
  // per parent layer: partitioned histogram (nb buckets x G chunks) or global atomics (nb = 0)
  std::vector<u32> hnb(D, 0);
  std::vector<u64> hG(D, 0);
  for (int cl = 0; cl < D; ++cl) {
    nmax = std::max(nmax, n_of[cl]);
    const u64 nw = 2 * c->info.layer_size[cl];
    const u64 nb = (n_of[cl] + (1ull << kHB) - 1) >> kHB;
    // partition when parents reference their children many times over in random order (the
    // leaves: ~20 references each at 1 Gbase); a layer whose children are referenced about once
    // is referenced in near position order (ids are first occurrences), where atomics coalesce
    if (nw >= (1ull << 20) && nw >= 4 * n_of[cl] && nb >= 1 && nb <= kHMaxBuckets) {
      hnb[cl] = u32(nb);
      hG[cl] = (nw + kHChunk - 1) / kHChunk;
      nwmax = std::max(nwmax, nw);
      matmax = std::max(matmax, nb * hG[cl] + 1);
    }
  }
  // the partitioned layer with the most references keeps its records (histogrammed last):
  // its rewire reads new children back through them (k_hremap)
  int scl = -1;
  for (int cl = 0; cl < D; ++cl)
    if (hnb[cl] && (scl < 0 || c->info.layer_size[cl] > c->info.layer_size[scl])) scl = cl;
  const u64 cs_tiles = (nmax + kCsTile - 1) / kCsTile;
  matmax = std::max(matmax, 256 * cs_tiles + 1);
  int rc;   // (the buffers: gcz_sort_reserve, same sizes)
  S_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_hbucket), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int((1u << kHB) * 4)));
  S_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(k_hremap), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int((1u << kHB) * 4)));
  hipEvent_t e0{};
  c->prof_begin(KID_SORT, e0);
  u32* cnt = s.cnt.as<u32>();
  u32* mm = s.mm.as<u32>();
  u32* mat = s.hmat.as<u32>();
  u32* off = s.hoff.as<u32>();
  u64* sdesc = s.desc.as<u64>();
  // exclusive scan of m matrix entries (+ the total at off[m])
  auto scan = [&](u64 m) -> int {
    const u64 t = scan_tiles(m + 1);
    S_HIP(hipMemsetAsync(sdesc, 0, t * 8 + 16, c->stream));
    hipLaunchKernelGGL(k_scan_excl<ScanU32>, dim3(unsigned(t)), dim3(kScanThreads), 0, c->stream, ScanU32{mat, m},
                       m + 1, off, sdesc, reinterpret_cast<u32*>(sdesc + t), static_cast<u64*>(nullptr));
    S_HIP(hipGetLastError());
    return GCZ_OK;
  };
  hipLaunchKernelGGL(k_mm_init, dim3(1), dim3(64), 0, c->stream, mm, D);   // [min, max] per child layer
  const uint2* nodes = c->nodes_out.as<uint2>();
  // Every child is referenced at least once by its parent layer's stored words (each id
  // occurs in the parent layer's input, and a pair stored or not holds the same ids as
  // the node it is an instance of), so when the parent holds no more non-null words than
  // there are children, every count is 1 and the order stays.  The parent's input pairs
  // up with a null at its end when it is odd (reader-buffer builds hold more: the bound
  // only grows), so 2 * nodes - (input & 1) bounds its non-null words from above.
  std::vector<bool> once(D);
  for (int cl = 0; cl < D; ++cl) {
    const u64 in = cl == 0 ? c->info.n_strands : c->layer_off[cl] - c->layer_off[cl - 1];
    once[cl] = 2 * c->info.layer_size[cl] - (in & 1) <= n_of[cl];
  }
  // the other layers: partitioned (the leaves' parents) or atomics, zeroed / counted /
  // reduced in one launch each for all of them
  RangePlan zp{}, hp{}, mp{};
  auto add = [](RangePlan& p, u64 lo, u64 n, u64 aux, u64 per_block) {
    const u32 nb = u32(std::min<u64>(2048, std::max<u64>(1, (n + per_block - 1) / per_block)));
    p.lo[p.m] = lo;
    p.n[p.m] = n;
    p.aux[p.m] = aux;
    p.b0[p.m + 1] = p.b0[p.m] + nb;
    ++p.m;
  };
  std::vector<int> order;
  for (int cl = 0; cl < D; ++cl)
    if (cl != scl) order.push_back(cl);
  if (scl >= 0) order.push_back(scl);
  // workgroups per bucket of a partitioned layer: enough to fill the part
  std::vector<u32> hS(D, 1);
  for (int cl : order) {
    if (once[cl] || n_of[cl] == 0) continue;
    const u64 nw = 2 * c->info.layer_size[cl];   // words of parent layer cl
    if (hnb[cl]) {
      hS[cl] = u32(std::max<u64>(1, std::min<u64>((1024 + hnb[cl] - 1) / hnb[cl], nw / (hnb[cl] * 32768ull))));
      if (hS[cl] > 1) {
        add(zp, coff[cl], n_of[cl], 0, u64(kBlock) * 8);
        add(mp, coff[cl], n_of[cl], u64(cl), u64(kBlock) * 8);
      }
    } else {
      add(zp, coff[cl], n_of[cl], 0, u64(kBlock) * 8);
      add(hp, 2 * c->layer_off[cl], nw, coff[cl], u64(kBlock) * 8);
      add(mp, coff[cl], n_of[cl], u64(cl), u64(kBlock) * 8);
    }
  }
  if (zp.m) hipLaunchKernelGGL(k_zero_ranges, dim3(zp.b0[zp.m]), dim3(kBlock), 0, c->stream, zp, cnt);
  for (int cl : order) {
    if (once[cl] || n_of[cl] == 0 || !hnb[cl]) continue;
    const u64 nw = 2 * c->info.layer_size[cl];
    const u32* words = reinterpret_cast<const u32*>(nodes + c->layer_off[cl]);
    const u32 nb = hnb[cl];
    const u64 G = hG[cl];
    const bool keep = cl == scl;
    hipLaunchKernelGGL(k_hcount, dim3(unsigned(G)), dim3(kHThreads), 0, c->stream, words, nw, nb, G, mat);
    if ((rc = scan(u64(nb) * G))) return rc;
    if (nb <= kHStagedMax)
      hipLaunchKernelGGL(k_hscatter_lds, dim3(unsigned(G)), dim3(kHThreads), 0, c->stream, words, nw, nb, G, mat,
                         off, s.hrec.as<unsigned short>(), keep ? s.hslot.as<u32>() : nullptr);
    else
      hipLaunchKernelGGL(k_hscatter, dim3(unsigned(G)), dim3(kHThreads), 0, c->stream, words, nw, nb, G, off,
                         s.hrec.as<unsigned short>(), keep ? s.hslot.as<u32>() : nullptr);
    hipLaunchKernelGGL(k_hbucket, dim3(nb * hS[cl]), dim3(kHThreads), (1u << kHB) * 4, c->stream,
                       s.hrec.as<unsigned short>(), off, G, n_of[cl], hS[cl], cnt + coff[cl], mm + 2 * cl,
                       keep ? s.hbs.as<u32>() : nullptr);
    S_HIP(hipGetLastError());
  }
  if (hp.m)
    hipLaunchKernelGGL(k_hist_ranges, dim3(hp.b0[hp.m]), dim3(kBlock), 0, c->stream, hp,
                       reinterpret_cast<const u32*>(nodes), cnt);
  if (mp.m) {
    hipLaunchKernelGGL(k_minmax_ranges, dim3(mp.b0[mp.m]), dim3(kBlock), 0, c->stream, mp, cnt, s.hpart.as<u32>());
    hipLaunchKernelGGL(k_minmax_fold, dim3(1), dim3(1024), 0, c->stream, mp, s.hpart.as<u32>(), mm);
  }
  S_HIP(hipGetLastError());
  S_HIP(hipMemcpyAsync(s.h_mm, mm, size_t(D) * 8, hipMemcpyDeviceToHost, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));
  std::vector<bool> ident(D);
  for (int cl = 0; cl < D; ++cl) ident[cl] = once[cl] || n_of[cl] <= 1 || s.h_mm[2 * cl] == s.h_mm[2 * cl + 1];
  // stable descending sort of (count, index) per non-trivial child layer: newpos[old] = new
  for (int cl = 0; cl < D; ++cl) {
    if (ident[cl]) continue;
    const u64 n = n_of[cl];
    const u32 lo = s.h_mm[2 * cl], hi = s.h_mm[2 * cl + 1];
    const u32 bits = bit_width(u64(hi - lo));
    const u32 npass = (bits + 7) / 8, db = (bits + npass - 1) / npass;
    const u64 nt = (n + kCsTile - 1) / kCsTile;
    u32 *kin = nullptr, *vin = nullptr, *kout = s.keys.as<u32>(), *vout = s.vals.as<u32>();
    for (u32 ps = 0; ps < npass; ++ps) {
      CsPass P{};
      P.cnt = ps == 0 ? cnt + coff[cl] : nullptr;
      P.keys = kin;
      P.vals = vin;
      P.hi = hi;
      P.shift = ps * db;
      P.bits = std::min(db, bits - ps * db);
      P.n = n;
      hipLaunchKernelGGL(k_cs_count, dim3(unsigned(nt)), dim3(kCsThreads), 0, c->stream, P, nt, mat);
      if ((rc = scan(u64(1u << P.bits) * nt))) return rc;
      const bool last = ps + 1 == npass;
      hipLaunchKernelGGL(k_cs_scatter, dim3(unsigned(nt)), dim3(kCsThreads), 0, c->stream, P, nt, off, kout, vout,
                         last ? s.newpos.as<u32>() + coff[cl] : nullptr);
      S_HIP(hipGetLastError());
      kin = kout;
      vin = vout;
      kout = kout == s.keys.as<u32>() ? s.keys2.as<u32>() : s.keys.as<u32>();
      vout = vout == s.vals.as<u32>() ? s.vals2.as<u32>() : s.vals.as<u32>();
    }
  }
  // apply: leaves, then every node layer (rewire children, permute itself)
  if (!ident[0] && nl) {
    hipLaunchKernelGGL(k_perm_leaves, grid_of(nl), dim3(kBlock), 0, c->stream, c->leaves_out.as<u64>(), nl,
                       s.newpos.as<u32>(), s.leaves2.as<u64>());
    std::swap(c->leaves_out, s.leaves2);
  }
  const bool remap = scl >= 0 && !once[scl] && !ident[scl];
  if (remap) {
    const u32 S = u32(std::max<u64>(1, (1024 + hnb[scl] - 1) / hnb[scl]));
    hipLaunchKernelGGL(k_hremap, dim3(hnb[scl] * S), dim3(kHThreads), (1u << kHB) * 4, c->stream,
                       s.hrec.as<unsigned short>(), s.hbs.as<u32>(), s.newpos.as<u32>() + coff[scl], n_of[scl], S,
                       s.hval.as<u32>());
    S_HIP(hipGetLastError());
  }
  // node layers: rewired in place where their own order stays, permuted into nodes2 (and
  // copied back) where it changes -- or, when that moves more bytes, every layer into
  // nodes2 and the buffers swapped
  u64 moved_inplace = 0, moved_swap = 0;
  for (int k = 0; k < D; ++k) {
    const bool child = !ident[k], own = k + 1 < D && !ident[k + 1];
    const u64 n = c->info.layer_size[k];
    moved_swap += 2 * n;
    moved_inplace += own ? 4 * n : child ? 2 * n : 0;
  }
  const bool swap_all = moved_swap < moved_inplace;
  PermPlan pp{};
  for (int k = 0; k < D; ++k) {
    const bool child = !ident[k], own = k + 1 < D && !ident[k + 1];
    const u64 n = c->info.layer_size[k];
    if (n == 0 || (!swap_all && !child && !own)) continue;
    pp.node[pp.m] = c->layer_off[k];
    pp.count[pp.m] = n;
    pp.child[pp.m] = child ? (long long)coff[k] : -1;
    pp.via_slot[pp.m] = child && remap && k == scl;
    pp.own[pp.m] = own ? (long long)coff[k + 1] : -1;
    pp.b0[pp.m + 1] = pp.b0[pp.m] + u32((n + kBlock * kPermItems - 1) / (kBlock * kPermItems));
    ++pp.m;
  }
  if (pp.m) {
    uint2* in = c->nodes_out.as<uint2>();
    uint2* tmp = s.nodes2.as<uint2>();
    hipLaunchKernelGGL(k_perm_nodes, dim3(pp.b0[pp.m]), dim3(kBlock), 0, c->stream, in, pp, s.newpos.as<u32>(),
                       s.hslot.as<u32>(), s.hval.as<u32>(),
                       swap_all ? tmp : in, tmp);
    S_HIP(hipGetLastError());
    if (swap_all) {
      std::swap(c->nodes_out, s.nodes2);
    } else {
      for (int e = 0; e < pp.m; ++e)
        if (pp.own[e] >= 0)
          S_HIP(hipMemcpyAsync(in + pp.node[e], tmp + pp.node[e], pp.count[e] * 8, hipMemcpyDeviceToDevice,
                               c->stream));
    }
  }
  c->prof_end(KID_SORT, e0);
  S_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

int gcz_bytes_device(gcz_ctx* c, uint64_t* out) {
  if (!c || !out || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  if (int rc = c->ensure(s.acc, kStatBytes + 8)) return rc;
  S_HIP(hipMemsetAsync(s.acc.ptr, 0, kStatBytes, c->stream));
  const int D = c->info.n_layers;
  const LayerStarts ls = layer_starts(c);
  const u64 M = ls.cstart[D];
  hipLaunchKernelGGL(k_node_bytes, dim3(unsigned(std::max<u64>(1, (M + kDagTile - 1) / kDagTile))), dim3(kDagThreads),
                     0, c->stream, c->nodes_out.as<uint2>(), M, ls, D, s.acc.as<unsigned long long>());
  u64* total = s.acc.as<u64>() + kStatBytes / 8;
  hipLaunchKernelGGL(k_stats_sum, dim3(1), dim3(1024), 0, c->stream, s.acc.as<u64>(), total);
  S_HIP(hipGetLastError());
  u64 nb = 0;
  S_HIP(hipMemcpyAsync(&nb, total, 8, hipMemcpyDeviceToHost, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));
  *out = host_ptr_bytes(c->info.root) + 8 + c->info.n_leaves * u64((c->info.L + 1) / 2) +
         8 * u64(c->info.n_layers) + nb;
  return GCZ_OK;
}

// The .dag bytes into device memory (d_out == null: a context buffer); *written = size.
static int serialize_on_device(gcz_ctx* c, unsigned char** d_dag, uint64_t* written) {
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  const int D = c->info.n_layers;
  for (int k = 0; k < D; ++k)   // (every layer count is written before its first node)
    if (c->info.layer_size[k] == 0) return c->fail(GCZ_ERR_ARG, "serialize", "empty node layer");
  const LayerStarts ls = layer_starts(c);
  const u64 M = ls.cstart[D];
  const int lb = (c->info.L + 1) / 2;
  const u64 hdr = host_ptr_bytes(c->info.root) + 8 + c->info.n_leaves * u64(lb);
  const u64 cap = hdr + 8 * u64(D) + 8 * M;   // (pointers of at most 4 bytes)
  const u64 t = (M + kDagTile - 1) / kDagTile;
  const u64 st = scan_tiles(t + 1);
  int rc;
  if ((rc = c->ensure(s.dag, cap + 16)) || (rc = c->ensure(s.desc, std::max<u64>(s.desc.bytes, st * 8 + 16))) ||
      (rc = c->ensure(s.cnt, std::max<u64>(s.cnt.bytes, t * 4 + 16))) ||
      (rc = c->ensure(s.keys, std::max<u64>(s.keys.bytes, (t + 1) * 8 + 16))))
    return rc;
  if (!s.h_tot) S_HIP(hipHostMalloc((void**)&s.h_tot, 8, hipHostMallocDefault));
  hipEvent_t e0{};
  c->prof_begin(KID_DAG, e0);
  unsigned char* out = s.dag.as<unsigned char>();
  u32* tsum = s.cnt.as<u32>();
  u64* tpre = s.keys.as<u64>();   // t + 1 prefixes (the last: the section's size)
  hipLaunchKernelGGL(k_write_leaves, grid_of(c->info.n_leaves), dim3(kBlock), 0, c->stream,
                     c->leaves_out.as<u64>(), c->info.n_leaves, lb, c->info.root, out);
  hipLaunchKernelGGL(k_dag_sizes, dim3(unsigned(t)), dim3(kDagThreads), 0, c->stream, c->nodes_out.as<uint2>(), M, ls,
                     D, tsum);
  S_HIP(hipMemsetAsync(s.desc.ptr, 0, st * 8 + 16, c->stream));
  hipLaunchKernelGGL((k_scan_excl<ScanU32, u64>), dim3(unsigned(st)), dim3(kScanThreads), 0, c->stream,
                     ScanU32{tsum, t}, t + 1, tpre, s.desc.as<u64>(), reinterpret_cast<u32*>(s.desc.as<u64>() + st),
                     static_cast<u64*>(nullptr));
  hipLaunchKernelGGL(k_dag_nodes, dim3(unsigned(t)), dim3(kDagThreads), 0, c->stream, c->nodes_out.as<uint2>(), M,
                     ls, D, hdr, tpre, out);
  S_HIP(hipGetLastError());
  S_HIP(hipMemcpyAsync(s.h_tot, tpre + t, 8, hipMemcpyDeviceToHost, c->stream));
  c->prof_end(KID_DAG, e0);
  S_HIP(hipStreamSynchronize(c->stream));
  *d_dag = out;
  *written = hdr + *s.h_tot;
  return GCZ_OK;
}

int gcz_serialize_device(gcz_ctx* c, uint8_t* host_buf, uint64_t cap, uint64_t* written) {
  if (!c || !written || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  unsigned char* d = nullptr;
  uint64_t n = 0;
  if (int rc = serialize_on_device(c, &d, &n)) return rc;
  *written = n;
  if (!host_buf || cap < n) {
    S_HIP(hipStreamSynchronize(c->stream));
    return GCZ_ERR_ARG;
  }
  S_HIP(hipMemcpyAsync(host_buf, d, n, hipMemcpyDeviceToHost, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

int gcz_decompress_device(gcz_ctx* c, void* d_out, uint64_t cap) {
  if (!c || !d_out || c->info.status != GCZ_OK || c->info.n_layers < 1) return GCZ_ERR_ARG;
  const u64 S = c->info.n_strands;
  const int L = c->info.L;
  if (cap < S * u64(L)) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  gcz_sort_state& s = *c->sortst;
  if (int rc = c->ensure(s.dw1, S * 4 + 16)) return rc;
  if (int rc = c->ensure(s.dw2, S * 4 + 16)) return rc;
  const int D = c->info.n_layers;
  // element counts: the input of node layer k has n[k] words (n[0] = S), its output n[k + 1]
  std::vector<u64> n(D + 1);
  n[0] = S;
  for (int k = 0; k < D; ++k) n[k + 1] = (n[k] + 1) / 2;
  u32* cur = s.dw1.as<u32>();
  u32* nxt = s.dw2.as<u32>();
  S_HIP(hipMemcpyAsync(cur, &c->info.root, 4, hipMemcpyHostToDevice, c->stream));
  S_HIP(hipStreamSynchronize(c->stream));   // the root came from a host variable
  for (int k = D - 1; k >= 0; --k) {
    hipLaunchKernelGGL(k_expand, grid_of(n[k + 1]), dim3(kBlock), 0, c->stream, cur, n[k + 1],
                       c->nodes_out.as<uint2>() + c->layer_off[k], nxt, n[k]);
    std::swap(cur, nxt);
  }
  hipLaunchKernelGGL(k_leaves_text, grid_of(S), dim3(kBlock), 0, c->stream, cur, S, c->leaves_out.as<u64>(), L,
                     static_cast<unsigned char*>(d_out));
  S_HIP(hipGetLastError());
  S_HIP(hipStreamSynchronize(c->stream));
  return GCZ_OK;
}

int gcz_decompress(gcz_ctx* c, uint8_t* host_out, uint64_t cap) {
  if (!c || !host_out || c->info.status != GCZ_OK) return GCZ_ERR_ARG;
  const u64 n = c->info.n_strands * u64(c->info.L);
  if (cap < n) return GCZ_ERR_ARG;
  S_HIP(hipSetDevice(c->device));
  if (!c->sortst) c->sortst = new gcz_sort_state();
  if (int rc = c->ensure(c->sortst->text, n + 16)) return rc;
  if (int rc = gcz_decompress_device(c, c->sortst->text.ptr, n)) return rc;
  S_HIP(hipMemcpy(host_out, c->sortst->text.ptr, n, hipMemcpyDeviceToHost));
  return GCZ_OK;
}

const uint8_t* gcz_device_dag(gcz_ctx* c, uint64_t* written) {
  if (!c || !written || c->info.status != GCZ_OK || hipSetDevice(c->device) != hipSuccess) return nullptr;
  unsigned char* d = nullptr;
  if (serialize_on_device(c, &d, written)) return nullptr;
  return hipStreamSynchronize(c->stream) == hipSuccess ? d : nullptr;
}

}  // extern "C"
