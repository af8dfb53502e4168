// Device code of the multi-rank build (gcz_dist.hip).
//
// R ranks own contiguous strand ranges (rank order = position order).  Every
// hash-consed level runs the single-device kernels on the rank's own elements
// (local ids = local first-occurrence ranks), then reconciles keys across
// ranks through their owner rank (owner = mix(key) mod R):
//
//   A  every locally-first element that went through the table sends its key
//      (bit 63: "repeats locally", node levels) to the owner;
//   B  the owner replies per record: not-globally-first (another rank with a
//      smaller rank id has the key), globally-repeated, held by >= 2 ranks;
//   -  each rank ranks its globally-first keys in local order; an allgather of
//      those counts gives every rank its id offset (rank order = position
//      order, so offset + local rank = global first-occurrence rank);
//   C  the first holder of every key held by >= 2 ranks sends its global id;
//   D  the owner returns that id to every other holder
//      (C and D carry only those records, compacted in record order on both
//      sides, so a layer of mostly rank-unique keys moves almost nothing);
//   -  local words are remapped to global ids, and globally-first uniques are
//      compacted into the rank's slice of the output layer.
//
// Elements whose pair holds a child that occurs once globally (singleton
// propagation, gcz_device.h) are unique everywhere and send nothing.
#pragma once

#include "gcz_device.h"
#include "gcz_dense.h"

namespace gcz_dev {

constexpr int kMaxRanks = 31;              // owner slot state: one bit per rank + local-multi bit
constexpr int kSyncWords = kMaxRanks + 6;  // per-rank sync vector (see DistHdr)
constexpr int kFinalWords = 4 + GCZ_MAX_LAYERS;

struct DistHdr {
  // per-level sync vector: [0, R) records per owner, [R] overflow, [R+1] local uniques,
  // [R+2] first bad symbol offset (local bytes), [R+3] that symbol, [R+4] repetitive
  // data (the leaf probe's pre-dedupe decision), [R+5] a strand that is not pure ACGT
  u64 sync[kSyncWords];
  // second sync vector: [0] globally-first local uniques, [1, 1+R) C records per owner,
  // [1+R, 1+2R) D records per owner, [1+2R] pairs of the next level with two repeated
  // children (look-ahead, see k_lookahead; 0 = the next level is direct)
  u64 sync2[2 + 2 * kMaxRanks];
  u64 tot[4];                           // selected counts of the four compaction scans
  u32 ticket;                           // look-back tickets of k_dist_rank
  u32 tick[4];                          // ... of the compaction scans
  u32 lcnt[2];                          // list lengths: C records (sender), D records (owner dedupe)
  u32 nnf;                              // positions not globally first (k_dist_flags; listed up to kNfListCap)
  u32 ccur[kMaxRanks + 1];              // append cursors: C records per owner (sender side)
  u32 dcur[kMaxRanks + 1];              // ... D records per source (owner side)
  u64 cell[GCZ_MAX_LAYERS + 1];         // direct flags: n_local when the layer is direct, else ~0
  u64 final_vec[kFinalWords];           // [0] overflow, [1] root, [2] tail first layer, [4 + k] tail counts
  // fused leaf + layer-0 schedule (gcz_dist_fast.h)
  u64 fl_onf[kMaxRanks];                // this owner's not-first layer-0 records per source (R3's allgather)
  u64 fl_r4[2];                         // {layer-1 pairs with two repeated children, failure} (R4's allgather)
  u64 fl_guard;                         // 0: layer 1 is direct on every rank and none failed
  u64 fl_leaf[3];                       // this rank's leaf id offset, r-first count, all ranks' total
  u32 fl_bad;                           // a C / D slot overflowed
};
constexpr size_t kDistHdrBytes = (sizeof(DistHdr) + 15) & ~size_t(15);   // (its buffer: whole 16-B stores)

struct Displ {   // segment starts of the R source (or destination) ranks in a buffer, plus the end
  u64 d[kMaxRanks + 1];
};

__device__ __forceinline__ u32 seg_of(const Displ& D, u32 R, u64 k) {
  u32 s = 0;
  while (s + 1 < R && k >= D.d[s + 1]) ++s;
  return s;
}

__device__ __forceinline__ u32 owner_of(u64 key, u32 R) {
  u64 h = key * 0xff51afd7ed558ccdull;
  h ^= h >> 33;
  h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 29;
  return u32(((h >> 32) * u64(R)) >> 32);
}

constexpr u64 kLocalMulti = 1ull << 63;

// (PreKey, the fused schedule's layer-0 record keys: gcz_dense.h)

// The elements of a level that send a record.
struct RecSrc {
  // leaf levels: local unique ids [0, *ucount), key = leaves[lid]
  const u64* leaves;
  const u64* ucount;
  // node levels: positions [0, p)
  const u32* in;
  u64 n, p;
  const u32* words;                    // final local words
  const unsigned char* nf;
  const unsigned char* multi;
  const unsigned char* prev_nf;        // null: every locally-first pair sends
  const unsigned char* prev_multi;
  const uint2* canon;                  // levels without the local dedupe: canonical pairs (k_node_keys)
  u32 R;
  // the fused schedule's layer 0 (gcz_dist_fast.h): pairs of the dense pack's pre-words (code
  // labels), canonicalised on the fly; every pair but the null one is a record, lid = position
  const u32* pre;
  PreKey pk;     // ... with pk.on: 6-byte records, the key = owner << 48 | record
};



__device__ __forceinline__ bool rec_get(const RecSrc& s, u64 e, u64& key, u32& lid) {
  if (s.leaves) {
    if (e >= *s.ucount) return false;
    key = s.leaves[e];
    lid = u32(e);
    return true;
  }
  if (e >= s.p || s.nf[e] != kNfMaybe) return false;
  if (s.prev_nf) {
    bool single;
    if (2 * e + 1 < s.n) {
      const uchar2 f = reinterpret_cast<const uchar2*>(s.prev_nf)[e];
      const uchar2 g = reinterpret_cast<const uchar2*>(s.prev_multi)[e];
      single = (f.x == 0 && g.x == 0) || (f.y == 0 && g.y == 0);
    } else {
      single = s.prev_nf[2 * e] == 0 && s.prev_multi[2 * e] == 0;
    }
    if (single) return false;
  }
  u32 cl, cr;
  if (s.canon) {
    const uint2 c = s.canon[e];
    cl = c.x;
    cr = c.y;
  } else {
    u32 l, r, m, t;
    load_pair(s.in, s.n, e, l, r);
    node_canonical(l, r, cl, cr, m, t);
  }
  key = ((u64(ulw(cl)) << 31) | ulw(cr)) | (s.multi[e] ? kLocalMulti : 0ull);
  lid = s.words[e] & kIdx;
  return true;
}

__device__ __forceinline__ u64 rec_key(const RecSrc& s, u64 key) { return s.leaves ? key : (key & ~kLocalMulti); }

// destination rank of a record's key
__device__ __forceinline__ u32 rec_dest(const RecSrc& s, u64 key) {
  return s.pre && s.pk.on ? u32(key >> 48) : owner_of(rec_key(s, key), s.R);
}

// rec_get for levels without the local dedupe (canonical pairs given): every load of the
// record issued at once, none behind the not-first mark.
// the record of a pre-word pair (l, r) (in: a pair of the level); false: no record (the null
// pair, or out of the level)
__device__ __forceinline__ bool pre_rec(const RecSrc& s, u32 l, u32 r, bool in, u64& key) {
  u32 cl, cr, m, t;
  node_canonical(l, r, cl, cr, m, t);
  const bool ok = in && (r & kIdx) != kIdx;
  if (s.pk.on) {
    if (!ok) {
      key = 0;
      return false;
    }
    pre_key_of(s.pk, cl, cr, key);
    return true;
  }
  key = (u64(ulw(cl)) << 31) | ulw(cr);
  return ok;
}

__device__ __forceinline__ bool rec_get_canon(const RecSrc& s, u64 e, u64& key, u32& lid) {
  if (s.pre) {
    u32 l = kNullWord, r = kNullWord;
    if (e < s.p) load_pair(s.pre, s.n, e, l, r);
    lid = u32(e);
    return pre_rec(s, l, r, e < s.p, key);
  }
  const u64 es = e < s.p ? e : 0;   // (in bounds; used only when e < p)
  const unsigned char f = s.nf[es], mu = s.multi[es];
  const uint2 c = s.canon[es];
  const u32 w = s.words[es];
  bool single = false;
  if (s.prev_nf) {
    if (2 * es + 1 < s.n) {
      const uchar2 pf = reinterpret_cast<const uchar2*>(s.prev_nf)[es];
      const uchar2 pm = reinterpret_cast<const uchar2*>(s.prev_multi)[es];
      single = (pf.x == 0 && pm.x == 0) || (pf.y == 0 && pm.y == 0);
    } else {
      single = s.prev_nf[2 * es] == 0 && s.prev_multi[2 * es] == 0;
    }
  }
  key = ((u64(ulw(c.x)) << 31) | ulw(c.y)) | (mu ? kLocalMulti : 0ull);
  lid = w & kIdx;
  return e < s.p && f == kNfMaybe && !single;
}

// Bucketing by owner, deterministic two-pass: per-block counts, one scan, scatter.
static __global__ __launch_bounds__(kBlock) void k_bucket_count(RecSrc s, u32* __restrict__ blockcnt, u32 nb) {
  __shared__ u32 h[kMaxRanks];
  const int tid = threadIdx.x;
  if (tid < int(s.R)) h[tid] = 0;
  __syncthreads();
#pragma unroll 4
  for (int e = 0; e < kItems; ++e) {
    const u64 idx = u64(blockIdx.x) * kTile + u64(e) * kBlock + tid;
    u64 key;
    u32 lid;
    if (rec_get(s, idx, key, lid)) atomicAdd(&h[owner_of(rec_key(s, key), s.R)], 1u);
  }
  __syncthreads();
  if (tid < int(s.R)) blockcnt[u64(tid) * nb + blockIdx.x] = h[tid];
}

// Exclusive scan of blockcnt[R * nb] (destination-major) in place, per-destination totals
// into tot[0..R): each destination row is cut into chunks of kScanChunk entries; pass 1 sums
// every chunk, pass 2 (one block) scans the R * cpr chunk sums, pass 3 rescans each chunk from
// its offset.  Coalesced and spread over R * cpr blocks (a one-block scan of the 81 K counts of
// a 1 Gbase leaf level took 130 us).
constexpr u32 kScanChunk = 16 * kBlock;

__device__ __forceinline__ u32 wave_incl_scan(u32 v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const u32 t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

static __global__ __launch_bounds__(kBlock) void k_bscan_sum(const u32* __restrict__ a, u32 nb, u32 cpr,
                                                             u32* __restrict__ csum) {
  __shared__ u32 ws[kBlock / 64];
  const u32 row = blockIdx.x / cpr, c = blockIdx.x % cpr;
  const u32* r = a + u64(row) * nb;
  const u32 j1 = min((c + 1) * kScanChunk, nb);
  u32 v = 0;
  for (u32 j = c * kScanChunk + threadIdx.x; j < j1; j += kBlock) v += r[j];
  const int lane = threadIdx.x & 63;
  v = wave_incl_scan(v, lane);
  if (lane == 63) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    u32 t = 0;
    for (int w = 0; w < kBlock / 64; ++w) t += ws[w];
    csum[blockIdx.x] = t;
  }
}

// One block of 1024 threads, R * cpr <= 1024 chunk sums -> exclusive chunk offsets (global
// over the destination-major order), row totals.
static __global__ __launch_bounds__(1024) void k_bscan_top(u32* __restrict__ csum, u32 R, u32 cpr,
                                                           u64* __restrict__ tot) {
  __shared__ u32 part[1024];
  __shared__ u32 ws[1024 / 64];
  const u32 n = R * cpr, tid = threadIdx.x;
  const int lane = tid & 63;
  const u32 v = tid < n ? csum[tid] : 0u;
  const u32 inc = wave_incl_scan(v, lane);
  if (lane == 63) ws[tid >> 6] = inc;
  __syncthreads();
  u32 add = 0;
  for (u32 w = 0; w < (tid >> 6); ++w) add += ws[w];
  part[tid] = inc + add - v;   // exclusive
  __syncthreads();
  if (tid < n) csum[tid] = part[tid];
  if (tid < R) {
    u32 all = 0;
    for (u32 w = 0; w < 1024 / 64; ++w) all += ws[w];
    const u32 s0 = part[tid * cpr];
    const u32 s1 = tid + 1 < R ? part[(tid + 1) * cpr] : all;
    tot[tid] = u64(s1 - s0);
  }
}

// The whole bucketing scan in one block when the count matrix is small (R x nb <= kBscanSmall
// entries, e.g. 8 ranks x 636 tiles at 1 Gbase over 8 ranks): exclusive offsets in place in
// destination-major order, the per-destination totals into tot[0, R) -- k_bscan_sum / top /
// down in one launch -- and the rest of the sync vector (k_dist_pack's words, thread 0).
constexpr u32 kBscanSmall = 16384;
static __global__ __launch_bounds__(1024) void k_bscan_small(u32* __restrict__ a, u32 R, u32 nb, u64* __restrict__ tot,
                                                             const Header* __restrict__ h,
                                                             const u64* __restrict__ ucount,
                                                             const unsigned char* __restrict__ bases) {
  __shared__ u32 ws[1024 / 64];
  __shared__ u32 rowst[kMaxRanks + 1];
  const u32 n = R * nb, tid = threadIdx.x, per = (n + 1023) / 1024, j0 = tid * per;
  const int lane = tid & 63;
  u32 x[kBscanSmall / 1024];
  u32 sum = 0;
#pragma unroll
  for (u32 i = 0; i < kBscanSmall / 1024; ++i) {
    x[i] = i < per && j0 + i < n ? a[j0 + i] : 0u;
    sum += x[i];
  }
  const u32 inc = wave_incl_scan(sum, lane);
  if (lane == 63) ws[tid >> 6] = inc;
  __syncthreads();
  u32 run = inc - sum;
  for (u32 w = 0; w < (tid >> 6); ++w) run += ws[w];
#pragma unroll
  for (u32 i = 0; i < kBscanSmall / 1024; ++i) {
    if (i < per && j0 + i < n) {
      const u32 j = j0 + i;
      if (j % nb == 0) rowst[j / nb] = run;   // a destination row starts here
      a[j] = run;
    }
    run += x[i];
  }
  if (tid == 1023) rowst[R] = run;   // (the last thread's run is the grand total)
  __syncthreads();
  if (tid < R) tot[tid] = u64(rowst[tid + 1] - rowst[tid]);
  if (tid == 0) {
    tot[R] = u64(h->overflow | h->leaf_overflow);
    tot[R + 1] = ucount ? *ucount : 0ull;
    const u64 e = h->err_offset;
    tot[R + 2] = e;
    tot[R + 3] = (e != ~0ull && bases) ? u64(bases[e]) : 0ull;
    tot[R + 4] = u64(h->predup);
    tot[R + 5] = u64(h->dense_fail);
  }
}

static __global__ __launch_bounds__(kBlock) void k_bscan_down(u32* __restrict__ a, u32 nb, u32 cpr,
                                                              const u32* __restrict__ coff) {
  constexpr int kPer = kScanChunk / kBlock;
  __shared__ u32 ws[kBlock / 64];
  const u32 row = blockIdx.x / cpr, c = blockIdx.x % cpr;
  u32* r = a + u64(row) * nb;
  const u32 j0 = c * kScanChunk + threadIdx.x * kPer;
  u32 x[kPer];
  u32 sum = 0;
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    x[i] = j0 + i < nb ? r[j0 + i] : 0u;
    sum += x[i];
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const u32 inc = wave_incl_scan(sum, lane);
  if (lane == 63) ws[wave] = inc;
  __syncthreads();
  u32 run = coff[blockIdx.x] + inc - sum;
  for (int w = 0; w < wave; ++w) run += ws[w];
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    if (j0 + i < nb) r[j0 + i] = run;
    run += x[i];
  }
}

// Stable: a block's records keep their order inside each destination segment (items
// in order, waves in order within an item, lanes in order within a wave), so every
// owner receives each source's records in the source's order.  Owners of levels that
// skip the local dedupe rely on it: the first record of a key is its first occurrence.
// split (the fused schedule's 6-byte records): record low 32 bits to skey as u32 [0, n), the
// high 16 to the u16 array `split`.
static __global__ __launch_bounds__(kBlock) void k_bucket_scatter(RecSrc s, const u32* __restrict__ boff, u32 nb,
                                                                  u64* __restrict__ skey, u32* __restrict__ sidx,
                                                                  unsigned short* __restrict__ split = nullptr) {
  constexpr int kWaves = kBlock / 64;
  // kPre items per round: their records loaded together (canonical-pair levels: straight-line,
  // in flight at once), one ballot pass per item, then ONE block-wide exclusive prefix over
  // the round's (item, wave, destination) counts -- two barriers per kPre items instead of
  // three per item.  Double-buffered counts: a round zeroes the previous round's buffer.
  constexpr int kPre = 8;
  __shared__ u32 cur[kMaxRanks];
  __shared__ u32 wcnt[2][kPre][kWaves][kMaxRanks];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < int(s.R)) cur[tid] = boff[u64(tid) * nb + blockIdx.x];
  for (int q = tid; q < 2 * kPre * kWaves * kMaxRanks; q += kBlock) (&wcnt[0][0][0][0])[q] = 0;
  __syncthreads();
  const u64 lt = (1ull << lane) - 1;
  const bool pre = (s.canon != nullptr || s.pre != nullptr) && s.leaves == nullptr;
  const u32 dbits = s.R > 1 ? 32u - u32(__clz(int(s.R - 1))) : 0u;   // bits of a destination
  int buf = 0;
  for (int e0 = 0; e0 < kItems; e0 += kPre, buf ^= 1) {
    u64 key[kPre];
    u32 lid[kPre], d[kPre], before[kPre];
    bool ok[kPre];
    if (pre) {
#pragma unroll
      for (int q = 0; q < kPre; ++q)
        ok[q] = rec_get_canon(s, u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid, key[q], lid[q]);
    }
#pragma unroll
    for (int q = 0; q < kPre; ++q) {
      if (!pre) {
        key[q] = 0;
        lid[q] = 0;
        ok[q] = rec_get(s, u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid, key[q], lid[q]);
      }
      d[q] = ok[q] ? rec_dest(s, key[q]) : 0u;
      // the lanes sharing this lane's destination: one ballot per destination bit
      u64 m = __ballot(ok[q]);
      for (u32 bit = 0; bit < dbits; ++bit) {
        const bool set = (d[q] >> bit) & 1u;
        const u64 bb = __ballot(ok[q] && set);
        m &= set ? bb : ~bb;
      }
      before[q] = u32(__popcll(m & lt));
      if (ok[q] && before[q] == 0) wcnt[buf][q][wave][d[q]] = u32(__popcll(m));
    }
    __syncthreads();   // this round's counts
    if (tid < int(s.R)) {   // per destination: exclusive offsets in (item, wave) order
#pragma unroll
      for (int q = 0; q < kPre; ++q)
        for (int w = 0; w < kWaves; ++w) wcnt[buf ^ 1][q][w][tid] = 0;   // (last round's, all read)
      u32 run = cur[tid];
#pragma unroll
      for (int q = 0; q < kPre; ++q)
        for (int w = 0; w < kWaves; ++w) {
          const u32 c = wcnt[buf][q][w][tid];
          wcnt[buf][q][w][tid] = run;
          run += c;
        }
      cur[tid] = run;
    }
    __syncthreads();   // this round's offsets
#pragma unroll
    for (int q = 0; q < kPre; ++q)
      if (ok[q]) {
        const u32 o = wcnt[buf][q][wave][d[q]] + before[q];
        if (split) {
          reinterpret_cast<u32*>(skey)[o] = u32(key[q]);
          split[o] = (unsigned short)(key[q] >> 32);
        } else {
          skey[o] = key[q];
        }
        sidx[o] = lid[q];
      }
  }
}

// ---- owner side ----------------------------------------------------------------
// Packed (default when it fits): one 8-B word per slot,
//     word = key << (R + 2) | state << 1      (bit 0 = 0: occupied; EMPTY = ~0)
// with the key re-encoded in K bits (leaves: the 4L-bit value; nodes: per child
// B-bit index + mirror + transpose) and state bit r = rank r holds the key,
// bit R = some rank holds it more than once.  A new key costs one CAS, a key
// already claimed one atomicOr (skipped when its bits are set).  The ids of
// C / D live beside it in ids[slot].
// Wide (fallback): Slot = {key ^ 1, ~state, id}, state bit 31 = repeats locally.
// memset 0xff clears both.
struct OwnTab {
  Slot* tab;     // wide
  u64* ptab;     // packed
  u32* ids;      // packed: id per slot
  u32 mask;
  u32 packed;
  u32 R;
  u32 B;         // packed node keys: child index bits
  u32 sh;        // packed: R + 2
  u32 nolocal;   // the senders skipped the local dedupe: a key may arrive twice from one rank
  u32* omin;     // nolocal: first (lowest) receive index of the key in each slot
};

__device__ __forceinline__ u64 own_pack_key(u64 key, int leaves, u32 B) {
  if (leaves) return key;
  auto enc = [B](u32 u) -> u64 {
    const u32 idx = u & kIdx;
    const u32 code = idx == kIdx ? ((1u << B) - 1u) : idx;
    return (u64(code) << 2) | (((u >> 29) & 1u) << 1) | ((u >> 30) & 1u);
  };
  return (enc(u32(key >> 31)) << (B + 2)) | enc(u32(key & 0x7fffffffu));
}

// state of a slot: bits [0, R) ranks holding the key, bit 31 repeats locally
__device__ __forceinline__ u32 own_state(const OwnTab& T, u32 s) {
  if (T.packed) {
    const u64 w = T.ptab[s];
    const u32 st = u32(w >> 1) & ((1u << (T.R + 1)) - 1u);
    return (st & ((1u << T.R) - 1u)) | ((st >> T.R) << 31);
  }
  return ~T.tab[s].pos;
}
__device__ __forceinline__ void own_set_id(const OwnTab& T, u32 s, u32 id) {
  if (T.packed) T.ids[s] = id;
  else T.tab[s].pad = id;
}
__device__ __forceinline__ u32 own_id(const OwnTab& T, u32 s) { return T.packed ? T.ids[s] : T.tab[s].pad; }

static __global__ __launch_bounds__(kBlock) void k_own_insert(const u64* __restrict__ rkey, u64 nrecv, Displ D,
                                                              u32 R, int leaves, OwnTab T, u32* __restrict__ oslot,
                                                              u64* __restrict__ ovf) {
  const u64 k = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= nrecv) return;
  const u32 src = seg_of(D, R, k);
  const u64 raw = rkey[k];
  const u64 key = leaves ? raw : (raw & ~kLocalMulti);
  const u32 lm = leaves ? 0u : u32(raw >> 63);
  if (T.packed) {
    const u64 pk = own_pack_key(key, leaves, T.B);
    const u64 bits = (u64((1u << src) | (lm << R))) << 1;
    const u64 mine = (pk << T.sh) | bits;
    u32 s = slot_hash(pk) & T.mask;
    for (u32 probe = 0; probe <= T.mask; ++probe) {
      u64 cur = T.ptab[s];
      if (cur == kEmpty) {
        cur = atomicCAS(&T.ptab[s], kEmpty, mine);
        if (cur == kEmpty) {
          oslot[k] = s;
          return;
        }
      }
      if ((cur >> T.sh) == pk) {
        if (T.nolocal) {   // a second record: the key repeats (first found by k_own_reply / k_own_first)
          const u64 b2 = bits | (u64(1u << R) << 1);
          if ((cur & b2) != b2) atomicOr(&T.ptab[s], b2);
        } else {
          // the reply only needs: the lowest rank, >= 2 ranks, repeats anywhere.  Once the
          // word shows two ranks with a lower one than src, this record changes none of them.
          const u32 ranks = u32(cur >> 1) & ((1u << R) - 1u);
          const bool settled = __popc(ranks) >= 2 && (ranks & ((1u << src) - 1u)) != 0;
          if (!settled && (cur & bits) != bits) atomicOr(&T.ptab[s], bits);
        }
        oslot[k] = s;
        return;
      }
      s = (s + 1) & T.mask;
    }
  } else {
    const u64 skey = key ^ 1ull;
    u32 s = slot_hash(skey) & T.mask;
    for (u32 probe = 0; probe <= T.mask; ++probe) {
      u64 cur = T.tab[s].key;
      if (cur == kEmpty) cur = atomicCAS(&T.tab[s].key, kEmpty, skey);
      if (cur == kEmpty || cur == skey) {
        const u32 rep = T.nolocal && cur == skey ? 1u : lm;
        atomicAnd(&T.tab[s].pos, ~((1u << src) | (rep << 31)));
        oslot[k] = s;
        return;
      }
      s = (s + 1) & T.mask;
    }
  }
  atomicOr(ovf, 1ull);
  oslot[k] = 0;
}

// reply bit 0: another rank before this one holds the key; bit 1: the key repeats globally
static __global__ __launch_bounds__(kBlock) void k_own_reply(const u32* __restrict__ oslot, u64 nrecv, Displ D,
                                                             u32 R, OwnTab T, unsigned char* __restrict__ rflag) {
  const u64 k = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= nrecv) return;
  const u32 src = seg_of(D, R, k);
  const u32 s = oslot[k];
  const u32 st = own_state(T, s);
  const u32 ranks = st & 0x7fffffffu;
  const u32 minr = u32(__ffs(ranks) - 1);
  const u32 shared = __popc(ranks) > 1;
  const u32 gm = shared | (st >> 31);
  if (T.nolocal) {
    // first = lowest receive index among the key's records (k_own_first settles the
    // repeated keys, marked 0x80 here); C / D run whenever the key repeats
    if (gm) atomicMin(&T.omin[s], u32(k));
    rflag[k] = gm ? (unsigned char)(0x80 | 6) : (unsigned char)0;
  } else {
    rflag[k] = (unsigned char)((minr != src) | (gm << 1) | (shared << 2));
  }
}

static __global__ __launch_bounds__(kBlock) void k_own_first(const u32* __restrict__ oslot, u64 nrecv, OwnTab T,
                                                             unsigned char* __restrict__ rflag) {
  const u64 k = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= nrecv) return;
  const unsigned char f = rflag[k];
  if (f & 0x80) rflag[k] = (unsigned char)((f & 6) | (T.omin[oslot[k]] != u32(k) ? 1 : 0));
}

// A level without the local dedupe (OwnTab::nolocal) through a position-packed table:
// every source sends its records in position order and the sources arrive in rank
// (= position) order, so the receive index orders a key's occurrences like their genome
// positions.  The owner hash-conses the records exactly like a single-device level
// (PackedTab::insert: one CAS per new key, atomicMin + marks only for repeats); the
// reply then comes from the marks, streaming.
static __global__ __launch_bounds__(kBlock) void k_own_insert_pos(const u64* __restrict__ rkey, u64 nrecv, u32 B,
                                                                  PackedTab T, Marks mk, u32* __restrict__ oslot,
                                                                  u32* __restrict__ ovf) {
  const u64 k = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= nrecv) return;
  oslot[k] = T.insert(own_pack_key(rkey[k] & ~kLocalMulti, 0, B), u32(k), mk, ovf);
}

// The same owner hash-cons without a table (non-repetitive levels: almost every key is
// new): the received keys are partitioned into NB buckets by the top bits of
// h = T.mix(key) (a bijection on the K key bits), per chunk of kDC receive indices
// (count, scan, scatter of (h's low bits, index in chunk) records), and each bucket is
// hash-consed by one workgroup in LDS.  Only keys with several records write anything:
// not-first marks, the first index's multi mark, and oslot = the first index (the id
// slot of k_own_setid / k_own_getid).  A bucket over kObCap records (a hot key) sets
// *ovf: the level is redone through the table.
constexpr u32 kObCap = 6144;     // records per bucket held in registers (6 per thread)
constexpr u32 kObSlots = 8192;   // LDS table: 64 KB keys + 32 KB first indices

struct OwnBkt {
  PackedTab T;   // mix over K bits (plan_table of the level's owner keys)
  u32 B;         // child index bits (own_pack_key)
  u32 K, bb;     // key bits, bucket bits
  u32 nch;       // chunks of kDC receive indices
  u64 nr;
  __device__ __forceinline__ u64 hash(u64 raw) const { return T.mix(own_pack_key(raw & ~kLocalMulti, 0, B)); }
};

// The owner dedupe as the single-device two-pass partition (k_bkt_fine, k_bkt_dedupe2<true>
// follow): pass 1 sorts each chunk of kPartChunk receive indices by the b1 coarse bits of
// h = T.mix(packed key) in LDS and writes the records back contiguously with the chunk's
// run table -- whole runs instead of k_ob_scatter's scattered 8-B stores.
// hi != null (the fused schedule's 6-byte records): rkey holds the records' low 32 bits as u32,
// hi their high 16; the record IS the key's mix (h's bits below the owner's), no own_pack_key.
static __global__ __launch_bounds__(kBktThreads) void k_ob_part(const u64* __restrict__ rkey, u64 nr, Bkt2Plan bp,
                                                                u32 B, u64* __restrict__ seg, u32* __restrict__ rt,
                                                                unsigned char* __restrict__ rflag,
                                                                const unsigned short* __restrict__ hi = nullptr) {
  extern __shared__ u64 stage[];   // kPartChunk records (dynamic)
  __shared__ u32 cur[(1u << kPartMaxB1) + 1];
  const u32 nb1 = 1u << bp.b1;
  for (u32 q = threadIdx.x; q <= nb1; q += kBktThreads) cur[q] = 0;
  const u64 g = blockIdx.x, j0 = g * kPartChunk;
  {   // the reply flags of this chunk's records start at 0 (the dedupe writes the repeats'); 16 B a store
    const u64 end = blockIdx.x + 1 == gridDim.x ? nr + 16 : j0 + kPartChunk;   // (rflag holds nr + 32 bytes)
    const u64 e0 = j0 / 16, e1 = (end + 15) / 16;
    for (u64 e = e0 + threadIdx.x; e < e1; e += kBktThreads) reinterpret_cast<uint4*>(rflag)[e] = make_uint4(0, 0, 0, 0);
  }
  u64 x[kPartItems];
#pragma unroll
  for (int e = 0; e < kPartItems; ++e) {
    const u64 j = j0 + u64(e) * kBktThreads + threadIdx.x;
    x[e] = j >= nr ? 0ull : hi ? u64(reinterpret_cast<const u32*>(rkey)[j]) | (u64(hi[j]) << 32) : rkey[j];
  }
  __syncthreads();
  const u32 sh1 = bp.K - bp.b1;
  const u64 lowmask = sh1 >= 64 ? ~0ull : (1ull << sh1) - 1;
  u64 r[kPartItems];
  u32 slot[kPartItems];   // coarse bucket << 16 | rank in it
#pragma unroll
  for (int e = 0; e < kPartItems; ++e) {
    const u64 j = j0 + u64(e) * kBktThreads + threadIdx.x;
    slot[e] = ~0u;
    if (j >= nr) continue;
    const u64 h = hi ? x[e] : bp.T.mix(own_pack_key(x[e] & ~kLocalMulti, 0, B));
    const u32 c = bp.b1 ? u32(h >> sh1) : 0u;
    r[e] = ((h & lowmask) << kPartLog) | (j - j0);
    slot[e] = (c << 16) | atomicAdd(&cur[c], 1u);
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
}

static __global__ __launch_bounds__(1024) void k_ob_count(const u64* __restrict__ rkey, OwnBkt P,
                                                          u32* __restrict__ cnt) {
  __shared__ u32 hist[4096];
  const u32 NB = 1u << P.bb;
  for (u32 b = threadIdx.x; b < NB; b += 1024) hist[b] = 0;
  __syncthreads();
  const u64 k0 = u64(blockIdx.x) * kDC;
  for (u32 q0 = 0; q0 < kDC; q0 += 1024 * 8) {
    u64 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u64 k = k0 + q0 + u32(j) * 1024 + threadIdx.x;
      x[j] = k < P.nr ? rkey[k] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u64 k = k0 + q0 + u32(j) * 1024 + threadIdx.x;
      if (k < P.nr) atomicAdd(&hist[u32(P.hash(x[j]) >> (P.K - P.bb))], 1u);
    }
  }
  __syncthreads();
  for (u32 b = threadIdx.x; b < NB; b += 1024) cnt[u64(b) * P.nch + blockIdx.x] = hist[b];
}

static __global__ __launch_bounds__(1024) void k_ob_scatter(const u64* __restrict__ rkey, OwnBkt P,
                                                            const u32* __restrict__ off, u64* __restrict__ rec) {
  __shared__ u32 cur[4096];
  const u32 NB = 1u << P.bb, ch = blockIdx.x;
  for (u32 b = threadIdx.x; b < NB; b += 1024) cur[b] = off[u64(b) * P.nch + ch];
  __syncthreads();
  const u64 k0 = u64(ch) * kDC;
  const u64 lowmask = (1ull << (P.K - P.bb)) - 1ull;
  for (u32 q0 = 0; q0 < kDC; q0 += 1024 * 8) {
    u64 x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u64 k = k0 + q0 + u32(j) * 1024 + threadIdx.x;
      x[j] = k < P.nr ? rkey[k] : 0ull;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const u32 q = q0 + u32(j) * 1024 + threadIdx.x;
      if (k0 + q >= P.nr) continue;
      const u64 h = P.hash(x[j]);
      const u32 d = atomicAdd(&cur[u32(h >> (P.K - P.bb))], 1u);
      rec[d] = ((h & lowmask) << kDLog) | q;
    }
  }
}

static __global__ __launch_bounds__(1024) void k_ob_dedupe(const u64* __restrict__ rec, const u32* __restrict__ off,
                                                           OwnBkt P, Marks mk, u32* __restrict__ oslot,
                                                           u32* __restrict__ ovf) {
  __shared__ unsigned long long s_key[kObSlots];
  __shared__ u32 s_pos[kObSlots];
  __shared__ u32 s_dup[kObSlots / 32];
  extern __shared__ u32 s_run[];   // nch + 1 run starts of the bucket
  constexpr int E = kObCap / 1024;
  const u64 b = blockIdx.x;
  const u32 start = off[b * P.nch], end = off[(b + 1) * P.nch];
  if (end - start > kObCap) {
    if (threadIdx.x == 0) atomicOr(ovf, 1u);
    return;
  }
  for (u32 q = threadIdx.x; q <= P.nch; q += 1024) s_run[q] = off[b * P.nch + q];
  for (u32 q = threadIdx.x; q < kObSlots; q += 1024) {
    s_key[q] = kEmpty;
    s_pos[q] = ~0u;
  }
  for (u32 q = threadIdx.x; q < kObSlots / 32; q += 1024) s_dup[q] = 0;
  u64 x[E];
  u32 slot[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const u32 i = start + u32(e) * 1024 + threadIdx.x;
    x[e] = i < end ? rec[i] : kEmpty;
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (x[e] == kEmpty) continue;
    const u64 key = x[e] >> kDLog;
    u32 h = u32((u64(u32(bkt_hash(key))) * kObSlots) >> 32);
    for (;;) {
      unsigned long long c = s_key[h];
      if (c == kEmpty) c = atomicCAS(&s_key[h], kEmpty, (unsigned long long)key);
      if (c == key) atomicOr(&s_dup[h >> 5], 1u << (h & 31));
      if (c == kEmpty || c == key) break;
      h = h + 1 == kObSlots ? 0u : h + 1;
    }
    slot[e] = h;
  }
  __syncthreads();
  u32 pos[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {   // only keys with several records need their indices
    pos[e] = ~0u;
    if (x[e] == kEmpty || !((s_dup[slot[e] >> 5] >> (slot[e] & 31)) & 1u)) continue;
    const u32 i = start + u32(e) * 1024 + threadIdx.x;
    u32 lo = 0, hi = P.nch - 1;   // chunk: the last run starting at or before record i
    while (lo < hi) {
      const u32 mid = (lo + hi + 1) >> 1;
      if (s_run[mid] <= i) lo = mid;
      else hi = mid - 1;
    }
    pos[e] = (lo << kDLog) | u32(x[e] & (kDC - 1));
    atomicMin(&s_pos[slot[e]], pos[e]);
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if (pos[e] == ~0u) continue;
    const u32 first = s_pos[slot[e]];
    oslot[pos[e]] = first;
    if (pos[e] != first) mk.nf[pos[e]] = kNfNot;
    else mk.multi[pos[e]] = 1;
  }
}

// Reply from the marks: not first (1), repeats (2), and C / D whenever the key repeats (4),
// like k_own_reply + k_own_first.
static __global__ __launch_bounds__(kBlock) void k_own_reply_marks(const unsigned char* __restrict__ nf,
                                                                   const unsigned char* __restrict__ multi,
                                                                   u64 nrecv, unsigned char* __restrict__ rflag) {
  const u64 k = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (k >= nrecv) return;
  rflag[k] = nf[k] ? 7 : (multi[k] ? 6 : 0);
}

// Per-record flags (reply bits): 1 not globally first, 2 repeats globally, 4 held by >= 2 ranks.
// C: the first holder of a shared key sends its id; D: every other holder receives it.
__device__ __forceinline__ bool want_c(unsigned char f) { return (f & 1) == 0 && (f & 4); }
__device__ __forceinline__ bool want_d(unsigned char f) { return (f & 1) != 0; }

// C and D records travel as (index within the sender->owner segment, id) pairs, so
// neither side needs them in order: they are appended per segment with wave-aggregated
// cursors into the segment's span of the record layout (at most every record of a
// segment is selected) and sent from there (Transport::alltoallv_at).
__device__ __forceinline__ u32 wave_append(u32* __restrict__ cur, u32 q, bool want) {
  const int lane = threadIdx.x & 63;
  const u64 lt = (1ull << lane) - 1;
  u32 slot = 0;
  u64 left = __ballot(want);
  while (left) {                                   // one atomic per distinct segment in the wave
    const int leader = __ffsll((long long)left) - 1;
    const u32 ql = __shfl(q, leader, 64);
    const u64 m = __ballot(want && q == ql);
    u32 base = 0;
    if (lane == leader) base = atomicAdd(&cur[ql], u32(__popcll(m)));
    base = __shfl(base, leader, 64);
    if (want && q == ql) slot = base + u32(__popcll(m & lt));
    left &= ~m;
  }
  return slot;
}

// C at the owner: the first holder's global id of every shared key.  cnt.d[s] = C records
// from source s, packed at the start of s's segment; the grid covers their sum only.
__device__ __forceinline__ u64 packed_at(const Displ& D, const Displ& cnt, u32 R, u64 i) {   // i-th packed record
  u32 s = 0;
  while (s + 1 < R && i >= cnt.d[s]) i -= cnt.d[s++];
  return D.d[s] + i;
}
static __global__ __launch_bounds__(kBlock) void k_own_setid(const u64* __restrict__ rc, u64 ntot, Displ D,
                                                             Displ cnt, u32 R, const u32* __restrict__ oslot,
                                                             OwnTab T) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= ntot) return;
  const u64 k = packed_at(D, cnt, R, i);
  const u32 s = seg_of(D, R, k);
  const u64 v = rc[k];
  own_set_id(T, oslot[D.d[s] + u32(v)], u32(v >> 32));
}

// Per-segment append over a tile of kTile records: pass 1 counts the selected records per
// segment (wave ballots into LDS), one global atomic per segment reserves the block's
// span, pass 2 recomputes the selection and writes.  `sel(k, q)` -> selected, segment q.
template <class Sel, class Put>
__device__ __forceinline__ void tile_append(u64 n, u32 R, u32* __restrict__ gcur, Sel sel, Put put) {
  __shared__ u32 cnt[kMaxRanks], base[kMaxRanks];
  const int tid = threadIdx.x;
  if (tid < int(R)) cnt[tid] = 0;
  __syncthreads();
  const u64 k0 = u64(blockIdx.x) * kTile;
  for (int e = 0; e < kItems; ++e) {
    const u64 k = k0 + u64(e) * kBlock + tid;
    u32 q = 0;
    const bool want = k < n && sel(k, q);
    (void)wave_append(cnt, q, want);
  }
  __syncthreads();
  if (tid < int(R)) {
    base[tid] = cnt[tid] ? atomicAdd(&gcur[tid], cnt[tid]) : 0u;
    cnt[tid] = 0;
  }
  __syncthreads();
  for (int e = 0; e < kItems; ++e) {
    const u64 k = k0 + u64(e) * kBlock + tid;
    u32 q = 0;
    const bool want = k < n && sel(k, q);
    const u32 slot = wave_append(cnt, q, want);
    if (want) put(k, q, base[q] + slot);
  }
}

// D at the owner: every other holder's record gets the id back (appended per source).
static __global__ __launch_bounds__(kBlock) void k_own_getid(const u32* __restrict__ oslot, u64 nrecv, Displ D,
                                                             u32 R, const unsigned char* __restrict__ rflag,
                                                             OwnTab T, u32* __restrict__ dcur,
                                                             u64* __restrict__ dval) {
  tile_append(
      nrecv, R, dcur,
      [&](u64 k, u32& s) {
        if (!want_d(rflag[k])) return false;
        s = seg_of(D, R, k);
        return true;
      },
      [&](u64 k, u32 s, u32 slot) { dval[D.d[s] + slot] = u64(k - D.d[s]) | (u64(own_id(T, oslot[k])) << 32); });
}

// ... the same from the owner dedupe's list of not-first records (k_bkt_dedupe2<true>), in
// any order: the D records of a segment need no order.
static __global__ __launch_bounds__(kBlock) void k_own_getid_list(const u32* __restrict__ list, u64 n,
                                                                  const u32* __restrict__ oslot, Displ D, u32 R,
                                                                  OwnTab T, u32* __restrict__ dcur,
                                                                  u64* __restrict__ dval) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const u32 k = list[i];
  const u32 s = seg_of(D, R, k);
  const u32 slot = atomicAdd(&dcur[s], 1u);
  dval[D.d[s] + slot] = u64(k - D.d[s]) | (u64(own_id(T, oslot[k])) << 32);
}

// ---- sender side ---------------------------------------------------------------

// Reply flags -> per local unique (gnf: not globally first, gmul: repeats globally), and
// the C / D record counts per owner (cnt[q], cnt[R + q]: the sync2 vector).  One tile of
// kTile records per block.
// gnf / gmul arrive zeroed (k_node_keys, or the exchange's memsets): only the set flags are
// written.  nfl (optional): the positions not globally first, counted in *nnf and listed while
// there are at most kNfListCap of them (k_dist_rank's sparse path).
// Owner replies packed 2 bits per record (the fused schedule, gcz_dist_fast.h): per source
// segment s of the owner's receive layout D, ceil(n_s / 4) bytes at P4.d[s]; codes 0 (a single
// key), 1 (the first of a repeated key: reply 6), 2 (not first: reply 7).
// (sd / p4: the two Displ's starts staged in LDS -- a kernel argument indexed by a register
// would go through scratch)
// (the segment search first, for every record of a round, then the loads together)
__device__ __forceinline__ u64 reply_at2(const u64* sd, const u64* p4, u32 R, u64 k, u32& q, u32& sh) {
  while (q + 1 < R && k >= sd[q + 1]) ++q;   // (k only grows along a thread's records)
  const u64 i = k - sd[q];
  sh = 2 * u32(i & 3);
  return p4[q] + (i >> 2);
}
__device__ __forceinline__ unsigned char reply_code2(unsigned char byte, u32 sh) {
  const u32 c = (u32(byte) >> sh) & 3u;
  return c == 0 ? 0 : c == 1 ? 6 : 7;
}

// p2 != null: the replies arrive packed (reply_at2 / reply_code2, P4 the packed segment starts), sflag unused;
// the send buffer's segments may have gaps: owner q's records are [SD.d[q], SE.d[q]).
static __global__ __launch_bounds__(kBlock) void k_dist_flags(const u32* __restrict__ sidx, u64 nsent,
                                                              const unsigned char* __restrict__ sflag,
                                                              unsigned char* __restrict__ gnf,
                                                              unsigned char* __restrict__ gmul, Displ SD, u32 R,
                                                              u64* __restrict__ cnt, u32* __restrict__ clist,
                                                              u32* __restrict__ lcnt, u32* __restrict__ nfl,
                                                              u32* __restrict__ nnf,
                                                              const unsigned char* __restrict__ p2 = nullptr,
                                                              Displ P4 = {}, Displ SE = {}) {
  __shared__ u32 hc[kMaxRanks], hd[kMaxRanks];
  __shared__ u64 s_sd[kMaxRanks + 1], s_p4[kMaxRanks + 1], s_se[kMaxRanks + 1];
  const int tid = threadIdx.x;
  if (tid < int(R)) { hc[tid] = 0; hd[tid] = 0; }
  if (tid <= kMaxRanks) {
    s_sd[tid] = SD.d[tid];
    s_p4[tid] = P4.d[tid];
    s_se[tid] = SE.d[tid];
  }
  __syncthreads();
  const u64 k0 = u64(blockIdx.x) * kTile;
  constexpr int kB = 8;   // records whose index and flag are loaded together
  u32 q2 = 0;   // the packed replies' segment of this thread's records
  if (p2)
    while (q2 + 1 < R && k0 >= s_sd[q2 + 1]) ++q2;
  for (int e0 = 0; e0 < kItems; e0 += kB) {
    u32 li[kB];
    unsigned char fl[kB];
    u64 at[kB];
    u32 sh[kB];
    bool ok[kB];   // a record (p2: segments with gaps -- [SD.d[q], SE.d[q]) holds owner q's records)
    if (p2) {
#pragma unroll
      for (int b = 0; b < kB; ++b) {
        const u64 k = k0 + u64(e0 + b) * kBlock + tid;
        sh[b] = 0;
        at[b] = k < nsent ? reply_at2(s_sd, s_p4, R, k, q2, sh[b]) : 0ull;
        ok[b] = k < nsent && k < s_se[q2];
      }
    } else {
#pragma unroll
      for (int b = 0; b < kB; ++b) ok[b] = k0 + u64(e0 + b) * kBlock + tid < nsent;
    }
#pragma unroll
    for (int b = 0; b < kB; ++b) {
      const u64 k = k0 + u64(e0 + b) * kBlock + tid;
      li[b] = ok[b] ? sidx[k] : 0u;
      fl[b] = !ok[b] ? 0 : p2 ? p2[at[b]] : sflag[k];
    }
    if (p2) {
#pragma unroll
      for (int b = 0; b < kB; ++b) fl[b] = reply_code2(fl[b], sh[b]);   // (no record: byte 0 -> 0)
    }
#pragma unroll
    for (int b = 0; b < kB; ++b) {
      const u64 k = k0 + u64(e0 + b) * kBlock + tid;
      const unsigned char f = fl[b];
      if (ok[b]) {
        if (f & 1) gnf[li[b]] = 1;
        if (f & 2) gmul[li[b]] = 1;
      }
      if (nfl) {   // (one atomic per wave with such records, none once the list is over its cap)
        const bool nf = ok[b] && (f & 1);
        const u64 m = __ballot(nf);
        if (m) {
          const int lane = tid & 63, lead = __ffsll((long long)m) - 1;
          u32 base = 0;
          if (lane == lead)
            base = *reinterpret_cast<volatile u32*>(nnf) > kNfListCap ? ~0u : atomicAdd(nnf, u32(__popcll(m)));
          base = __shfl(base, lead, 64);
          if (nf && base != ~0u) {
            const u32 i = base + u32(__popcll(m & ((1ull << lane) - 1ull)));
            if (i < kNfListCap) nfl[i] = li[b];
          }
        }
      }
      const u32 q = (want_c(f) || want_d(f)) ? seg_of(SD, R, k) : 0u;
      (void)wave_append(hc, q, ok[b] && want_c(f));
      (void)wave_append(hd, q, ok[b] && want_d(f));
      const u32 cs = wave_append(lcnt, 0u, ok[b] && want_c(f));   // (k_dist_cvals' list)
      if (ok[b] && want_c(f)) clist[cs] = u32(k);
    }
  }
  __syncthreads();
  if (tid < int(R)) {
    if (hc[tid]) atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[tid]), (unsigned long long)hc[tid]);
    if (hd[tid]) atomicAdd(reinterpret_cast<unsigned long long*>(&cnt[R + tid]), (unsigned long long)hd[tid]);
  }
}

// Look-ahead on a level without the local dedupe (lid = position): pairs (2j, 2j+1) of the
// next level whose children both repeat globally (the odd tail pairs with null and goes
// through the table when its left child repeats; rec_get's singleton test).  None on any
// rank: every next-level pair holds a singleton, so the next level is direct.
static __global__ __launch_bounds__(kBlock) void k_lookahead(const unsigned char* __restrict__ gmul, u64 n,
                                                             u64* __restrict__ out) {
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  bool hashed = false;
  if (2 * j < n) hashed = gmul[2 * j] && (2 * j + 1 >= n || gmul[2 * j + 1]);
  const u64 m = __ballot(hashed);
  if ((threadIdx.x & 63) == 0 && m)
    atomicAdd(reinterpret_cast<unsigned long long*>(out), (unsigned long long)__popcll(m));
}

// Rank of each globally-first local unique among them (local order); total -> *count_out.
// Such a unique goes straight to its place in the rank's output slice; gid keeps its local
// rank tagged kLocalId (the global offset is known only after the count allgather and is
// added where the id is used: k_dist_cvals, k_dist_remap).
constexpr u32 kLocalId = kLocalIdBit;
// nfl / nnf (optional): k_dist_flags' list of the positions not globally first; at most
// kNfListCap of them: ranked without the look-back chain (SparseTile).
template <class T>
__global__ __launch_bounds__(kBlock) void k_dist_rank(const unsigned char* __restrict__ gnf,
                                                      const u64* __restrict__ ucount, u32* __restrict__ gid,
                                                      u64* __restrict__ desc, u32* __restrict__ ticket,
                                                      u64* __restrict__ count_out, const T* __restrict__ scratch,
                                                      T* __restrict__ out, const u32* __restrict__ nfl = nullptr,
                                                      const u32* __restrict__ nnf = nullptr) {
  __shared__ u32 s_tile;
  __shared__ u32 s_pre[kGroupsPerTile];
  const u64 u = *ucount;
  if (u64(blockIdx.x) * kTile >= u) {          // grid sized for the capacity: surplus tiles leave
    return;
  }
  if (nfl && *nnf <= kNfListCap) {
    const u32 c = *nnf;
    const SparseTile<kItems> st = sparse_tile<kItems>(nfl, c, u64(blockIdx.x) * kTile);
    if (blockIdx.x == 0 && threadIdx.x == 0) *count_out = u - c;
#pragma unroll
    for (int e = 0; e < kItems; ++e) {
      const u32 k = u32(e) * kBlock + threadIdx.x;
      const u64 j = st.base + k;
      if (j < u && !st.listed(k)) {
        const u32 r = u32(j - st.nb(k));
        gid[j] = r | kLocalId;
        if (out) out[r] = scratch[j];
      }
    }
    return;
  }
  TileScan<kItems> ts;
  tile_scan(ts, &s_tile, s_pre, gnf, 0, u, 0, desc, ticket, count_out);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const u64 lt = (1ull << lane) - 1;
#pragma unroll
  for (int e = 0; e < kItems; ++e) {
    const u64 j = ts.base + u64(e) * kBlock + tid;
    if (j < u && ((ts.mask[e] >> lane) & 1ull)) {
      const u32 r = s_pre[e * 4 + wave] + u32(__popcll(ts.mask[e] & lt));
      gid[j] = r | kLocalId;
      if (out) out[r] = scratch[j];   // (null: the fused schedule writes the nodes later, k_fl_l0)
    }
  }
}

// C at the sender: the first holder of a shared key sends (segment index, global id); the
// grid covers k_dist_flags' list of those records only.
static __global__ __launch_bounds__(kBlock) void k_dist_cvals(const u32* __restrict__ clist, u64 n,
                                                              const u32* __restrict__ sidx, Displ SD, u32 R,
                                                              const u32* __restrict__ gid, u32 off,
                                                              u32* __restrict__ ccur, u64* __restrict__ cval) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= n) return;
  const u32 k = clist[i];
  const u32 q = seg_of(SD, R, k);
  const u32 slot = atomicAdd(&ccur[q], 1u);
  cval[SD.d[q] + slot] = u64(k - SD.d[q]) | (u64(off + (gid[sidx[k]] & ~kLocalId)) << 32);
}

// D at the sender: cnt.d[q] records from owner q, packed at the start of q's segment; the
// grid covers their sum only.
static __global__ __launch_bounds__(kBlock) void k_dist_dvals(const u32* __restrict__ sidx, u64 ntot, Displ SD,
                                                              Displ cnt, u32 R, const u64* __restrict__ dval,
                                                              u32* __restrict__ gid) {
  const u64 i = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (i >= ntot) return;
  const u64 k = packed_at(SD, cnt, R, i);
  const u32 q = seg_of(SD, R, k);
  const u64 v = dval[k];
  gid[sidx[SD.d[q] + u32(v)]] = u32(v >> 32);
}

// Local words -> global ids; locally-first elements whose key repeats on
// another rank are marked multi (the next level's singleton test).
static __global__ __launch_bounds__(kBlock) void k_dist_remap(u32* __restrict__ words, u64 p,
                                                              const unsigned char* __restrict__ nf,
                                                              unsigned char* __restrict__ multi,
                                                              const u32* __restrict__ gid,
                                                              const unsigned char* __restrict__ gmul, u32 off,
                                                              const unsigned char* __restrict__ gmark) {
  const u64 j = u64(blockIdx.x) * kBlock + threadIdx.x;
  if (j >= p) return;
  // the word, its marks and the seeding mark in one round trip, then the id lookups
  const unsigned char gm = gmark ? gmark[j] : 0;
  const u32 w = words[j];
  const unsigned char f = multi ? nf[j] : 0;
  if (gmark && gm == kNfGlobal) return;   // seeded leaf: the word holds its global id
  const u32 lid = w & kIdx;
  const u32 g = gid[lid];
  const unsigned char gmu = multi && f == kNfMaybe ? gmul[lid] : 0;
  words[j] = ((g & kLocalId) ? (g & ~kLocalId) + off : g) | (w & kBits);
  if (gmu) multi[j] = 1;
}

static __global__ void k_dist_pack(const Header* __restrict__ h, const u64* __restrict__ ucount,
                                   const unsigned char* __restrict__ bases, DistHdr* __restrict__ dh, u32 R) {
  dh->sync[R] = u64(h->overflow | h->leaf_overflow);
  dh->sync[R + 1] = ucount ? *ucount : 0ull;
  const u64 e = h->err_offset;
  dh->sync[R + 2] = e;
  dh->sync[R + 3] = (e != ~0ull && bases) ? u64(bases[e]) : 0ull;
  dh->sync[R + 4] = u64(h->predup);
  dh->sync[R + 5] = u64(h->dense_fail);
}

// A node level without the local dedupe: every pair is its own local unique (local id =
// position), so the owners alone hash-cons it.  Writes what node_level would leave
// behind for the exchange: local words, canonical pairs (the finalize source), marks
// (all locally first, none known to repeat) and the local unique count.
// gid != null: the input words still hold the previous level's LOCAL ids (its remap was
// deferred to here, k_dist_remap's translation), so the pass reads each word once.
// blockcnt != null: also the bucketing's per-tile owner counts (k_bucket_count over `rs`,
// the level's record source, whose canonical pairs and marks this pass writes); one tile of
// kTile pairs per block, like the bucketing grid.
static __global__ __launch_bounds__(kBlock) void k_node_keys(const u32* __restrict__ in, u64 n, u64 p,
                                                             u32* __restrict__ words, uint2* __restrict__ pairs,
                                                             unsigned char* __restrict__ nf,
                                                             unsigned char* __restrict__ multi,
                                                             u64* __restrict__ count_out,
                                                             const u32* __restrict__ gid, u32 off, RecSrc rs,
                                                             u32* __restrict__ blockcnt, u32 nb,
                                                             const unsigned char* __restrict__ gmark,
                                                             unsigned char* __restrict__ gnf,
                                                             unsigned char* __restrict__ gmul, u64* __restrict__ ddesc,
                                                             u32 skip_null = 0) {
  __shared__ u32 h[kMaxRanks];
  const int tid = threadIdx.x;
  // what the exchange's sender side expects zeroed for this tile (local uniques = positions):
  // the global flags (k_dist_flags sets the sent ones) and the rank scan's look-back word
  if (gnf) {
    const u64 end = blockIdx.x + 1 == gridDim.x ? p + 1 : std::min<u64>(u64(blockIdx.x + 1) * kTile, p + 1);
    const u64 e0 = u64(blockIdx.x) * kTile / 16, e1 = (end + 15) / 16;
    for (u64 e = e0 + tid; e < e1; e += kBlock) {
      reinterpret_cast<uint4*>(gnf)[e] = make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint4*>(gmul)[e] = make_uint4(0, 0, 0, 0);
    }
    if (tid == 0) ddesc[blockIdx.x] = 0;
  }
  if (blockcnt) {
    if (tid < int(rs.R)) h[tid] = 0;
    __syncthreads();
  }
  if (blockIdx.x == 0 && tid == 0) *count_out = p;
  // kB items at a time: their pairs (and the previous level's marks) loaded together, then
  // their leaf-id lookups together, then the work -- no dependent loads per item.  The
  // bucketing count takes the record straight from registers (a pair with a singleton
  // child is not sent: rec_get's rule).
  constexpr int kB = 8;
  auto glob = [&](u32 w, u64 strand, unsigned char gm, u32 g) {
    if ((w & kIdx) == kIdx) return w;                            // the odd tail's null
    if (gmark && gm == kNfGlobal) return w;                      // seeded: already global
    (void)strand;
    return ((g & kLocalId) ? (g & ~kLocalId) + off : g) | (w & kBits);
  };
  for (int e0 = 0; e0 < kItems; e0 += kB) {
    u32 L[kB], Rw[kB];
    uchar2 pf[kB], pm[kB];
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      const u64 j = u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid;
      L[q] = Rw[q] = kNullWord;
      pf[q] = pm[q] = make_uchar2(1, 1);
      if (j < p) {
        load_pair(in, n, j, L[q], Rw[q]);
        if (blockcnt && rs.prev_nf) {
          if (2 * j + 1 < n) {
            pf[q] = reinterpret_cast<const uchar2*>(rs.prev_nf)[j];
            pm[q] = reinterpret_cast<const uchar2*>(rs.prev_multi)[j];
          } else {
            pf[q] = make_uchar2(rs.prev_nf[2 * j], 1);
            pm[q] = make_uchar2(rs.prev_multi[2 * j], 1);
          }
        }
      }
    }
    if (gid) {
      u32 gl[kB], gr[kB];
      unsigned char ml[kB], mr[kB];
#pragma unroll
      for (int q = 0; q < kB; ++q) {
        const u64 j = u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid;
        const bool okj = j < p;
        gl[q] = okj && (L[q] & kIdx) != kIdx ? gid[L[q] & kIdx] : 0u;
        gr[q] = okj && (Rw[q] & kIdx) != kIdx ? gid[Rw[q] & kIdx] : 0u;
        ml[q] = okj && gmark ? gmark[2 * j] : 0;
        mr[q] = okj && gmark && 2 * j + 1 < n ? gmark[2 * j + 1] : 0;
      }
#pragma unroll
      for (int q = 0; q < kB; ++q) {
        const u64 j = u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid;
        L[q] = glob(L[q], 2 * j, ml[q], gl[q]);
        Rw[q] = glob(Rw[q], 2 * j + 1, mr[q], gr[q]);
      }
    }
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      const u64 j = u64(blockIdx.x) * kTile + u64(e0 + q) * kBlock + tid;
      if (j >= p) continue;
      const u32 l = L[q], r = Rw[q];
      u32 cl, cr, m, t;
      node_canonical(l, r, cl, cr, m, t);
      const u32 v = ulw(l) == ulw(xf(r, 1, 0));
      pairs[j] = make_uint2(cl, cr);
      words[j] = make_word(u32(j), m, t, v);
      // skip_null (the fused schedule, whose keys carry code labels without a null code): the
      // genome's last pair, with the null child, is the only pair of its class -- globally
      // first and unique without an exchange
      const bool lone = skip_null && (r & kIdx) == kIdx;
      nf[j] = lone ? kNfDone : kNfMaybe;
      multi[j] = 0;
      if (blockcnt && !lone) {
        const bool single = rs.prev_nf && ((pf[q].x == 0 && pm[q].x == 0) || (pf[q].y == 0 && pm[q].y == 0));
        if (!single) atomicAdd(&h[owner_of((u64(ulw(cl)) << 31) | ulw(cr), rs.R)], 1u);
      }
    }
  }
  if (blockcnt) {
    __syncthreads();
    if (tid < int(rs.R)) blockcnt[u64(tid) * nb + blockIdx.x] = h[tid];
  }
}

static __global__ void k_dist_final(const Header* __restrict__ h, DistHdr* __restrict__ dh, int tail0, int D,
                                    int has_tail) {
  dh->final_vec[0] = u64(h->overflow | h->leaf_overflow);
  dh->final_vec[1] = has_tail ? u64(h->root) : 0ull;
  dh->final_vec[2] = u64(tail0);
  for (int k = 0; k < GCZ_MAX_LAYERS; ++k)
    dh->final_vec[4 + k] = (has_tail && k >= tail0 && k < D) ? h->count[kLayerSlot + k] : 0ull;
}

static __global__ void k_set_u64(u64* p, u64 v) { *p = v; }

}  // namespace gcz_dev
